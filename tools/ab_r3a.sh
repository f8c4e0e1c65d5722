tools/ab.sh r3a "base:X=1" "e1:PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_e1.so" "j1:PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_j1.so" "ej:PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_ej.so" "base2:X=1"
