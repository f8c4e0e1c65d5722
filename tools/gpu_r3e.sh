#!/bin/bash
# Round-3 session e: sponge cost attribution with diagnostic builds (tools/sponge_ab.py).
set -u
mkdir -p gpurun_out
run() {  # run LABEL ENV...
  local l=$1; shift
  env "$@" timeout -k 10 240 python -u tools/sponge_ab.py --label $l >> gpurun_out/sponge_r3e.log 2> gpurun_out/sponge_r3e_$l.err
  local r=$?
  tail -1 gpurun_out/sponge_r3e.log
  [ $r -ne 0 ] && { tail -5 gpurun_out/sponge_r3e_$l.err; exit $r; }
  return 0
}
run base X=1
run nospec PRIO3GPU_SPECULATE=0
run nold PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_nold.so
run noab PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_noab.so
run both PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_both.so
run both_nospec PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_both.so PRIO3GPU_SPECULATE=0
run nost PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_nost.so
run base2 X=1
exit 0
