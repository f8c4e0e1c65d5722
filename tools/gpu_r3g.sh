#!/bin/bash
# Round-3 session g: where k_jr's window fills cost (diagnostic builds, timing only).
set -u
mkdir -p gpurun_out
run() {
  local l=$1; shift
  env "$@" timeout -k 10 240 python -u tools/sponge_ab.py --label $l >> gpurun_out/sponge_r3g.log 2> gpurun_out/sponge_r3g.err || { tail -5 gpurun_out/sponge_r3g.err; exit 1; }
  tail -1 gpurun_out/sponge_r3g.log
}
run base X=1
run nowait PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_nowait.so
run nold PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_nold.so
run noldab PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_nospec_nold.so
run noldab_nospec PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_nospec_nold.so PRIO3GPU_SPECULATE=0
run base2 X=1
