#!/bin/bash
# Round-3 session k: where the FLP query time goes (inversion share), per config.
set -u
mkdir -p gpurun_out
for c in sumvec histogram sum; do
  for v in base noinv; do
    e=X=1; [ $v = noinv ] && e=PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_noinv.so
    env $e timeout -k 10 300 python -u tools/sponge_ab.py --config $c --query 1 --reps 2 --label ${c}_$v >> gpurun_out/flp_r3k.log 2> gpurun_out/flp_r3k.err || { tail -5 gpurun_out/flp_r3k.err; exit 1; }
    tail -1 gpurun_out/flp_r3k.log
  done
done
