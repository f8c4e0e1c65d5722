#!/bin/bash
# Round-6 sponge floor: per-launch times of the SumVec sponge kernels (tools/sponge_ab.py) in the
# product build and in timing-only variant builds (wrong bytes), alternated so box drift shows:
#   jrnl  k_jr issues no window fills            exns   k_expand stores nothing
#   jrfix k_jr refills block 1's window always   exfix  k_expand stores over the row's first bytes
# (the *fix variants keep every instruction but take HBM out: the same lines every block).
#   usage: tools/r6_diag.sh LIB...   (janus_amd/lib/libprio3gpu_LIB.so; "prod" = the product build)
set -o pipefail
O=gpurun_out/r6_diag; mkdir -p $O
for rep in 1 2; do
  for lib in "$@"; do
    if [ $lib = prod ]; then P=janus_amd/lib/libprio3gpu.so; else P=janus_amd/lib/libprio3gpu_$lib.so; fi
    PRIO3GPU_LIB=$P timeout -k 10 300 python -u tools/sponge_ab.py --config sumvec --reps 3 \
      --label $lib > $O/${lib}_$rep.log 2>&1 || { tail -5 $O/${lib}_$rep.log; exit 1; }
    tail -1 $O/${lib}_$rep.log
  done
done
