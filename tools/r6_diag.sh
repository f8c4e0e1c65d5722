#!/bin/bash
# Round-6 sponge floor: per-launch times of the SumVec sponge kernels in the default build and in
# the timing-only diagnostic builds (k_jr without window fills, k_expand without stores), two
# alternations each so box drift shows.  Output: gpurun_out/r6_diag/*.log
set -o pipefail
O=gpurun_out/r6_diag; mkdir -p $O
for rep in 1 2; do
  for lib in base0 jrnl exns; do
    E="PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_$lib.so"
    env $E timeout -k 10 300 python -u tools/sponge_ab.py --config sumvec --reps 3 --label $lib \
      > $O/${lib}_$rep.log 2>&1 || { tail -5 $O/${lib}_$rep.log; exit 1; }
    tail -1 $O/${lib}_$rep.log
  done
done
