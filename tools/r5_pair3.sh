#!/bin/bash
# config E at 10,752 reports: lane-pair chains (default) vs the unpaired kernels
set -o pipefail
O=gpurun_out/r5_pair3; mkdir -p $O
for v in pair unpaired pair; do
  extra=""; [ $v = unpaired ] && extra="--opt pair_chains=0"
  timeout -k 10 300 python3 tools/bench_fpvec.py --reports 10752 --unique 16 --steps 2 --warmup 1 --opt snap_chunk=256 $extra > $O/b_$v.log 2>&1 || { tail -20 $O/b_$v.log; exit 1; }
  echo "== $v"; grep '^{' $O/b_$v.log | cut -c1-300
done
