#!/bin/bash
# config E at 10,752 reports, lane-pair chains: repeated runs, then a kernel-trace timeline
set -o pipefail
O=gpurun_out/r5_pair4; mkdir -p $O
for k in 1 2 3; do
  timeout -k 10 300 python3 tools/bench_fpvec.py --reports 10752 --unique 16 --steps 3 --warmup 1 --opt snap_chunk=256 > $O/b_pair_$k.log 2>&1 || { tail -20 $O/b_pair_$k.log; exit 1; }
  echo "== pair $k"; grep '^{' $O/b_pair_$k.log | cut -c1-260
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 tools/bench_fpvec.py --reports 10752 --unique 16 --steps 1 --warmup 1 --opt snap_chunk=256 > $O/b_trace.log 2>&1 || { tail -20 $O/b_trace.log; exit 1; }
grep '^{' $O/b_trace.log | cut -c1-200
