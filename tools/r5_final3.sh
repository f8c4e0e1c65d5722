#!/bin/bash
# round-5 final check after the lane-pair chains, wait-free publishes and the overlapped helper query: GPU suite, smoke, bench lines, then config E at
# 10,240 distinct GPU-sharded reports (unshard == plaintext checked by bench_fpvec)
set -o pipefail
O=gpurun_out/final3; mkdir -p $O
./tools/final_check.sh $O || exit 1
timeout -k 10 400 python3 tools/bench_fpvec.py --reports 10240 --distinct 1 --steps 2 --warmup 1 --opt snap_chunk=256 > $O/fpvec_10240_distinct.log 2>&1 || { tail -20 $O/fpvec_10240_distinct.log; exit 1; }
grep '^{' $O/fpvec_10240_distinct.log | cut -c1-330
