#!/bin/bash
# round-5 close: GPU suite, smoke and bench lines on the final build, then a config E kernel trace
# at 10,240 reports (rocprofv3 --kernel-trace --stats)
set -o pipefail
O=gpurun_out/final4; mkdir -p $O
./tools/final_check.sh $O || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 tools/bench_fpvec.py --reports 10240 --unique 16 --steps 1 --warmup 1 --opt snap_chunk=256 > $O/fpvec_trace.log 2>&1 || { tail -20 $O/fpvec_trace.log; exit 1; }
grep '^{' $O/fpvec_trace.log | cut -c1-200
