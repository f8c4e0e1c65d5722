set -o pipefail
# Config E kernel trace at 10,240 reports (default options), for the timeline.
O=gpurun_out/r5_fpv8; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 tools/bench_fpvec.py --reports 10240 --unique 16 --steps 1 --warmup 1 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
grep '^{' $O/b.log | cut -c1-200
