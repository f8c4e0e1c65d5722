set -o pipefail
# Config E kernel trace at 10,752 reports (snap_chunk 256), default schedule: the timeline.
O=gpurun_out/r5_fpv_final; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 tools/bench_fpvec.py --reports 10752 --unique 16 --steps 1 --warmup 1 --opt snap_chunk=256 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
grep '^{' $O/b.log | cut -c1-200
