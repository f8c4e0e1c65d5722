set -o pipefail
# Config E kernel traces at 8,192 reports: serial (--overlap 0) and co-run (--overlap 1).
O=gpurun_out/r5_fpv4; mkdir -p $O
for ov in 0 1; do
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr$ov -o run -- python3 tools/bench_fpvec.py --reports 8192 --unique 16 --steps 1 --warmup 1 --overlap $ov > $O/b_ov$ov.log 2>&1 || { tail -20 $O/b_ov$ov.log; exit 1; }
  grep '^{' $O/b_ov$ov.log | cut -c1-300
done
