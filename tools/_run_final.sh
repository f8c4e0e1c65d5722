set -o pipefail
R=$(pwd)
timeout -k 10 420 python -u bench.py > gpurun_out/final_bench_sumvec.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/final_bench_sumvec.log; exit 1; }
tail -c 400 gpurun_out/final_bench_sumvec.log
for c in sum histogram count; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 1 --hpke 0 > gpurun_out/final_bench_$c.log 2>&1 || { echo "bench $c rc=$?"; tail -5 gpurun_out/final_bench_$c.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/final_bench_$c.log'):
    if l.startswith('{'): d=json.loads(l); print('$c', d['value'], d['ms_per_step'], d['cpu_baseline']['value'], d['speedup_vs_cpu'])
"
done
mkdir -p gpurun_out/prof_final
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_final/trace -o run -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 --hpke 0 --helper-only 0 > $R/gpurun_out/prof_final/trace.log 2>&1 || { echo "rocprof rc=$?"; tail -5 $R/gpurun_out/prof_final/trace.log; exit 1; }
find $R/gpurun_out/prof_final/trace -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/final_kernel_stats.csv \;
grep "^{\"metric\"" $R/gpurun_out/prof_final/trace.log > $R/gpurun_out/final_bench_under_rocprof.json || true
head -12 $R/gpurun_out/final_kernel_stats.csv
