set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final_pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/final_pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/final_smoke.log; [ $rc -ne 0 ] && exit $rc
for c in sum histogram count; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 1 --hpke 0 > gpurun_out/final2_bench_$c.log 2>&1 || { echo "bench $c rc=$?"; tail -5 gpurun_out/final2_bench_$c.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/final2_bench_$c.log'):
    if l.startswith('{'): d=json.loads(l); print('$c', d['value'], d['ms_per_step'], d['cpu_baseline']['value'], d['cpu_baseline']['one_thread'], d['speedup_vs_cpu'], d['helper_only']['value'])
"
done
