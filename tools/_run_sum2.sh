set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_sum2.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_sum2.log; [ $rc -ne 0 ] && exit $rc
for c in sum count; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --hpke 0 --cpu-baseline 0 --helper-only 1 > gpurun_out/bench_sum2_$c.log 2>&1 || { echo "bench $c rc=$?"; tail -5 gpurun_out/bench_sum2_$c.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/bench_sum2_$c.log'):
    if l.startswith('{'): d=json.loads(l); print('$c', d['value'], d['ms_per_step'], d['helper_only']['value'], {k:v for k,v in d['kernels_ms_per_step'].items() if v>0.1})
"
done
