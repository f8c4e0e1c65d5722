set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "sum or turbo or spec or parity" > gpurun_out/pytest_sum3.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_sum3.log; [ $rc -ne 0 ] && exit $rc
for v in sum3 lane; do
  E=X=0; [ $v = lane ] && E=PRIO3GPU_FLPQ_SUM3=0
  env $E timeout -k 10 300 python -u bench.py --config sum --steps 3 --warmup 1 --hpke 0 --cpu-baseline 0 --helper-only 1 > gpurun_out/bench_sum3_$v.log 2>&1 || { echo "bench $v rc=$?"; tail -5 gpurun_out/bench_sum3_$v.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/bench_sum3_$v.log'):
    if l.startswith('{'): d=json.loads(l); print('$v', d['value'], d['ms_per_step'], d['helper_only']['value'], {k:v for k,v in d['kernels_ms_per_step'].items() if v>0.1})
"
done
