set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_lane.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_lane.log; [ $rc -ne 0 ] && exit $rc
for c in sum count; do
 for v in lane block; do
  E=X=0; [ $v = block ] && E=PRIO3GPU_FLPQ_BLOCK=1
  env $E timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --hpke 0 --cpu-baseline 0 --helper-only 1 > gpurun_out/bench_lane_${c}_$v.log 2>&1 || { echo "bench $c $v rc=$?"; tail -5 gpurun_out/bench_lane_${c}_$v.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/bench_lane_${c}_$v.log'):
    if l.startswith('{'): d=json.loads(l); print('$c $v', d['value'], d['ms_per_step'], d['helper_only']['value'], {k:v for k,v in d['kernels_ms_per_step'].items() if v>0.2})
"
 done
done
