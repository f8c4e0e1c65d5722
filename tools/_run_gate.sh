set -o pipefail
bash tools/gpu_check.sh r02d || exit $?
for c in sum histogram count; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --hpke 0 > gpurun_out/bench_r02d_$c.log 2>&1 || { echo "bench $c rc=$?"; tail -5 gpurun_out/bench_r02d_$c.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/bench_r02d_$c.log'):
    if l.startswith('{'): d=json.loads(l); print('$c', d['value'], d['ms_per_step'], d['cpu_baseline']['value'] if d['cpu_baseline'] else None, d['parity'][:60])
"
done
