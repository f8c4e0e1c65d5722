set -o pipefail
O=gpurun_out/r5b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for c in sum sumvec; do
  timeout -k 10 400 python -u bench.py --config $c --cpu-baseline 0 --hpke 0 > $O/bench_$c.log 2>&1 || { tail -20 $O/bench_$c.log; exit 1; }
  python3 -c "
import json
for l in open('$O/bench_$c.log'):
    if l.startswith('{'): d=json.loads(l); r=d['roofline']; print('$c', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac'], d['serial_pass'])
"
done
