#!/bin/bash
# Round-end check on one GPU box: full GPU test suite, smoke(), and the bench lines.
set -o pipefail
O=${1:-gpurun_out/final}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for c in sumvec sum histogram count; do
  timeout -k 10 400 python -u bench.py --config $c > $O/bench_$c.log 2>&1 || { tail -20 $O/bench_$c.log; exit 1; }
  python3 -c "
import json
for l in open('$O/bench_$c.log'):
    if l.startswith('{'): d=json.loads(l); r=d['roofline']; print('$c', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r.get('avg_launch_ms_timed_span'), r['frac'], d['serial_pass'])
"
done
