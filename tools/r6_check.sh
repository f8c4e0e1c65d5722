#!/bin/bash
# Round-6 check on one GPU box: the whole GPU test suite and smoke() on the product build, then
# the default bench line of the product build and of a reference build, alternated.
#   usage: tools/r6_check.sh OUTDIR [REFLIB] [CONFIGS]
set -o pipefail
O=${1:-gpurun_out/r6_check}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for c in ${3:-sumvec}; do
  for lib in prod $2; do
    if [ $lib = prod ]; then E=""; else E="PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_$lib.so"; fi
    env $E timeout -k 10 400 python -u bench.py --config $c > $O/bench_${c}_$lib.log 2>&1 || { tail -20 $O/bench_${c}_$lib.log; exit 1; }
    python3 -c "
import json
for l in open('$O/bench_${c}_$lib.log'):
    if l.startswith('{\"metric'):
        d=json.loads(l); r=d['roofline']
        print('$c $lib', round(d['value']), d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac'], {k: round(v, 2) for k, v in d['kernels_ms_per_step'].items() if v > 0.5})
"
  done
done
