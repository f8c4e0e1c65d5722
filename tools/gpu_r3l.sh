#!/bin/bash
# Round-3 session l: Field128 inversion by divsteps -- parity, FLP timing vs exponentiation, benches.
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_flp_branches.py tests/test_gpu_turboshake.py tests/test_gpu_spec.py > gpurun_out/pytest_r3l.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3l.log
[ $rc -ne 0 ] && exit $rc
for c in sumvec histogram sum; do
  for v in gcd exp; do
    e=X=1; [ $v = exp ] && e=PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_exp.so
    env $e timeout -k 10 300 python -u tools/sponge_ab.py --config $c --query 1 --reps 2 --label ${c}_$v >> gpurun_out/flp_r3l.log 2> gpurun_out/flp_r3l.err || { tail -5 gpurun_out/flp_r3l.err; exit 1; }
    tail -1 gpurun_out/flp_r3l.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['label'], {k:v for k,v in d['ms_per_launch_min'].items() if 'flp' in k})"
  done
done
for c in sum histogram sumvec; do
  timeout -k 10 400 python -u bench.py --config $c --steps 4 --warmup 1 --cpu-baseline 0 --hpke 0 --helper-only 0 > gpurun_out/bench_r3l_$c.log 2>&1 || { tail -5 gpurun_out/bench_r3l_$c.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/bench_r3l_$c.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$c', d['value'], 'ms/step', d['ms_per_step']); print(' ', d['kernels_ms_per_step'])
"
done
