#!/bin/bash
# Round-3 session i: fused helper sponge -- parity in all modes, then timing.
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_helper_sponge.py tests/test_gpu_spec.py tests/test_gpu_parity.py tests/test_gpu_squeeze.py > gpurun_out/pytest_r3i.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_r3i.log
[ $rc -ne 0 ] && exit $rc
for l in fused twopass; do
  e=X=1; [ $l = twopass ] && e=PRIO3GPU_HELPER_SPONGE=0
  env $e timeout -k 10 240 python -u tools/sponge_ab.py --label $l >> gpurun_out/sponge_r3i.log 2> gpurun_out/sponge_r3i.err || { tail -5 gpurun_out/sponge_r3i.err; exit 1; }
  tail -1 gpurun_out/sponge_r3i.log
done
for l in fused twopass; do
  e=X=1; [ $l = twopass ] && e=PRIO3GPU_HELPER_SPONGE=0
  env $e timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --cpu-baseline 0 --hpke 0 --helper-only 0 > gpurun_out/bench_r3i_$l.log 2>&1 || { tail -5 gpurun_out/bench_r3i_$l.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/bench_r3i_$l.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$l bench', d['value'], 'ms/step', d['ms_per_step']); print(' ', d['kernels_ms_per_step'])
"
done
