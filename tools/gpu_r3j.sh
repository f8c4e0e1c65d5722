#!/bin/bash
# Round-3 session j: v_perm byte rotations (microbench + variant), fused helper on small types.
set -u
mkdir -p gpurun_out
timeout -k 10 120 ./tools/microbench > gpurun_out/microbench_r3j.log 2>&1 || exit 1
timeout -k 10 120 ./tools/microbench_perm > gpurun_out/microbench_perm_r3j.log 2>&1 || exit 1
cat gpurun_out/microbench_r3j.log; grep Keccak gpurun_out/microbench_perm_r3j.log
PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_perm.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_turboshake.py tests/test_gpu_helper_sponge.py > gpurun_out/pytest_r3j_perm.log 2>&1
rc=$?
echo "pytest perm rc=$rc"; tail -3 gpurun_out/pytest_r3j_perm.log
[ $rc -ne 0 ] && exit $rc
for v in base perm base2 perm2; do
  e=X=1; case $v in perm*) e=PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_perm.so;; esac
  env $e PRIO3GPU_HELPER_SPONGE=0 timeout -k 10 240 python -u tools/sponge_ab.py --label $v >> gpurun_out/sponge_r3j.log 2> gpurun_out/sponge_r3j.err || { tail -5 gpurun_out/sponge_r3j.err; exit 1; }
  tail -1 gpurun_out/sponge_r3j.log
done
for c in histogram sum; do
  for m in 0 1; do
    PRIO3GPU_HELPER_SPONGE=$m timeout -k 10 400 python -u bench.py --config $c --steps 4 --warmup 1 --cpu-baseline 0 --hpke 0 --helper-only 0 > gpurun_out/bench_r3j_${c}_$m.log 2>&1 || { tail -5 gpurun_out/bench_r3j_${c}_$m.log; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/bench_r3j_${c}_$m.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$c sponge=$m', d['value'], 'ms/step', d['ms_per_step']); print(' ', d['kernels_ms_per_step'])
"
  done
done
