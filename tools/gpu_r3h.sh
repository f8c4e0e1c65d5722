#!/bin/bash
# Round-3 session h: k_flp_wires with loads ahead of the MACs -- parity (both wire kernels), bench.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_spec.py tests/test_gpu_parity.py > gpurun_out/pytest_r3h.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3h.log
[ $rc -ne 0 ] && exit $rc
PRIO3GPU_WIRES_COLS=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "hist or countvec or sumvec" > gpurun_out/pytest_r3h_nocols.log 2>&1
rc=$?
echo "pytest (wires for histogram) rc=$rc"; tail -3 gpurun_out/pytest_r3h_nocols.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --cpu-baseline 0 --hpke 0 --helper-only 0 > gpurun_out/bench_r3h_$i.log 2>&1 || { tail -5 gpurun_out/bench_r3h_$i.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/bench_r3h_$i.log'):
    if l.startswith('{'):
        d=json.loads(l); print('bench', d['value'], 'ms/step', d['ms_per_step']); print(' ', d['kernels_ms_per_step']); print(' ', d['roofline']['hbm'])
"
done
timeout -k 10 400 python -u bench.py --config histogram --steps 4 --warmup 1 --cpu-baseline 0 --hpke 0 --helper-only 0 > gpurun_out/bench_r3h_hist.log 2>&1 || { tail -5 gpurun_out/bench_r3h_hist.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/bench_r3h_hist.log'):
    if l.startswith('{'):
        d=json.loads(l); print('hist', d['value'], 'ms/step', d['ms_per_step']); print(' ', d['kernels_ms_per_step'])
"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_leader.py > gpurun_out/pytest_r3h_leader.log 2>&1 || { tail -20 gpurun_out/pytest_r3h_leader.log; exit 1; }
tail -1 gpurun_out/pytest_r3h_leader.log
timeout -k 10 400 python -u tools/bench_leader_e2e.py --jobs 4 --job-size 32768 --reps 1 --cycle 4 > gpurun_out/leader_e2e_r3h.log 2>&1 || { tail -5 gpurun_out/leader_e2e_r3h.log; exit 1; }
tail -1 gpurun_out/leader_e2e_r3h.log
PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_a2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "transcript or aggregate" > gpurun_out/pytest_r3h_a2.log 2>&1 || { tail -20 gpurun_out/pytest_r3h_a2.log; exit 1; }
tail -1 gpurun_out/pytest_r3h_a2.log
PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_a2.so timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --cpu-baseline 0 --hpke 0 --helper-only 0 > gpurun_out/bench_r3h_a2.log 2>&1 || { tail -5 gpurun_out/bench_r3h_a2.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/bench_r3h_a2.log'):
    if l.startswith('{'):
        d=json.loads(l); print('a2 bench', d['value'], 'ms/step', d['ms_per_step']); print(' ', d['kernels_ms_per_step'])
"
