#!/bin/bash
# Round-3 session p: one wire per thread (k_flp_wires_split) -- parity, A/B.
set -u
mkdir -p gpurun_out
PRIO3GPU_WIRES_SPLIT=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_spec.py > gpurun_out/pytest_r3p.log 2>&1
rc=$?; echo "pytest split rc=$rc"; tail -2 gpurun_out/pytest_r3p.log; [ $rc -ne 0 ] && exit $rc
PRIO3GPU_WIRES_SPLIT=1 PRIO3GPU_WIRES_COLS=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "hist or noncanonical or countvec or sumvec" > gpurun_out/pytest_r3p_nocols.log 2>&1 || { tail -20 gpurun_out/pytest_r3p_nocols.log; exit 1; }
tail -1 gpurun_out/pytest_r3p_nocols.log
for v in base split base2 split2; do
  e=X=1; case $v in split*) e=PRIO3GPU_WIRES_SPLIT=1;; esac
  env $e timeout -k 10 300 python -u tools/sponge_ab.py --config sumvec --query 1 --reps 2 --label $v >> gpurun_out/flp_r3p.log 2> gpurun_out/flp_r3p.err || { tail -5 gpurun_out/flp_r3p.err; exit 1; }
  tail -1 gpurun_out/flp_r3p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['label'], {k:v for k,v in d['ms_per_launch_min'].items() if 'flp' in k})"
done
