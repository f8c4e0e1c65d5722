#!/bin/bash
# Round-3 session m: k_flp_wires canonical pre-filter -- parity, A/B vs the previous build.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/pytest_r3m.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r3m.log
[ $rc -ne 0 ] && exit $rc
PRIO3GPU_WIRES_COLS=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "hist or noncanonical or countvec" > gpurun_out/pytest_r3m_nocols.log 2>&1 || { tail -20 gpurun_out/pytest_r3m_nocols.log; exit 1; }
tail -1 gpurun_out/pytest_r3m_nocols.log
for v in new orig new2 orig2; do
  e=X=1; case $v in orig*) e=PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_orig.so;; esac
  env $e timeout -k 10 300 python -u tools/sponge_ab.py --config sumvec --query 1 --reps 2 --label $v >> gpurun_out/flp_r3m.log 2> gpurun_out/flp_r3m.err || { tail -5 gpurun_out/flp_r3m.err; exit 1; }
  tail -1 gpurun_out/flp_r3m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['label'], {k:v for k,v in d['ms_per_launch_min'].items() if 'flp' in k})"
done
