#!/bin/bash
# Round-3 session t: k_flp_wires_mfma with the first load batch issued before the weight
# conversion (WM_PREFETCH) -- parity, A/B against the build without it.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_wires_mfma.py > gpurun_out/pytest_r3t.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r3t.log; [ $rc -ne 0 ] && exit $rc
for v in pf nopf pfu8 pf2 nopf2 pfu82; do
  e=X=1; case $v in nopf*) e=PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_nopf.so;; pfu8*) e=PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_pfu8.so;; esac
  env $e timeout -k 10 300 python -u tools/sponge_ab.py --config sumvec --query 1 --reps 2 --label $v >> gpurun_out/flp_r3t.log 2> gpurun_out/flp_r3t.err || { tail -5 gpurun_out/flp_r3t.err; exit 1; }
  tail -1 gpurun_out/flp_r3t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['label'], {k:v for k,v in d['ms_per_launch_min'].items() if 'wires' in k})"
done
