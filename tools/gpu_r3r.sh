#!/bin/bash
# Round-3 session r: k_flp_wires_mfma tile loop (<= 4 waves per block) -- parity, and A/B of the
# loads issued together per K-step batch (WM_U = 2 / 4 / 8 / 16) against the VALU pass.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_wires_mfma.py > gpurun_out/pytest_r3r.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r3r.log; [ $rc -ne 0 ] && exit $rc
for v in u4 u2 u8 u16 valu nored noloop u4b u8b u16b; do
  e=X=1
  case $v in valu) e=PRIO3GPU_WIRES_MFMA=0;; u4*) e=X=1;; u*|nored|noloop) e=PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_${v%b}.so;; esac
  env $e timeout -k 10 300 python -u tools/sponge_ab.py --config sumvec --query 1 --reps 2 --label $v >> gpurun_out/flp_r3r.log 2> gpurun_out/flp_r3r.err || { tail -5 gpurun_out/flp_r3r.err; exit 1; }
  tail -1 gpurun_out/flp_r3r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['label'], {k:v for k,v in d['ms_per_launch_min'].items() if 'wires' in k})"
done
