#!/bin/bash
# Round-3 session x: FLP weight rows at a 128-B pitch (PRIO3GPU_WROW_ALIGN=1) -- parity, A/B of
# k_flp_weights + the wire pass (SumVec, Histogram).
set -u
mkdir -p gpurun_out
PRIO3GPU_WROW_ALIGN=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_wires_mfma.py -k "sumvec or hist or mfma" > gpurun_out/pytest_r3x.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r3x.log; [ $rc -ne 0 ] && exit $rc
for cfg in sumvec histogram; do
for v in packed align packed2 align2; do
  e=PRIO3GPU_WROW_ALIGN=0; case $v in align*) e=PRIO3GPU_WROW_ALIGN=1;; esac
  env $e timeout -k 10 300 python -u tools/sponge_ab.py --config $cfg --query 1 --reps 2 --label ${cfg}_$v >> gpurun_out/wrow_r3x.log 2> gpurun_out/wrow_r3x.err || { tail -5 gpurun_out/wrow_r3x.err; exit 1; }
  tail -1 gpurun_out/wrow_r3x.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['label'], {k:v for k,v in d['ms_per_launch_min'].items() if 'flp' in k})"
done
done
