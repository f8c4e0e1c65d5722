#!/bin/bash
# Round-3 session q: k_flp_wires_mfma (byte-limb convolution on the i8 matrix cores) -- parity,
# A/B against the VALU wire pass (PRIO3GPU_WIRES_MFMA=0).
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_wires_mfma.py tests/test_gpu_parity.py tests/test_gpu_spec.py > gpurun_out/pytest_r3q.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3q.log
[ $rc -ne 0 ] && exit $rc
for v in mfma valu mfma2 valu2; do
  e=X=1; case $v in valu*) e=PRIO3GPU_WIRES_MFMA=0;; esac
  env $e timeout -k 10 300 python -u tools/sponge_ab.py --config sumvec --query 1 --reps 2 --label $v >> gpurun_out/flp_r3q.log 2> gpurun_out/flp_r3q.err || { tail -5 gpurun_out/flp_r3q.err; exit 1; }
  tail -1 gpurun_out/flp_r3q.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['label'], {k:v for k,v in d['ms_per_launch_min'].items() if 'flp' in k})"
done
