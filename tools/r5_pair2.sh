#!/bin/bash
# lane-pair config E kernels: FixedPoint parity (pair default + unpaired variants)
set -o pipefail
mkdir -p gpurun_out/r5_pair2
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "fpvec or fixedpoint or fp16 or fp64 or fp32" \
  > gpurun_out/r5_pair2/pytest.log 2>&1; rc=$?
tail -40 gpurun_out/r5_pair2/pytest.log
exit $rc
