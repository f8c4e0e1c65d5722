#!/bin/bash
# One GPU session: the GPU test suite (own time limit), then bench A/B runs (tools/ab_bench.sh
# specs as arguments).  Stops at the first failure.
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error" $O/pytest_gpu.log | head -20; exit $rc; }
[ $# -gt 0 ] && bash tools/ab_bench.sh "$@"
