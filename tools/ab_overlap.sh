#!/bin/bash
# A/B of the bench's overlap schedules (tests first; any GPU fault/timeout ends the session).
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_leader.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > $O/pt_ov.log 2>&1
rc=$?; tail -2 $O/pt_ov.log
[ $rc -ne 0 ] && exit $rc
for ov in "$@"; do
  timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --cpu-baseline 0 --hpke 0 \
    --helper-only 0 --overlap $ov > $O/ov$ov.log 2>&1
  rc=$?
  echo "== overlap $ov rc=$rc"; tail -c 1200 $O/ov$ov.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
