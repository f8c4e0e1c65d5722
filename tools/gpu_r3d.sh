#!/bin/bash
# Round-3 session d: pitched-input tests, then the leader-pitch A/B (packed rows vs 128-B rows).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "pitched or transcript_bit_exact" > gpurun_out/pytest_r3d.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_r3d.log
case $rc in 0|1) ;; *) exit $rc ;; esac
ab() {  # ab LABEL ARGS...
  local l=$1; shift
  timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --cpu-baseline 0 --hpke 0 --helper-only 0 "$@" > gpurun_out/ab_r3d_$l.log 2>&1
  local r=$?
  python3 -c "
import json
for l in open('gpurun_out/ab_r3d_$l.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$l value', d['value'], 'ms/step', d['ms_per_step']); print(' ', d['kernels_ms_per_step'])
" || tail -3 gpurun_out/ab_r3d_$l.log
  [ $r -ne 0 ] && exit $r
  return 0
}
ab packed --leader-pitch 0
ab p128 --leader-pitch -1
ab packed2 --leader-pitch 0
ab p128b --leader-pitch -1
exit 0
