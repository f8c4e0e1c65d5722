#!/bin/bash
# Round-3 session u: k_flp_wires_mfma<SHORT> (Histogram / chunk 8..32: a wave per report) --
# parity, A/B against k_flp_wires_cols, Histogram bench.
set -u
mkdir -p gpurun_out
PRIO3GPU_WIRES_MFMA_SHORT=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_wires_mfma.py tests/test_gpu_parity.py tests/test_gpu_spec.py > gpurun_out/pytest_r3u.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r3u.log; [ $rc -ne 0 ] && exit $rc
for v in mfma cols mfma2 cols2; do
  e=PRIO3GPU_WIRES_MFMA_SHORT=1; case $v in cols*) e=PRIO3GPU_WIRES_MFMA=0;; esac
  env $e timeout -k 10 300 python -u tools/sponge_ab.py --config histogram --query 1 --reps 2 --label $v >> gpurun_out/flp_r3u.log 2> gpurun_out/flp_r3u.err || { tail -5 gpurun_out/flp_r3u.err; exit 1; }
  tail -1 gpurun_out/flp_r3u.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['label'], {k:v for k,v in d['ms_per_launch_min'].items() if 'flp' in k})"
done
for v in mfma cols; do
  e=PRIO3GPU_WIRES_MFMA_SHORT=1; case $v in cols*) e=PRIO3GPU_WIRES_MFMA=0;; esac
  env $e timeout -k 10 400 python -u bench.py --config histogram > gpurun_out/bench_r3u_hist_$v.log 2>&1 || { tail -20 gpurun_out/bench_r3u_hist_$v.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/bench_r3u_hist_$v.log'):
    if l.startswith('{'): d=json.loads(l); print('hist $v', d['value'], d['ms_per_step'])
"
done
