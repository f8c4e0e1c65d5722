#!/bin/bash
# Round-3 session o: the self-launching N-rank bench on the one-GPU box (gloo rehearsal).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --gpus 2 --merge gloo --steps 2 --warmup 1 --reports 65536 --cpu-baseline 0 --hpke 0 --helper-only 0 > gpurun_out/bench_r3o_gpus2_gloo.log 2>&1
rc=$?
echo "rc=$rc"; grep '^{' gpurun_out/bench_r3o_gpus2_gloo.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('n_gpus', d['n_gpus'], 'value', d['value'], 'ms/step', d['ms_per_step'], d['config']['parallelism'])
"; tail -3 gpurun_out/bench_r3o_gpus2_gloo.log
exit $rc
