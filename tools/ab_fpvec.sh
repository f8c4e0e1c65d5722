#!/bin/bash
# FixedPoint GPU tests, then config E (B distinct reports through the GPU shard) on one box.
#   tools/ab_fpvec.sh TAG B
set -o pipefail
TAG=$1; B=${2:-4800}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_squeeze.py tests/test_codec.py -k "fp" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pt_$TAG.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/bench_fpvec.py --reports $B --unique 16 --distinct 1 --steps 2 --warmup 1 --shard-chunk 1600 > gpurun_out/fpvec_$TAG.log 2>&1
rc=$?
python3 -c "
import json
for l in open('gpurun_out/fpvec_$TAG.log'):
    if l.startswith('{'): d=json.loads(l); print(d['reports_per_sec'], d['ms_per_step'], d['kernels_ms_per_step'])
" || tail -3 gpurun_out/fpvec_$TAG.log
exit $rc
