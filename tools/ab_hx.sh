#!/bin/bash
# k_helper_xof consumer-wave placement A/B (PRIO3GPU_HX_CWAVE = 1, 2, 3): FixedPoint GPU tests
# with the candidate, then config E once per placement.   tools/ab_hx.sh "1 2 3" [B]
set -o pipefail
WAVES=${1:-"1 2"}; B=${2:-4800}
for w in $WAVES; do
  PRIO3GPU_HX_CWAVE=$w timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fp" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_hx$w.log 2>&1
  rc=$?; tail -1 gpurun_out/pt_hx$w.log; [ $rc -ne 0 ] && exit $rc
  PRIO3GPU_HX_CWAVE=$w timeout -k 10 400 python -u tools/bench_fpvec.py --reports $B --unique 16 --distinct 1 --steps 2 --warmup 1 --shard-chunk 1600 > gpurun_out/fpvec_hx$w.log 2>&1
  rc=$?
  python3 -c "
import json
for l in open('gpurun_out/fpvec_hx$w.log'):
    if l.startswith('{'): d=json.loads(l); k=d['kernels_ms_per_step']; print('cwave $w', round(d['reports_per_sec'],1), round(d['ms_per_step'],1), 'hx', k.get('k_helper_xof'), 'jr', k.get('k_jr'))
" || tail -3 gpurun_out/fpvec_hx$w.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
