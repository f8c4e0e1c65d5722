#!/bin/bash
# Config E A/B over engine environment knobs: FixedPoint GPU tests once, then one bench per
# configuration.   tools/ab_fpvec_env.sh "base: jr96:PRIO3GPU_JR_LDS=98304 ..." [B]
set -o pipefail
CONFS=$1; B=${2:-4800}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fp" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_env.log 2>&1
rc=$?; tail -1 gpurun_out/pt_env.log; [ $rc -ne 0 ] && exit $rc
for c in $CONFS; do
  [ -n "$QUIET" ] || true
  tag=${c%%:*}; envs=${c#*:}
  env ${envs//,/ } timeout -k 10 400 python -u tools/bench_fpvec.py --reports $B --unique 16 --distinct 1 --steps 2 --warmup 1 --shard-chunk 1600 > gpurun_out/fpvec_$tag.log 2>&1
  rc=$?
  python3 -c "
import json
for l in open('gpurun_out/fpvec_$tag.log'):
    if l.startswith('{'): d=json.loads(l); k=d['kernels_ms_per_step']; print('$tag', round(d['reports_per_sec'],1), round(d['ms_per_step'],1), 'hx', k.get('k_helper_xof'), 'jr', k.get('k_jr'), 'jr_ring', k.get('k_jr_ring'), 'accum', k.get('k_accum_spec'), k.get('k_accum_partial'))
" || tail -3 gpurun_out/fpvec_$tag.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
