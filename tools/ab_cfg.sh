#!/bin/bash
# A/B timing of library variants for one bench config (bench.py, no CPU baseline).
#   tools/ab_cfg.sh TAG CONFIG "label1:ENV=..;ENV2=.." "label2:..." ...
set -uo pipefail
TAG=$1; CFG=$2; shift 2
O=gpurun_out; mkdir -p $O
for spec in "$@"; do
  label=${spec%%:*}; envs=${spec#*:}
  echo "== $label ($envs)"
  env $(echo "$envs" | tr ';' ' ') timeout -k 10 300 python -u bench.py --config $CFG --steps 5 --warmup 1 --cpu-baseline 0 --hpke 0 --helper-only 0 > $O/ab_${TAG}_$label.log 2>&1
  rc=$?
  python3 -c "
import json,sys
for l in open('$O/ab_${TAG}_$label.log'):
    if l.startswith('{'):
        d=json.loads(l); print(' value', d['value'], 'ms/step', d['ms_per_step']); print(' ', d['kernels_ms_per_step'])
" || tail -3 $O/ab_${TAG}_$label.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
