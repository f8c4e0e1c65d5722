#!/bin/bash
# Round-6 Sum-query A/B: parity of the Sum configs on each variant build, then the query phase
# timing (tools/sponge_ab.py --config sum --query 1), alternated.  usage: tools/r6_sq.sh LIB...
set -o pipefail
O=gpurun_out/r6_sq; mkdir -p $O
for lib in "$@"; do
  if [ $lib = prod ]; then P=janus_amd/lib/libprio3gpu.so; else P=janus_amd/lib/libprio3gpu_$lib.so; fi
  PRIO3GPU_LIB=$P timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 \
    --timeout-method thread -k "sum" > $O/pytest_$lib.log 2>&1 || { tail -20 $O/pytest_$lib.log; exit 1; }
  echo "$lib $(tail -1 $O/pytest_$lib.log)"
done
for rep in 1 2; do
  for lib in "$@"; do
    if [ $lib = prod ]; then P=janus_amd/lib/libprio3gpu.so; else P=janus_amd/lib/libprio3gpu_$lib.so; fi
    PRIO3GPU_LIB=$P timeout -k 10 300 python -u tools/sponge_ab.py --config sum --query 1 --reps 3 \
      --label $lib > $O/${lib}_$rep.log 2>&1 || { tail -5 $O/${lib}_$rep.log; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/${lib}_$rep.log').read().strip().splitlines()[-1])
print(d['label'], {k:v for k,v in d['ms_per_launch_min'].items() if 'query_lane' in k})"
  done
done
