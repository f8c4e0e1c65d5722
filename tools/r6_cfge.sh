#!/bin/bash
# Config E determinism (round 6): the FixedPoint16 100k-entry bench at the documented batch and
# above it, several runs each -- every run's value, to show
# the spread.  usage: tools/r6_cfge.sh "B1 B2 ..." RUNS [extra bench_fpvec args]
set -o pipefail
O=gpurun_out/r6_cfge${TAG:+/$TAG}; mkdir -p $O
BS=$1; RUNS=$2; shift 2
for r in $(seq 1 $RUNS); do
  for b in $BS; do
    timeout -k 10 240 python -u tools/bench_fpvec.py --reports $b --unique 16 --steps 2 --warmup 1 \
      --opt snap_chunk=256 "$@" > $O/e_${b}_$r.log 2>&1 || { tail -5 $O/e_${b}_$r.log; exit 1; }
    python3 - "$O/e_${b}_$r.log" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print(sys.argv[1], round(d.get("reports_per_sec", 0), 1), round(d.get("ms_per_step"), 1))
PY
  done
done
