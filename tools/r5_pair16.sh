#!/bin/bash
# config E lane-pair chains at 10,496 reports: five more runs (placement check)
set -o pipefail
O=gpurun_out/r5_pair16; mkdir -p $O
run() {  # name reports
  timeout -k 10 300 python3 tools/bench_fpvec.py --reports $2 --unique 16 --steps 2 --warmup 1 --opt snap_chunk=256 > $O/b_$1.log 2>&1 || { tail -20 $O/b_$1.log; exit 1; }
  echo "== $1 $(grep '^{' $O/b_$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels_ms_per_step"]; print(round(d["ms_per_step"],1), round(d["reports_per_sec"]), k.get("k_helper_xof"), k.get("k_jr_ring"))')"
}
for k in 1 2 3 4 5; do run r$k 10496 || exit 1; done
