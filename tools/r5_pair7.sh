#!/bin/bash
# config E lane-pair chains: run-to-run spread at 10,752 (252 chain workgroups) vs 10,240 (240)
set -o pipefail
O=gpurun_out/r5_pair7; mkdir -p $O
run() {  # name reports chunk
  timeout -k 10 300 python3 tools/bench_fpvec.py --reports $2 --unique 16 --steps 2 --warmup 1 --opt snap_chunk=$3 > $O/b_$1.log 2>&1 || { tail -20 $O/b_$1.log; exit 1; }
  echo "== $1 $(grep '^{' $O/b_$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels_ms_per_step"]; print(round(d["ms_per_step"],1), round(d["reports_per_sec"]), k.get("k_jr_ring"), k.get("k_helper_xof"))')"
}
run a10240 10240 256 && run a10752 10752 256 && run b10240 10240 256 && run b10752 10752 256 && \
run c10240 10240 256 && run c10752 10752 256 && run d10240 10240 256 && run d10752 10752 256
