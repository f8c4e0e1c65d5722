#!/bin/bash
# config E 10,240: the helper's storer cost -- base vs a timing-only build whose storer neither
# zips nor sums columns (hxp1, -DP3G_DIAG_HXP=1; wrong bytes, so --no-check)
set -o pipefail
O=gpurun_out/r5_pair14; mkdir -p $O
run() {  # name
  timeout -k 10 300 python3 tools/bench_fpvec.py --reports 10240 --unique 16 --steps 2 --warmup 1 --opt snap_chunk=256 --no-check 1 > $O/b_$1.log 2>&1 || { tail -20 $O/b_$1.log; exit 1; }
  echo "== $1 $(grep '^{' $O/b_$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels_ms_per_step"]; print(round(d["ms_per_step"],1), k.get("k_helper_xof"), k.get("k_jr_ring"))')"
}
run base1 && PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_hxp1.so run hxp1_1 && run base2 && \
PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_hxp1.so run hxp1_2
