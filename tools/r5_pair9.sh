#!/bin/bash
# config E 10,240 lane-pair chains with the helper's query_overlap: wait-free (default) vs waiting
# ring publishes (pw0, -DP3G_PAIR_NOWAIT=0) vs the leader's column sums on their own waves (cs1,
# -DP3G_JRP_COLSUM=1); snap_chunk 256, each twice, and 384 once
set -o pipefail
O=gpurun_out/r5_pair9; mkdir -p $O
run() {  # name args
  timeout -k 10 300 python3 tools/bench_fpvec.py --reports 10240 --unique 16 --steps 2 --warmup 1 $2 > $O/b_$1.log 2>&1 || { tail -20 $O/b_$1.log; exit 1; }
  echo "== $1 $(grep '^{' $O/b_$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels_ms_per_step"]; print(round(d["ms_per_step"],1), round(d["reports_per_sec"]), k.get("k_fpv_regen"), k.get("k_helper_xof"), k.get("k_jr_ring"))')"
}
A="--opt snap_chunk=256 --hopt query_overlap=1"
for k in 1 2; do
  run nw_$k "$A" || exit 1
  PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_pw0.so run w_$k "$A" || exit 1
  PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_cs1.so run cs_$k "$A" || exit 1
done
run nw384 "--opt snap_chunk=384 --hopt query_overlap=1"
