#!/bin/bash
# config E 10,240 lane-pair chains: k_fpv_regen with and without its row stores (timing-only
# build rgn1, -DP3G_DIAG_REGEN=1: the row stores replaced by an XOR fold -- it ran 401 vs 231 ms,
# inconclusive, and the macro was removed), and snap_chunk 384 vs 256
set -o pipefail
O=gpurun_out/r5_regen2; mkdir -p $O
run() {  # name chunk
  timeout -k 10 300 python3 tools/bench_fpvec.py --reports 10240 --unique 16 --steps 2 --warmup 1 --opt snap_chunk=$2 --no-check 1 > $O/b_$1.log 2>&1 || { tail -20 $O/b_$1.log; exit 1; }
  echo "== $1 $(grep '^{' $O/b_$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels_ms_per_step"]; print(round(d["ms_per_step"],1), round(10240e3/d["ms_per_step"]), k.get("k_fpv_regen"), k.get("k_fpv_wires0_mfma"), k.get("k_fpv_wires1_mfma"), k.get("k_helper_xof"), k.get("k_jr_ring"))')"
}
run base 256 && PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_rgn1.so run rgn1 256 && run c384 384 && run base2 256
