#!/bin/bash
# lane-pair chains: cached counter polls (then the default; removed after this run: no gain) vs a
# poll per block (pc0, -DP3G_PAIR_POLLCACHE=0); FixedPoint parity first
set -o pipefail
O=gpurun_out/r5_pair17; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "fpvec or fixedpoint or fp16 or fp64 or fp32" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # name
  timeout -k 10 300 python3 tools/bench_fpvec.py --reports 10240 --unique 16 --steps 2 --warmup 1 --opt snap_chunk=256 > $O/b_$1.log 2>&1 || { tail -20 $O/b_$1.log; exit 1; }
  echo "== $1 $(grep '^{' $O/b_$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels_ms_per_step"]; print(round(d["ms_per_step"],1), round(d["reports_per_sec"]), k.get("k_fpv_regen"), k.get("k_helper_xof"), k.get("k_jr_ring"))')"
}
for k in 1 2; do
  run c1_$k || exit 1
  PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_pc0.so run c0_$k || exit 1
done
