#!/bin/bash
# config E 10,752, lane-pair chains with the leader's ds counters and the v_perm zip / unzip:
# FixedPoint parity, then base vs timing-only builds without the loader's column sums (jrp1) /
# its unzip (jrp2)
set -o pipefail
O=gpurun_out/r5_pair6; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "fpvec or fixedpoint or fp16 or fp64 or fp32" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # name
  timeout -k 10 300 python3 tools/bench_fpvec.py --reports 10752 --unique 16 --steps 2 --warmup 1 --opt snap_chunk=256 --no-check 1 > $O/b_$1.log 2>&1 || { tail -20 $O/b_$1.log; exit 1; }
  echo "== $1 $(grep '^{' $O/b_$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels_ms_per_step"]; print(round(d["ms_per_step"],1), round(10752e3/d["ms_per_step"]), k.get("k_jr_ring"), k.get("k_helper_xof"))')"
}
run base && PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_jrp1.so run jrp1 && \
PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_jrp2.so run jrp2 && run base2
