#!/bin/bash
# config E 10,752, lane-pair chains: wave_prio 1 (sponges only, default) / 2 (every wave) / 0,
# and a build with the leader's ring counters through ds instructions (P3G_JR_CTR_LDS=1)
set -o pipefail
O=gpurun_out/r5_pair5; mkdir -p $O
run() {  # name, extra args
  timeout -k 10 300 python3 tools/bench_fpvec.py --reports 10752 --unique 16 --steps 2 --warmup 1 --opt snap_chunk=256 $2 > $O/b_$1.log 2>&1 || { tail -20 $O/b_$1.log; exit 1; }
  echo "== $1 $(grep '^{' $O/b_$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels_ms_per_step"]; print(round(d["ms_per_step"],1), round(d["reports_per_sec"]), k.get("k_jr_ring"), k.get("k_helper_xof"))')"
}
run prio1 "" && run prio2 "--opt wave_prio=2" && run prio0 "--opt wave_prio=0" && \
PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_jrlds.so run jrlds "" && run prio1b ""
