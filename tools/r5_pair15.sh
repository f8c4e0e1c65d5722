#!/bin/bash
# config E lane-pair chains: 10,496 reports (246 chain workgroups) three times, then one PMC pass
# over a 10,240-report run (VALU / LDS instructions and wait cycles of the chain kernels)
set -o pipefail
O=gpurun_out/r5_pair15; mkdir -p $O
run() {  # name reports
  timeout -k 10 300 python3 tools/bench_fpvec.py --reports $2 --unique 16 --steps 2 --warmup 1 --opt snap_chunk=256 > $O/b_$1.log 2>&1 || { tail -20 $O/b_$1.log; exit 1; }
  echo "== $1 $(grep '^{' $O/b_$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels_ms_per_step"]; print(round(d["ms_per_step"],1), round(d["reports_per_sec"]), k.get("k_helper_xof"), k.get("k_jr_ring"))')"
}
run a10496 10496 && run b10496 10496 && run c10496 10496 || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc -o run -- python3 tools/bench_fpvec.py --reports 10240 --unique 16 --steps 1 --warmup 1 --opt snap_chunk=256 > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
grep '^{' $O/pmc.log | cut -c1-160
