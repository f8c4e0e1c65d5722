#!/bin/bash
# Round-3 session w: k_expand occupancy vs its wave quantisation (6,144 waves of 64 reports at
# 4 waves/SIMD = 1.5 rounds of the chip): base (98 VGPRs, 4 waves), an LDS cap to 3 waves
# (2 full rounds), 5 waves (96 VGPRs, launch bound).  Timing only.
set -u
mkdir -p gpurun_out
for v in base lds3 ew5 base2 lds32 ew52; do
  e=X=1
  case $v in lds3*) e=PRIO3GPU_EXPAND_LDS=53248;; ew5*) e=PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_ew5.so;; esac
  env $e timeout -k 10 300 python -u tools/sponge_ab.py --config sumvec --reps 2 --label $v >> gpurun_out/expand_r3w.log 2> gpurun_out/expand_r3w.err || { tail -5 gpurun_out/expand_r3w.err; exit 1; }
  tail -1 gpurun_out/expand_r3w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['label'], d['ms_per_launch_min'])"
done
