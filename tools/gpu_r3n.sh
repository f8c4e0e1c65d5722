#!/bin/bash
# Round-3 session n: is k_expand's store cost L2 line churn or per-instruction scatter?
set -u
mkdir -p gpurun_out
for v in base fixed tile nost base2; do
  e=X=1; case $v in base*) ;; *) e=PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_$v.so;; esac
  env $e timeout -k 10 240 python -u tools/sponge_ab.py --label $v >> gpurun_out/sponge_r3n.log 2> gpurun_out/sponge_r3n.err || { tail -5 gpurun_out/sponge_r3n.err; exit 1; }
  tail -1 gpurun_out/sponge_r3n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['label'], d['ms_per_launch_min'])"
done
