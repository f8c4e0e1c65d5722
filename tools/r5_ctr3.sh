set -o pipefail
# k_jr_ring with ds counters and a throttled loader (sleep 8 / 32 quanta) vs the FLAT default.
O=gpurun_out/r5_ctr3; mkdir -p $O
for v in "" jrl8 jrl32; do
  lib=""; [ -n "$v" ] && lib="PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_$v.so"
  for ov in 0 1; do
    env $lib timeout -k 10 300 python -u tools/bench_fpvec.py --reports 10240 --unique 16 --steps 2 --warmup 1 --overlap $ov > $O/e_${v}_$ov.log 2>&1 || { tail -5 $O/e_${v}_$ov.log; exit 1; }
    python3 -c "
import json
for l in open('$O/e_${v}_$ov.log'):
    if l.startswith('{'): d=json.loads(l); k=d['kernels_ms_per_step']; print('${v:-flat} ov$ov', round(d['reports_per_sec'],1), round(d['ms_per_step'],1), 'ring', k.get('k_jr_ring'), 'hx', k.get('k_helper_xof'))
"
  done
done
