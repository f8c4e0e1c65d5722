set -o pipefail
# Which role bounds the helper chain: timing-only builds (P3G_DIAG_HX) at 10,240 reports, serial.
O=gpurun_out/r5_fpv13; mkdir -p $O
for v in "" hx1 hx2 hx3; do
  lib=""; [ -n "$v" ] && lib="PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_$v.so"
  env $lib timeout -k 10 300 python -u tools/bench_fpvec.py --reports 10240 --unique 16 --steps 2 --warmup 1 --overlap 0 --no-check 1 > $O/b_$v.log 2>&1 || { tail -5 $O/b_$v.log; exit 1; }
  python3 -c "
import json
for l in open('$O/b_$v.log'):
    if l.startswith('{'): d=json.loads(l); k=d['kernels_ms_per_step']; print('$v', round(d['ms_per_step'],1), k.get('k_helper_xof'), k.get('k_jr_ring'))
"
done
