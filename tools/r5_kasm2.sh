set -o pipefail
# Rolled asm Keccak (P3G_KECCAK_ASM=2): GPU parity, SumVec A/B, config E (10,240, serial) A/B.
O=gpurun_out/r5_kasm2; mkdir -p $O
PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_kroll.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_kroll.log 2>&1 || { tail -30 $O/pytest_kroll.log; exit 1; }
tail -1 $O/pytest_kroll.log
for v in "" kroll "" kroll; do
  lib=""; [ -n "$v" ] && lib="PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_$v.so"
  env $lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --prof-steps 2 > $O/b_$v.log 2>&1 || { tail -5 $O/b_$v.log; exit 1; }
  grep '^{' $O/b_$v.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); k=d.get('kernels_ms_per_step',{}); print('${v:-base}', d['value'], d['ms_per_step'], 'k_jr', k.get('k_jr'), 'k_expand', k.get('k_expand'))"
done
for v in "" kroll; do
  lib=""; [ -n "$v" ] && lib="PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_$v.so"
  env $lib timeout -k 10 300 python -u tools/bench_fpvec.py --reports 10240 --unique 16 --steps 2 --warmup 1 > $O/e_$v.log 2>&1 || { tail -5 $O/e_$v.log; exit 1; }
  python3 -c "
import json
for l in open('$O/e_$v.log'):
    if l.startswith('{'): d=json.loads(l); k=d['kernels_ms_per_step']; print('E ${v:-base}', round(d['reports_per_sec'],1), round(d['ms_per_step'],1), k.get('k_jr_ring'), k.get('k_helper_xof'), k.get('k_fpv_regen'))
"
done
