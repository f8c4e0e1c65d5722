set -o pipefail
# Bank-aware asm Keccak (P3G_KECCAK_ASM=1 variant): GPU parity, then the SumVec headline A/B.
O=gpurun_out/r5_kasm1; mkdir -p $O
PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_kasm.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_kasm.log 2>&1 || { tail -30 $O/pytest_kasm.log; exit 1; }
tail -1 $O/pytest_kasm.log
for v in "" kasm "" kasm; do
  lib=""; [ -n "$v" ] && lib="PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_$v.so"
  env $lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --prof-steps 2 > $O/b_$v.log 2>&1 || { tail -5 $O/b_$v.log; exit 1; }
  grep '^{' $O/b_$v.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); k=d.get('kernels_ms_per_step',{}); print('${v:-base}', d['value'], d['ms_per_step'], 'k_jr', k.get('k_jr'), 'k_expand', k.get('k_expand'), 'wires', k.get('k_flp_wires_mfma'))"
done
