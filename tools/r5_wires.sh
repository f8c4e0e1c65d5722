set -o pipefail
# SumVec MFMA wire pass: nt loads (aux 2) and 8 K-steps per load batch vs the default.
O=gpurun_out/r5_wires; mkdir -p $O
for v in "" nt2 u8 "" nt2 u8; do
  lib=""; [ -n "$v" ] && lib="PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_$v.so"
  env $lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --prof-steps 2 --cpu-baseline 0 --helper-only 0 --hpke 0 > $O/b_$v.log 2>&1 || { tail -5 $O/b_$v.log; exit 1; }
  grep '^{' $O/b_$v.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); k=d.get('kernels_ms_per_step',{}); print('${v:-base}', d['value'], d['ms_per_step'], 'wires', k.get('k_flp_wires_mfma'))"
done
