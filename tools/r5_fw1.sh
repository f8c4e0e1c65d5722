set -o pipefail
# k_flp_weights occupancy A/B on the headline (SumVec): default build vs amdgpu_waves_per_eu(3).
O=gpurun_out/r5_fw1; mkdir -p $O
for v in "" fw3 "" fw3; do
  lib=""; [ -n "$v" ] && lib="PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_$v.so"
  env $lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --prof-steps 2 > $O/b_$v.log 2>&1 || { tail -5 $O/b_$v.log; exit 1; }
  grep '^{' $O/b_$v.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); k=d.get('kernels_ms_per_step',{}); print('$v', d['value'], d['ms_per_step'], 'weights', k.get('k_flp_weights'), 'wires', k.get('k_flp_wires_mfma'))"
done
