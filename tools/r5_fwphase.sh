set -o pipefail
# k_flp_weights phase attribution (timing-only builds without one phase's products), SumVec
# query phase through tools/sponge_ab.py --query 1 (no parity checks).
O=gpurun_out/r5_fwphase; mkdir -p $O
for v in "" fwp1 fwp2 fwp3 ""; do
  lib=""; [ -n "$v" ] && lib="PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_$v.so"
  env $lib timeout -k 10 300 python -u tools/sponge_ab.py --query 1 --reps 3 > $O/s_$v.log 2>&1 || { tail -5 $O/s_$v.log; exit 1; }
  grep -o '"k_flp_weights": [0-9.]*' $O/s_$v.log | head -1 | sed "s/^/${v:-base} /"
done
