set -o pipefail
O=gpurun_out/r5_diag1; mkdir -p $O
for spec in "base|sum" "sqnl|sum" "base|sumvec" "fwnl|sumvec"; do
  IFS='|' read -r lib cfg <<< "$spec"
  if [ $lib = base ]; then E=""; else E="PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_$lib.so"; fi
  env $E timeout -k 10 300 python -u tools/sponge_ab.py --config $cfg --query 1 --reps 3 --label $lib > $O/${lib}_$cfg.log 2>&1 || { tail -5 $O/${lib}_$cfg.log; exit 1; }
  tail -1 $O/${lib}_$cfg.log
done
