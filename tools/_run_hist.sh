set -o pipefail
for sl in 256 64 128; do
  PRIO3GPU_WIRES_SLOTS=$sl timeout -k 10 300 python -u bench.py --config histogram --steps 3 --warmup 1 --hpke 0 --cpu-baseline 0 --helper-only 0 > gpurun_out/ab_hist_slots$sl.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/ab_hist_slots$sl.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/ab_hist_slots$sl.log'):
    if l.startswith('{'): d=json.loads(l); print('slots $sl', d['value'], d['ms_per_step'], {k:v for k,v in d['kernels_ms_per_step'].items() if v>0.3})
"
done
