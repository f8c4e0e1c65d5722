set -o pipefail
O=gpurun_out/r5_fpv; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "fpvec or fixedpoint or fp16 or fp32 or fp64" --timeout 300 --timeout-method thread > $O/pytest_fpv.log 2>&1 || { tail -30 $O/pytest_fpv.log; exit 1; }
tail -1 $O/pytest_fpv.log
for spec in "4800|helper_snap=0" "4800|helper_snap=1" "8192|helper_snap=1"; do
  IFS='|' read -r B opt <<< "$spec"
  timeout -k 10 400 python -u tools/bench_fpvec.py --reports $B --distinct 1 --steps 2 --warmup 1 --opt $opt > $O/bench_${B}_$opt.log 2>&1 || { tail -20 $O/bench_${B}_$opt.log; exit 1; }
  python3 -c "
import json
for l in open('$O/bench_${B}_$opt.log'):
    if l.startswith('{'): d=json.loads(l); print('$B $opt', round(d['reports_per_sec'],1), round(d['ms_per_step'],1), {k:v for k,v in d['kernels_ms_per_step'].items() if v>5})
"
done
