set -o pipefail
# Config E batch size at the HBM limit: 10,240 / 10,752 / 10,880 reports (snap_chunk 256).
O=gpurun_out/r5_fpv17; mkdir -p $O
for spec in "10240|--opt snap_chunk=256" "10752|--opt snap_chunk=256" "10880|--opt snap_chunk=256"; do
  IFS='|' read -r B opt <<< "$spec"
  tag=$(echo "$B $opt" | tr -c 'a-z0-9\n' '_')
  timeout -k 10 300 python -u tools/bench_fpvec.py --reports $B --unique 16 --steps 3 --warmup 1 $opt > $O/b_$tag.log 2>&1 || { tail -3 $O/b_$tag.log; continue; }
  python3 -c "
import json
for l in open('$O/b_$tag.log'):
    if l.startswith('{'): d=json.loads(l); k=d['kernels_ms_per_step']; print('$B $opt', round(d['reports_per_sec'],1), round(d['ms_per_step'],1), {a:b for a,b in k.items() if b>5})
"
done
