set -o pipefail
O=gpurun_out/r5_fpv3; mkdir -p $O
for spec in "8192|--pipeline 1 --opt snap_chunk=256" "4096|--pipeline 1 --opt snap_chunk=256"; do
  IFS='|' read -r B opt <<< "$spec"
  tag=$(echo "$B $opt" | tr -c 'a-z0-9\n' '_')
  timeout -k 10 600 python -u tools/bench_fpvec.py --reports $B --distinct 1 --steps 3 --warmup 1 $opt > $O/b_$tag.log 2>&1 || { tail -20 $O/b_$tag.log; exit 1; }
  python3 -c "
import json
for l in open('$O/b_$tag.log'):
    if l.startswith('{'): d=json.loads(l); print('$B $opt', round(d['reports_per_sec'],1), round(d['ms_per_step'],1), d['steps'])
"
done
