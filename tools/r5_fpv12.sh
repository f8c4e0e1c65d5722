set -o pipefail
# Chain-phase diagnostics at 10,240 reports, serial schedule: times with/without the storer's
# column sums, and SQ / GRBM counters of the chain kernels.
O=gpurun_out/r5_fpv12; mkdir -p $O
for spec in "10240|--overlap 0" "10240|--overlap 0 --opt speculate=0" "10240|"; do
  IFS='|' read -r B opt <<< "$spec"
  tag=$(echo "$B $opt" | tr -c 'a-z0-9\n' '_')
  timeout -k 10 300 python -u tools/bench_fpvec.py --reports $B --unique 16 --steps 3 --warmup 1 $opt > $O/b_$tag.log 2>&1 || { tail -5 $O/b_$tag.log; exit 1; }
  python3 -c "
import json
for l in open('$O/b_$tag.log'):
    if l.startswith('{'): d=json.loads(l); k=d['kernels_ms_per_step']; print('$B $opt', round(d['reports_per_sec'],1), round(d['ms_per_step'],1), {a:b for a,b in k.items() if b>5})
"
done
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/sq -o run -- python3 tools/bench_fpvec.py --reports 10240 --unique 16 --steps 1 --warmup 0 --overlap 0 > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 1; }
