set -o pipefail
# wave_prio A/B at 10,240 reports (x query_overlap), parity first.
O=gpurun_out/r5_fpv10; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wires_mfma.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "fpvec or fixedpoint16 or mfma" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for spec in "10240|" "10240|--opt wave_prio=0" "10240|--opt query_overlap=0" "10240|--opt wave_prio=0 --opt query_overlap=0"; do
  IFS='|' read -r B opt <<< "$spec"
  tag=$(echo "$B $opt" | tr -c 'a-z0-9\n' '_')
  timeout -k 10 300 python -u tools/bench_fpvec.py --reports $B --unique 16 --steps 3 --warmup 1 $opt > $O/b_$tag.log 2>&1 || { tail -5 $O/b_$tag.log; exit 1; }
  python3 -c "
import json
for l in open('$O/b_$tag.log'):
    if l.startswith('{'): d=json.loads(l); k=d['kernels_ms_per_step']; print('$B $opt', round(d['reports_per_sec'],1), round(d['ms_per_step'],1), {a:b for a,b in k.items() if b>5})
"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 tools/bench_fpvec.py --reports 10240 --unique 16 --steps 1 --warmup 1 > $O/b_tr.log 2>&1 || { tail -20 $O/b_tr.log; exit 1; }
