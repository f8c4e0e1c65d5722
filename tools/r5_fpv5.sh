set -o pipefail
# chain_pairs: parity, then config E at 8,192 / 10,240 / 11,264 reports per step.
O=gpurun_out/r5_fpv5; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "fpvec or fixedpoint16" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for spec in "8192|" "10240|" "10240|--opt snap_chunk=256" "11264|--opt snap_chunk=256"; do
  IFS='|' read -r B opt <<< "$spec"
  tag=$(echo "$B $opt" | tr -c 'a-z0-9\n' '_')
  timeout -k 10 300 python -u tools/bench_fpvec.py --reports $B --unique 16 --steps 3 --warmup 1 $opt > $O/b_$tag.log 2>&1 || { tail -20 $O/b_$tag.log; exit 1; }
  python3 -c "
import json
for l in open('$O/b_$tag.log'):
    if l.startswith('{'): d=json.loads(l); k=d['kernels_ms_per_step']; print('$B $opt', round(d['reports_per_sec'],1), round(d['ms_per_step'],1), 'jr_ring', k.get('k_jr_ring'), 'hx', k.get('k_helper_xof'), 'regen', k.get('k_fpv_regen'))
"
done
