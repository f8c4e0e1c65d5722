set -o pipefail
# k_fpv_wires1_mfma over tile groups: parity, then config E batch sizes.
O=gpurun_out/r5_fpv18; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wires_mfma.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "fpvec or fixedpoint16 or mfma" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for spec in "10240|" "10752|--opt snap_chunk=256" "10752|" "10880|--opt snap_chunk=128"; do
  IFS='|' read -r B opt <<< "$spec"
  tag=$(echo "$B $opt" | tr -c 'a-z0-9\n' '_')
  timeout -k 10 300 python -u tools/bench_fpvec.py --reports $B --unique 16 --steps 3 --warmup 1 $opt > $O/b_$tag.log 2>&1 || { tail -3 $O/b_$tag.log; continue; }
  python3 -c "
import json
for l in open('$O/b_$tag.log'):
    if l.startswith('{'): d=json.loads(l); k=d['kernels_ms_per_step']; print('$B $opt', round(d['reports_per_sec'],1), round(d['ms_per_step'],1), {a:b for a,b in k.items() if b>5})
"
done
