set -o pipefail
# Overlapped helper query (query_overlap 1) with k_fpv_regen occupancy capped by regen_lds.
O=gpurun_out/r5_regen; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "snapshot" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for opt in "--opt snap_chunk=256" "--opt snap_chunk=256 --hopt query_overlap=1" "--opt snap_chunk=256 --hopt query_overlap=1 --hopt regen_lds=49152" "--opt snap_chunk=256 --hopt query_overlap=1 --hopt regen_lds=65536" "--opt snap_chunk=256 --hopt query_overlap=1 --hopt regen_lds=73728"; do
  tag=$(echo "$opt" | tr -c 'a-z0-9\n' '_')
  timeout -k 10 300 python -u tools/bench_fpvec.py --reports 10752 --unique 16 --steps 3 --warmup 1 $opt > $O/e_$tag.log 2>&1 || { tail -5 $O/e_$tag.log; exit 1; }
  python3 -c "
import json
for l in open('$O/e_$tag.log'):
    if l.startswith('{'): d=json.loads(l); k=d['kernels_ms_per_step']; print('$opt', round(d['reports_per_sec'],1), round(d['ms_per_step'],1), 'regen', k.get('k_fpv_regen'), 'w0', k.get('k_fpv_wires0'), 'w1', k.get('k_fpv_wires1'))
"
done
