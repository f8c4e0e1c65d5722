set -o pipefail
# Interior-block fast path in jrp_absorb: parity, then config E at 10,752 (twice).
O=gpurun_out/r5_absorb; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wires_mfma.py -x -q --timeout 240 --timeout-method thread -k "fpvec or fixedpoint16" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  timeout -k 10 300 python -u tools/bench_fpvec.py --reports 10752 --unique 16 --steps 3 --warmup 1 --opt snap_chunk=256 > $O/e_$r.log 2>&1 || { tail -5 $O/e_$r.log; exit 1; }
  python3 -c "
import json
for l in open('$O/e_$r.log'):
    if l.startswith('{'): d=json.loads(l); k=d['kernels_ms_per_step']; print('run $r', round(d['reports_per_sec'],1), round(d['ms_per_step'],1), 'ring', k.get('k_jr_ring'), 'hx', k.get('k_helper_xof'))
"
done
