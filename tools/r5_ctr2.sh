set -o pipefail
# Helper ds counters + leader FLAT counters (default) vs both ds (jrlds): parity, config E.
O=gpurun_out/r5_ctr2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wires_mfma.py -x -q --timeout 240 --timeout-method thread -k "fpvec or fixedpoint16" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for spec in "|10240|" "|10240|--overlap 0" "jrlds|10240|" "|10752|--opt snap_chunk=256" "|10880|--opt snap_chunk=128"; do
  IFS='|' read -r v B opt <<< "$spec"
  lib=""; [ -n "$v" ] && lib="PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_$v.so"
  tag=$(echo "$v $B $opt" | tr -c 'a-z0-9\n' '_')
  env $lib timeout -k 10 300 python -u tools/bench_fpvec.py --reports $B --unique 16 --steps 3 --warmup 1 $opt > $O/e_$tag.log 2>&1 || { tail -5 $O/e_$tag.log; exit 1; }
  python3 -c "
import json
for l in open('$O/e_$tag.log'):
    if l.startswith('{'): d=json.loads(l); k=d['kernels_ms_per_step']; print('$v $B $opt', round(d['reports_per_sec'],1), round(d['ms_per_step'],1), 'ring', k.get('k_jr_ring'), 'hx', k.get('k_helper_xof'), 'regen', k.get('k_fpv_regen'))
"
done
