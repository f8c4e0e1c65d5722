#!/bin/bash
# Round-3 session f: k_jr scalar-based window fills -- parity (spec fold + transcripts), then timing.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_spec.py tests/test_gpu_parity.py tests/test_gpu_squeeze.py > gpurun_out/pytest_r3f.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_r3f.log
[ $rc -ne 0 ] && exit $rc
for l in a b; do
  timeout -k 10 240 python -u tools/sponge_ab.py --label jrbuf_$l >> gpurun_out/sponge_r3f.log 2> gpurun_out/sponge_r3f.err || { tail -5 gpurun_out/sponge_r3f.err; exit 1; }
  tail -1 gpurun_out/sponge_r3f.log
done
timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --cpu-baseline 0 --hpke 0 --helper-only 0 > gpurun_out/bench_r3f.log 2>&1 || { tail -5 gpurun_out/bench_r3f.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/bench_r3f.log'):
    if l.startswith('{'):
        d=json.loads(l); print('bench', d['value'], 'ms/step', d['ms_per_step']); print(' ', d['kernels_ms_per_step'])
"
for v in tile nost; do
  PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_$v.so timeout -k 10 240 python -u tools/sponge_ab.py --label $v >> gpurun_out/sponge_r3f.log 2> gpurun_out/sponge_r3f.err || { tail -5 gpurun_out/sponge_r3f.err; exit 1; }
  tail -1 gpurun_out/sponge_r3f.log
done
