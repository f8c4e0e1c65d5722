#!/bin/bash
# Round-6 k_flp_weights A/B: GPU parity of every ParallelSum config, then the FLP phase timing
# (tools/sponge_ab.py --query 1) of the product build against a reference build, alternated.
#   usage: tools/r6_fw.sh REFLIB [REPS]   (janus_amd/lib/libprio3gpu_REFLIB.so)
set -o pipefail
O=gpurun_out/r6_fw; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "sumvec or hist or countvec or transcript or aggregate_and_unshard or noncanonical" \
  > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in $(seq 1 ${2:-2}); do
  for lib in prod $1; do
    if [ $lib = prod ]; then P=janus_amd/lib/libprio3gpu.so; else P=janus_amd/lib/libprio3gpu_$lib.so; fi
    for cfg in sumvec histogram; do
      PRIO3GPU_LIB=$P timeout -k 10 300 python -u tools/sponge_ab.py --config $cfg --query 1 --reps 3 \
        --label $lib > $O/${lib}_${cfg}_$rep.log 2>&1 || { tail -5 $O/${lib}_${cfg}_$rep.log; exit 1; }
      python3 -c "
import json,sys
d=json.loads(open('$O/${lib}_${cfg}_$rep.log').read().strip().splitlines()[-1])
print(d['label'], d['config'], {k:v for k,v in d['ms_per_launch_min'].items() if 'weights' in k or 'wires' in k})"
    done
  done
done
