#!/bin/bash
# A/B of bench.py variants on one box, each run under its own time limit; stops at the first
# failure (GPU fault, abort, timeout).  Each argument is  LABEL|LIB|ENV|BENCH-ARGS  where LIB is a
# variant library name (tools/build_variant.sh NAME -> janus_amd/lib/libprio3gpu_NAME.so) or
# "base", ENV is "-" or space-separated VAR=value settings for that run only, e.g.
#   bash tools/ab_bench.sh "ov0|base|-|--overlap 0" "ov2cap|base|PRIO3GPU_JR_LDS=65536|--overlap 2"
# Output: gpurun_out/ab_LABEL.log, one summary line per run on stdout.
O=gpurun_out; mkdir -p $O
COMMON="--steps 6 --warmup 2 --cpu-baseline 0 --hpke 0 --helper-only 0"
for spec in "$@"; do
  IFS='|' read -r label libn envs args <<< "$spec"
  vars=()
  [ "$libn" != base ] && vars+=("PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_$libn.so")
  [ "$envs" != "-" ] && vars+=($envs)
  env "${vars[@]}" timeout -k 10 300 python -u bench.py $COMMON $args > $O/ab_$label.log 2>&1
  rc=$?
  python - "$O/ab_$label.log" "$label" "$rc" <<'PY'
import json, sys
path, label, rc = sys.argv[1:]
line = [l for l in open(path) if l.startswith("{")]
if not line:
    print(f"== {label} rc={rc} (no JSON line)"); sys.exit(0)
d = json.loads(line[-1])
k = {n: round(v, 2) for n, v in d["kernels_ms_per_step"].items() if v > 0.5}
print(f"== {label} rc={rc} value={d['value']:.0f} ms/step={d['ms_per_step']} kernels={k}")
PY
  [ $rc -ne 0 ] && { tail -20 $O/ab_$label.log; exit $rc; }
done
exit 0
