#!/bin/bash
# One rocprofv3 PMC pass over a short bench run (one counter group per run, as MI355X_MICROARCH.md
# prescribes), summarised per kernel.   usage: tools/pmc_pass.sh TAG "CTR1 CTR2 ..." [bench args]
set -uo pipefail
TAG=$1; CTRS=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/pmc_$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc $CTRS --output-format csv -d "$O/raw" -o run -- python3 "$R/bench.py" \
  --steps 1 --warmup 0 --cpu-baseline 0 --hpke 0 --helper-only 0 "$@" > "$O/run.log" 2>&1
rc=$?
[ $rc -ne 0 ] && { tail -5 "$O/run.log"; exit $rc; }
python3 "$R/tools/pmc_summary.py" --sq "$O/raw" --out "$R/gpurun_out/pmc_$TAG.json"
rm -rf "$O/raw"
