#!/bin/bash
# One rocprofv3 PMC pass over a short run (one counter group per run, as MI355X_MICROARCH.md
# prescribes), summarised per kernel (full-size dispatches).
#   tools/pmc_pass.sh TAG "CTR1 CTR2 ..." [script.py args...]   (default: bench.py, 1 step)
set -uo pipefail
TAG=$1; CTRS=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/pmc_$TAG
mkdir -p "$O"
if [ $# -gt 0 ] && [[ "$1" == *.py ]]; then SCRIPT=$R/$1; shift; ARGS="$*"
else SCRIPT=$R/bench.py; ARGS="--steps 1 --warmup 0 --cpu-baseline 0 --hpke 0 --helper-only 0 $*"; fi
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 600 rocprofv3 --pmc $CTRS --output-format csv -d "$O/raw" -o run -- python3 "$SCRIPT" $ARGS > "$O/run.log" 2>&1
rc=$?
[ $rc -ne 0 ] && { tail -5 "$O/run.log"; exit $rc; }
python3 "$R/tools/pmc_summary.py" --sq "$O/raw" --out "$R/gpurun_out/pmc_$TAG.json"
rm -rf "$O/raw"
