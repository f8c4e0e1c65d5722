#!/bin/bash
# Collect the round's rocprofv3 evidence on a GPU box (kernel trace + separate PMC passes, as
# MI355X_MICROARCH.md prescribes) and summarise into profiles/.
#   usage: tools/profile_round.sh TAG [CONFIG]   (CONFIG: a bench.py --config, default sumvec)
set -euo pipefail
TAG=${1:-r01}
CFG=${2:-sumvec}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/prof_${TAG}_$CFG
mkdir -p "$O" "$R/profiles"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --cpu-baseline 0 --hpke 0 --helper-only 0 --config $CFG"
ONE="--steps 1 --warmup 0 --cpu-baseline 0 --hpke 0 --helper-only 0 --config $CFG"
# the trace pass runs every kernel alone (--overlap 0: one context, one stream), so its durations
# are the kernels' own, like the PMC passes (which serialise dispatches) and bench.py's serial pass
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- python3 "$R/bench.py" $ARGS --overlap 0 > "$O/trace.log" 2>&1
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch" -o run -- python3 "$R/bench.py" $ONE > "$O/fetch.log" 2>&1
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write" -o run -- python3 "$R/bench.py" $ONE > "$O/write.log" 2>&1
timeout -k 10 500 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/sq" -o run -- python3 "$R/bench.py" $ONE > "$O/sq.log" 2>&1
python3 "$R/tools/pmc_summary.py" --trace "$O/trace" --fetch "$O/fetch" --write "$O/write" --sq "$O/sq" --out "$R/gpurun_out/pmc_${CFG}_$TAG.json" > "$O/summary.txt"
cp "$O"/trace/*kernel_stats.csv "$R/gpurun_out/kernel_stats_${CFG}_$TAG.csv" 2>/dev/null || find "$O/trace" -name "*kernel_stats.csv" -exec cp {} "$R/gpurun_out/kernel_stats_${CFG}_$TAG.csv" \;
grep "^{\"metric\"" "$O/trace.log" > "$R/gpurun_out/bench_under_rocprof_${CFG}_$TAG.json" || true
cat "$O/summary.txt"
