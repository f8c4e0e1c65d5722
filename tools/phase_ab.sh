#!/bin/bash
# A/B of engine builds on one box: optional GPU parity subset per build, then the XOF phase (and
# with QUERY=1 the FLP query phase) timed by tools/sponge_ab.py, builds alternated REPS times so
# box drift shows.  Builds: "prod" = janus_amd/lib/libprio3gpu.so, NAME =
# janus_amd/lib/libprio3gpu_NAME.so (tools/build_variant.sh, or a build of temporary source copies
# for timing-only diagnostics).
#   CONFIGS="sumvec histogram" QUERY=1 PYTEST_K="sumvec or hist" REPS=2 OUT=gpurun_out/ab \
#     bash tools/phase_ab.sh prod NAME...
set -o pipefail
O=${OUT:-gpurun_out/phase_ab}; mkdir -p $O
lib_path() { [ "$1" = prod ] && echo janus_amd/lib/libprio3gpu.so || echo janus_amd/lib/libprio3gpu_$1.so; }
if [ -n "$PYTEST_K" ]; then
  for lib in "$@"; do
    PRIO3GPU_LIB=$(lib_path $lib) timeout -k 10 400 python -u -m pytest tests -m gpu -x -q \
      --timeout 200 --timeout-method thread -k "$PYTEST_K" > $O/pytest_$lib.log 2>&1 \
      || { tail -20 $O/pytest_$lib.log; exit 1; }
    echo "$lib $(tail -1 $O/pytest_$lib.log)"
  done
fi
for rep in $(seq 1 ${REPS:-2}); do
  for lib in "$@"; do
    for cfg in ${CONFIGS:-sumvec}; do
      f=$O/${lib}_${cfg}_$rep.log
      PRIO3GPU_LIB=$(lib_path $lib) timeout -k 10 300 python -u tools/sponge_ab.py --config $cfg \
        --query ${QUERY:-0} --reps 3 --label $lib > $f 2>&1 || { tail -5 $f; exit 1; }
      tail -1 $f
    done
  done
done
