#!/bin/bash
# One GPU session: the -m gpu tests, then the default bench, each under its own time limit.
# A step that faults, aborts, segfaults, times out or hangs ends the session (no later GPU step);
# ordinary test failures (pytest rc 1) still let the bench run.   usage: tools/gpu_check.sh TAG [bench args]
TAG=${1:-r02}
shift
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/gpurun_out"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > "gpurun_out/pytest_gpu_$TAG.log" 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 "gpurun_out/pytest_gpu_$TAG.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 420 python -u bench.py "$@" > "gpurun_out/bench_$TAG.log" 2>&1
brc=$?
echo "bench rc=$brc"
tail -c 4000 "gpurun_out/bench_$TAG.log"
[ $rc -eq 0 ] && exit $brc
exit $rc
