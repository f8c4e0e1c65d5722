#!/bin/bash
# Round-3 GPU session b: the new GPU tests, then the sponge A/B (base / deferred k_expand stores /
# spread k_jr LDS-DMA / both).  A fault, abort, segfault or time limit ends the session.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_flp_branches.py tests/test_gpu_async.py tests/test_leader.py tests/test_hpke.py \
  > gpurun_out/pytest_r3b.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_r3b.log
case $rc in 0|1) ;; *) exit $rc ;; esac
bash tools/ab.sh r3b "base:X=1" "e1:PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_e1.so" \
  "j1:PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_j1.so" "ej:PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_ej.so" \
  "base2:X=1"
