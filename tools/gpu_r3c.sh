#!/bin/bash
# Round-3 first GPU session: the whole -m gpu suite + default bench (tools/gpu_check.sh), then the
# sponge A/B (base / deferred k_expand stores / spread k_jr LDS-DMA / both).  A fault, abort,
# segfault or time limit ends the session.
set -u
bash tools/gpu_check.sh r03a
rc=$?
case $rc in 0|1) ;; *) exit $rc ;; esac
bash tools/ab.sh r3c "base:X=1" "e1:PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_e1.so" \
  "j1:PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_j1.so" "ej:PRIO3GPU_LIB=janus_amd/lib/libprio3gpu_ej.so" \
  "base2:X=1"
