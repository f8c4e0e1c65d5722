#!/bin/bash
# Build an A/B variant of the engine library (same sources, extra -D flags) for PRIO3GPU_LIB:
#   tools/build_variant.sh NAME "-DFOO=1 ..."   ->  janus_amd/lib/libprio3gpu_NAME.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/janus_amd/csrc
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared $2 -o "$R/janus_amd/lib/libprio3gpu_$1.so" \
  "$C/engine.hip" "$C/codec.cpp" "$C/hpke.cpp" -lrccl -lcrypto
