#!/bin/bash
# Register / LDS / spill summary of selected kernels in a built library (measurement tooling).
#   tools/kinfo.sh LIB.so REGEX
set -e
T=$(mktemp -d)
cp "$1" "$T/lib.so"
cd "$T"
/opt/rocm/lib/llvm/bin/llvm-objdump --offloading lib.so > /dev/null 2>&1
CO=$(ls "$T"/*gfx950* | head -1)
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$CO" | grep -A40 "\.name:.*\($2\)" | grep -E "\.name|vgpr_count|sgpr_spill|vgpr_spill|group_segment_fixed|private_segment_fixed" || true
[ -n "$3" ] && /opt/rocm/lib/llvm/bin/llvm-objdump -d --no-show-raw-insn "$CO" > "$3"
rm -rf "$T"
