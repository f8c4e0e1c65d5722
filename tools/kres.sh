#!/bin/bash
# Print VGPR / occupancy of the main kernels (compile-only, no GPU):  tools/kres.sh [pattern]
cd /tmp && hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c --cuda-device-only -Rpass-analysis=kernel-resource-usage \
  -o /tmp/kres.o /root/repo/janus_amd/csrc/engine.hip 2>&1 | python3 -c '
import re,sys
pat=sys.argv[1] if len(sys.argv)>1 else "Field128"
cur=None
for l in sys.stdin:
    m=re.search(r"Function Name: (\S+)",l)
    if m: cur=m.group(1); continue
    m=re.search(r"remark:\s+(VGPRs|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]|ScratchSize \[bytes/lane\]): (\S+)",l)
    if m and cur and re.search(pat,cur): print(cur[:48].ljust(50), m.group(1), m.group(2))
' "${1:-Field128}"
