#!/bin/bash
# Round-3 session v: the short-row MFMA wire pass (gpu_r3u.sh), then the round-end check with it
# switched on (every GPU test, smoke, the four bench lines).
set -u
bash tools/gpu_r3u.sh || exit 1
PRIO3GPU_WIRES_MFMA_SHORT=1 bash tools/final_check.sh
