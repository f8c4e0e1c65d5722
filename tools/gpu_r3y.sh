#!/bin/bash
# Round-3 session y: the weight-row pitch A/B (gpu_r3x.sh), then the round-end check of the
# final tree with its defaults.
set -u
bash tools/gpu_r3x.sh || exit 1
bash tools/final_check.sh
