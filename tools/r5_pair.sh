#!/bin/bash
# lane-pair (bit-interleaved) Keccak chain latency vs keccak.h, tools/mb_pair.hip
set -o pipefail
mkdir -p gpurun_out/r5_pair
timeout -k 10 120 ./tools/mb_pair > gpurun_out/r5_pair/mb_pair.log 2>&1; rc=$?
cat gpurun_out/r5_pair/mb_pair.log
exit $rc
