#!/bin/bash
# Round-4 session g: GPU tests, Sum / SumVec bench, the round's rocprofv3 profile (trace + PMC
# passes) of the default bench command, and an SQ pass over the Sum config.
set -o pipefail
bash tools/gpu_session.sh "sum|base|-|--config sum" "sv|base|-|" || exit 1
timeout -k 10 900 bash tools/profile_round.sh r04 > gpurun_out/profile_r04.log 2>&1 || { tail -20 gpurun_out/profile_r04.log; exit 1; }
tail -30 gpurun_out/profile_r04.log
timeout -k 10 300 bash tools/pmc_pass.sh sumsq "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY" --config sum
