#!/bin/bash
# Round-3 attribution of the sponge kernels' stall cycles (k_jr, k_expand) and of k_flp_wires:
# separate rocprofv3 PMC passes (one counter group per run, MI355X_MICROARCH.md §rocprofv3 PMC slots)
# over a short bench run.  A pass that times out, aborts or faults ends the script (no later GPU step).
#   tools/attrib_r03.sh TAG [bench args...]
set -u
TAG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/attrib_$TAG
mkdir -p "$O"
ARGS="--steps 1 --warmup 0 --cpu-baseline 0 --hpke 0 --helper-only 0 --reports 131072 $*"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$O/counters_list.txt" 2>&1
echo "list rc=$?"
pass() {  # pass NAME "COUNTERS"
  timeout -s KILL 240 rocprofv3 --pmc $2 --output-format csv -d "$O/raw_$1" -o run -- python3 "$R/bench.py" $ARGS > "$O/$1.log" 2>&1
  local rc=$?
  echo "pass $1 rc=$rc"
  if [ $rc -eq 0 ]; then
    python3 "$R/tools/pmc_summary.py" --sq "$O/raw_$1" --out "$O/$1.json" > /dev/null 2>&1
    rm -rf "$O/raw_$1"
  else
    tail -3 "$O/$1.log"
  fi
  case $rc in 124|137|134|139|-6|-11) exit $rc ;; esac
  return 0
}
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d "$O/raw_trace" -o run -- python3 "$R/bench.py" $ARGS > "$O/trace.log" 2>&1
trc=$?
echo "trace rc=$trc"
case $trc in 124|137|134|139) exit $trc ;; esac
find "$O/raw_trace" -name "*kernel_trace.csv" -exec cp {} "$O/kernel_trace.csv" \;
rm -rf "$O/raw_trace"
pass sqA "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
pass sqB "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
pass sqC "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_FLAT SQ_INSTS_SMEM SQ_IFETCH"
pass tcc "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"
pass tcp "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum"
exit 0
