set -o pipefail
# Stall counters of the chain kernels at 10,240 reports, serial schedule (one SQ pass).
O=gpurun_out/r5_fpv14; mkdir -p $O
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_IFETCH SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/sq -o run -- python3 tools/bench_fpvec.py --reports 10240 --unique 16 --steps 1 --warmup 0 --overlap 0 > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 1; }
