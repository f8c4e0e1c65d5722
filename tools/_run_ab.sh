set -o pipefail
bash tools/ab.sh wl "base:X=0" "l4:PRIO3GPU_WIRES_LDS=4" "l6:PRIO3GPU_WIRES_LDS=6" "l8:PRIO3GPU_WIRES_LDS=8" "l12:PRIO3GPU_WIRES_LDS=12" || exit $?
PRIO3GPU_WIRES_LDS=8 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_spec.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_wl.log 2>&1; rc=$?; echo "pytest wires_lds rc=$rc"; tail -3 gpurun_out/pytest_wl.log; [ $rc -gt 1 ] && exit $rc
bash tools/ab_fpvec.sh storer 4800
