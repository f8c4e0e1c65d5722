set -o pipefail
bash tools/ab.sh hx "base:X=0" "hx2:PRIO3GPU_FUSED_HELPER=2" "hx4:PRIO3GPU_FUSED_HELPER=2;PRIO3GPU_HX_DEPTH=4" || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_hxa.log 2>&1; echo "pytest default rc=$?"; tail -3 gpurun_out/pytest_hxa.log
PRIO3GPU_FUSED_HELPER=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_spec.py tests/test_gpu_squeeze.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_hxb.log 2>&1; echo "pytest fused rc=$?"; tail -3 gpurun_out/pytest_hxb.log
