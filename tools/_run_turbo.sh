set -o pipefail
timeout -k 10 400 python -u bench.py --xof turboshake128 --steps 5 --warmup 1 > gpurun_out/bench_r02_turbo.log 2>&1; rc=$?; tail -c 2500 gpurun_out/bench_r02_turbo.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --cpu-baseline 0 --hpke 0 --helper-only 0 > gpurun_out/bench_r02_shake_check.log 2>&1; rc=$?; tail -c 600 gpurun_out/bench_r02_shake_check.log; exit $rc
