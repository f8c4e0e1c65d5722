set -o pipefail
export MASTER_ADDR=127.0.0.1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --merge gloo --reports 131072 --steps 2 --warmup 1 --hpke 0 --cpu-baseline 0 --helper-only 1 > gpurun_out/rehearse_n2.log 2>&1; rc=$?; echo "n2 rc=$rc"; grep '^{"metric"' gpurun_out/rehearse_n2.log | cut -c1-400; [ $rc -ne 0 ] && { tail -20 gpurun_out/rehearse_n2.log; exit $rc; }
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --merge gloo --reports 65536 --steps 2 --warmup 1 --hpke 0 --cpu-baseline 0 --helper-only 0 > gpurun_out/rehearse_n4.log 2>&1; rc=$?; echo "n4 rc=$rc"; grep '^{"metric"' gpurun_out/rehearse_n4.log | cut -c1-400; [ $rc -ne 0 ] && { tail -20 gpurun_out/rehearse_n4.log; exit $rc; }
exit 0
