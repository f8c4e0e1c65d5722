set -o pipefail
timeout -k 10 120 ./tools/mb_keccak_pair > gpurun_out/mb_keccak_pair.log 2>&1; rc=$?; cat gpurun_out/mb_keccak_pair.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_fpvec_env.sh "spec: nospec:PRIO3GPU_HX_SPEC=0 spec2:"
