set -o pipefail
bash tools/pmc_pass.sh r5_sum_sq "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" --config sum --overlap 0 --prof-steps 0 && \
bash tools/pmc_pass.sh r5_sum_tcc "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" --config sum --overlap 0 --prof-steps 0 && \
bash tools/pmc_pass.sh r5_sumvec_tcc "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" --config sumvec --prof-steps 0 && \
python3 - <<'PY'
import json
for t in ("r5_sum_sq","r5_sum_tcc","r5_sumvec_tcc"):
    d=json.load(open(f"gpurun_out/pmc_{t}.json"))
    for k in ("k_flp_query_lane","k_jr","k_expand","k_flp_wires_mfma"):
        if k in d: print(t,k,{a:round(b,3) if isinstance(b,float) else b for a,b in d[k].items()})
PY
