#!/bin/bash
# Round-3 counter passes at the bench's steady state (800 training steps): the march and the fused inference.
# Usage: bash scripts/gpu_r03_pmc.sh TAG   -> gpurun_out/pmc_TAG_<kernel>_p<k>.txt
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r03}
export WARM=800 ITERS=3 V=99
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAIT_INST_ANY"
P2="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_MFMA"
P3="TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TA_BUSY_avr TCP_TCP_TA_DATA_STALL_CYCLES_sum"
for kr in "0:k_march<" "3:k_nerf_infer"; do
  export K=${kr%%:*}; RX=${kr#*:}
  for p in 1 2 3; do
    eval CNT=\$P$p
    bash "$R/scripts/gpu_pmc_diag.sh" "${TAG}_k${K}_p$p" "$CNT" "$RX" || exit $?
    python3 "$R/scripts/pmc_table.py" --last 3 "$R/gpurun_out/pmcd_${TAG}_k${K}_p$p" > "$R/gpurun_out/pmc_${TAG}_k${K}_p$p.txt" 2>&1
    rm -rf "$R/gpurun_out/pmcd_${TAG}_k${K}_p$p"
    cat "$R/gpurun_out/pmc_${TAG}_k${K}_p$p.txt"
  done
done
echo PMC_DONE
