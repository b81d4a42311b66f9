#!/bin/bash
# Steady-state PMC passes for single kernels via diag_one.py (3 launches each after WARM steps).
# Usage: bash scripts/gpu_pmc_kernels.sh "K:REGEX K:REGEX ..."
R=${GRAFT_REPO_ROOT:-$(pwd)}
export WARM=${WARM:-800} ITERS=3 V=0
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAIT_INST_ANY"
P2="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_MFMA"
P3="TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TA_BUSY_avr TCP_TCP_TA_DATA_STALL_CYCLES_sum"
for kr in $1; do
  export K=${kr%%:*}; RX=${kr#*:}
  for p in 1 2 3; do
    eval CNT=\$P$p
    bash "$R/scripts/gpu_pmc_diag.sh" "k${K}_p$p" "$CNT" "$RX" || exit $?
  done
done
