#!/bin/bash
# Instruction / wait counters of the Adam / EMA pass (replayed, K=12) at the bench's steady state.
# Usage: bash scripts/gpu_pmc_adam.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-adam}
export WARM=800 ITERS=3 V=99 K=12
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAIT_INST_ANY"
P2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS"
for p in 1 2; do
  eval CNT=\$P$p
  bash "$R/scripts/gpu_pmc_diag.sh" "${TAG}_a$p" "$CNT" "k_adam_ema" || exit $?
  python3 "$R/scripts/pmc_table.py" --last 3 "$R/gpurun_out/pmcd_${TAG}_a$p" > "$R/gpurun_out/pmc_${TAG}_adam_p$p.txt" 2>&1
  rm -rf "$R/gpurun_out/pmcd_${TAG}_a$p"
  cat "$R/gpurun_out/pmc_${TAG}_adam_p$p.txt"
done
echo PMC_DONE
