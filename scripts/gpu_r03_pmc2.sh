#!/bin/bash
# Round-3 counter passes at the bench's steady state (800 training steps) over replayed launches of the grid scatter
# (K=7), the training MLP (5), its weight-gradient reduction (6) and the Adam / EMA pass (12): two instruction passes
# for the scatter kernels, then the four HBM-traffic passes (FETCH_SIZE / WRITE_SIZE / request sizes, as
# scripts/gpu_traffic.sh). Usage: bash scripts/gpu_r03_pmc2.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r03p}
export WARM=800 ITERS=3 V=99 K=7
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAIT_INST_ANY"
P2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS"
for p in 1 2; do
  eval CNT=\$P$p
  bash "$R/scripts/gpu_pmc_diag.sh" "${TAG}_s$p" "$CNT" "k_scatter" || exit $?
  python3 "$R/scripts/pmc_table.py" --last 3 "$R/gpurun_out/pmcd_${TAG}_s$p" > "$R/gpurun_out/pmc_${TAG}_scatter_p$p.txt" 2>&1
  rm -rf "$R/gpurun_out/pmcd_${TAG}_s$p"
  cat "$R/gpurun_out/pmc_${TAG}_scatter_p$p.txt"
done
export K=7,5,6,12
RX="k_scatter|k_mlp_train|k_mlp_grad_reduce|k_adam_ema"
i=0
for CNT in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  bash "$R/scripts/gpu_pmc_diag.sh" "${TAG}_t$i" "$CNT" "$RX" || exit $?
done
python3 "$R/scripts/pmc_table.py" --last 3 "$R"/gpurun_out/pmcd_${TAG}_t* > "$R/gpurun_out/${TAG}_traffic_table.txt" && rm -rf "$R"/gpurun_out/pmcd_${TAG}_t*
cat "$R/gpurun_out/${TAG}_traffic_table.txt"
echo PMC_DONE
