#!/bin/bash
# HBM-side traffic per launch of the hot kernels (MI355X_MICROARCH.md §HBM): separate rocprofv3 --pmc
# passes for FETCH_SIZE, WRITE_SIZE and the L2->fabric read-request size breakdown, over 3 replayed
# launches of each kernel after WARM training steps. Usage: bash scripts/gpu_traffic.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-traffic}
export WARM=${WARM:-800} ITERS=3 V=99 K=${K:-3,7,0,5,8,1,4}
RX=${RX:-"k_nerf_infer|k_scatter|k_march|k_ray_gen|k_mlp_train|k_grid_encode|k_loss_alpha|k_adam_ema|rocprim"}
i=0
for CNT in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  bash "$R/scripts/gpu_pmc_diag.sh" "${TAG}_p$i" "$CNT" "$RX" || exit $?
done
# summarise the replayed launches on the box and drop the per-dispatch CSVs of the warm-up steps
python3 "$R/scripts/pmc_table.py" --last 3 "$R"/gpurun_out/pmcd_${TAG}_p* > "$R/gpurun_out/${TAG}_table.txt" && rm -rf "$R"/gpurun_out/pmcd_${TAG}_p*
