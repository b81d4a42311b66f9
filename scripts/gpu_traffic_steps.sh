#!/bin/bash
# HBM-side traffic per launch of the training step's OWN kernels at the bench state (MI355X_MICROARCH.md §HBM):
# separate rocprofv3 --pmc passes over scripts/diag_steps.py (WARM steps, then STEPS measured steps); each kernel's
# last LAST dispatches are summarised (the measured steps' launches: 4 progressive k_nerf_infer rounds per step).
# Usage: bash scripts/gpu_traffic_steps.sh TAG [LAST]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-steps}
LAST=${2:-20}
export WARM=${WARM:-800} STEPS=${STEPS:-5}
RX=${RX:-"k_nerf_infer"}
mkdir -p "$R/gpurun_out"
i=0
for CNT in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc $CNT --kernel-include-regex "$RX" --output-format csv \
     -d "$R/gpurun_out/pmcs_${TAG}_p$i" -o run -- python3 "$R/scripts/diag_steps.py" > "$R/gpurun_out/pmcs_${TAG}_p$i.log" 2>&1) || { echo "pmc pass $i failed"; exit 1; }
  echo "pmc pass $i ok"
done
python3 "$R/scripts/pmc_table.py" --last "$LAST" "$R"/gpurun_out/pmcs_${TAG}_p* > "$R/gpurun_out/${TAG}_table.txt" && rm -rf "$R"/gpurun_out/pmcs_${TAG}_p*/
