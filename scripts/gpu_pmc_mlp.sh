#!/bin/bash
# Instruction-mix / stall counters of the training-MLP kernels (9 colour, 10 density) and the march (0), replayed on the
# bench state (scripts/diag_one.py, V=99: only the timed kernel is launched). Usage: bash scripts/gpu_pmc_mlp.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-mlp}
mkdir -p "$R/gpurun_out"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 60 rocprofv3 --list-avail > "$R/gpurun_out/counters_avail.txt" 2>&1) || echo "list-avail rc=$?"
export WARM=${WARM:-800} ITERS=3 V=99 K=${K:-9,10,0}
RX=${RX:-"k_mlp_train|k_march<"}
i=0
for CNT in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_BUSY_CYCLES" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  bash "$R/scripts/gpu_pmc_diag.sh" "${TAG}_p$i" "$CNT" "$RX" || exit $?
done
python3 "$R/scripts/pmc_table.py" --last 3 "$R"/gpurun_out/pmcd_${TAG}_p* > "$R/gpurun_out/${TAG}_pmc_table.txt" && rm -rf "$R"/gpurun_out/pmcd_${TAG}_p*/
cat "$R/gpurun_out/${TAG}_pmc_table.txt"
