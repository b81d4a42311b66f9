#!/bin/bash
# L2 hit / miss and memory-side reads of the training step's inference rounds (k_nerf_infer, progressive, all levels)
# per value of an environment variable: bash scripts/gpu_l2_ab.sh TAG VAR v1 v2 ...   (scripts/diag_steps.py, WARM=800)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=$1; VAR=$2; shift 2
export WARM=${WARM:-800} STEPS=${STEPS:-5}
for V in "$@"; do
  (cd /tmp && export TMPDIR=/tmp && export "$VAR=$V" && timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum \
     --kernel-include-regex k_nerf_infer --output-format csv -d "$R/gpurun_out/pmcl2_${TAG}_$V" -o run -- python3 "$R/scripts/diag_steps.py" \
     > "$R/gpurun_out/pmcl2_${TAG}_$V.log" 2>&1) || { echo "pmc failed for $V"; exit 1; }
  python3 scripts/pmc_table.py --last 15 gpurun_out/pmcl2_${TAG}_$V > gpurun_out/pmcl2_${TAG}_${V}_table.txt && rm -rf gpurun_out/pmcl2_${TAG}_$V/
  echo "== $VAR=$V"; grep -A5 "Lb1ELb1E" gpurun_out/pmcl2_${TAG}_${V}_table.txt
done
echo L2_OK
