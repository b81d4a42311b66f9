#!/bin/bash
# PMC pass over scripts/diag_one.py. Usage: bash scripts/gpu_pmc_diag.sh TAG "COUNTERS" KERNEL_REGEX  (env K, V, WARM)
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; CNT=$2; RX=${3:-.*}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc $CNT --kernel-include-regex "$RX" --output-format csv -d "$R/gpurun_out/pmcd_$TAG" -o run -- python3 "$R/scripts/diag_one.py" > "$R/gpurun_out/pmcd_$TAG.log" 2>&1
rc=$?; echo "pmc $TAG rc=$rc"; exit $rc
