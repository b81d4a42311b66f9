#!/bin/bash
# rocprofv3 PMC passes (counters only with kernel-trace; never combined with runtime/hip/sys traces).
# Usage: bash scripts/gpu_pmc.sh TAG "COUNTERS..." [kernel regex]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; CNT=$2; RX=${3:-.*}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc $CNT --kernel-include-regex "$RX" --output-format csv -d "$R/gpurun_out/pmc_$TAG" -o run -- python3 "$R/bench.py" --steps 5 --warmup 800 --cpu-baseline 0 > "$R/gpurun_out/pmc_$TAG.log" 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
