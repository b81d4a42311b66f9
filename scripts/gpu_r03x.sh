#!/bin/bash
# Round-3 iteration: scatter-mode determinism stress, level-partitioned gather timing, then the scatter tests and the
# steady-state kernel-trace summary (scripts/gpu_iter3.sh). Usage: bash scripts/gpu_r03x.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r03x}
REPS=4 timeout -k 10 250 python -u scripts/stress_scatter_modes.py > gpurun_out/stress_$TAG.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/stress_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/diag_levelpart.py > gpurun_out/levelpart_$TAG.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/levelpart_$TAG.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_iter3.sh $TAG "scatter or bitwise"
