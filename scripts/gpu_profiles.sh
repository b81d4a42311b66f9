#!/bin/bash
# rocprofv3 kernel-trace summaries of the driver-shaped bench and of a steady-state run (main config only: --l16 0).
# Usage: bash scripts/gpu_profiles.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 > "$R/gpurun_out/prof_$TAG.log" 2>&1 || { echo PROF_FAIL; exit 1; }
python3 "$R/scripts/prof_summary.py" "$R/gpurun_out/prof_$TAG" "$R/gpurun_out/prof_${TAG}_drv_summary.md" --last-steps 20 > /dev/null && rm -rf "$R/gpurun_out/prof_$TAG"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 50 --warmup 800 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 > "$R/gpurun_out/prof_${TAG}_steady.log" 2>&1 || { echo PROF2_FAIL; exit 1; }
python3 "$R/scripts/prof_summary.py" "$R/gpurun_out/prof_$TAG" "$R/gpurun_out/prof_${TAG}_steady_summary.md" --last-steps 50 > /dev/null && rm -rf "$R/gpurun_out/prof_$TAG"
echo PROF_OK
