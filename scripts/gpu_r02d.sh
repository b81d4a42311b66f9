#!/bin/bash
# Kernel-trace summary of the driver-shaped bench (warmup 5, steps 20) + PMC traffic of the inference and march
# kernels at that state (4 active levels) and at steady state (14 levels).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r02d}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 > "$R/gpurun_out/prof_$TAG.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 "$R/scripts/prof_summary.py" "$R/gpurun_out/prof_$TAG" "$R/gpurun_out/prof_${TAG}_summary.md" --last-steps 20 && rm -rf "$R/gpurun_out/prof_$TAG"
cd "$R"
WARM=5 K=3,0 bash scripts/gpu_traffic.sh ${TAG}_w5 || exit $?
WARM=800 K=3,0 bash scripts/gpu_traffic.sh ${TAG}_w800 || exit $?
echo ALL_OK
