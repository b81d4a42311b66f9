#!/bin/bash
# Bench + rocprofv3 kernel-trace summary on the GPU box (no tests). Usage: bash scripts/gpu_bench.sh [steps] [warmup] [tag]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
STEPS=${1:-50}; WARM=${2:-100}; TAG=${3:-run}
timeout -k 10 600 python bench.py --steps $STEPS --warmup $WARM --cpu-steps 6 > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 20 --warmup 800 --cpu-baseline 0 > "$R/gpurun_out/prof_$TAG.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
[ $rc -eq 0 ] && python3 "$R/scripts/prof_summary.py" "$R/gpurun_out/prof_$TAG" --last-steps 16 > "$R/gpurun_out/prof_${TAG}_summary.md" && rm -rf "$R/gpurun_out/prof_$TAG"
exit $rc
