#!/bin/bash
# Round 6: kernel trace of the bench after a 1600-step prepare (the march at a late state, with the march cut).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06t1600}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --prepare 1600 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "$R/gpurun_out/prof_$TAG.log" 2>&1 || { echo PROF_FAIL; exit 1; }
python3 "$R/scripts/prof_summary.py" "$R/gpurun_out/prof_$TAG" "$R/gpurun_out/prof_${TAG}_summary.md" --last-steps 20 --seq-back 6 > /dev/null && rm -rf "$R/gpurun_out/prof_$TAG"
head -12 "$R/gpurun_out/prof_${TAG}_summary.md"
echo ALL_OK
