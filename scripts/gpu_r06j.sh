#!/bin/bash
# Round 6, iteration j: the later step-1600 state with the compaction cut - the driver-flag bench after a 1600-step
# prepare, and its kernel trace (the march there).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06j}
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --prepare 1600 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > gpurun_out/bench_${TAG}_step1600.log 2>&1 || { echo BENCH_FAIL; tail -5 gpurun_out/bench_${TAG}_step1600.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_step1600.log | cut -c1-160
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --prepare 1600 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "$R/gpurun_out/prof_$TAG.log" 2>&1 || { echo PROF_FAIL; exit 1; }
python3 "$R/scripts/prof_summary.py" "$R/gpurun_out/prof_$TAG" "$R/gpurun_out/prof_${TAG}_step1600_summary.md" --last-steps 20 > /dev/null && rm -rf "$R/gpurun_out/prof_$TAG"
head -16 "$R/gpurun_out/prof_${TAG}_step1600_summary.md"
echo ALL_OK
