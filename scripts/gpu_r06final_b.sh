#!/bin/bash
# Round 6 final evidence, part b: the driver-flag bench (step 800 and step 1600), the kernel trace of the driver-shaped
# bench (summary + timelines + queue gaps), and the PMC traffic of the training step's inference launches at HEAD.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06fb}
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 > gpurun_out/bench_driver_$TAG.log 2>&1 || { echo BENCH_FAIL; exit 1; }
tail -1 gpurun_out/bench_driver_$TAG.log | cut -c1-200
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 --prepare 1600 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > gpurun_out/bench_step1600_$TAG.log 2>&1 || { echo BENCH1600_FAIL; exit 1; }
tail -1 gpurun_out/bench_step1600_$TAG.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "$R/gpurun_out/prof_$TAG.log" 2>&1 || { echo PROF_FAIL; exit 1; }
python3 "$R/scripts/prof_gaps.py" "$R/gpurun_out/prof_$TAG" --last-steps 20 > "$R/gpurun_out/prof_${TAG}_gaps.txt" 2>&1
python3 "$R/scripts/prof_summary.py" "$R/gpurun_out/prof_$TAG" "$R/gpurun_out/prof_${TAG}_summary.md" --last-steps 20 --seq-back 6,7 > /dev/null && rm -rf "$R/gpurun_out/prof_$TAG"
head -14 "$R/gpurun_out/prof_${TAG}_summary.md"
cd "$R"
WARM=800 STEPS=20 bash scripts/gpu_traffic_steps.sh ${TAG}_steps 60 || exit $?
head -40 gpurun_out/${TAG}_steps_table.txt
echo ALL_OK
