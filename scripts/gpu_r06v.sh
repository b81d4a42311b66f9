#!/bin/bash
# Round 6, iteration v: the march-cut rerun tests (with short calls), then the driver-shaped trace at step 800: timelines of
# mid-call steps and the idle gaps between consecutive kernels of each queue.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06v}
timeout -k 10 600 python -u -m pytest tests/test_gpu_overlap.py -v --timeout 400 --timeout-method thread -k march_cut > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|^E " gpurun_out/pytest_$TAG.log | tail -8; tail -1 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --prepare 800 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "$R/gpurun_out/prof_$TAG.log" 2>&1 || { echo PROF_FAIL; exit 1; }
python3 "$R/scripts/prof_gaps.py" "$R/gpurun_out/prof_$TAG" --last-steps 20 > "$R/gpurun_out/prof_${TAG}_gaps.txt" 2>&1
python3 "$R/scripts/prof_summary.py" "$R/gpurun_out/prof_$TAG" "$R/gpurun_out/prof_${TAG}_timeline.md" --last-steps 20 --seq-back 6,7,8 > /dev/null && rm -rf "$R/gpurun_out/prof_$TAG"
head -30 "$R/gpurun_out/prof_${TAG}_gaps.txt"
echo ALL_OK
