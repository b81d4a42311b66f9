#!/bin/bash
# Round 6, iteration s: the whole GPU suite with the march cut on by default, then the driver-shaped trace at step 800
# with the timelines of mid-call steps.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06s}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|^E " gpurun_out/pytest_$TAG.log | tail -8; tail -2 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --prepare 800 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "$R/gpurun_out/prof_$TAG.log" 2>&1 || { echo PROF_FAIL; exit 1; }
python3 "$R/scripts/prof_summary.py" "$R/gpurun_out/prof_$TAG" "$R/gpurun_out/prof_${TAG}_timeline.md" --last-steps 20 --seq-back 6,7,8 > /dev/null && rm -rf "$R/gpurun_out/prof_$TAG"
head -30 "$R/gpurun_out/prof_${TAG}_timeline.md"
echo ALL_OK
