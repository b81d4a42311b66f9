#!/bin/bash
# Quick GPU check (run from the repo root on the box): parity tests (stop at the first failure), then a
# rocprofv3 kernel-trace summary of the driver-shaped bench (--warmup 5 --steps 20) and of a steady-state run.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-quick}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 > "$R/gpurun_out/prof_${TAG}_drv.log" 2>&1 || { echo PROF_FAIL; exit 1; }
python3 "$R/scripts/prof_summary.py" "$R/gpurun_out/prof_$TAG" "$R/gpurun_out/prof_${TAG}_drv_summary.md" --last-steps 20 > /dev/null && rm -rf "$R/gpurun_out/prof_$TAG"
tail -1 "$R/gpurun_out/prof_${TAG}_drv.log" | cut -c1-200
if [ "${STEADY:-1}" = "1" ]; then
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 50 --warmup 800 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 > "$R/gpurun_out/prof_${TAG}_steady.log" 2>&1 || { echo PROF2_FAIL; exit 1; }
python3 "$R/scripts/prof_summary.py" "$R/gpurun_out/prof_$TAG" "$R/gpurun_out/prof_${TAG}_steady_summary.md" --last-steps 50 > /dev/null && rm -rf "$R/gpurun_out/prof_$TAG"
tail -1 "$R/gpurun_out/prof_${TAG}_steady.log" | cut -c1-200
fi
echo ALL_OK
