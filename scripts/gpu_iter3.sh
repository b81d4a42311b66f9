#!/bin/bash
# Iteration pass (repo root on the box): a GPU test subset, then a rocprofv3 kernel-trace summary of the steady-state
# bench (prepare 800, 50 timed steps) and its bench line. Usage: bash scripts/gpu_iter3.sh TAG "pytest -k expr"
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-iter}
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$K" > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 50 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "$R/gpurun_out/prof_${TAG}_steady.log" 2>&1 || { echo PROF_FAIL; exit 1; }
python3 "$R/scripts/prof_summary.py" "$R/gpurun_out/prof_$TAG" "$R/gpurun_out/prof_${TAG}_steady_summary.md" --last-steps 50 > /dev/null && rm -rf "$R/gpurun_out/prof_$TAG"
tail -1 "$R/gpurun_out/prof_${TAG}_steady.log" | cut -c1-300
head -30 "$R/gpurun_out/prof_${TAG}_steady_summary.md"
echo ALL_OK
