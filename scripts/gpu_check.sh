#!/bin/bash
# One GPU-box pass: parity tests, the default bench, and a rocprofv3 kernel-trace summary of the bench.
# Usage (from the repo root on the box): bash scripts/gpu_check.sh [tag] [bench steps] [bench warmup]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-run}; STEPS=${2:-200}; WARM=${3:-800}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps $STEPS --warmup $WARM --cpu-steps 6 > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 20 --warmup 800 --cpu-baseline 0 > "$R/gpurun_out/prof_$TAG.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
[ $rc -eq 0 ] && python3 "$R/scripts/prof_summary.py" "$R/gpurun_out/prof_$TAG" --last-steps 16 > "$R/gpurun_out/prof_${TAG}_summary.md" && rm -rf "$R/gpurun_out/prof_$TAG"
exit $rc
