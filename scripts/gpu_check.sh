#!/bin/bash
# One GPU-box pass: parity tests, a short bench, and a rocprofv3 kernel-trace summary of the bench.
# Usage (from the repo root on the box): bash scripts/gpu_check.sh [bench steps] [bench warmup]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
STEPS=${1:-50}; WARM=${2:-100}
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps $STEPS --warmup $WARM --cpu-steps 6 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --steps 20 --warmup 30 --cpu-baseline 0 > "$R/gpurun_out/prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
