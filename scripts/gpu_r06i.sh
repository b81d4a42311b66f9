#!/bin/bash
# Round 6, iteration i: the GPU suite with the bench-shape cut test, then the default bench (all legs).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06i}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|^E " gpurun_out/pytest_$TAG.log | tail -8; tail -2 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --cpu-steps 6 > gpurun_out/bench_$TAG.log 2>&1 || { echo BENCH_FAIL; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-300
