#!/bin/bash
# Iteration check on the GPU box: parity tests (stop on failure), driver-shaped bench, kernel-trace summaries.
# Usage: bash scripts/gpu_iter.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-iter}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 > gpurun_out/bench_drv_$TAG.log 2>&1 || { echo BENCH_DRV_FAIL; exit 1; }
tail -1 gpurun_out/bench_drv_$TAG.log | cut -c1-400
bash scripts/gpu_profiles.sh $TAG
