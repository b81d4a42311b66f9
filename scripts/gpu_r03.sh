#!/bin/bash
# Round-3 GPU pass (run from the repo root on the box): the GPU tests, the driver-shaped bench and the default bench.
# Usage: bash scripts/gpu_r03.sh TAG [pytest -k expression]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r03}
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$K" > gpurun_out/pytest_$TAG.log 2>&1
else
  timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
fi
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ "${BENCH:-1}" = "1" ] || exit $rc
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --psnr-steps 0 --cpu-baseline 0 --l16 0 > gpurun_out/bench_drv_$TAG.log 2>&1 || { echo BENCH_DRV_FAIL; exit 1; }
tail -1 gpurun_out/bench_drv_$TAG.log | cut -c1-400
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1 || { echo BENCH_FAIL; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-400
echo ALL_OK
