#!/bin/bash
# Round-4 pass b: selected GPU tests (-k), the driver-shaped bench, then the march diagnostics (scripts/gpu_r04_march.sh).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r04b}
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$K" > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --psnr-steps 0 --cpu-baseline 0 --l16 0 --early 0 --mc-res 0 > gpurun_out/bench_drv_$TAG.log 2>&1 || { echo BENCH_DRV_FAIL; exit 1; }
tail -1 gpurun_out/bench_drv_$TAG.log | cut -c1-300
[ "${MARCH:-1}" = "1" ] && { bash scripts/gpu_r04_march.sh ${TAG}m || exit 1; }
echo ALL_OK
