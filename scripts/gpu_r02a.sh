#!/bin/bash
# Round-2 first pass: GPU parity tests, then the driver-shaped bench (warmup 5, steps 20) and the default bench (with PSNR).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r02a}
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 > gpurun_out/bench_drv_$TAG.log 2>&1
rc=$?; echo "bench_drv rc=$rc"; tail -2 gpurun_out/bench_drv_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --cpu-steps 6 > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench_$TAG.log
exit $rc
