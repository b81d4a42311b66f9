#!/bin/bash
# One full GPU evidence pass (run from the repo root on the box): parity tests, the driver-shaped bench
# (--warmup 5 --steps 20), the default bench (PSNR leg, marching cubes 1024^3, CPU baseline), a rocprofv3
# kernel-trace summary of the driver-shaped bench, and PMC traffic of the inference kernel at 4 and 14 levels.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-round}
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_drv_$TAG.log 2>&1 || { echo BENCH_DRV_FAIL; exit 1; }
tail -1 gpurun_out/bench_drv_$TAG.log | cut -c1-300
timeout -k 10 600 python -u bench.py --cpu-steps 6 > gpurun_out/bench_$TAG.log 2>&1 || { echo BENCH_FAIL; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 > "$R/gpurun_out/prof_$TAG.log" 2>&1 || { echo PROF_FAIL; exit 1; }
python3 "$R/scripts/prof_summary.py" "$R/gpurun_out/prof_$TAG" "$R/gpurun_out/prof_${TAG}_drv_summary.md" --last-steps 20 > /dev/null && rm -rf "$R/gpurun_out/prof_$TAG"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 50 --warmup 800 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 > "$R/gpurun_out/prof_${TAG}_steady.log" 2>&1 || { echo PROF2_FAIL; exit 1; }
python3 "$R/scripts/prof_summary.py" "$R/gpurun_out/prof_$TAG" "$R/gpurun_out/prof_${TAG}_steady_summary.md" --last-steps 50 > /dev/null && rm -rf "$R/gpurun_out/prof_$TAG"
cd "$R"
WARM=5 K=3 bash scripts/gpu_traffic.sh ${TAG}_w5 || exit $?
WARM=800 K=3 bash scripts/gpu_traffic.sh ${TAG}_w800 || exit $?
echo ALL_OK
