#!/bin/bash
# Round-4 GPU pass (run from the repo root on the box): GPU tests (optionally -k), the driver-shaped bench, a
# rocprofv3 kernel-trace summary of the bench's main leg only (no early / L16 / PSNR / MC legs), the PMC traffic of
# the training step's own inference rounds, and the GPU side of the PSNR anchor.
# Usage: bash scripts/gpu_r04.sh TAG [pytest -k expression]   (env: BENCH=0 skips the bench; PROF=0, PMC=0, ANCHOR=0)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r04}
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$K" > gpurun_out/pytest_$TAG.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
fi
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --psnr-steps 0 --cpu-baseline 0 --l16 0 --early 0 --mc-res 0 > gpurun_out/bench_drv_$TAG.log 2>&1 || { echo BENCH_DRV_FAIL; exit 1; }
  tail -1 gpurun_out/bench_drv_$TAG.log | cut -c1-600
fi
if [ "${PROF:-1}" = "1" ]; then
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 \
     --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "$R/gpurun_out/prof_$TAG.log" 2>&1) || { echo PROF_FAIL; exit 1; }
  python3 scripts/prof_summary.py gpurun_out/prof_$TAG gpurun_out/prof_${TAG}_main_summary.md --last-steps 20 > /dev/null && rm -rf gpurun_out/prof_$TAG
  tail -1 gpurun_out/prof_$TAG.log | cut -c1-300
fi
if [ "${PMC:-1}" = "1" ]; then
  bash scripts/gpu_traffic_steps.sh ${TAG}_steps 20 || exit 1
fi
if [ "${ANCHOR:-1}" = "1" ]; then
  timeout -k 10 300 python -u scripts/psnr_anchor.py --side gpu --steps 2000 --checkpoints 250,500,1000,1500 > gpurun_out/psnr_anchor_gpu_$TAG.jsonl 2>&1 || { echo ANCHOR_FAIL; exit 1; }
  cat gpurun_out/psnr_anchor_gpu_$TAG.jsonl
fi
echo ALL_OK
