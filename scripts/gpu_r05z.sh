#!/bin/bash
# Round-5 final pass. Part 1 (PART=1): the whole GPU suite, smoke, the default bench (all legs) and the driver-shaped
# bench. Part 2 (PART=2): kernel-trace summaries of the bench's main leg and of the step-1600 state, and the PMC traffic
# of the training step's own inference rounds (for traffic.json).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${TAG:-r05z}
if [ "${PART:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE_FAIL; tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
  tail -1 gpurun_out/smoke_$TAG.log
  timeout -k 10 600 python -u bench.py > gpurun_out/bench_default_$TAG.log 2>&1 || { echo BENCH_DEFAULT_FAIL; exit 1; }
  tail -1 gpurun_out/bench_default_$TAG.log | cut -c1-400
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_drv_$TAG.log 2>&1 || { echo BENCH_DRV_FAIL; exit 1; }
  tail -1 gpurun_out/bench_drv_$TAG.log | cut -c1-400
else
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 \
     --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "$R/gpurun_out/prof_$TAG.log" 2>&1) || { echo PROF_FAIL; exit 1; }
  python3 scripts/prof_summary.py gpurun_out/prof_$TAG gpurun_out/prof_${TAG}_main_summary.md --last-steps 20 > /dev/null && rm -rf gpurun_out/prof_$TAG
  head -14 gpurun_out/prof_${TAG}_main_summary.md
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}s" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 \
     --prepare 1600 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "$R/gpurun_out/prof_${TAG}_1600.log" 2>&1) || { echo PROF1600_FAIL; exit 1; }
  python3 scripts/prof_summary.py gpurun_out/prof_${TAG}s gpurun_out/prof_${TAG}_step1600_summary.md --last-steps 20 > /dev/null && rm -rf gpurun_out/prof_${TAG}s
  head -8 gpurun_out/prof_${TAG}_step1600_summary.md
  bash scripts/gpu_traffic_steps.sh ${TAG}_steps ${LAST:-15} || exit 1
  cat gpurun_out/${TAG}_steps_table.txt | head -20
fi
echo ALL_OK
