#!/bin/bash
# Round-4 pass m: parity / march / progressive tests, then A/B benches of the round's switches at the step-800 and
# step-1600 states (driver shape), then the balanced march's diagnostics.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -k "progressive or teacher_forced or bitwise or health or parity or forward" > gpurun_out/pytest_r04m.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r04m.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/gpu_sweep_env.sh bal800 NEUS_MARCH_BALANCE 1 0 || exit 1
bash scripts/gpu_sweep_env.sh pipe800 NEUS_INFER_PIPE 1 0 || exit 1
BENCH_ARGS="--prepare 1600" bash scripts/gpu_sweep_env.sh bal1600 NEUS_MARCH_BALANCE 1 0 || exit 1
BENCH_ARGS="--prepare 1600" bash scripts/gpu_sweep_env.sh pipe1600 NEUS_INFER_PIPE 0 || exit 1
for W in 800 1600; do
  WARM=$W timeout -k 10 300 python -u scripts/diag_march_prof.py > gpurun_out/march_prof_r04m_w$W.log 2>&1 || { echo "march prof $W failed"; exit 1; }
  head -12 gpurun_out/march_prof_r04m_w$W.log
done
echo ALL_OK
