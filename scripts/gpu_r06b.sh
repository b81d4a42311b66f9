#!/bin/bash
# Round 6, iteration b: the GPU suite; Adam beside the scatter (NEUS_ADAM_OVERLAP) A/B; the inference state diagnostic;
# the default bench (PSNR leg with the scaled scatter records).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06b}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR" gpurun_out/pytest_$TAG.log | tail -8; tail -2 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/gpu_env_ab.sh $TAG 800 NEUS_ADAM_OVERLAP=0 NEUS_ADAM_OVERLAP=1 NEUS_MLP_BLOCKS_PCT=200 NEUS_MLP_BLOCKS_PCT=400 NEUS_ADAM_OVERLAP=0 NEUS_ADAM_OVERLAP=1 NEUS_MLP_BLOCKS_PCT=200 NEUS_MLP_BLOCKS_PCT=400 || exit 1
timeout -k 10 300 python -u scripts/diag_infer_state.py > gpurun_out/diag_infer_state_$TAG.log 2>&1; echo "diag rc=$?"
timeout -k 10 600 python -u bench.py --cpu-steps 6 > gpurun_out/bench_$TAG.log 2>&1 || { echo BENCH_FAIL; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-400
