#!/bin/bash
# Round 6, iteration c: the new overlap tests, the Adam-beside-the-scatter A/B on the step's side stream, the inference state diagnostic.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06c}
timeout -k 10 600 python -u -m pytest tests/test_gpu_overlap.py tests/test_gpu_dp.py tests/test_gpu_dp_procs.py -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR" gpurun_out/pytest_$TAG.log | tail -8; tail -2 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/gpu_env_ab.sh $TAG 800 NEUS_ADAM_OVERLAP=0 NEUS_ADAM_OVERLAP=1 NEUS_ADAM_OVERLAP=0 NEUS_ADAM_OVERLAP=1 || exit 1
timeout -k 10 300 python -u scripts/diag_infer_state.py > gpurun_out/diag_infer_state_$TAG.log 2>&1; echo "diag rc=$?"
