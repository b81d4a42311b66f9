#!/bin/bash
# Round 6, iteration a: scaled scatter records (grid.hip record format) - the GPU suite, then a bench A/B against the
# previous commit's library (golden_ref/libneus2_hip_base.so) with the working tree copied as golden_ref/libneus2_hip_new.so.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06a}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR" gpurun_out/pytest_$TAG.log | grep -v "^tests.*PASSED" | tail -8; tail -2 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cp neus2_amd/libneus2_hip.so golden_ref/libneus2_hip_new.so
bash scripts/gpu_lib_ab.sh $TAG libneus2_hip_base libneus2_hip_new libneus2_hip_base libneus2_hip_new
timeout -k 10 300 python -u scripts/diag_infer_state.py > gpurun_out/diag_infer_state_$TAG.log 2>&1; echo "diag rc=$?"
