#!/bin/bash
# Round-3 iteration: scatter / bitwise GPU tests, concurrent-testbed determinism diagnostics, steady-state kernel
# trace (gpu_iter3.sh), then the counter passes of gpu_r03_pmc2.sh. Usage: bash scripts/gpu_r03y.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r03y}
timeout -k 10 300 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -k "scatter or backward or bitwise" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
AB=0 REPS=3 timeout -k 10 250 python -u scripts/det_concurrent.py > gpurun_out/detc0_$TAG.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/detc0_$TAG.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_iter3.sh $TAG || exit $?
bash scripts/gpu_r03_pmc2.sh $TAG > gpurun_out/pmc2_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pmc2_$TAG.log; exit $rc
