#!/bin/bash
# r05f: the operator-API generality tests (GridMlp, Identity scale/offset, fp32 encoding), then the launch-lock experiment
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_grid_mlp.py tests/test_gpu_module.py \
  > gpurun_out/r05f_pytest_module.log 2>&1 &&
bash scripts/gpu_r05e.sh &&
timeout -k 10 380 python -u scripts/diag_recycle.py > gpurun_out/diag_recycle_r05f.log 2>&1
