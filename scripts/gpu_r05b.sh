#!/bin/bash
# round 5 pass b: the whole-step determinism test (LDS garbage before every kernel, concurrent testbeds) and the
# stale-LDS / health tests it extends
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD:$PWD/tests:$PWD/oracle
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_determinism.py tests/test_gpu_health.py \
  tests/test_gpu_progressive.py > gpurun_out/pytest_r05b.log 2>&1
