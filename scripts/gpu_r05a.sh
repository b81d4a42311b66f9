#!/bin/bash
# round 5, first GPU pass: the new multi-process / health / bench-shape parity tests, then the whole GPU suite, then a
# two-process same-device bench with the host backend
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD:$PWD/tests:$PWD/oracle
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_dp_procs.py \
  "tests/test_gpu_train_parity.py::test_teacher_forced_bench_shape" > gpurun_out/pytest_r05a_new.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
  --deselect "tests/test_gpu_train_parity.py::test_teacher_forced_bench_shape" --deselect tests/test_gpu_dp_procs.py > gpurun_out/pytest_r05a_all.log 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 2 --dp-backend host --same-device 1 --steps 12 --warmup 2 --prepare 50 --psnr-steps 0 --l16 0 --early 0 --cpu-baseline 0 > gpurun_out/bench_r05a_host2.log 2>&1
