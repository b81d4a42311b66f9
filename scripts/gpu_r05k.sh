#!/bin/bash
# r05k: bitwise A/B of the working tree (no packed fp32, cooperative sample-map fill in k_loss_ray, sRGB byte table)
# against the packed-fp32 build of round-5 commit 22d9b67's kernels (libneus2_hip_base.so), then the GPU suite, the
# driver-shaped bench and a kernel trace of it
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
NEUS2_HIP_LIB=$PWD/neus2_amd/libneus2_hip_base.so timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_base_r05k.npz > gpurun_out/golden_base_r05k.log 2>&1 &&
timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_new_r05k.npz --compare gpurun_out/golden_base_r05k.npz > gpurun_out/golden_new_r05k.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_r05k.log 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_drv_r05k.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05k -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > gpurun_out/prof_r05k.log 2>&1
