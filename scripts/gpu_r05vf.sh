#!/bin/bash
# r05vf: MFMA results in VGPRs (-amdgpu-mfma-vgpr-form): bitwise fingerprint against the build before it
# (libneus2_hip_prev.so), then alternating benches at the default and step-1600 states
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
NEUS2_HIP_LIB=$PWD/neus2_amd/libneus2_hip_prev.so timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_prev_r05vf.npz > gpurun_out/golden_prev_r05vf.log 2>&1 &&
timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_new_r05vf.npz --compare gpurun_out/golden_prev_r05vf.npz > gpurun_out/golden_new_r05vf.log 2>&1 || { tail -5 gpurun_out/golden_new_r05vf.log; exit 1; }
tail -4 gpurun_out/golden_new_r05vf.log
T=r05vf bash scripts/gpu_r05ab.sh
