#!/bin/bash
# Bitwise A/B of the working tree's library against golden_ref/libneus2_hip_base.so (a build of the previous
# commit, development only; golden_ref/libneus2_hip_new.so, if present, stands for the working tree, e.g. both built
# with -ffp-contract=off so that a restructuring is compared without contraction changes): fingerprints of both (scripts/golden_params.py), then the iteration check.
# Usage: bash scripts/gpu_ab.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-ab}
NEUS2_HIP_LIB="$R/golden_ref/libneus2_hip_base.so" timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_base_$TAG.npz > gpurun_out/golden_base_$TAG.log 2>&1 || { echo GOLDEN_BASE_FAIL; exit 1; }
NEW="$R/golden_ref/libneus2_hip_new.so"; [ -f "$NEW" ] || NEW="$R/neus2_amd/libneus2_hip.so"
NEUS2_HIP_LIB="$NEW" timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_new_$TAG.npz --compare gpurun_out/golden_base_$TAG.npz > gpurun_out/golden_new_$TAG.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/golden_new_$TAG.log | tail -12
[ $rc -eq 0 ] || { echo GOLDEN_MISMATCH; [ $rc -eq 1 ] || exit $rc; }
bash scripts/gpu_iter.sh $TAG
