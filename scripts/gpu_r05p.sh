#!/bin/bash
# r05p: (1) the march write without the unused sample->ray map: bitwise A/B against 22d9b67's build; (2) the training MLP
# kernels at two waves per SIMD (libneus2_hip_mlp2.so: amdgpu_waves_per_eu(2, 2), spilling to scratch) against one:
# alternating bench runs and a kernel trace of each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
NEUS2_HIP_LIB=$PWD/neus2_amd/libneus2_hip_base.so timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_base_r05p.npz > gpurun_out/golden_base_r05p.log 2>&1 &&
timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_new_r05p.npz --compare gpurun_out/golden_base_r05p.npz > gpurun_out/golden_new_r05p.log 2>&1 || exit 1
o=gpurun_out/ab_r05p.txt
: > $o
B="--gpus 1 --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0"
for i in 1 2; do
  for v in new mlp2; do
    if [ $v = new ]; then L=$PWD/neus2_amd/libneus2_hip.so; else L=$PWD/neus2_amd/libneus2_hip_$v.so; fi
    NEUS2_HIP_LIB=$L timeout -k 10 200 python -u bench.py $B > gpurun_out/bench_ab_${v}_$i.log 2>&1 || exit 1
    echo "$v $i $(tail -1 gpurun_out/bench_ab_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["mfma_mlp_train"])')" >> $o
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
NEUS2_HIP_LIB=$PWD/neus2_amd/libneus2_hip_mlp2.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05p_mlp2 -o run --output-format csv -- python3 bench.py $B > gpurun_out/prof_r05p_mlp2.log 2>&1
