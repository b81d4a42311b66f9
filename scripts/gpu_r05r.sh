#!/bin/bash
# r05r: 16-bit saturating Adam step counts: bitwise A/B against 22d9b67's build, the optimizer / snapshot / parity tests,
# alternating bench runs against the previous commit's build (libneus2_hip_prev.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
NEUS2_HIP_LIB=$PWD/neus2_amd/libneus2_hip_base.so timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_base_r05r.npz > gpurun_out/golden_base_r05r.log 2>&1 &&
timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_new_r05r.npz --compare gpurun_out/golden_base_r05r.npz > gpurun_out/golden_new_r05r.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_r05r.log 2>&1 || exit 1
o=gpurun_out/ab_r05r.txt
: > $o
B="--gpus 1 --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0"
for i in 1 2; do
  for v in prev new; do
    if [ $v = new ]; then L=$PWD/neus2_amd/libneus2_hip.so; else L=$PWD/neus2_amd/libneus2_hip_$v.so; fi
    NEUS2_HIP_LIB=$L timeout -k 10 200 python -u bench.py $B > gpurun_out/bench_ab_${v}_$i.log 2>&1 || exit 1
    echo "$v $i $(tail -1 gpurun_out/bench_ab_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" >> $o
  done
done
