#!/bin/bash
# r05q: per-ray wave loops for the round lists (k_ray_sort_place, k_loss_scan_chunk) and a 4-deep fetch in the later
# chunk scans (NEUS_SCAN_NB_LATER=2: the former 2-deep): bitwise A/B against 22d9b67's build, the progressive bitwise
# tests, alternating bench runs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
NEUS2_HIP_LIB=$PWD/neus2_amd/libneus2_hip_base.so timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_base_r05q.npz > gpurun_out/golden_base_r05q.log 2>&1 &&
timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_new_r05q.npz --compare gpurun_out/golden_base_r05q.npz > gpurun_out/golden_new_r05q.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_progressive.py tests/test_gpu_determinism.py > gpurun_out/pytest_prog_r05q.log 2>&1 || exit 1
o=gpurun_out/ab_r05q.txt
: > $o
B="--gpus 1 --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0"
for i in 1 2; do
  for v in 2 4; do
    NEUS_SCAN_NB_LATER=$v timeout -k 10 200 python -u bench.py $B > gpurun_out/bench_nb${v}_$i.log 2>&1 || exit 1
    echo "NB_later=$v $i $(tail -1 gpurun_out/bench_nb${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" >> $o
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05q -o run --output-format csv -- python3 bench.py $B > gpurun_out/prof_r05q.log 2>&1
