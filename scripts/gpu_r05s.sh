#!/bin/bash
# r05s: chunk scans with 4-sample groups (NEUS_SCAN_U=4: 98 VGPRs, 6 KB LDS per wave) against 8: alternating bench runs,
# then the progressive bitwise tests with U = 4
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
o=gpurun_out/ab_r05s.txt
: > $o
B="--gpus 1 --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0"
for i in 1 2; do
  for v in 8 4; do
    NEUS_SCAN_U=$v timeout -k 10 200 python -u bench.py $B > gpurun_out/bench_u${v}_$i.log 2>&1 || exit 1
    echo "U=$v $i $(tail -1 gpurun_out/bench_u${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" >> $o
  done
done
NEUS_SCAN_U=4 timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_progressive.py > gpurun_out/pytest_prog_r05s.log 2>&1
