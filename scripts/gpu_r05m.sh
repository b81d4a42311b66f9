#!/bin/bash
# r05m: chunk-scan U = 16 for the later progressive rounds (NEUS_SCAN_U_LATER=8: the former U = 8 everywhere): the
# progressive bitwise tests, then alternating bench runs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_progressive.py > gpurun_out/pytest_prog_r05m.log 2>&1 || exit 1
o=gpurun_out/ab_r05m.txt
: > $o
B="--gpus 1 --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0"
for i in 1 2; do
  for v in 8 16; do
    NEUS_SCAN_U_LATER=$v timeout -k 10 200 python -u bench.py $B > gpurun_out/bench_u${v}_$i.log 2>&1 || exit 1
    echo "U_later=$v $i $(tail -1 gpurun_out/bench_u${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" >> $o
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05m -o run --output-format csv -- python3 bench.py $B > gpurun_out/prof_r05m.log 2>&1
