#!/bin/bash
# r05w: k_march_bal's work-profile weight of non-skippable blocks (NEUS_MARCH_PROF_W) at the step-1600 and default states
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
o=gpurun_out/ab_r05w.txt
: > $o
B="--gpus 1 --steps 50 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0"
for i in 1 2; do
  for v in 2 4 6 10; do
    NEUS_MARCH_PROF_W=$v timeout -k 10 300 python -u bench.py $B --prepare 1600 > gpurun_out/bench_w${v}_1600_$i.log 2>&1 || exit 1
    echo "1600 w=$v $i $(tail -1 gpurun_out/bench_w${v}_1600_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" >> $o
  done
done
for v in 2 4 6 10; do
  NEUS_MARCH_PROF_W=$v timeout -k 10 200 python -u bench.py $B > gpurun_out/bench_w${v}_main.log 2>&1 || exit 1
  echo "main w=$v $(tail -1 gpurun_out/bench_w${v}_main.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" >> $o
done
cat $o
echo ALL_OK
