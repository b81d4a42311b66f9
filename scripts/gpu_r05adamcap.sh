#!/bin/bash
# r05adamcap: Adam's grid capped (NEUS_ADAM_BLOCKS) so that the low-priority lookahead march finds wave slots beside it
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
o=gpurun_out/ab_r05adamcap.txt
: > $o
B="--gpus 1 --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0"
for i in 1 2; do
  for v in 16384 2048 1024 512; do
    NEUS_ADAM_BLOCKS=$v timeout -k 10 200 python -u bench.py $B > gpurun_out/bench_ac_${v}_$i.log 2>&1 || exit 1
    echo "main blocks=$v $i $(tail -1 gpurun_out/bench_ac_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["loss"], d["kernels"]["adam_ema"]["ms"])')" >> $o
  done
done
cat $o
echo ALL_OK
