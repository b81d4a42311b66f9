#!/bin/bash
# r05l16c: stream priorities after the early leg: main at the highest + lookahead lowest / lookahead default / off
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
o=gpurun_out/ab_r05l16c.txt
: > $o
B="--steps 200 --warmup 20 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --early 1 --l16 1"
for v in hi_lo hi_def; do
  unset NEUS_LA_PRIO; export NEUS_MAIN_PRIO=1
  if [ $v = hi_def ]; then export NEUS_LA_PRIO=0; fi
  timeout -k 10 400 python -u bench.py $B > gpurun_out/bench_l16c_${v}.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/bench_l16c_${v}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("main", d["ms_per_step"], "early", d["early_steps"]["ms_per_step"], "l16", d["levels16"]["ms_per_step"])')" >> $o
done
cat $o
echo ALL_OK
