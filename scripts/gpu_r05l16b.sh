#!/bin/bash
# r05l16b: the 16-level leg after the early leg (as the default bench runs them), lookahead variants
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
o=gpurun_out/ab_r05l16b.txt
: > $o
B="--steps 200 --warmup 20 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --early 1 --l16 1"
for v in 1 p0 0; do
  if [ $v = p0 ]; then export NEUS_LOOKAHEAD=1 NEUS_LA_PRIO=0; else export NEUS_LOOKAHEAD=$v; unset NEUS_LA_PRIO; fi
  timeout -k 10 400 python -u bench.py $B > gpurun_out/bench_l16b_${v}.log 2>&1 || exit 1
  echo "la=$v $(tail -1 gpurun_out/bench_l16b_${v}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("main", d["ms_per_step"], "early", d["early_steps"]["ms_per_step"], "l16", d["levels16"]["ms_per_step"])')" >> $o
done
cat $o
echo ALL_OK
