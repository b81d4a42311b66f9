#!/bin/bash
# r05l16: the 16-level leg with the lookahead off / on (and at the default priority)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
o=gpurun_out/ab_r05l16.txt
: > $o
B="--gpus 1 --steps 50 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 1 --early 0"
for i in 1 2; do
  for v in 0 1 p0; do
    if [ $v = p0 ]; then export NEUS_LOOKAHEAD=1 NEUS_LA_PRIO=0; else export NEUS_LOOKAHEAD=$v; unset NEUS_LA_PRIO; fi
    timeout -k 10 300 python -u bench.py $B > gpurun_out/bench_l16_${v}_$i.log 2>&1 || exit 1
    echo "la=$v $i $(tail -1 gpurun_out/bench_l16_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("main", d["ms_per_step"], "l16", d["levels16"]["ms_per_step"])')" >> $o
  done
done
cat $o
echo ALL_OK
