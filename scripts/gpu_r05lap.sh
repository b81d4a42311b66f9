#!/bin/bash
# r05lap: the lookahead stream's priority (NEUS_LA_PRIO -1 / 0 / 1) and the lookahead off, alternating benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
o=gpurun_out/ab_r05lap.txt
: > $o
B="--gpus 1 --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0"
for i in 1 2; do
  for v in off -1 0 1; do
    if [ "$v" = off ]; then export NEUS_LOOKAHEAD=0; unset NEUS_LA_PRIO; else export NEUS_LOOKAHEAD=1 NEUS_LA_PRIO=$v; fi
    timeout -k 10 200 python -u bench.py $B > gpurun_out/bench_lap_${v}_$i.log 2>&1 || exit 1
    echo "main prio=$v $i $(tail -1 gpurun_out/bench_lap_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["loss"])')" >> $o
  done
done
cat $o
echo ALL_OK
