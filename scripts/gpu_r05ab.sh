#!/bin/bash
# r05ab: alternating benches of the previous commit's build (libneus2_hip_prev.so) against HEAD's, at the default (step
# 800) and step-1600 states, plus kernel traces of both builds at step 1600
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
T=${T:-r05ab}
o=gpurun_out/ab_$T.txt
: > $o
B="--gpus 1 --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0"
for i in 1 2; do
  for v in prev new; do
    if [ $v = new ]; then L=$PWD/neus2_amd/libneus2_hip.so; else L=$PWD/neus2_amd/libneus2_hip_$v.so; fi
    NEUS2_HIP_LIB=$L timeout -k 10 200 python -u bench.py $B > gpurun_out/bench_${T}_${v}_$i.log 2>&1 || exit 1
    echo "main $v $i $(tail -1 gpurun_out/bench_${T}_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" >> $o
    NEUS2_HIP_LIB=$L timeout -k 10 300 python -u bench.py $B --prepare 1600 > gpurun_out/bench_${T}_${v}_1600_$i.log 2>&1 || exit 1
    echo "1600 $v $i $(tail -1 gpurun_out/bench_${T}_${v}_1600_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" >> $o
  done
done
cat $o
echo ALL_OK
