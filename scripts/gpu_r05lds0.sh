#!/bin/bash
# r05lds0 (timing experiment, wrong results): level pair 0 gathered from an LDS copy of level 0's table instead of global
# memory; the bench's inference replay per sample against the production build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
o=gpurun_out/ab_r05lds0.txt
: > $o
B="--gpus 1 --steps 30 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0"
for i in 1 2; do
  for v in prev lds0; do
    NEUS2_HIP_LIB=$PWD/neus2_amd/libneus2_hip_$v.so timeout -k 10 200 python -u bench.py $B > gpurun_out/bench_lds0_${v}_$i.log 2>&1 || exit 1
    echo "$v $i $(tail -1 gpurun_out/bench_lds0_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels"]["inference"]; r=d["roofline"]; print(d["ms_per_step"], k["ms"], k["units"], round(k["ms"]/k["units"]*1e9,1), "ns/Msample;", r["launch_ms"], r["units_per_launch"], round(r["launch_ms"]/r["units_per_launch"]*1e9,1))')" >> $o
  done
done
cat $o
echo ALL_OK
