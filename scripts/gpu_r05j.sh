#!/bin/bash
# r05j: cost of dropping packed fp32 (default build now) against the packed build (libneus2_hip_pk.so): alternating bench
# runs and one kernel trace each; then the concurrency diagnostic and the determinism test on the new default build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
o=gpurun_out/pk_ab_r05j.txt
: > $o
B="--gpus 1 --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0"
for i in 1 2; do
  for v in pk nopk; do
    if [ $v = pk ]; then L=$PWD/neus2_amd/libneus2_hip_pk.so; else L=$PWD/neus2_amd/libneus2_hip.so; fi
    NEUS2_HIP_LIB=$L timeout -k 10 200 python -u bench.py $B > gpurun_out/bench_pkab_${v}_$i.log 2>&1 || exit 1
    echo "$v $i $(tail -1 gpurun_out/bench_pkab_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" >> $o
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
NEUS2_HIP_LIB=$PWD/neus2_amd/libneus2_hip_pk.so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pk -o run -- python3 bench.py $B > gpurun_out/prof_pk.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_nopk -o run -- python3 bench.py $B > gpurun_out/prof_nopk.log 2>&1 &&
timeout -k 10 200 python -u scripts/diag_concurrency_batch.py --steps 1 --pairs 12 --buffers 0 > gpurun_out/diag_conc_nopk_r05j.jsonl 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 380 --timeout-method thread tests/test_gpu_determinism.py > gpurun_out/pytest_determinism_r05j.log 2>&1
