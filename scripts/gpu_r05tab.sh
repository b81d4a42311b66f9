#!/bin/bash
# r05tab: inference level pair 0 from an LDS copy of its tables: the parity / progressive / render / determinism tests, the
# training fingerprint against the build before (libneus2_hip_prev.so), alternating benches with the inference replays
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_progressive.py > gpurun_out/pytest_r05tab.log 2>&1 || { tail -30 gpurun_out/pytest_r05tab.log; exit 1; }
tail -2 gpurun_out/pytest_r05tab.log
NEUS2_HIP_LIB=$PWD/neus2_amd/libneus2_hip_prev.so timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_prev_r05tab.npz > gpurun_out/golden_prev_r05tab.log 2>&1 &&
timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_new_r05tab.npz --compare gpurun_out/golden_prev_r05tab.npz > gpurun_out/golden_new_r05tab.log 2>&1 || { tail -5 gpurun_out/golden_new_r05tab.log; exit 1; }
echo "fingerprint: $(grep -c identical gpurun_out/golden_new_r05tab.log) identical of 8"
o=gpurun_out/ab_r05tab.txt
: > $o
B="--gpus 1 --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0"
for i in 1 2; do
  for v in prev new; do
    if [ $v = new ]; then L=$PWD/neus2_amd/libneus2_hip.so; else L=$PWD/neus2_amd/libneus2_hip_$v.so; fi
    NEUS2_HIP_LIB=$L timeout -k 10 200 python -u bench.py $B > gpurun_out/bench_tab_${v}_$i.log 2>&1 || exit 1
    echo "main $v $i $(tail -1 gpurun_out/bench_tab_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels"]["inference"]; r=d["roofline"]; print(d["ms_per_step"], k["ms"], r["ms_per_step"], r["launch_ms"])')" >> $o
    NEUS2_HIP_LIB=$L timeout -k 10 300 python -u bench.py $B --prepare 1600 > gpurun_out/bench_tab_${v}_1600_$i.log 2>&1 || exit 1
    echo "1600 $v $i $(tail -1 gpurun_out/bench_tab_${v}_1600_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels"]["inference"]; r=d["roofline"]; print(d["ms_per_step"], k["ms"], r["ms_per_step"], r["launch_ms"])')" >> $o
  done
done
cat $o
echo ALL_OK
