#!/bin/bash
# r05nb: chunk scans with one group in flight (NEUS_SCAN_NB=1: 130 VGPRs, 3 waves per SIMD; with NEUS_SCAN_WPE=4: 128
# VGPRs + 5 spilled dwords, 4 waves) against the default two (170 VGPRs, 2 waves): fingerprints, alternating benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_def_r05nb.npz > gpurun_out/golden_def_r05nb.log 2>&1 || exit 1
for v in nb1 nb1w4; do
  NEUS2_HIP_LIB=$PWD/neus2_amd/libneus2_hip_$v.so timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_${v}_r05nb.npz --compare gpurun_out/golden_def_r05nb.npz > gpurun_out/golden_${v}_r05nb.log 2>&1 || exit 1
  echo "$v: $(grep -c identical gpurun_out/golden_${v}_r05nb.log) identical of 8"
done
o=gpurun_out/ab_r05nb.txt
: > $o
B="--gpus 1 --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0"
for i in 1 2; do
  for v in def nb1 nb1w4; do
    if [ $v = def ]; then L=$PWD/neus2_amd/libneus2_hip.so; else L=$PWD/neus2_amd/libneus2_hip_$v.so; fi
    NEUS2_HIP_LIB=$L timeout -k 10 200 python -u bench.py $B > gpurun_out/bench_nb_${v}_$i.log 2>&1 || exit 1
    echo "main $v $i $(tail -1 gpurun_out/bench_nb_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" >> $o
    NEUS2_HIP_LIB=$L timeout -k 10 300 python -u bench.py $B --prepare 1600 > gpurun_out/bench_nb_${v}_1600_$i.log 2>&1 || exit 1
    echo "1600 $v $i $(tail -1 gpurun_out/bench_nb_${v}_1600_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" >> $o
  done
done
cat $o
echo ALL_OK
