#!/bin/bash
# r05combo: against the build before (libneus2_hip_prev.so): "new" = the density training kernel reading the density
# forward's fragments stored by the colour kernel; max-ilp / max-memory-clause = mlp.hip built with those scheduler
# strategies. Fingerprints, then alternating benches with the MLP kernel replays.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
NEUS2_HIP_LIB=$PWD/neus2_amd/libneus2_hip_prev.so timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_prev_combo.npz > gpurun_out/golden_prev_combo.log 2>&1 || exit 1
for v in new max-ilp max-memory-clause; do
  if [ $v = new ]; then L=$PWD/neus2_amd/libneus2_hip.so; else L=$PWD/neus2_amd/libneus2_hip_$v.so; fi
  NEUS2_HIP_LIB=$L timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_${v}_combo.npz --compare gpurun_out/golden_prev_combo.npz > gpurun_out/golden_${v}_combo.log 2>&1 || exit 1
  echo "$v: $(grep -c identical gpurun_out/golden_${v}_combo.log) identical of 8"
done
o=gpurun_out/ab_combo.txt
: > $o
B="--gpus 1 --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0"
for i in 1 2; do
  for v in prev new max-ilp max-memory-clause; do
    if [ $v = new ]; then L=$PWD/neus2_amd/libneus2_hip.so; else L=$PWD/neus2_amd/libneus2_hip_$v.so; fi
    NEUS2_HIP_LIB=$L timeout -k 10 200 python -u bench.py $B > gpurun_out/bench_combo_${v}_$i.log 2>&1 || exit 1
    echo "main $v $i $(tail -1 gpurun_out/bench_combo_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels"]; print(d["ms_per_step"], k["inference"]["ms"], k["mlp_train_rgb"]["ms"], k["mlp_train_density"]["ms"])')" >> $o
  done
done
cat $o
echo ALL_OK
