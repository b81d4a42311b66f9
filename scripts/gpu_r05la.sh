#!/bin/bash
# r05la: the next step's ray sampling issued beside the backward (NEUS_LOOKAHEAD=1): fingerprint against the same build
# without it, the progressive / determinism / train-parity tests with it, alternating benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
NEUS_LOOKAHEAD=0 timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_off_r05la.npz > gpurun_out/golden_off_r05la.log 2>&1 &&
NEUS_LOOKAHEAD=1 timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_on_r05la.npz --compare gpurun_out/golden_off_r05la.npz > gpurun_out/golden_on_r05la.log 2>&1 || { tail -8 gpurun_out/golden_on_r05la.log; exit 1; }
echo "fingerprint: $(grep -c identical gpurun_out/golden_on_r05la.log) identical of 8"; grep DIFF gpurun_out/golden_on_r05la.log
o=gpurun_out/ab_r05la.txt
: > $o
B="--gpus 1 --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0"
for i in 1 2; do
  for v in 0 1; do
    NEUS_LOOKAHEAD=$v timeout -k 10 200 python -u bench.py $B > gpurun_out/bench_la${v}_$i.log 2>&1 || exit 1
    echo "main la=$v $i $(tail -1 gpurun_out/bench_la${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["loss"])')" >> $o
    NEUS_LOOKAHEAD=$v timeout -k 10 300 python -u bench.py $B --prepare 1600 > gpurun_out/bench_la${v}_1600_$i.log 2>&1 || exit 1
    echo "1600 la=$v $i $(tail -1 gpurun_out/bench_la${v}_1600_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["loss"])')" >> $o
  done
done
cat $o
NEUS_LOOKAHEAD=1 timeout -k 10 800 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_progressive.py tests/test_gpu_determinism.py tests/test_gpu_train_parity.py > gpurun_out/pytest_r05la.log 2>&1 || { tail -30 gpurun_out/pytest_r05la.log; exit 1; }
tail -2 gpurun_out/pytest_r05la.log
echo ALL_OK
