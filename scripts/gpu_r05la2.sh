#!/bin/bash
# r05la2: the lookahead at the lowest priority as the default: fingerprint against it off, the whole GPU suite, smoke,
# alternating benches at both states
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
NEUS_LOOKAHEAD=0 timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_off_r05la2.npz > gpurun_out/golden_off_r05la2.log 2>&1 &&
timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_on_r05la2.npz --compare gpurun_out/golden_off_r05la2.npz > gpurun_out/golden_on_r05la2.log 2>&1 || { tail -8 gpurun_out/golden_on_r05la2.log; exit 1; }
echo "fingerprint: $(grep -c identical gpurun_out/golden_on_r05la2.log) identical of 8"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > gpurun_out/pytest_r05la2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r05la2.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/pytest_r05la2.log | head; exit 1; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r05la2.log 2>&1 || { tail -5 gpurun_out/smoke_r05la2.log; exit 1; }
tail -1 gpurun_out/smoke_r05la2.log
o=gpurun_out/ab_r05la2.txt
: > $o
B="--gpus 1 --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0"
for i in 1 2; do
  for v in 0 1; do
    NEUS_LOOKAHEAD=$v timeout -k 10 300 python -u bench.py $B --prepare 1600 > gpurun_out/bench_la2_${v}_1600_$i.log 2>&1 || exit 1
    echo "1600 la=$v $i $(tail -1 gpurun_out/bench_la2_${v}_1600_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["loss"])')" >> $o
  done
done
cat $o
echo ALL_OK
