#!/bin/bash
# r05v: empty-block skip + work-profiled lane slices: march parity tests, fingerprint off/on, event diagnostics and
# alternating benches at the step-1600 and default states
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
T=${T:-r05v}
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "sample_rays or multilane" > gpurun_out/pytest_$T.log 2>&1 || { tail -30 gpurun_out/pytest_$T.log; exit 1; }
tail -2 gpurun_out/pytest_$T.log
NEUS_MARCH_MACRO=0 timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_off_$T.npz > gpurun_out/golden_off_$T.log 2>&1 &&
timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_on_$T.npz --compare gpurun_out/golden_off_$T.npz > gpurun_out/golden_on_$T.log 2>&1 || { tail -5 gpurun_out/golden_on_$T.log; exit 1; }
tail -3 gpurun_out/golden_on_$T.log
for v in 0 1; do
  NEUS_MARCH_MACRO=$v WARM=1600 timeout -k 10 200 python -u scripts/diag_march_prof.py > gpurun_out/march_prof_m${v}_$T.log 2>&1 || exit 1
  grep -E "kernel span|segment events|segment march" gpurun_out/march_prof_m${v}_$T.log
done
o=gpurun_out/ab_$T.txt
: > $o
B="--gpus 1 --steps 50 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0"
for i in 1 2; do
  for v in 0 1; do
    NEUS_MARCH_MACRO=$v timeout -k 10 300 python -u bench.py $B --prepare 1600 > gpurun_out/bench_m${v}_1600_$i.log 2>&1 || exit 1
    echo "1600 macro=$v $i $(tail -1 gpurun_out/bench_m${v}_1600_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" >> $o
    NEUS_MARCH_MACRO=$v timeout -k 10 200 python -u bench.py $B > gpurun_out/bench_m${v}_$i.log 2>&1 || exit 1
    echo "main macro=$v $i $(tail -1 gpurun_out/bench_m${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" >> $o
  done
done
cat $o
echo ALL_OK
