#!/bin/bash
# r05t: exact empty-block skip in the march (march.hip macro_skip): march parity tests (oracle, multi-lane, block-skip
# off), a bitwise training fingerprint with the skip off / on, alternating benches at the default and step-1600 states
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "sample_rays or multilane" > gpurun_out/pytest_r05t.log 2>&1 || { tail -30 gpurun_out/pytest_r05t.log; exit 1; }
tail -3 gpurun_out/pytest_r05t.log
NEUS_MARCH_MACRO=0 timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_off_r05t.npz > gpurun_out/golden_off_r05t.log 2>&1 &&
timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_on_r05t.npz --compare gpurun_out/golden_off_r05t.npz > gpurun_out/golden_on_r05t.log 2>&1 || { tail -5 gpurun_out/golden_on_r05t.log; exit 1; }
tail -3 gpurun_out/golden_on_r05t.log
o=gpurun_out/ab_r05t.txt
: > $o
B="--gpus 1 --steps 50 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0"
for i in 1 2; do
  for v in 0 1; do
    NEUS_MARCH_MACRO=$v timeout -k 10 200 python -u bench.py $B > gpurun_out/bench_m${v}_$i.log 2>&1 || exit 1
    echo "main macro=$v $i $(tail -1 gpurun_out/bench_m${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" >> $o
    NEUS_MARCH_MACRO=$v timeout -k 10 300 python -u bench.py $B --prepare 1600 > gpurun_out/bench_m${v}_1600_$i.log 2>&1 || exit 1
    echo "1600 macro=$v $i $(tail -1 gpurun_out/bench_m${v}_1600_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" >> $o
  done
done
cat $o
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r05ts" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 \
   --prepare 1600 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "$GRAFT_REPO_ROOT/gpurun_out/prof_r05t_1600.log" 2>&1) || { echo PROF1600_FAIL; exit 1; }
python3 scripts/prof_summary.py gpurun_out/prof_r05ts gpurun_out/prof_r05t_step1600_summary.md --last-steps 20 > /dev/null && rm -rf gpurun_out/prof_r05ts
head -12 gpurun_out/prof_r05t_step1600_summary.md
echo ALL_OK
