#!/bin/bash
# Round 6: k_loss_ray limited to the marched slots on cut-march steps - the overlap / cut / parity tests, the bench-shape
# fingerprint against no cuts, the bench at steps 800 / 1600.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06lr}
timeout -k 10 900 python -u -m pytest tests/test_gpu_overlap.py tests/test_gpu_parity.py -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|^E " gpurun_out/pytest_$TAG.log | tail -8; tail -1 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
NEUS_MARCH_CUT=0 NEUS_PROG_CUT=0 timeout -k 10 300 python -u scripts/fingerprint_bench_shape.py gpurun_out/fp_nocut_$TAG.json > gpurun_out/fp_nocut_$TAG.log 2>&1 || { echo FP0_FAIL; exit 1; }
timeout -k 10 300 python -u scripts/fingerprint_bench_shape.py gpurun_out/fp_def_$TAG.json --compare gpurun_out/fp_nocut_$TAG.json > gpurun_out/fp_def_$TAG.log 2>&1
echo "fingerprint rc=$?"; grep FINGERPRINT gpurun_out/fp_def_$TAG.log
for P in 800 1600; do
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --prepare $P --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "gpurun_out/bench_${TAG}.log" 2>&1 || { echo "BENCH_FAIL"; exit 1; }
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/bench_${TAG}.log') if l.startswith('{')][-1]);print('prepare $P', 'ms/step %.4f' % d['ms_per_step'])"
done; done
echo ALL_OK
