#!/bin/bash
# Round 6: occupancy-biased samples binned by coarse cell - GPU tests (parity incl. the occupancy updates), bench-shape
# fingerprint with the binning off / on, the density pass split, bench A/B at step 800.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06occ}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_overlap.py tests/test_gpu_determinism.py -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|^E " gpurun_out/pytest_$TAG.log | tail -8; tail -1 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
NEUS_OCC_NU_SORT=0 timeout -k 10 300 python -u scripts/fingerprint_bench_shape.py gpurun_out/fp_nu0_$TAG.json > gpurun_out/fp_nu0_$TAG.log 2>&1 || { echo FP0_FAIL; exit 1; }
timeout -k 10 300 python -u scripts/fingerprint_bench_shape.py gpurun_out/fp_nu1_$TAG.json --compare gpurun_out/fp_nu0_$TAG.json > gpurun_out/fp_nu1_$TAG.log 2>&1
echo "fingerprint rc=$?"; grep FINGERPRINT gpurun_out/fp_nu1_$TAG.log
for E in NEUS_OCC_NU_SORT=0 NEUS_OCC_NU_SORT=1 NEUS_OCC_NU_SORT=0 NEUS_OCC_NU_SORT=1; do
  env $E timeout -k 10 300 python -u bench.py --prepare 800 --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "gpurun_out/bench_${TAG}.log" 2>&1 || { echo "BENCH_FAIL $E"; exit 1; }
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/bench_${TAG}.log') if l.startswith('{')][-1]);print('$E', 'ms/step %.4f' % d['ms_per_step'])"
done
echo ALL_OK
