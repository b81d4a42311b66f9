#!/bin/bash
# Round 6, iteration t: the overlap / cut tests, the bench-shape fingerprint (march cut on vs off), the bench at steps
# 800 / 1600.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06t}
timeout -k 10 900 python -u -m pytest tests/test_gpu_overlap.py -v --timeout 400 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|^E " gpurun_out/pytest_$TAG.log | tail -8; tail -1 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
NEUS_MARCH_CUT=0 timeout -k 10 300 python -u scripts/fingerprint_bench_shape.py gpurun_out/fp_mc0_$TAG.json > gpurun_out/fp_mc0_$TAG.log 2>&1 || { echo FP0_FAIL; exit 1; }
NEUS_MARCH_CUT=1 timeout -k 10 300 python -u scripts/fingerprint_bench_shape.py gpurun_out/fp_mc1_$TAG.json --compare gpurun_out/fp_mc0_$TAG.json > gpurun_out/fp_mc1_$TAG.log 2>&1
echo "fingerprint rc=$?"; grep FINGERPRINT gpurun_out/fp_mc1_$TAG.log
for P in 800 1600; do
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --prepare $P --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "gpurun_out/bench_${TAG}_${P}_$rep.log" 2>&1 || { echo "BENCH_FAIL"; exit 1; }
  python3 - "$P" "gpurun_out/bench_${TAG}_${P}_$rep.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print("prepare", sys.argv[1], "ms/step %.4f" % d["ms_per_step"], "non_rollover %.4f" % d["non_rollover_fraction"])
PY
done; done
echo ALL_OK
