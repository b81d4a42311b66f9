#!/bin/bash
# Development: progressive-inference chunk schedules (NEUS_CHUNK_ENDS) on the in-tree library: steady-state bench
# lines, after the progressive / scan GPU tests. Usage: bash scripts/gpu_sched_ab.sh TAG "32,80" "32,64,96" ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "progressive or bitwise or loss" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
for E in "$@"; do
  NEUS_CHUNK_ENDS="$E" timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "gpurun_out/bench_${TAG}_$E.log" 2>&1 || { echo "BENCH_FAIL $E"; exit 1; }
  python3 - "$E" "gpurun_out/bench_${TAG}_$E.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print("ends", sys.argv[1], "ms/step %.4f" % d["ms_per_step"])
PY
done
echo SCHED_OK
