#!/bin/bash
# Round 6, iteration n: the march cut - its tests (bitwise against no cut; the re-run path, one rank and two), a bench-shape
# fingerprint with it off / on, then the bench at steps 800 / 1600 with it off / on.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06n}
timeout -k 10 900 python -u -m pytest tests/test_gpu_overlap.py -v --timeout 400 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|^E " gpurun_out/pytest_$TAG.log | tail -14; tail -2 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
NEUS_MARCH_CUT=0 timeout -k 10 300 python -u scripts/fingerprint_bench_shape.py gpurun_out/fp_mc0_$TAG.json > gpurun_out/fp_mc0_$TAG.log 2>&1 || { echo FP0_FAIL; exit 1; }
NEUS_MARCH_CUT=1 timeout -k 10 300 python -u scripts/fingerprint_bench_shape.py gpurun_out/fp_mc1_$TAG.json --compare gpurun_out/fp_mc0_$TAG.json > gpurun_out/fp_mc1_$TAG.log 2>&1
echo "fingerprint rc=$?"; grep FINGERPRINT gpurun_out/fp_mc1_$TAG.log; grep -o '"work": {[^}]*}' gpurun_out/fp_mc0_$TAG.json gpurun_out/fp_mc1_$TAG.json
for P in 800 1600; do
for E in NEUS_MARCH_CUT=0 NEUS_MARCH_CUT=1 NEUS_MARCH_CUT=0 NEUS_MARCH_CUT=1; do
  env $E timeout -k 10 300 python -u bench.py --prepare $P --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "gpurun_out/bench_${TAG}_${P}_$E.log" 2>&1 || { echo "BENCH_FAIL $E"; exit 1; }
  python3 - "$E" "$P" "gpurun_out/bench_${TAG}_${P}_$E.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[3]) if l.startswith("{")][-1])
print("prepare", sys.argv[2], sys.argv[1], "ms/step %.4f" % d["ms_per_step"], "non_rollover %.4f" % d["non_rollover_fraction"],
      "cut_steps", d["compaction_cut_steps_timed"], "eval/step %.0f" % d["roofline_step"]["per_step"]["evaluated_samples"])
PY
done; done
echo ALL_OK
