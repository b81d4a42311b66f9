#!/bin/bash
# Round 6, iteration y: the fused scan + cut (tests, fingerprint), then two-round chunk ends by first-chunk scale at steps
# 800 / 1600.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06y}
timeout -k 10 900 python -u -m pytest tests/test_gpu_overlap.py tests/test_gpu_parity.py -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|^E " gpurun_out/pytest_$TAG.log | tail -8; tail -1 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
NEUS_MARCH_CUT=0 NEUS_PROG_CUT=0 timeout -k 10 300 python -u scripts/fingerprint_bench_shape.py gpurun_out/fp_nocut_$TAG.json > gpurun_out/fp_nocut_$TAG.log 2>&1 || { echo FP0_FAIL; exit 1; }
timeout -k 10 300 python -u scripts/fingerprint_bench_shape.py gpurun_out/fp_def_$TAG.json --compare gpurun_out/fp_nocut_$TAG.json > gpurun_out/fp_def_$TAG.log 2>&1
echo "fingerprint rc=$?"; grep FINGERPRINT gpurun_out/fp_def_$TAG.log
for P in 800 1600; do
for E in "NEUS_CHUNK_SCALE=1 NEUS_CHUNK_ROUNDS=2" "NEUS_CHUNK_SCALE=1.5 NEUS_CHUNK_ROUNDS=2" "NEUS_CHUNK_SCALE=2 NEUS_CHUNK_ROUNDS=2" "NEUS_CHUNK_SCALE=2.5 NEUS_CHUNK_ROUNDS=2" "NEUS_CHUNK_SCALE=1"; do
  env $E timeout -k 10 300 python -u bench.py --prepare $P --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "gpurun_out/bench_${TAG}.log" 2>&1 || { echo "BENCH_FAIL $E"; exit 1; }
  python3 - "$E" "$P" "gpurun_out/bench_${TAG}.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[3]) if l.startswith("{")][-1])
print("prepare", sys.argv[2], sys.argv[1], "ms/step %.4f" % d["ms_per_step"], "chunk_end", d["progressive_chunk_end"],
      "eval/step %.0f" % d["roofline_step"]["per_step"]["evaluated_samples"], "mcut", d["march_cut_steps_timed"], "reruns", d["march_cut_reruns_timed"])
PY
done; done
echo ALL_OK
