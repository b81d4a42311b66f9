#!/bin/bash
# Round 6, iteration x: the progressive chunk ends with the cuts - first-chunk scale and round count, at steps 800 / 1600.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06x}
for P in 800 1600; do
for E in "NEUS_CHUNK_SCALE=1" "NEUS_CHUNK_SCALE=1.5" "NEUS_CHUNK_SCALE=2" "NEUS_CHUNK_SCALE=2.5" "NEUS_CHUNK_SCALE=3" "NEUS_CHUNK_SCALE=2 NEUS_CHUNK_ROUNDS=2" "NEUS_CHUNK_SCALE=3 NEUS_CHUNK_ROUNDS=2" "NEUS_CHUNK_SCALE=1.5"; do
  env $E timeout -k 10 300 python -u bench.py --prepare $P --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "gpurun_out/bench_${TAG}.log" 2>&1 || { echo "BENCH_FAIL $E"; exit 1; }
  python3 - "$E" "$P" "gpurun_out/bench_${TAG}.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[3]) if l.startswith("{")][-1])
print("prepare", sys.argv[2], sys.argv[1], "ms/step %.4f" % d["ms_per_step"], "chunk_end", d["progressive_chunk_end"],
      "eval/step %.0f" % d["roofline_step"]["per_step"]["evaluated_samples"], "cut", d["compaction_cut_steps_timed"], "mcut", d["march_cut_steps_timed"])
PY
done; done
echo ALL_OK
