#!/bin/bash
# Round 6: the lookahead's issue point with the cut march, alternating A/B (0: after the loss; 1: after the encode).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06la}
for P in 800 1600; do
for E in NEUS_LA_AT=0 NEUS_LA_AT=1 NEUS_LA_AT=0 NEUS_LA_AT=1 NEUS_LA_AT=0 NEUS_LA_AT=1; do
  env $E timeout -k 10 300 python -u bench.py --prepare $P --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "gpurun_out/bench_${TAG}.log" 2>&1 || { echo "BENCH_FAIL $E"; exit 1; }
  python3 - "$E" "$P" "gpurun_out/bench_${TAG}.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[3]) if l.startswith("{")][-1])
print("prepare", sys.argv[2], sys.argv[1], "ms/step %.4f" % d["ms_per_step"])
PY
done; done
echo LA_OK
