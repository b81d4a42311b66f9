#!/bin/bash
# The lookahead started once every block of the density training kernel is resident (NEUS_LA_AT=5, a signal-memory
# count) against the start right after the loss (0), alternating on one box; then the bitwise A/B of the two.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
F="--cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 --steps 200 --warmup 20"
: > gpurun_out/ab_r05la5.txt
for rep in 1 2; do for at in 5 0; do
  NEUS_LA_STAT=1 NEUS_LA_AT=$at timeout -k 10 120 python -u bench.py $F > gpurun_out/la5_${at}_$rep.log 2>&1 || { echo FAIL $at; tail -5 gpurun_out/la5_${at}_$rep.log; exit 1; }
  python3 - "$at" "$rep" gpurun_out/la5_${at}_$rep.log >> gpurun_out/ab_r05la5.txt <<'PY'
import json, sys
lines = open(sys.argv[3]).read().splitlines()
d = json.loads(lines[-1]); st = [l for l in lines if l.startswith("la_stat n=1")]
print("at", sys.argv[1], "rep", sys.argv[2], "ms", round(d["ms_per_step"], 4), st[-1] if st else "")
PY
  tail -1 gpurun_out/ab_r05la5.txt
done; done
echo ALL_OK
