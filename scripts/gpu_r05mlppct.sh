#!/bin/bash
# The training MLP kernels on a smaller persistent grid (NEUS_MLP_BLOCKS_PCT of the resident capacity) beside the lookahead,
# alternating on one box, at the bench state (main leg only).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
F="--cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 --steps 200 --warmup 20"
: > gpurun_out/ab_r05mlppct.txt
for rep in 1 2; do for m in ${PCTV:-100 75 50}; do
  NEUS_LA_STAT=1 NEUS_MLP_BLOCKS_PCT=$m timeout -k 10 300 python -u bench.py $F > gpurun_out/mlppct_${m}_$rep.log 2>&1 || exit 1
  python3 - "$m" "$rep" gpurun_out/mlppct_${m}_$rep.log >> gpurun_out/ab_r05mlppct.txt <<'PY'
import json, sys
lines = open(sys.argv[3]).read().splitlines()
d = json.loads(lines[-1]); st = [l for l in lines if l.startswith("la_stat n=1")]
print("pct", sys.argv[1], "rep", sys.argv[2], "ms", round(d["ms_per_step"], 4), st[-1] if st else "")
PY
  tail -1 gpurun_out/ab_r05mlppct.txt
done; done
echo ALL_OK
