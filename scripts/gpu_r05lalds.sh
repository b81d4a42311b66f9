#!/bin/bash
# The lookahead march with dynamic LDS (NEUS_LA_LDS bytes) to cap its workgroups per CU beside the training kernels,
# alternating on one box, at the bench state (main leg only).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
F="--cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 --steps 200 --warmup 20"
: > gpurun_out/ab_r05lalds.txt
for rep in 1 2; do for m in ${LDSV:-0 24576 40960 57344}; do
  NEUS_LA_STAT=1 NEUS_LA_LDS=$m timeout -k 10 300 python -u bench.py $F > gpurun_out/lalds_${m}_$rep.log 2>&1 || exit 1
  python3 - "$m" "$rep" gpurun_out/lalds_${m}_$rep.log >> gpurun_out/ab_r05lalds.txt <<'PY'
import json, sys
lines = open(sys.argv[3]).read().splitlines()
d = json.loads(lines[-1]); st = [l for l in lines if l.startswith("la_stat n=1")]
print("lds", sys.argv[1], "rep", sys.argv[2], "ms", round(d["ms_per_step"], 4), st[-1] if st else "")
PY
  tail -1 gpurun_out/ab_r05lalds.txt
done; done
echo ALL_OK
