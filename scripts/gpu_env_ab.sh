#!/bin/bash
# Development: steady-state bench lines under environment variants. Usage: bash scripts/gpu_env_ab.sh TAG PREPARE "VAR=a" "VAR=b" ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=$1; P=$2; shift 2
for E in "$@"; do
  env $E timeout -k 10 300 python -u bench.py --prepare $P --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "gpurun_out/bench_${TAG}_$P_$E.log" 2>&1 || { echo "BENCH_FAIL $E"; exit 1; }
  python3 - "$E" "$P" "gpurun_out/bench_${TAG}_$P_$E.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[3]) if l.startswith("{")][-1])
print("prepare", sys.argv[2], sys.argv[1], "ms/step %.4f" % d["ms_per_step"], "march %.1f" % (1000 * d["kernels"]["march"]["ms"]))
PY
done
echo ENV_OK
