#!/bin/bash
# Main-leg kernel-trace summary per value of an environment variable: bash scripts/gpu_trace_env.sh TAG VAR v1 v2 ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=$1; VAR=$2; shift 2
for V in "$@"; do
  (cd /tmp && export TMPDIR=/tmp && export "$VAR=$V" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_$V" -o run -- python3 "$R/bench.py" \
     --steps 20 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 ${BENCH_ARGS:-} > "$R/gpurun_out/prof_${TAG}_$V.log" 2>&1) || { echo "PROF_FAIL $V"; exit 1; }
  python3 scripts/prof_summary.py gpurun_out/prof_${TAG}_$V gpurun_out/prof_${TAG}_${V}_summary.md --last-steps 20 > /dev/null && rm -rf gpurun_out/prof_${TAG}_$V
  echo "== $VAR=$V"; head -24 gpurun_out/prof_${TAG}_${V}_summary.md
done
echo TRACE_OK
