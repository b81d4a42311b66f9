#!/bin/bash
# March diagnostics at the bench state (WARM=800) and the later step-1600 state: per-wave phase timing and lane event
# balance (scripts/diag_march_prof.py), and a kernel-trace summary of 20 steps at step 1600.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r04m}
for W in 800 1600; do
  WARM=$W timeout -k 10 300 python -u scripts/diag_march_prof.py > gpurun_out/march_prof_${TAG}_w$W.log 2>&1 || { echo "march prof $W failed"; exit 1; }
  head -8 gpurun_out/march_prof_${TAG}_w$W.log
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 \
   --prepare 1600 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "$R/gpurun_out/prof_${TAG}_1600.log" 2>&1) || { echo PROF_FAIL; exit 1; }
python3 scripts/prof_summary.py gpurun_out/prof_$TAG gpurun_out/prof_${TAG}_step1600_summary.md --last-steps 20 > /dev/null && rm -rf gpurun_out/prof_$TAG
head -12 gpurun_out/prof_${TAG}_step1600_summary.md
echo ALL_OK
