#!/bin/bash
# Round 6, iteration l: kernel traces of the driver-shaped bench at step 800 and step 1600 with the launch timelines of
# two mid-call steps (the lookahead's sampling beside the backward, the cut rounds).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06l}
cd /tmp && export TMPDIR=/tmp
for P in 800 1600; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_$P" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --prepare $P --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "$R/gpurun_out/prof_${TAG}_$P.log" 2>&1 || { echo PROF_FAIL; exit 1; }
  python3 "$R/scripts/prof_summary.py" "$R/gpurun_out/prof_${TAG}_$P" "$R/gpurun_out/prof_${TAG}_${P}_timeline.md" --last-steps 20 --seq-back 2,5 > /dev/null && rm -rf "$R/gpurun_out/prof_${TAG}_$P"
done
echo ALL_OK
