#!/bin/bash
# Round 6, iteration q: kernel traces (timelines of two mid-call steps) of the driver-shaped bench at step 800 with the
# march cut, with and without the host's wait for the witness word (the latter an unsafe timing experiment).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06q}
cd /tmp && export TMPDIR=/tmp
for W in 0 1; do
  NEUS_DBG_ABORT_NOWAIT=$W timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_w$W" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --prepare 800 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "$R/gpurun_out/prof_${TAG}_w$W.log" 2>&1 || { echo PROF_FAIL; exit 1; }
  python3 "$R/scripts/prof_summary.py" "$R/gpurun_out/prof_${TAG}_w$W" "$R/gpurun_out/prof_${TAG}_nowait${W}_timeline.md" --last-steps 20 --seq-back 2,3,5 > /dev/null && rm -rf "$R/gpurun_out/prof_${TAG}_w$W"
done
echo ALL_OK
