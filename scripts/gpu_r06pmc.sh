#!/bin/bash
# Round 6: memory-side traffic of the training step's own k_nerf_infer launches at the bench state (with the compaction
# cut; 20 steps after an 800-step prepare, the last 77 dispatches = those 20 steps), and the rocprofv3 kernel trace of the
# driver-shaped bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06pmc}
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE_FAIL; tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
WARM=800 STEPS=20 bash scripts/gpu_traffic_steps.sh ${TAG}_steps 77 || exit $?
cat gpurun_out/${TAG}_steps_table.txt | head -30
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "$R/gpurun_out/prof_$TAG.log" 2>&1 || { echo PROF_FAIL; exit 1; }
python3 "$R/scripts/prof_summary.py" "$R/gpurun_out/prof_$TAG" "$R/gpurun_out/prof_${TAG}_summary.md" --last-steps 20 > /dev/null && rm -rf "$R/gpurun_out/prof_$TAG"
head -12 "$R/gpurun_out/prof_${TAG}_summary.md"; tail -1 "$R/gpurun_out/prof_$TAG.log" | cut -c1-200
echo ALL_OK
