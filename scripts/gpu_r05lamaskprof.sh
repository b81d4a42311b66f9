#!/bin/bash
# Kernel-trace summary of the bench's main leg with the lookahead stream CU-masked (NEUS_LA_CUMASK=$M): is the mask
# honoured (the march slower, the density training kernel back near its serial time)?
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
M=${M:-8}
(cd /tmp && export TMPDIR=/tmp && NEUS_LA_CUMASK=$M timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_lamask$M" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 \
   --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "$R/gpurun_out/prof_lamask$M.log" 2>&1) || { echo PROF_FAIL; exit 1; }
python3 scripts/prof_summary.py gpurun_out/prof_lamask$M gpurun_out/prof_lamask${M}_summary.md --last-steps 20 > /dev/null && rm -rf gpurun_out/prof_lamask$M
head -16 gpurun_out/prof_lamask${M}_summary.md
echo ALL_OK
