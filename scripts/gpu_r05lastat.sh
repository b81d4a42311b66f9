#!/bin/bash
# Where the lookahead's time goes (NEUS_LA_STAT=1): the next step's wait for the sampling, the sampling's duration beside
# the backward, and the slack between its end and the wait; at the bench state and at step 1600.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
F="--cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0"
NEUS_LA_STAT=1 timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 $F > gpurun_out/lastat_main.log 2>&1 || exit 1
grep la_stat gpurun_out/lastat_main.log | tail -3; tail -1 gpurun_out/lastat_main.log | cut -c1-200
NEUS_LA_STAT=1 timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --prepare 1600 $F > gpurun_out/lastat_1600.log 2>&1 || exit 1
grep la_stat gpurun_out/lastat_1600.log | tail -3; tail -1 gpurun_out/lastat_1600.log | cut -c1-200
echo ALL_OK
