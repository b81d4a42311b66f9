#!/bin/bash
# r05n: PSNR anchor by segments (the oracle continues the device's state for 500 steps; both rendered)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 1100 python -u scripts/psnr_anchor_segments.py --starts ${STARTS:-250,500,750,1000,1250,1500,1750} --length ${LEN:-250} > gpurun_out/r05_psnr_anchor_segments.jsonl 2> gpurun_out/r05_psnr_anchor_segments.err
