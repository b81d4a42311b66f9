#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
o=gpurun_out/diag_conc_r05h.jsonl
: > $o
echo '{"variant": "default queues"}' >> $o
timeout -k 10 200 python -u scripts/diag_concurrency_batch.py --steps 1 --pairs 8 --buffers 0 >> $o 2>&1 &&
echo '{"variant": "GPU_MAX_HW_QUEUES=8"}' >> $o &&
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u scripts/diag_concurrency_batch.py --steps 1 --pairs 8 --buffers 0 >> $o 2>&1 &&
echo '{"variant": "GPU_MAX_HW_QUEUES=16"}' >> $o &&
GPU_MAX_HW_QUEUES=16 timeout -k 10 200 python -u scripts/diag_concurrency_batch.py --steps 1 --pairs 8 --buffers 0 >> $o 2>&1 &&
timeout -k 10 300 python -u scripts/psnr_anchor.py --side gpu --steps 2000 --checkpoints 250,500,1000,1500 --fixed-rays 512 > gpurun_out/r05_psnr_anchor_fixedR512_gpu.jsonl 2>&1
