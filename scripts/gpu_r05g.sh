#!/bin/bash
# r05g: fp32 denormal probe alone / beside two training testbeds; the concurrent-testbed batch diagnostic again; the
# PSNR-anchor ensemble (GPU runs with 1-ulp perturbed initial parameters)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 240 python -u scripts/diag_denorm.py > gpurun_out/diag_denorm_r05g.jsonl 2>&1 &&
timeout -k 10 240 python -u scripts/diag_concurrency_batch.py --steps 1 --pairs 10 --buffers 0 > gpurun_out/diag_conc_r05g2.jsonl 2>&1 &&
timeout -k 10 300 python -u scripts/psnr_anchor.py --side gpu --steps 2000 --checkpoints 250,500,1000,1500 --fixed-rays 512 --ensemble 6 \
  > gpurun_out/r05_psnr_anchor_fixedR512_gpu_ensemble.jsonl 2>&1
