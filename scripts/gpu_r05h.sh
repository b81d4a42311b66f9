#!/bin/bash
# r05h: the concurrent-testbed batch diagnostic with the loss-gradient kernel's variance-term intermediates recorded
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
NEUS_DBG_LOSS_VALS=1 timeout -k 10 300 python -u scripts/diag_concurrency_batch.py --steps 1 --pairs 10 --buffers 0 > gpurun_out/diag_conc_r05h2.jsonl 2>&1
