#!/bin/bash
# round 5 pass c: locate the divergence of concurrently trained testbeds (scripts/diag_concurrency.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
o=gpurun_out/diag_conc_r05c2.jsonl
: > $o
timeout -k 10 200 python -u scripts/diag_concurrency.py --steps 300 --progressive 2 >> $o 2>&1 &&
timeout -k 10 300 python -u scripts/diag_concurrency.py --steps 816 --sync-every 16 >> $o 2>&1 &&
timeout -k 10 400 python -u scripts/diag_concurrency.py --steps 816 --sync-every 1 >> $o 2>&1
