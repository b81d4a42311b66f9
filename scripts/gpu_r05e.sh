#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
o=gpurun_out/diag_conc_lock_r05e.jsonl
: > $o
echo '{"variant": "NEUS_LAUNCH_LOCK=1"}' >> $o
NEUS_LAUNCH_LOCK=1 timeout -k 10 300 python -u scripts/diag_concurrency_procs.py --trials 16 --threads >> $o 2>&1 &&
echo '{"variant": "no lock"}' >> $o &&
timeout -k 10 300 python -u scripts/diag_concurrency_procs.py --trials 8 --threads >> $o 2>&1
