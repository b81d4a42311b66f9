#!/bin/bash
# r05i: A/B of the concurrent-testbed divergence: the default build against march.o without packed-fp32 instructions
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
o=gpurun_out/diag_conc_pk_ab_r05i.jsonl
: > $o
echo '{"variant": "default build"}' >> $o &&
timeout -k 10 200 python -u scripts/diag_concurrency_batch.py --steps 1 --pairs 12 --buffers 0 >> $o 2>&1 &&
echo '{"variant": "march.o without packed fp32 (NEUS2_HIP_LIB=libneus2_hip_nopk.so)"}' >> $o &&
NEUS2_HIP_LIB=$PWD/neus2_amd/libneus2_hip_nopk.so timeout -k 10 200 python -u scripts/diag_concurrency_batch.py --steps 1 --pairs 12 --buffers 0 >> $o 2>&1 &&
echo '{"variant": "default build, again"}' >> $o &&
timeout -k 10 200 python -u scripts/diag_concurrency_batch.py --steps 1 --pairs 12 --buffers 0 >> $o 2>&1
