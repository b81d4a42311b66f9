#!/bin/bash
# Round 6, iteration f: the compaction-cut tests and a bench-shape bitwise fingerprint with the cut off / on.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06f}
timeout -k 10 600 python -u -m pytest tests/test_gpu_overlap.py -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|^E " gpurun_out/pytest_$TAG.log | tail -8; tail -2 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
NEUS_PROG_CUT=0 timeout -k 10 300 python -u scripts/fingerprint_bench_shape.py gpurun_out/fp_cut0_$TAG.json > gpurun_out/fp_cut0_$TAG.log 2>&1 || { echo FP0_FAIL; exit 1; }
NEUS_PROG_CUT=1 timeout -k 10 300 python -u scripts/fingerprint_bench_shape.py gpurun_out/fp_cut1_$TAG.json --compare gpurun_out/fp_cut0_$TAG.json > gpurun_out/fp_cut1_$TAG.log 2>&1
echo "fingerprint rc=$?"; grep FINGERPRINT gpurun_out/fp_cut1_$TAG.log; grep -o '"work": {[^}]*}' gpurun_out/fp_cut0_$TAG.json gpurun_out/fp_cut1_$TAG.json
