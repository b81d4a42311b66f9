#!/bin/bash
# Round 6, iteration h: the cut test; where the lookahead is issued now that the inference is shorter (NEUS_LA_AT), and the
# training MLP kernels on half their grid beside it (NEUS_MLP_BLOCKS_PCT=50).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06h}
timeout -k 10 600 python -u -m pytest tests/test_gpu_overlap.py -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|^E " gpurun_out/pytest_$TAG.log | tail -8; tail -2 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/gpu_env_ab.sh $TAG 800 NEUS_LA_AT=0 NEUS_LA_AT=2 NEUS_LA_AT=3 NEUS_MLP_BLOCKS_PCT=50 NEUS_LA_AT=0 NEUS_LA_AT=2 NEUS_LA_AT=3 NEUS_MLP_BLOCKS_PCT=50 || exit 1
