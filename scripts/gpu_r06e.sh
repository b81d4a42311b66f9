#!/bin/bash
# Round 6, iteration e: the compaction cut with the split round 0 - the GPU suite, then the bench A/B (NEUS_PROG_CUT).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06e}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR" gpurun_out/pytest_$TAG.log | tail -8; tail -2 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/gpu_env_ab.sh $TAG 800 NEUS_PROG_CUT=0 NEUS_PROG_CUT=1 NEUS_PROG_CUT=0 NEUS_PROG_CUT=1 || exit 1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_drv_$TAG.log 2>&1 || { echo BENCH_DRV_FAIL; exit 1; }
tail -1 gpurun_out/bench_drv_$TAG.log | cut -c1-300
