#!/bin/bash
# Round 6 end check of the in-tree library: smoke, the whole GPU suite, one default-shape bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06end}
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE_FAIL; tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|^E " gpurun_out/pytest_$TAG.log | tail -8; tail -1 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > gpurun_out/bench_$TAG.log 2>&1 || { echo BENCH_FAIL; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-220
echo ALL_OK
