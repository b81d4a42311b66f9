#!/bin/bash
# March parity (bit-exact sampling tests) then the march launch time over persistent-wave counts at two states.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "sample_rays or loss_compaction or render or dynamic" > gpurun_out/pytest_march.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_march.log; [ $rc -ne 0 ] && exit $rc
for W in 5 800; do for MW in 0 2048; do
  NEUS_MARCH_WAVES=$MW WARM=$W K=0,1 ITERS=9 timeout -k 10 120 python -u scripts/diag_one.py > gpurun_out/march_w${W}_mw${MW}.log 2>&1 || exit 1
  echo "warm $W waves $MW: $(tr '\n' ' ' < gpurun_out/march_w${W}_mw${MW}.log)"
done; done
