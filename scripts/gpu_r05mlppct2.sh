#!/bin/bash
# NEUS_MLP_BLOCKS_PCT=50 as a candidate default: the GPU suite with it, then the bench legs (main, early steps, 16
# levels) with it and without, alternating on one box.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
NEUS_MLP_BLOCKS_PCT=50 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_pct50.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_pct50.log; [ $rc -eq 0 ] || exit $rc
F="--cpu-baseline 0 --psnr-steps 0 --mc-res 0"
: > gpurun_out/ab_r05mlppct2.txt
for rep in 1 2; do for m in 50 100; do
  NEUS_MLP_BLOCKS_PCT=$m timeout -k 10 300 python -u bench.py $F > gpurun_out/mlppct2_${m}_$rep.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/mlppct2_${m}_$rep.log').read().strip().splitlines()[-1]); print('pct', $m, 'rep', $rep, 'main', round(d['ms_per_step'],4), 'early', round(d['early_steps']['ms_per_step'],4), 'l16', round(d['levels16']['ms_per_step'],4))" >> gpurun_out/ab_r05mlppct2.txt
  tail -1 gpurun_out/ab_r05mlppct2.txt
done; done
echo ALL_OK
