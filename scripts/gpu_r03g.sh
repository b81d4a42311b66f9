#!/bin/bash
# tests subset + steady-state profile + the scatter replay at the two wide-binning block sizes
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r03g}
bash scripts/gpu_iter3.sh $TAG "${2:-scatter or module or config or teacher or reproducible or dp}" || exit $?
for C in 512 1024; do
  NEUS_SCATTER_CHUNK=$C timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > gpurun_out/bench_${TAG}_c$C.log 2>&1 || { echo BENCH_FAIL; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_${TAG}_c$C.log').read().strip().splitlines()[-1]); print('chunk $C', round(d['ms_per_step'],4), {k: v['ms'] for k, v in d['kernels'].items()})"
done
echo DONE_G
