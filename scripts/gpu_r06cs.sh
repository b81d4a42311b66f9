#!/bin/bash
# Round 6: the cut steps' first-chunk scale around the default 2 (two rounds), at steps 800 / 1600, alternating.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06cs}
for P in 800 1600; do
for E in NEUS_CHUNK_SCALE=2 NEUS_CHUNK_SCALE=1.75 NEUS_CHUNK_SCALE=2.25 NEUS_CHUNK_SCALE=2 NEUS_CHUNK_SCALE=1.75 NEUS_CHUNK_SCALE=2.25; do
  env $E timeout -k 10 300 python -u bench.py --prepare $P --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "gpurun_out/bench_${TAG}.log" 2>&1 || { echo "BENCH_FAIL $E"; exit 1; }
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/bench_${TAG}.log') if l.startswith('{')][-1]);print('prepare $P $E', 'ms/step %.4f' % d['ms_per_step'])"
done; done
echo ALL_OK
