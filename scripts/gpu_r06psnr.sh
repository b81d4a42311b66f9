#!/bin/bash
# Round 6: the PSNR leg's training time (adaptive rays: no cuts, full-march lookahead) by the full march's lookahead issue
# point (NEUS_LA_AT_FULL 0: after the loss, the default; 1: after the encode), and the step-800 bench of this build.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06psnr}
for E in NEUS_LA_AT_FULL=1 NEUS_LA_AT_FULL=0 NEUS_LA_AT_FULL=1 NEUS_LA_AT_FULL=0; do
  env $E timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --cpu-baseline 0 --mc-res 0 --l16 0 --early 0 > "gpurun_out/bench_${TAG}.log" 2>&1 || { echo "BENCH_FAIL $E"; exit 1; }
  python3 - "$E" "gpurun_out/bench_${TAG}.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(sys.argv[1], "psnr", d["psnr"]["value"], "train_wall_s", d["psnr"]["train_wall_s"])
PY
done
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --prepare 800 --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "gpurun_out/bench_${TAG}_800.log" 2>&1 || { echo "BENCH_FAIL"; exit 1; }
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/bench_${TAG}_800.log') if l.startswith('{')][-1]);print('prepare 800 ms/step %.4f' % d['ms_per_step'])"
done
echo ALL_OK
