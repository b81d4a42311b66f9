#!/bin/bash
# Round 6: queue gaps of kernels replayed back to back without events (k_nerf_infer at its resident grid and capped at
# 256 / 128 workgroups, the grid encode, the loss scan), then the step-800 bench with the inference grid capped.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06gap}
cd /tmp && export TMPDIR=/tmp
for G in 0 256; do
  NEUS_INFER_GRID=$G timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/prof_${TAG}_g$G" -o run -- python3 "$R/scripts/diag_launch_gaps.py" > "$R/gpurun_out/prof_${TAG}_g$G.log" 2>&1 || { echo REPLAY_FAIL; tail -3 "$R/gpurun_out/prof_${TAG}_g$G.log"; exit 1; }
  python3 "$R/scripts/prof_gaps.py" "$R/gpurun_out/prof_${TAG}_g$G" --all > "$R/gpurun_out/prof_${TAG}_g${G}_gaps.txt" 2>&1 && rm -rf "$R/gpurun_out/prof_${TAG}_g$G"
  echo "grid cap $G"; grep -E "k_nerf_infer -> k_nerf_infer|k_grid_encode -> k_grid_encode|k_loss_scan_list -> k_loss_scan_list|k_loss_scan" "$R/gpurun_out/prof_${TAG}_g${G}_gaps.txt" | head -6
  grep kernel "$R/gpurun_out/prof_${TAG}_g$G.log"
done
cd "$R"
for E in NEUS_INFER_GRID=0 NEUS_INFER_GRID=256 NEUS_INFER_GRID=0 NEUS_INFER_GRID=256; do
  env $E timeout -k 10 300 python -u bench.py --prepare 800 --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "gpurun_out/bench_${TAG}.log" 2>&1 || { echo "BENCH_FAIL $E"; exit 1; }
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/bench_${TAG}.log') if l.startswith('{')][-1]);print('$E', 'ms/step %.4f' % d['ms_per_step'])"
done
echo ALL_OK
