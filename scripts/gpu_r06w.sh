#!/bin/bash
# Round 6, iteration w: (1) launch gaps of single kernels replayed back to back (k_nerf_infer, k_grid_encode, loss scan);
# (2) the lookahead's hand-off events without / with the system-scope fence (NEUS_EV_SYSFENCE), bench at step 800;
# (3) the step's queue gaps with the new events.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06w}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/prof_${TAG}_replay" -o run -- python3 "$R/scripts/diag_launch_gaps.py" > "$R/gpurun_out/prof_${TAG}_replay.log" 2>&1 || { echo REPLAY_FAIL; tail -3 "$R/gpurun_out/prof_${TAG}_replay.log"; exit 1; }
python3 "$R/scripts/prof_gaps.py" "$R/gpurun_out/prof_${TAG}_replay" --all > "$R/gpurun_out/prof_${TAG}_replay_gaps.txt" 2>&1 && rm -rf "$R/gpurun_out/prof_${TAG}_replay"
head -14 "$R/gpurun_out/prof_${TAG}_replay_gaps.txt"
cd "$R"
for E in NEUS_EV_SYSFENCE=1 NEUS_EV_SYSFENCE=0 NEUS_EV_SYSFENCE=1 NEUS_EV_SYSFENCE=0 NEUS_CHUNK_ROUNDS=2 NEUS_CHUNK_SCALE=1.5 NEUS_CHUNK_SCALE=0.75 NEUS_CHUNK_ROUNDS=3; do
  env $E timeout -k 10 300 python -u bench.py --prepare 800 --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "gpurun_out/bench_${TAG}_$E.log" 2>&1 || { echo "BENCH_FAIL $E"; exit 1; }
  python3 - "$E" "gpurun_out/bench_${TAG}_$E.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(sys.argv[1], "ms/step %.4f" % d["ms_per_step"], "mcut", d.get("march_cut_steps_timed"), "reruns", d.get("march_cut_reruns_timed"))
PY
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --prepare 800 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "$R/gpurun_out/prof_$TAG.log" 2>&1 || { echo PROF_FAIL; exit 1; }
python3 "$R/scripts/prof_gaps.py" "$R/gpurun_out/prof_$TAG" --last-steps 20 > "$R/gpurun_out/prof_${TAG}_gaps.txt" 2>&1 && rm -rf "$R/gpurun_out/prof_$TAG"
head -14 "$R/gpurun_out/prof_${TAG}_gaps.txt"
echo ALL_OK
