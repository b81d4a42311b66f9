#!/bin/bash
# Round 6, iteration m: timing experiment - the march limited to the compaction cut's split estimate (NEUS_MARCH_CUT_EXP=1,
# later slots dropped: not exact, an upper bound of what a cut march could save) against the default, at steps 800 / 1600.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06m}
for P in 800 1600; do
for rep in 1 2; do
for E in NEUS_MARCH_CUT_EXP=0 NEUS_MARCH_CUT_EXP=1; do
  env $E timeout -k 10 300 python -u bench.py --prepare $P --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "gpurun_out/bench_${TAG}_${P}_$E.log" 2>&1 || { echo "BENCH_FAIL $E"; exit 1; }
  python3 - "$E" "$P" "gpurun_out/bench_${TAG}_${P}_$E.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[3]) if l.startswith("{")][-1])
print("prepare", sys.argv[2], sys.argv[1], "ms/step %.4f" % d["ms_per_step"], "non_rollover %.4f" % d["non_rollover_fraction"],
      "cut_steps", d["compaction_cut_steps_timed"], "eval/step %.0f" % d["roofline_step"]["per_step"]["evaluated_samples"])
PY
done; done; done
echo ALL_OK
