#!/bin/bash
# Round 6: a long bitwise check - the bench-shape fingerprint after 3000 steps with every cut on (the default) against
# both cuts off (several view-window rotations, occupancy updates, re-runs if any).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06long}
NEUS_MARCH_CUT=0 NEUS_PROG_CUT=0 STEPS=3000 timeout -k 10 400 python -u scripts/fingerprint_bench_shape.py gpurun_out/fp_nocut_$TAG.json > gpurun_out/fp_nocut_$TAG.log 2>&1 || { echo FP0_FAIL; tail -3 gpurun_out/fp_nocut_$TAG.log; exit 1; }
STEPS=3000 timeout -k 10 400 python -u scripts/fingerprint_bench_shape.py gpurun_out/fp_def_$TAG.json --compare gpurun_out/fp_nocut_$TAG.json > gpurun_out/fp_def_$TAG.log 2>&1
echo "fingerprint rc=$?"; grep FINGERPRINT gpurun_out/fp_def_$TAG.log
python3 -c "
import json
for f in ('gpurun_out/fp_nocut_$TAG.json', 'gpurun_out/fp_def_$TAG.json'):
    d = json.load(open(f)); print(f, d.get('work'), d.get('counters'))"
echo ALL_OK
