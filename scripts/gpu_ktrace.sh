#!/bin/bash
# rocprofv3 kernel trace of diag_one.py (env K, V, WARM, ITERS); prints the last launches' durations.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-kt}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/kt_$TAG" -o run -- python3 "$R/scripts/diag_one.py" > "$R/gpurun_out/kt_$TAG.log" 2>&1 || exit $?
python3 - "$R/gpurun_out/kt_$TAG" "${NLAST:-40}" <<'PY'
import csv, glob, sys, re
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
for r in rows[-int(sys.argv[2]):]:
    n = re.sub(r"\(.*", "", r["Kernel_Name"])[:60]
    print(f"{n:60s} {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:9.1f} us")
PY
rm -rf "$R/gpurun_out/kt_$TAG"
