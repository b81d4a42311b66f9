#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/diag_overhead.py > gpurun_out/diag_overhead5.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_m" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 > "$R/gpurun_out/prof_m.log" 2>&1 || exit 1
python3 "$R/scripts/prof_summary.py" "$R/gpurun_out/prof_m" "$R/gpurun_out/prof_m_summary.md" --last-steps 20 > /dev/null
python3 - "$R/gpurun_out/prof_m" <<'PY'
import sqlite3, glob, sys
db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
con = sqlite3.connect(db)
tabs = [r[0] for r in con.execute("select name from sqlite_master where type in ('table','view')")]
print([t for t in tabs if 'kernel' in t.lower()][:10])
PY
rm -rf "$R/gpurun_out/prof_m"
