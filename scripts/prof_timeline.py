"""Kernel timeline of the last training steps of a rocprofv3 --kernel-trace run (rocpd SQLite db): start / end
relative to the first listed launch, duration and the stream / queue columns the db has, so overlap between the
step's stream and the lookahead stream is visible. Usage: prof_timeline.py <dir-with-db or db> [--steps K]"""
import glob
import os
import sqlite3
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import short, step_ends  # noqa: E402


def main():
    path = sys.argv[1]
    k = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 3
    if os.path.isdir(path):
        path = sorted(glob.glob(os.path.join(path, "**", "*.db"), recursive=True))[0]
    con = sqlite3.connect(path)
    cur = con.execute("select * from kernels limit 1")
    cols = [d[0] for d in cur.description]
    extra = [c for c in cols if "stream" in c.lower() or "queue" in c.lower()]
    sel = ", ".join(["name", "start", "end"] + extra)
    ks = list(con.execute(f"select {sel} from kernels order by start"))
    adam = step_ends(ks)
    lo = adam[-k - 1] + 1 if len(adam) > k else 0
    rows = ks[lo:adam[-1] + 1]
    t0 = rows[0][1]
    print("start_us end_us dur_us " + " ".join(extra) + " kernel")
    for r in rows:
        print(f"{(r[1] - t0) / 1e3:9.1f} {(r[2] - t0) / 1e3:9.1f} {(r[2] - r[1]) / 1e3:7.1f} " +
              " ".join(str(x) for x in r[3:]) + " " + short(r[0]))
    print(f"span of the last {k} steps: {(rows[-1][2] - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
