"""Gaps between consecutive kernels of one queue in a rocprofv3 kernel trace (development tool): for every (previous,
next) kernel pair on the same queue over the final K training steps, the number of transitions and the median idle gap
between the previous kernel's end and the next one's start.
Usage: prof_gaps.py <trace dir or .db> [--last-steps K | --all]"""
import glob
import os
import sqlite3
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import short, step_ends  # noqa: E402


def main():
    args = sys.argv[1:]
    k = 20
    if "--last-steps" in args:
        i = args.index("--last-steps")
        k = int(args[i + 1])
        del args[i:i + 2]
    path = [a for a in args if not a.startswith("--")][0]
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)[0]
    con = sqlite3.connect(path)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    qcol = next((c for c in ("queue_id", "stream_id", "queue") if c in cols), None)
    ks = list(con.execute(f"select name, start, end, {qcol or 0} from kernels order by start"))
    if "--all" in args:  # every kernel of the trace (replays, diagnostics)
        t0, t1, k = ks[0][1], ks[-1][2], 1
    else:
        adam = step_ends([(n, s, e) for n, s, e, _ in ks])
        t0, t1 = ks[adam[-k - 1]][2], ks[adam[-1]][2]
    byq = defaultdict(list)
    for n, s, e, q in ks:
        if t0 <= s <= t1:
            byq[q].append((short(n), s, e))
    pairs = defaultdict(list)
    for q, lst in byq.items():
        for (a, _, ea), (b, sb, _) in zip(lst, lst[1:]):
            pairs[(q, a, b)].append((sb - ea) / 1e3)
    print(f"queue column: {qcol}; kernels per queue: " + ", ".join(f"{q}: {len(v)}" for q, v in byq.items()))
    print("queue | previous -> next | transitions | median gap us | total gap us per step")
    rows = []
    for (q, a, b), g in pairs.items():
        g = sorted(g)
        rows.append((sum(g) / k, q, a, b, len(g), g[len(g) // 2]))
    for tot, q, a, b, n, med in sorted(rows, reverse=True)[:40]:
        print(f"{q} | {a} -> {b} | {n} | {med:.1f} | {tot:.1f}")


if __name__ == "__main__":
    main()
