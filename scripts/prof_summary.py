"""Summarise a rocprofv3 --kernel-trace --stats run (rocpd SQLite db or kernel_stats.csv) into a
markdown table: kernel, calls, total ms, average us, share. Usage: prof_summary.py <db|csv> [out.md]"""
import csv
import re
import sqlite3
import sys


def short(name):
    name = re.sub(r"^void ", "", name)
    m = re.match(r"_ZN4neus(\d+)", name)  # mangled (template) kernels: length-prefixed identifier
    if m:
        n = int(m.group(1))
        return name[m.end():m.end() + n]
    m = re.search(r"neus::(k_\w+)", name)
    if m:
        return m.group(1)
    if "rocprim" in name:
        kind = "scan" if "scan" in name else ("reduce" if "reduce" in name else "rocprim")
        return f"rocprim::{kind}" + ("_init" if "init_lookback" in name else "")
    return name[:60]


def rows_from(path):
    if path.endswith(".db"):
        con = sqlite3.connect(path)
        # rocpd top_kernels durations are in microseconds; normalise to ns like kernel_stats.csv
        return [(r[0], int(r[1]), float(r[2]) * 1e3, float(r[3]) * 1e3) for r in
                con.execute("select name, total_calls, total_duration, average from top_kernels")]
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"])))
    return out


def main():
    rows = rows_from(sys.argv[1])
    agg = {}
    for name, calls, tot, _ in rows:
        k = short(name)
        c, t = agg.get(k, (0, 0.0))
        agg[k] = (c + calls, t + tot)
    total = sum(t for _, t in agg.values())
    lines = ["| kernel | calls | total ms | avg us | share |", "|---|---:|---:|---:|---:|"]
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        lines.append(f"| {k} | {c} | {t / 1e6:.3f} | {t / c / 1e3:.1f} | {100 * t / total:.1f}% |")
    text = "\n".join(lines) + "\n"
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text)
    print(text)


if __name__ == "__main__":
    main()
