"""Summarise a rocprofv3 --kernel-trace --stats run (rocpd SQLite db or kernel_stats.csv) into a
markdown table: kernel, calls, total ms, average us, share.
Usage: prof_summary.py <db|csv> [out.md] [--last-steps K]
--last-steps K (db only): only the final K training steps (delimited by the optimizer launches), i.e. the final K
training steps (the steady state after the bench warm-up), with the per-step time of each kernel."""
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


def replay_start(ks):
    """Index of the first launch of bench.py's kernel replays (kernel_rooflines): each replay regenerates the step's
    samples with k_loss_alpha, which the static-scene training step no longer launches (its alpha terms are in the
    inference epilogue); len(ks) when there are none."""
    return next((i for i, r in enumerate(ks) if "k_loss_alpha" in r[0]), len(ks))


def step_ends(ks):
    """Indices of the training steps' optimizer launches (one k_adam_ema per step), before the replays (which replay
    the optimizer too)."""
    end = replay_start(ks)
    return [i for i, r in enumerate(ks[:end]) if "k_adam_ema" in r[0]]


def rows_last_steps(path, k):
    """Kernels of the last k training steps: the launches after the (k+1)-th last k_adam_ema of the training up to and
    including the last one."""
    con = sqlite3.connect(path)
    ks = list(con.execute("select name, start, end from kernels order by start"))
    adam = step_ends(ks)
    begin, last = adam[-k - 1] + 1, adam[-1]
    out = {}
    for name, st, en in ks[begin:last + 1]:
        c, t = out.get(name, (0, 0.0))
        out[name] = (c + 1, t + float(en - st))
    return [(n, c, t, t / c) for n, (c, t) in out.items()]


def main():
    args = [a for a in sys.argv[1:]]
    last = None
    back = [1]
    if "--seq-back" in args:  # also print the launch sequences of these steps counted from the end (1 = the final step)
        i = args.index("--seq-back")
        back = [int(x) for x in args[i + 1].split(",")]
        del args[i:i + 2]
    if "--last-steps" in args:
        i = args.index("--last-steps")
        last = int(args[i + 1])
        del args[i:i + 2]
    sys.argv = [sys.argv[0]] + args
    import glob, os
    if os.path.isdir(sys.argv[1]):
        sys.argv[1] = (glob.glob(os.path.join(sys.argv[1], "**", "*.db"), recursive=True) or
                       glob.glob(os.path.join(sys.argv[1], "**", "*kernel_stats.csv"), recursive=True))[0]
    rows = rows_last_steps(sys.argv[1], last) if last else rows_from(sys.argv[1])
    agg = {}
    for name, calls, tot, _ in rows:
        k = short(name)
        c, t = agg.get(k, (0, 0.0))
        agg[k] = (c + calls, t + tot)
    total = sum(t for _, t in agg.values())
    hdr = "| kernel | calls | total ms | avg us | share |" + (" us/step |" if last else "")
    lines = [hdr, "|---|---:|---:|---:|---:|" + ("---:|" if last else "")]
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        extra = f" {t / last / 1e3:.1f} |" if last else ""
        lines.append(f"| {k} | {c} | {t / 1e6:.3f} | {t / c / 1e3:.1f} | {100 * t / total:.1f}% |" + extra)
    if last:
        lines.append(f"\nGPU kernel time per step over the last {last} steps: {total / last / 1e6:.3f} ms")
        # the launch sequence of the final step (start offset, duration), e.g. the progressive-inference rounds
        con = sqlite3.connect(sys.argv[1])
        ks = list(con.execute("select name, start, end from kernels order by start"))
        adam = step_ends(ks)
        for j in back:
            # from the end of the previous step's optimizer launch: the kernels that started after it (the lookahead's
            # sampling for this step, issued beside that step's backward, started before it and is listed there)
            seq = ks[adam[-j - 1] + 1:adam[-j] + 1]
            t0 = ks[adam[-j - 1]][2]
            lines.append(f"\nLaunch sequence of step -{j} (start us after the previous step's optimizer ended, end us, duration us):\n")
            lines += [f"    {(st - t0) / 1e3:9.1f} {(en - t0) / 1e3:9.1f} {(en - st) / 1e3:8.1f}  {short(n)}" for n, st, en in seq]
        # bench.py's per-kernel replays (kernel_rooflines) run after the last training step: their median launch is
        # the `launch_ms` of the bench line's roofline / kernels entries
        tail = {}
        for n, st, en in ks[adam[-1] + 1:]:
            tail.setdefault(short(n), []).append((en - st) / 1e3)
        if tail:
            lines.append("\nReplayed launches after the timed steps (bench.py kernel_rooflines): kernel, launches, median us\n")
            for k, v in sorted(tail.items(), key=lambda kv: -sorted(kv[1])[len(kv[1]) // 2]):
                v = sorted(v)
                lines.append(f"    {k:28s} {len(v):4d} {v[len(v) // 2]:9.1f}")
    text = "\n".join(lines) + "\n"
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text)
    print(text)


if __name__ == "__main__":
    main()
