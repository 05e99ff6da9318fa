"""Summarise a rocprofv3 --kernel-trace --stats SQLite output (rocpd format) per kernel.

    python tools/prof_summary.py gpurun_out/prof5/run_results.db [--csv out.csv] [--steps N]

Per-step figures divide by the number of train steps seen in the trace (Adam launches / 2,
one per network per step) unless --steps is given.  Durations in the db are nanoseconds.
"""
import argparse
import collections
import csv
import re
import sqlite3


def short(name):
    name = re.sub(r"\(tpg::\w+\)$", "", name)
    name = name.replace("void tpg::", "")
    return name[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--steps", type=int, default=0)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, duration, grid_x, grid_y, grid_z, workgroup_x from kernels").fetchall()
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 1e30])
    for name, dur, gx, gy, gz, wx in rows:
        e = agg[short(name)]
        e[0] += 1
        e[1] += dur
        e[2] = max(e[2], dur)
        e[3] = min(e[3], dur)
    steps = a.steps or max(1, agg.get("adam_kernel", [2])[0] // 2)
    total = sum(v[1] for v in agg.values())
    items = sorted(agg.items(), key=lambda kv: -kv[1][1])
    print("steps in trace: %d   total kernel time %.2f ms  (%.2f ms/step)" % (steps, total / 1e6, total / 1e6 / steps))
    print("%-90s %7s %10s %9s %6s" % ("kernel", "calls", "ms/step", "avg_us", "%"))
    for k, (n, t, mx, mn) in items[:a.top]:
        print("%-90s %7d %10.3f %9.1f %6.2f" % (k, n, t / 1e6 / steps, t / n / 1e3, 100 * t / total))
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "calls", "total_ns", "avg_ns", "min_ns", "max_ns", "percent", "ms_per_step"])
            for k, (n, t, mx, mn) in items:
                w.writerow([k, n, int(t), round(t / n, 1), int(mn), int(mx), round(100 * t / total, 3),
                            round(t / 1e6 / steps, 4)])


if __name__ == "__main__":
    main()
