"""Summarise a rocprofv3 --kernel-trace run (CSV kernel trace) per kernel over the timed steps.

    python tools/prof_summary.py gpurun_out/x/prof/run_kernel_trace.csv --steps 10 [--csv out.csv]

The train step ends with one Adam launch per network (D then G), so the window of the last
`--steps` steps starts right after the G Adam launch of the step before it; warm-up and
weight-gradient autotuning trials fall outside the window.  Durations are nanoseconds.
"""
import argparse
import collections
import csv
import re

BY_GRID = False


def short(name):
    name = re.sub(r"\(tpg::\w+\)$", "", name)
    name = name.replace("void tpg::", "").replace("tpg::", "")
    return name[:90]


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if BY_GRID:
                name = short(name)[:60] + " g%sx%sx%s" % (r.get("Grid_Size_X", "?"), r.get("Grid_Size_Y", "?"),
                                                        r.get("Grid_Size_Z", "?"))
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    return rows


def window(rows, steps):
    adam = [i for i, r in enumerate(rows) if "adam_kernel" in r[2]]
    if steps <= 0 or len(adam) < 2 * steps + 1:
        return rows, max(1, len(adam) // 2)
    first = adam[-(2 * steps + 1)] + 1
    return rows[first:adam[-1] + 1], steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--csv")
    ap.add_argument("--steps", type=int, default=0)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--by-grid", action="store_true", help="group by (kernel, grid size): one line per layer shape")
    a = ap.parse_args()
    global BY_GRID
    BY_GRID = a.by_grid
    rows, steps = window(load(a.trace), a.steps)
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 1e30])
    for t0, t1, name in rows:
        dur = t1 - t0
        e = agg[short(name)]
        e[0] += 1
        e[1] += dur
        e[2] = max(e[2], dur)
        e[3] = min(e[3], dur)
    total = sum(v[1] for v in agg.values())
    span = (rows[-1][1] - rows[0][0]) if rows else 0
    # union of kernel intervals (streams overlap) and the idle gaps between them
    busy, cur0, cur1, gaps = 0, None, None, collections.Counter()
    for t0, t1, name in rows:
        if cur1 is None or t0 > cur1:
            if cur1 is not None:
                busy += cur1 - cur0
                g = t0 - cur1
                gaps["<5us" if g < 5000 else "5-20us" if g < 20000 else "20-100us" if g < 100000 else ">100us"] += g
            cur0, cur1 = t0, t1
        else:
            cur1 = max(cur1, t1)
    if cur1 is not None:
        busy += cur1 - cur0
    print("GPU busy (union) %.2f ms/step, idle %.2f ms/step; idle by gap size: %s" % (
        busy / 1e6 / steps, (span - busy) / 1e6 / steps,
        ", ".join("%s %.2f ms" % (k, v / 1e6 / steps) for k, v in sorted(gaps.items()))))
    items = sorted(agg.items(), key=lambda kv: -kv[1][1])
    print("steps in window: %d   kernel time %.2f ms/step   wall span %.2f ms/step   (busy %.1f%%)   launches %.0f/step" % (
        steps, total / 1e6 / steps, span / 1e6 / steps, 100 * total / max(span, 1), len(rows) / steps))
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
