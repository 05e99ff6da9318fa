"""Wall-time share of each kernel (by name + grid) in a rocprofv3 kernel trace of graph-replayed
steps: at every instant the wall clock is split evenly among the kernels running then, so the
shares sum to the GPU-busy wall time (streams overlap under graph replay; a kernel's plain
duration double-counts).  Also: wall time with exactly one kernel running (the serial stretches).

    python tools/wall_share.py gpurun_out/x/prof/run_kernel_trace.csv --steps 10 [--top 50]
"""
import argparse
import collections
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import prof_summary as PS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--top", type=int, default=50)
    ap.add_argument("--family", action="store_true", help="group by kernel template name only")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            nm = PS.short(r["Kernel_Name"])
            if not a.family:
                nm = nm[:60] + " g%sx%sx%s" % (r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
            else:
                nm = nm.split("<")[0].split("(")[0]
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), nm))
    rows.sort()
    rows, steps = PS.window(rows, a.steps)
    ev = []
    for i, (t0, t1, nm) in enumerate(rows):
        ev.append((t0, 1, i))
        ev.append((t1, -1, i))
    ev.sort(key=lambda e: (e[0], e[1]))
    share = collections.Counter()
    solo = collections.Counter()
    active = set()
    last = None
    conc_hist = collections.Counter()
    for t, d, i in ev:
        if last is not None and active and t > last:
            dt = t - last
            k = len(active)
            conc_hist[min(k, 6)] += dt
            for j in active:
                share[rows[j][2]] += dt / k
                if k == 1:
                    solo[rows[j][2]] += dt
        if d > 0:
            active.add(i)
        else:
            active.discard(i)
        last = t
    busy = sum(conc_hist.values())
    print("busy wall %.2f ms/step; by concurrency: %s" % (busy / 1e6 / steps, ", ".join(
        "%s%d %.2f" % ("" if k < 6 else ">=", k, v / 1e6 / steps) for k, v in sorted(conc_hist.items()))))
    calls = collections.Counter(r[2] for r in rows)
    print("%-80s %6s %9s %9s" % ("kernel (grid)", "calls", "wall ms", "solo ms"))
    for nm, v in share.most_common(a.top):
        print("%-80s %6d %9.3f %9.3f" % (nm, calls[nm] // steps, v / 1e6 / steps, solo[nm] / 1e6 / steps))


if __name__ == "__main__":
    main()
