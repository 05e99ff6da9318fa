"""Per-kernel ms/step difference between two rocprofv3 kernel traces (same window rules as
prof_summary.py).   python tools/prof_diff.py A.csv B.csv --steps 5 [--by-grid]"""
import argparse
import collections
import re
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import prof_summary as PS  # noqa: E402


def agg(path, steps, strip):
    rows, st = PS.window(PS.load(path), steps)
    out = collections.defaultdict(float)
    cnt = collections.defaultdict(int)
    for t0, t1, name in rows:
        k = PS.short(name)
        if strip:
            k = re.sub(r", (true|false)>", ">", k)
        out[k] += (t1 - t0) / 1e6 / st
        cnt[k] += 1.0 / st
    return out, cnt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--by-grid", action="store_true")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    PS.BY_GRID = a.by_grid
    A, ca = agg(a.a, a.steps, True)
    B, cb = agg(a.b, a.steps, True)
    keys = sorted(set(A) | set(B), key=lambda k: -abs(B.get(k, 0) - A.get(k, 0)))
    print("total A %.2f ms  B %.2f ms  diff %+.2f" % (sum(A.values()), sum(B.values()), sum(B.values()) - sum(A.values())))
    for k in keys[:a.top]:
        print("%-80s %7.3f %7.3f %+7.3f  calls %5.0f %5.0f" % (k[:80], A.get(k, 0), B.get(k, 0), B.get(k, 0) - A.get(k, 0),
                                                          ca.get(k, 0), cb.get(k, 0)))


if __name__ == "__main__":
    main()
