"""Per-stream time split of a rocprofv3 kernel trace over the timed steps (window as
tools/prof_summary.py): kernel time and busy union per HIP stream, and the main stream's idle
gaps (where it waits for side streams or the host)."""
import collections
import csv
import sys


def main(path, steps=10):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Stream_Id"]), r["Kernel_Name"]))
    rows.sort()
    adam = [i for i, r in enumerate(rows) if "adam_kernel" in r[3]]
    first = adam[-(2 * steps + 1)] + 1
    rows = rows[first:adam[-1] + 1]
    span = rows[-1][1] - rows[0][0]
    by = collections.defaultdict(list)
    for r in rows:
        by[r[2]].append(r)
    print("window %.2f ms/step" % (span / 1e6 / steps))
    for sid, rs in sorted(by.items(), key=lambda kv: -sum(r[1] - r[0] for r in kv[1])):
        kt = sum(r[1] - r[0] for r in rs)
        busy, c0, c1 = 0, None, None
        gaps = 0
        for t0, t1, _, _ in rs:
            if c1 is None or t0 > c1:
                if c1 is not None:
                    busy += c1 - c0
                    gaps += t0 - c1
                c0, c1 = t0, t1
            else:
                c1 = max(c1, t1)
        busy += c1 - c0
        print("stream %3d: %5d launches/step  kernel %.2f ms/step  busy %.2f ms/step  idle-between %.2f ms/step" % (
            sid, len(rs) // steps, kt / 1e6 / steps, busy / 1e6 / steps, gaps / 1e6 / steps))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 10)
