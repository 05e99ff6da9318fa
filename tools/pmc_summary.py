"""Per-dispatch HBM traffic of one kernel from rocprofv3 --pmc runs (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_summary.py --fetch DIR1 --write DIR2 --kernel halo_kernel [--grid X] [--slice A:B]
                                [--set key=value ...] [--out json]

--slice keeps the dispatches A..B-1 (in dispatch order) of those that match: tools/bench_layers.py
runs its passes back to back, so the forward and input-gradient dispatches of one halo kernel
(same grid) are the first and second block of 9.

FETCH_SIZE / WRITE_SIZE are kilobytes per dispatch.  gfx950 correction (MI355X_MICROARCH.md,
HBM section): FETCH_SIZE reports half of the bytes of wide (16 B/lane) coalesced reads,
so it is doubled; WRITE_SIZE is exact for 16-byte stores.
"""
import argparse
import csv
import glob
import json
import os
import statistics


def values(d, counter, kernel, grid, sl=None):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = []
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                if r.get("Counter_Name") != counter or kernel not in r.get("Kernel_Name", ""):
                    continue
                if grid and int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0) != grid:
                    continue
                vals.append((int(r.get("Dispatch_Id", 0) or 0), float(r["Counter_Value"])))
    vals = [v for _, v in sorted(vals)]
    if sl:
        a, b = (int(t) for t in sl.split(":"))
        vals = vals[a:b]
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--grid", type=int, default=0)
    ap.add_argument("--algorithmic-bytes", type=float, default=0.0)
    ap.add_argument("--slice")
    ap.add_argument("--set", action="append", default=[], help="extra key=value fields of the summary")
    ap.add_argument("--out")
    a = ap.parse_args()
    fv = values(a.fetch, "FETCH_SIZE", a.kernel, a.grid, a.slice)
    wv = values(a.write, "WRITE_SIZE", a.kernel, a.grid, a.slice)
    if not fv or not wv:
        raise SystemExit("no dispatches of %r found (fetch %d, write %d)" % (a.kernel, len(fv), len(wv)))
    fetch_b = statistics.median(fv) * 1024 * 2  # KB -> B, x2 gfx950 wide-read correction
    write_b = statistics.median(wv) * 1024
    res = {"kernel": a.kernel, "dispatches": [len(fv), len(wv)], "fetch_bytes": fetch_b, "write_bytes": write_b,
           "traffic_bytes": fetch_b + write_b, "raw_fetch_kb_median": statistics.median(fv),
           "raw_write_kb_median": statistics.median(wv),
           "correction": "FETCH_SIZE x2 (gfx950 wide coalesced reads), WRITE_SIZE x1; KB = 1024 B"}
    if a.algorithmic_bytes:
        res["algorithmic_bytes"] = a.algorithmic_bytes
        res["traffic_over_algorithmic"] = (fetch_b + write_b) / a.algorithmic_bytes
    for kv in a.set:
        k, v = kv.split("=", 1)
        res[k] = v
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
