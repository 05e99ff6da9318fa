"""Per-kernel counter table from several rocprofv3 --pmc passes (one run per pass).

    python tools/kernel_counters.py DIR [DIR ...] [--match wgrad] [--out json]

Dispatches are grouped by (kernel name, grid size); each counter is the median over the group's
dispatches.  Derived columns (where the counters are present):
  us        kernel duration (median of the counter rows' timestamps; counter collection
            serialises dispatches, so this is the kernel alone)
  mfma      SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs): MFMA-pipe busy
  valu/mf   SQ_INSTS_VALU / SQ_INSTS_MFMA
  lds/mf    SQ_INSTS_LDS / SQ_INSTS_MFMA
  wait      SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
  waves     SQ_WAVES
  wr_MB     WRITE_SIZE (KB -> MB; exact for 16-B stores and f32 atomics, MI355X_MICROARCH.md)
  rd_MB     FETCH_SIZE x2 (gfx950 wide-read correction)
"""
import argparse
import collections
import csv
import glob
import json
import os
import statistics


def load(d):
    groups = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    seen = set()
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                grid = int(r.get("Grid_Size", 0) or r.get("Grid_Size_X", 0) or 0)
                groups[(r["Kernel_Name"], grid)][r["Counter_Name"]].append(float(r["Counter_Value"]))
                if r.get("Start_Timestamp") and r["Dispatch_Id"] not in seen:
                    seen.add(r["Dispatch_Id"])
                    durs[(r["Kernel_Name"], grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return groups, durs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default="tpg::")
    ap.add_argument("--out")
    a = ap.parse_args()
    table = collections.defaultdict(dict)
    dur = collections.defaultdict(list)
    for d in a.dirs:
        g, du = load(d)
        for k, cs in g.items():
            if a.match not in k[0]:
                continue
            for c, v in cs.items():
                table[k][c] = statistics.median(v)
        for k, v in du.items():
            if a.match in k[0]:
                dur[k] += v
    rows = []
    for (name, grid), c in sorted(table.items(), key=lambda kv: -statistics.median(dur.get(kv[0], [0]) or [0])):
        e = {"kernel": name.split("(")[0].replace("void ", ""), "grid": grid, "counters": c}
        ds = dur.get((name, grid), [])
        e["us"] = statistics.median(ds) if ds else None
        cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8
        if cyc and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            e["mfma_busy"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc)
        if c.get("SQ_INSTS_MFMA"):
            if "SQ_INSTS_VALU" in c:
                e["valu_per_mfma"] = c["SQ_INSTS_VALU"] / c["SQ_INSTS_MFMA"]
            if "SQ_INSTS_LDS" in c:
                e["lds_per_mfma"] = c["SQ_INSTS_LDS"] / c["SQ_INSTS_MFMA"]
        if c.get("SQ_WAVE_CYCLES") and "SQ_WAIT_INST_ANY" in c:
            e["wait_frac"] = c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"]
        if "WRITE_SIZE" in c:
            e["write_MB"] = c["WRITE_SIZE"] / 1024
        if "FETCH_SIZE" in c:
            e["fetch_MB_x2"] = c["FETCH_SIZE"] * 2 / 1024
        rows.append(e)
    print("%-58s %8s %8s %6s %7s %6s %6s %7s %9s %9s" % ("kernel", "grid", "us", "mfma", "valu/mf", "lds/mf", "wait",
                                                        "waves", "write_MB", "fetchMBx2"))

    def f(v, fmt):
        return fmt % v if v is not None else "-"
    for e in rows:
        c = e["counters"]
        print("%-58s %8d %8s %6s %7s %6s %6s %7s %9s %9s" % (
            e["kernel"][:58], e["grid"], f(e["us"], "%.1f"), f(e.get("mfma_busy"), "%.3f"),
            f(e.get("valu_per_mfma"), "%.2f"), f(e.get("lds_per_mfma"), "%.2f"), f(e.get("wait_frac"), "%.2f"),
            f(c.get("SQ_WAVES"), "%.0f"), f(e.get("write_MB"), "%.1f"), f(e.get("fetch_MB_x2"), "%.1f")))
    if a.out:
        with open(a.out, "w") as fo:
            json.dump({"method": __doc__, "kernels": rows}, fo, indent=1)


if __name__ == "__main__":
    main()
