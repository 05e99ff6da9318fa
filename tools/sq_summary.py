"""MFMA utilisation of the dominant kernels from rocprofv3 SQ counter passes.

    python tools/sq_summary.py --pass fwd DIR_A DIR_B --pass dgrad ... [--out json]

DIR_A holds SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS, DIR_B SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT
SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE (tools/gpu_r2pmc.sh; tools/bench_layers.py enhance_128, one
pass per run).  Medians per dispatch of the tpg kernel of the pass.  Derived:
  mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)
    (SQ_VALU_MFMA_BUSY_CYCLES sums the 1024 SIMDs; GRBM_GUI_ACTIVE sums the 8 XCDs; checked:
    busy cycles = 16 x SQ_INSTS_MFMA, the v_mfma_f32_16x16x32_bf16 issue cost, and
    GRBM_GUI_ACTIVE / 8 / 2.4 GHz = the kernel's trace duration)
  mfma_padding = SQ_INSTS_MFMA / (algorithmic flops / 16384 flop per 16x16x32 MFMA)
  wait_inst_frac = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES, lds_conflict_frac = conflicts / LDS active
"""
import argparse
import csv
import glob
import json
import os
import statistics

FLOPS = {  # enhance_128: 32 x 128 x 128 x 206 x 206 x 25 x 2 per pass
    "enhance_128": 2 * 32 * 128 * 128 * 206 * 206 * 25,
}


def counters(d):
    agg = {}
    name = None
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"]
                if "tpg::" not in k or "pack" in k:
                    continue
                name = k
                agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return name, {c: statistics.median(v) for c, v in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pass", dest="passes", nargs=3, action="append", metavar=("NAME", "DIR_A", "DIR_B"),
                    required=True)
    ap.add_argument("--layer", default="enhance_128")
    ap.add_argument("--out")
    a = ap.parse_args()
    res = {"layer": a.layer, "algorithmic_flops_per_launch": FLOPS[a.layer],
           "method": __doc__.split("Derived:")[1].strip(), "passes": {}}
    for name, da, db in a.passes:
        ka, ca = counters(da)
        kb, cb = counters(db)
        c = dict(ca)
        c.update(cb)
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        e = {"kernel": ka, "counters_median_per_dispatch": c,
             "kernel_cycles_per_xcd": cyc, "kernel_ms_at_2p4ghz": cyc / 2.4e6,
             "mfma_busy_frac": c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc),
             "mfma_busy_per_inst": c["SQ_VALU_MFMA_BUSY_CYCLES"] / c["SQ_INSTS_MFMA"],
             "mfma_padding": c["SQ_INSTS_MFMA"] / (FLOPS[a.layer] / 16384),
             "wait_inst_frac": c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"],
             "valu_per_mfma": c["SQ_INSTS_VALU"] / c["SQ_INSTS_MFMA"],
             "lds_conflict_frac": c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_LDS_IDX_ACTIVE"], 1)}
        res["passes"][name] = e
        print("%-6s mfma busy %.3f  (x%.2f padding, %.1f cyc/inst)  wait %.2f  valu/mfma %.2f  lds conflicts %.3f  %.3f ms  %s"
              % (name, e["mfma_busy_frac"], e["mfma_padding"], e["mfma_busy_per_inst"], e["wait_inst_frac"],
                 e["valu_per_mfma"], e["lds_conflict_frac"], e["kernel_ms_at_2p4ghz"], (ka or "")[:60]))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
