"""Per-kernel VGPR / scratch / occupancy of one HIP source (hipcc kernel-resource-usage remarks).

    python tools/resource_usage.py tp-gan_amd/csrc/tpg_wgrad_rh.hip [--filter wgrad_rh] [--spills]
"""
import argparse
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def usage(src):
    cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", os.devnull,
           "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True, cwd=os.path.join(REPO, "tp-gan_amd"))
    if out.returncode:
        sys.exit(out.stderr[-4000:])
    rows, cur = [], None
    for line in out.stderr.splitlines():
        m = re.search(r"remark: (.*?)(?: \[-Rpass-analysis.*)?$", line)
        if not m:
            continue
        kv = m.group(1).strip()
        if kv.startswith("Function Name:"):
            cur = {"name": kv.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in kv:
            k, v = kv.split(":", 1)
            cur[k.strip()] = v.strip()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--filter", default="")
    ap.add_argument("--spills", action="store_true", help="only kernels with scratch")
    a = ap.parse_args()
    for r in usage(os.path.abspath(a.src)):
        if a.filter not in r["name"]:
            continue
        scratch = int(r.get("ScratchSize [bytes/lane]", "0"))
        if a.spills and not scratch:
            continue
        print("%-70s vgpr %4s agpr %3s scratch %4d occ %s" % (r["name"][:70], r.get("VGPRs"), r.get("AGPRs"), scratch,
                                                           r.get("Occupancy [waves/SIMD]")))


if __name__ == "__main__":
    main()
