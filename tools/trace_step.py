"""Per-conv timing of one real TP-GAN G+D train step (bs32, bf16) on the GPU.

    python tools/trace_step.py [--batch 32] [--top 60]

Every conv launch (fwd / dgrad / wgrad) of one step is bracketed by HIP events on the
launch stream (tpgan_ops.PROBE); launches are grouped by (pass, shape) and sorted by time.
The un-probed step time is printed for comparison, so the remainder is glue (activation
backward, packs, adds, fills, copies, Adam).
"""
import argparse
import collections
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tp-gan_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--top", type=int, default=70)
    ap.add_argument("--no-multistream", action="store_true",
                    help="serialise the local pathways (per-op event times are only exact without overlap)")
    a = ap.parse_args()
    import D_and_G_model as DG
    import tpgan_ops
    import tpgan_train
    if a.no_multistream:
        tpgan_ops.MULTISTREAM = False
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    G = DG.Generator(64, 347, use_batchnorm=False).to(dev)
    D = DG.Discriminator().to(dev)
    tr = tpgan_train.TPGANTrainer(G, D, compute_dtype=torch.bfloat16)
    b = tpgan_train.synthetic_batch(a.batch, dev)
    for _ in range(3):
        tr.step(b)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        tr.step(b)
    torch.cuda.synchronize()
    step_ms = (time.perf_counter() - t0) / 5 * 1e3

    tpgan_ops.PROBE["match"] = lambda d, w: True
    tpgan_ops.PROBE["events"] = []
    tr.step(b)
    torch.cuda.synchronize()
    tpgan_ops.PROBE["match"] = None
    agg = collections.defaultdict(lambda: [0, 0.0, 0])
    per_pass = collections.defaultdict(float)
    for e0, e1, fl, which, key in tpgan_ops.PROBE["events"]:
        ms = e0.elapsed_time(e1)
        g = agg[(which, key)]
        g[0] += 1
        g[1] += ms
        g[2] += fl
        per_pass[which] += ms
    conv_ms = sum(v for k, v in per_pass.items() if k != "actb")
    print("step %.2f ms (unprobed); conv launches %.2f ms (%s); glue ~%.2f ms" % (
        step_ms, conv_ms, ", ".join("%s %.2f" % kv for kv in sorted(per_pass.items())), step_ms - conv_ms))
    print("%-6s %-44s %5s %9s %8s %6s" % ("pass", "shape", "calls", "ms", "TF/s", "%pk"))
    for (which, key), (n, ms, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        tf = fl / (ms * 1e-3) / 1e12
        if which == "actb":  # bf16 activation backward: HBM-bound, report GB/s
            print("%-6s %-44s %5d %9.3f %8.0f GB/s %5.1f%% of 8 TB/s" % (which, key, n, ms, tf * 1e3, tf * 1e3 / 80))
        else:
            print("%-6s %-44s %5d %9.3f %8.1f %6.1f" % (which, key, n, ms, tf, 100 * tf / 2500))
    # totals by pass and output map size
    tot = collections.defaultdict(float)
    for (which, key), (n, ms, fl) in agg.items():
        hw = key.split("->")[1].split("x", 1)[1]
        tot[(which, hw)] += ms
    print("by pass and output map:")
    for (which, hw), ms in sorted(tot.items(), key=lambda kv: -kv[1]):
        print("  %-6s %-10s %8.3f ms" % (which, hw, ms))


if __name__ == "__main__":
    main()
