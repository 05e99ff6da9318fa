"""What the forward / input-gradient k-split tuner (tpgan_ops._tuned_data_split) measured and
picked over one configs[1] train step: one line per tuned shape, the candidate times from
graph replays, and the in-step per-layer times with and without the picks.

    python tools/data_tune_report.py [--batch 32]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tp-gan_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    import D_and_G_model as DG
    import tpgan_ops
    import tpgan_train
    from config import G as GCFG
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    G = DG.Generator(GCFG["zdim"], GCFG["num_classes"], use_batchnorm=False).to(dev)
    D = DG.Discriminator().to(dev)
    tr = tpgan_train.TPGANTrainer(G, D, lr=1e-4, compute_dtype=torch.bfloat16)
    b = tpgan_train.synthetic_batch(a.batch, dev, seed=1000)
    log = tpgan_ops.DATA_TUNE["log"] = []
    tr.step(b, next_b=b)
    torch.cuda.synchronize()
    names = {0: "fwd", 1: "dgrad"}
    print("op     n  cin  h    w  cout oh   ow   pick  t(0) ms   t(pick) ms  candidates")
    for op, shp, times, best in sorted(log, key=lambda e: -(e[2].get((0, 0), 0.0))):
        t0 = times.get((0, 0), float("nan"))
        tb = times.get(best, float("nan"))
        cand = " ".join("%s/%s:%.4f" % (k[1], k[0], v) for k, v in sorted(times.items()))
        print("%-5s %s  %s  %.4f  %.4f  %s" % (names.get(op, op), " ".join("%4d" % v for v in shp[:7]), best, t0,
                                                 tb, cand))
    for en in (True, False):
        tpgan_ops.DATA_TUNE["enabled"] = en
        for _ in range(3):
            tr.step(b, next_b=b)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            tr.step(b, next_b=b)
        e1.record()
        e1.synchronize()
        print("data tuning %s: %.3f ms/step" % ("on" if en else "off", e0.elapsed_time(e1) / 10))


if __name__ == "__main__":
    main()
