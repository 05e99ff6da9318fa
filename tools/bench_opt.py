"""The optimizer tail of the configs[1] networks: one flat Adam launch and one re-pack of every
weight image (FlatParams.adam's two launches), timed with HIP events.  --vars runs the same
timing once per value of TPG_OPT_VAR (for a temporary kernel-variant switch in the library
while an A/B is open; the product has none) and compares results bit for bit with the first.

    python tools/bench_opt.py [--reps 20] [--vars 0]
"""
import argparse
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tp-gan_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--vars", default="0")
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
    for _ in range(2):
        tr.step(b, next_b=b)
    torch.cuda.synchronize()
    variants = [int(v) for v in a.vars.split(",")]
    for name, f in (("G", tr.fG), ("D", tr.fD)):
        n = f.data.numel()
        saved = [t.clone() for t in (f.data, f.exp_avg, f.exp_avg_sq, f.adam_state)]
        images = [e for e in f.pack_entries.values() if e is not None and e.njobs]
        pbytes = sum(e.buf.numel() for e in images)
        ref = None
        for var in variants:
            os.environ["TPG_OPT_VAR"] = str(var)
            ta, tp = [], []
            for r in range(a.reps + 2):
                for t, s in zip((f.data, f.exp_avg, f.exp_avg_sq, f.adam_state), saved):
                    t.copy_(s)
                e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                e0.record()
                tpgan_ops.adam_step(f.data, f.grad, f.exp_avg, f.exp_avg_sq, 1e-4, 0.5, 0.999, 1e-8, 0.0,
                                    f.adam_state, 0, 1.0)
                e1.record()
                f.epoch += 1
                tpgan_ops.repack(f)
                e2.record()
                torch.cuda.synchronize()
                if r >= 2:
                    ta.append(e0.elapsed_time(e1))
                    tp.append(e1.elapsed_time(e2))
            out = (f.data.clone(), f.exp_avg.clone(), f.exp_avg_sq.clone(), [e.buf.clone() for e in images])
            if ref is None:
                ref = out
                same = "ref"
            else:
                same = "bit-exact" if (all(torch.equal(x, y) for x, y in zip(out[:3], ref[:3])) and
                                       all(torch.equal(x, y) for x, y in zip(out[3], ref[3]))) else "DIFFERS"
            ma, mp = statistics.median(ta), statistics.median(tp)
            print("%s var %2d  adam %.3f ms (%.2f TB/s, %d params x 28 B)  pack %.3f ms (%d images, %.0f MB written)  %s"
                  % (name, var, ma, n * 28 / ma / 1e9, n, mp, len(images), pbytes / 1e6, same), flush=True)
        for t, s in zip((f.data, f.exp_avg, f.exp_avg_sq, f.adam_state), saved):
            t.copy_(s)
    os.environ.pop("TPG_OPT_VAR", None)


if __name__ == "__main__":
    main()
