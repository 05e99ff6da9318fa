"""Census of the C-ABI calls one configs[1] train step makes: every tpg_* entry point of the
loaded library is wrapped, and each call is counted by (function, the tpgan_ops / model line
that made it, shape arguments).  Finds where the glue launches (copies, activation-backward
passes, fills) come from.

    python tools/call_census.py [--batch 32] [--fn tpg_copy4d,tpg_act_bwd]
"""
import argparse
import collections
import os
import sys
import traceback

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tp-gan_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--fn", default="", help="comma-separated entry points to list by call site (default: all)")
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
    for _ in range(3):
        tr.step(b, next_b=b)
    torch.cuda.synchronize()
    lib = tpgan_ops.load()
    counts = collections.Counter()
    sites = collections.Counter()
    want = set(filter(None, a.fn.split(",")))
    names = [n for n in dir(lib) if n.startswith("tpg_")] if not want else sorted(want)
    names = [n for n in names if callable(getattr(lib, n, None))]
    orig = {}

    def wrap(name, fn):
        def w(*args):
            counts[name] += 1
            if not want or name in want:
                st = traceback.extract_stack(limit=8)[:-1]
                fr = [f for f in st if "tp-gan_amd" in f.filename or "tpgan" in f.filename]
                site = " < ".join("%s:%d" % (os.path.basename(f.filename), f.lineno) for f in reversed(fr[-3:]))
                shp = tuple(x for x in args[:4] if isinstance(x, int))
                sites[(name, site, shp)] += 1
            return fn(*args)
        return w
    for n in names:
        try:
            orig[n] = getattr(lib, n)
            setattr(lib, n, wrap(n, orig[n]))
        except (AttributeError, TypeError):
            pass
    tr.step(b, next_b=b)
    torch.cuda.synchronize()
    for n, f in orig.items():
        setattr(lib, n, f)
    print("entry point calls in one step:")
    for n, c in counts.most_common():
        print("  %-28s %4d" % (n, c))
    print("\nby call site:")
    for (n, site, shp), c in sorted(sites.items(), key=lambda kv: (kv[0][0], -kv[1])):
        print("  %-22s %3d  %-18s %s" % (n, c, shp, site))


if __name__ == "__main__":
    main()
