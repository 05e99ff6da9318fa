"""Which aten ops one configs[1] train step still runs (every HIP kernel of the product is a
tpg_* C-ABI call; the rest is aten glue): torch.profiler over one step, CPU-side op events with
their Python call sites, counted by (op, shapes, the innermost tp-gan_amd frame).

    python tools/aten_census.py [--batch 32] [--top 60]
"""
import argparse
import collections
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tp-gan_amd")]

import torch  # noqa: E402

# ops that launch device work (views, metadata and allocator calls do not)
KERNEL_OPS = ("add", "sub", "mul", "div", "neg", "abs", "sign", "mean", "sum", "fill_", "zero_", "zeros", "copy_",
              "to", "_to_copy", "clone", "cat", "flip", "cross_entropy", "nll", "log_softmax", "_softmax", "ones",
              "where", "rsub", "pow", "sqrt", "norm", "linalg_vector_norm", "masked_fill", "dropout", "native_dropout",
              "fused_dropout", "index", "contiguous", "expand", "empty_like", "rand", "uniform_", "lerp", "addcmul")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--top", type=int, default=60)
    a = ap.parse_args()
    import D_and_G_model as DG
    import tpgan_train
    from config import G as GCFG
    from torch.profiler import ProfilerActivity, profile
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    G = DG.Generator(GCFG["zdim"], GCFG["num_classes"], use_batchnorm=False).to(dev)
    D = DG.Discriminator().to(dev)
    tr = tpgan_train.TPGANTrainer(G, D, lr=1e-4, compute_dtype=torch.bfloat16)
    b = tpgan_train.synthetic_batch(a.batch, dev, seed=1000)
    for _ in range(3):
        tr.step(b, next_b=b)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU], record_shapes=True, with_stack=True) as prof:
        tr.step(b, next_b=b)
        torch.cuda.synchronize()
    cnt = collections.Counter()
    for ev in prof.events():
        name = ev.name.replace("aten::", "")
        if not ev.name.startswith("aten::") or not any(name == k or name.startswith(k) for k in KERNEL_OPS):
            continue
        if ev.cpu_parent is not None and ev.cpu_parent.name.startswith("aten::"):
            continue  # (count the outermost aten op only)
        st = [f for f in (ev.stack or []) if "tp-gan_amd" in f or "tools/" in f]
        site = st[0].split("/")[-1] if st else "?"
        shp = str(ev.input_shapes[:2])[:60] if ev.input_shapes else ""
        cnt[(name, site, shp)] += 1
    print("outermost aten ops with device work in one step: %d" % sum(cnt.values()))
    for (name, site, shp), c in cnt.most_common(a.top):
        print("%4d  %-28s %-40s %s" % (c, name, site, shp))


if __name__ == "__main__":
    main()
