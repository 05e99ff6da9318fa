"""Interleaved A/B of tpgan_ops / tpgan_train module switches on the real train step (one
process, one trainer, variants alternated round by round: cdna_hip_programming.md §5.4 rule 24).

    python tools/ab_step.py [--steps 10] [--rounds 5] VARIANT [VARIANT ...]

VARIANT = name[:module.ATTR[.key]=value,...], e.g.
    base   nolink:tpgan_ops.ACT_LINK.enabled=0   nogroup:tpgan_ops.GROUP.enabled=0
Values are parsed as int / float / bool literals.  Prints per-variant median and min ms/step.
"""
import argparse
import importlib
import os
import statistics
import sys
import time

TRAINER = [None]  # "trainer.ATTR=value" sets an attribute of the trainer (e.g. trainer.real_ahead=1)
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tp-gan_amd")]

import torch  # noqa: E402


def parse_variant(spec):
    """-> (name, settings, stream priority or None)."""
    name, _, rest = spec.partition(":")
    sets = []
    prio = None
    for kv in filter(None, rest.split(",")):
        path, _, val = kv.partition("=")
        if path == "stream.priority":  # the step itself runs on a stream of this priority
            prio = int(val)
            continue
        parts = path.split(".")
        if parts[0] == "env":  # env.NAME=value: an environment variable the library reads per launch
            sets.append(("env", [parts[1]], val))
            continue
        mod = TRAINER if parts[0] == "trainer" else importlib.import_module(parts[0])
        lv = val.lower()
        if lv in ("true", "false", "none"):
            v = {"true": True, "false": False, "none": None}[lv]
        else:
            v = float(val) if "." in val else int(val)
        sets.append((mod, parts[1:], v))
    return name, sets, prio


def apply(sets):
    old = []
    for mod, attrs, v in sets:
        if mod == "env":
            old.append(("env", attrs[0], os.environ.get(attrs[0]), None))
            os.environ[attrs[0]] = v
            continue
        obj = TRAINER[0] if mod is TRAINER else mod
        for a in attrs[:-1]:
            obj = getattr(obj, a) if not isinstance(obj, dict) else obj[a]
        last = attrs[-1]
        if isinstance(obj, dict):
            old.append((obj, last, obj[last], True))
            obj[last] = type(obj[last])(v) if isinstance(obj[last], (bool, int, float)) else v
        else:
            old.append((obj, last, getattr(obj, last), False))
            setattr(obj, last, v)
    return old


def restore(old):
    for obj, last, v, is_dict in reversed(old):
        if obj == "env":
            if v is None:
                os.environ.pop(last, None)
            else:
                os.environ[last] = v
        elif is_dict:
            obj[last] = v
        else:
            setattr(obj, last, v)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--identity", default="none", choices=["none", "resnet50", "mobilenetv2"])
    ap.add_argument("--gp", action="store_true")
    a = ap.parse_args()
    import D_and_G_model as DG
    import tpgan_train
    from config import G as GCFG
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    G = DG.Generator(GCFG["zdim"], GCFG["num_classes"], use_batchnorm=False).to(dev)
    D = DG.Discriminator().to(dev)
    idf = None
    if a.identity != "none":
        import FeatureExtract as FE
        idf = FE.IdentityPreservingLoss(FE.FeatureExtractModel(a.identity, 347).to(dev), torch.bfloat16)
    tr = tpgan_train.TPGANTrainer(G, D, lr=1e-4, compute_dtype=torch.bfloat16, identity_fn=idf, gradient_penalty=a.gp)
    TRAINER[0] = tr
    b = tpgan_train.synthetic_batch(a.batch, dev, seed=1000)
    variants = [parse_variant(v) for v in a.variants]  # (after TRAINER is set)
    streams = {}

    def run_steps(prio, n):
        if prio is None:
            for _ in range(n):
                tr.step(b, next_b=b)
            return
        st = streams.get(prio)
        if st is None:
            st = streams[prio] = torch.cuda.Stream(priority=prio)
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            for _ in range(n):
                tr.step(b, next_b=b)
        torch.cuda.current_stream().wait_stream(st)

    for name, sets, prio in variants:  # warm-up under every variant (autotuning, first-use packing)
        old = apply(sets)
        run_steps(prio, a.warmup)
        restore(old)
    torch.cuda.synchronize()
    res = {name: [] for name, _, _ in variants}
    for r in range(a.rounds):
        for name, sets, prio in variants:
            old = apply(sets)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run_steps(prio, a.steps)
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) / a.steps * 1e3)
            restore(old)
        print("round %d: %s" % (r, "  ".join("%s %.3f" % (n, res[n][-1]) for n, _, _ in variants)), flush=True)
    for name, _, _ in variants:
        v = res[name]
        print("%-12s median %.3f ms/step  min %.3f  (%s)" % (name, statistics.median(v), min(v),
                                                          " ".join("%.2f" % x for x in v)))


if __name__ == "__main__":
    main()
