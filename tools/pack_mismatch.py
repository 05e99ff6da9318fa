"""Where do pre-packed and call-packed weight images give different forward outputs?

Replays tests/test_gpu_train.py::test_prepacked_weights_match_inline_packing's setup (two bf16
train steps on the deterministic-init G / D at B=2), then runs G's forward with
tpgan_ops.PACK on and off and compares every leaf module's output (forward hooks), printing the
modules whose outputs differ, in execution order, with the op plans involved.

    python tools/pack_mismatch.py [--det]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tp-gan_amd"), os.path.join(REPO, "tests")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--det", action="store_true", help="deterministic mode for the comparison runs")
    ap.add_argument("--requires-grad", action="store_true", help="the test's x.requires_grad_(True)")
    a = ap.parse_args()
    import D_and_G_model as DG
    import tpgan_ops
    import tpgan_train
    from _cases import load_det
    gpu = torch.device("cuda", 0)
    G = DG.Generator(64, 347, use_batchnorm=False)
    D = DG.Discriminator()
    load_det(G, "G/", torch.float32)
    load_det(D, "D/", torch.float32)
    G, D = G.to(gpu), D.to(gpu)
    tr = tpgan_train.TPGANTrainer(G, D, compute_dtype=torch.bfloat16, use_dropout=False)
    b = tpgan_train.synthetic_batch(2, gpu, seed=21)
    tr.step(b)
    tr.step(b)
    torch.cuda.synchronize()
    outs = {}
    names = {m: n for n, m in G.named_modules()}
    order = []

    def hook(m, inp, out):
        t = out[0] if isinstance(out, (tuple, list)) else out
        if torch.is_tensor(t):
            outs.setdefault(names[m], []).append(t.detach().float().clone())
            if names[m] not in order:
                order.append(names[m])

    hs = [m.register_forward_hook(hook) for m in G.modules()]

    def run():
        x = b["I128"].clone()
        if a.requires_grad:
            x.requires_grad_(True)
        with tpgan_ops.compute_dtype(torch.bfloat16):
            o = G(x, b["left_eye"], b["right_eye"], b["nose"], b["mouth"], b["z"], False)
        torch.cuda.synchronize()
        return o[0].detach().float().clone()

    import contextlib
    with tpgan_ops.deterministic() if a.det else contextlib.nullcontext():
        y0 = run()
        y1 = run()
        tpgan_ops.PACK["enabled"] = False
        try:
            y2 = run()
        finally:
            tpgan_ops.PACK["enabled"] = True
    for h in hs:
        h.remove()

    def rel(p, q):
        return float((p - q).norm() / max(float(q.norm()), 1e-30))

    print("G output: run-to-run %.3e  packed vs call-packed %.3e" % (rel(y1, y0), rel(y2, y0)), flush=True)
    shown = 0
    for n in order:
        v = outs[n]
        if len(v) < 3:
            continue
        r01, r02 = rel(v[1], v[0]), rel(v[2], v[0])
        if r02 > max(3 * r01, 1e-6):
            print("  %-70s shape %-22s run-to-run %.3e  call-packed %.3e" % (n, tuple(v[0].shape), r01, r02), flush=True)
            shown += 1
            if shown >= 25:
                break
    print("modules compared: %d, differing shown: %d" % (len(order), shown))


if __name__ == "__main__":
    main()
