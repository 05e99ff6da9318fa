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
    ap.add_argument("--rounds", type=int, default=4, help="PACK on / on / off triples to compare")
    ap.add_argument("--backward", action="store_true", help="also run the test's backward after each forward")
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
    names = {m: n for n, m in G.named_modules()}
    calls = []  # (module name, output) of the current run, in call order

    def hook(m, inp, out):
        t = out[0] if isinstance(out, (tuple, list)) else out
        if torch.is_tensor(t):
            calls.append((names[m], t.detach().float().clone()))

    hs = [m.register_forward_hook(hook) for m in G.modules()]

    def run():
        calls.clear()
        x = b["I128"].clone()
        if a.requires_grad:
            x.requires_grad_(True)
        with tpgan_ops.compute_dtype(torch.bfloat16):
            o = G(x, b["left_eye"], b["right_eye"], b["nose"], b["mouth"], b["z"], False)
            if a.backward:
                d = D(o[0])
                (o[0].float().sum() + d.float().sum()).backward()
        torch.cuda.synchronize()
        return o[0].detach().float().clone(), list(calls)

    def rel(p, q):
        return float((p - q).norm() / max(float(q.norm()), 1e-30))

    import contextlib
    bad = 0
    for rnd in range(a.rounds):
        with tpgan_ops.deterministic() if a.det else contextlib.nullcontext():
            y0, c0 = run()
            y1, c1 = run()
            tpgan_ops.PACK["enabled"] = False
            try:
                y2, c2 = run()
            finally:
                tpgan_ops.PACK["enabled"] = True
        print("round %d  G output: run-to-run %.3e  packed vs call-packed %.3e" % (rnd, rel(y1, y0), rel(y2, y0)),
              flush=True)
        shown = 0
        for (n, t0), (_, t1), (_, t2) in zip(c0, c1, c2):
            r01, r02 = rel(t1, t0), rel(t2, t0)
            if r02 > max(3 * r01, 1e-6) or r01 > 1e-6:
                print("  %-60s shape %-22s run-to-run %.3e  call-packed %.3e" % (n, tuple(t0.shape), r01, r02),
                      flush=True)
                shown += 1
                if shown >= 12:
                    break
        bad += shown > 0
    for h in hs:
        h.remove()
    print("rounds with a difference: %d of %d" % (bad, a.rounds))


if __name__ == "__main__":
    main()
