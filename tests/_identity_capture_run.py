"""Child process of tests/test_gpu_identity_capture.py (not collected by pytest).

BASELINE configs[2] shape: bs32, ResNet-50 identity-preserving loss, bf16, deterministic mode.
Eager steps with the identity fork on its side stream (tpgan_train.IDENTITY_STREAM), then ONE
unsegmented hipGraph capture of the whole step with the fork inside it, then replays from the
same state; the replays must land on the eager steps' weights and losses bit for bit.  Run
with bench.py's graph-replay environment (packet capture off, 8 graph queues), which is read
when HIP initialises -- hence a process of its own.  Prints one JSON line.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tp-gan_amd"), os.path.join(REPO, "tests")]

import torch  # noqa: E402


def main():
    import FeatureExtract as FE
    import tpgan_ops
    import tpgan_train
    from _cases import load_det
    import D_and_G_model as DG
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    dev = torch.device("cuda", 0)
    res = {"batch": batch, "identity_stream": dict(tpgan_train.IDENTITY_STREAM)}
    with tpgan_ops.deterministic():
        G = DG.Generator(64, 347, use_batchnorm=False)
        D = DG.Discriminator()
        load_det(G, "G/", torch.float32)
        load_det(D, "D/", torch.float32)
        G, D = G.to(dev), D.to(dev)
        torch.manual_seed(0)
        ext = FE.FeatureExtractModel("resnet50", 347).to(dev)
        tr = tpgan_train.TPGANTrainer(G, D, lr=1e-3, betas=(0.5, 0.999), compute_dtype=torch.bfloat16,
                                      use_dropout=False, identity_fn=FE.IdentityPreservingLoss(ext, torch.bfloat16))
        b = tpgan_train.synthetic_batch(batch, dev, seed=23)
        tr.step(b)  # (eager, the fork on its side stream; tunes nothing in deterministic mode)
        torch.cuda.synchronize()
        snap = [t.clone() for f in (tr.fG, tr.fD) for t in (f.data, f.exp_avg, f.exp_avg_sq, f.adam_state)]

        def restore():
            ts = [t for f in (tr.fG, tr.fD) for t in (f.data, f.exp_avg, f.exp_avg_sq, f.adam_state)]
            for t, s in zip(ts, snap):
                t.copy_(s)
            for f in (tr.fG, tr.fD):
                f.weights_loaded()

        eager = [tr.step(b) for _ in range(2)]
        torch.cuda.synchronize()
        ref = (tr.fG.data.clone(), tr.fD.data.clone())
        restore()
        tr.capture(b, warmup=0, segmented=False)
        res["graphs"] = len(tr._graphs)
        res["fork_in_capture"] = bool(tr.identity_forks_captured)
        restore()
        outs = [tr.step_graphed() for _ in range(2)]
        torch.cuda.synchronize()
    res["G_equal"] = bool(torch.equal(tr.fG.data, ref[0]))
    res["D_equal"] = bool(torch.equal(tr.fD.data, ref[1]))
    res["losses"] = [[float(o[k]) for k in ("loss_D", "loss_G")] for o in outs]
    res["losses_eager"] = [[float(o[k]) for k in ("loss_D", "loss_G")] for o in eager]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
