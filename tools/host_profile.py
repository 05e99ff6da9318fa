"""Where the host time of a train step goes: cProfile over a few steady-state steps
(bs32, bf16), sorted by own time.  The GPU runs ahead, so this is the enqueue cost.

    python tools/host_profile.py [--steps 4] [--top 40]
"""
import argparse
import cProfile
import os
import pstats
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tp-gan_amd")]
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--top", type=int, default=45)
    a = ap.parse_args()
    import D_and_G_model as DG
    import tpgan_train
    dev = torch.device("cuda", 0)
    G = DG.Generator(64, 347, use_batchnorm=False).to(dev)
    D = DG.Discriminator().to(dev)
    tr = tpgan_train.TPGANTrainer(G, D, compute_dtype=torch.bfloat16)
    b = tpgan_train.synthetic_batch(32, dev)
    for _ in range(4):
        tr.step(b)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.steps):
        tr.step(b)
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(a.top)
    st.sort_stats("cumulative").print_stats(25)


if __name__ == "__main__":
    main()
