"""CPU baseline: the oracle's G+D train step on host cores (TEST INFRASTRUCTURE).

Used only by bench.py's cpu_baseline leg.  Same step as tp-gan_amd/tpgan_train.py
(G forward, D-step on [real; fake.detach()], G-step through D with the config.py loss
weights), restated with the functional oracle (aten CPU, float32), without the optimizer
update (parameter-sized elementwise work, <1% of the step).
"""
import time

import torch
import torch.nn.functional as F

from . import tpgan_oracle as O

W = dict(weight_128=1.0, weight_pixelwise=1.0, weight_pixelwise_local=3.0, weight_symmetry=0.3, weight_adv_G=1e-3,
         weight_total_varation=1e-3, weight_cross_entropy=10.0)


def cpu_train_step(PG, PD, b):
    fake, pred, fused_fake, le, re, no, mo, _ = O.generator(PG, b["I128"], b["left_eye"], b["right_eye"], b["nose"],
                                                           b["mouth"], b["z"])
    B = fake.shape[0]
    d = O.discriminator(PD, torch.cat([b["frontal"], fake.detach()], 0))
    loss_D = d[B:].mean() - d[:B].mean()
    gD = torch.autograd.grad(loss_D, list(PD.values()))
    d_gen = O.discriminator(PD, fake)
    l_tv = (fake[:, :, 1:] - fake[:, :, :-1]).abs().mean() + (fake[:, :, :, 1:] - fake[:, :, :, :-1]).abs().mean()
    loss_G = (W["weight_pixelwise"] * (fake - b["frontal"]).abs().mean() +
              W["weight_pixelwise_local"] * ((le - b["frontal_left_eye"]).abs().mean() +
                                             (re - b["frontal_right_eye"]).abs().mean() +
                                             (no - b["frontal_nose"]).abs().mean() +
                                             (mo - b["frontal_mouth"]).abs().mean()) / 4 +
              W["weight_symmetry"] * (fake - fake.flip(3)).abs().mean() - W["weight_adv_G"] * d_gen.mean() +
              W["weight_total_varation"] * l_tv + W["weight_cross_entropy"] * F.cross_entropy(pred, b["label"]))
    gG = torch.autograd.grad(loss_G, list(PG.values()))
    return float(loss_D.detach()), float(loss_G.detach()), gD, gG


def time_cpu_step(B=2, iters=2, threads=None, seed=0):
    """faces/s of the oracle step on the host: one untimed warm-up, then `iters` steps."""
    if threads:
        torch.set_num_threads(threads)
    PG, PD = O.make_params(torch.float32, seed)
    for p in list(PG.values()) + list(PD.values()):
        p.requires_grad_(True)
    g = torch.Generator().manual_seed(seed)

    def u(*s):
        return torch.rand(*s, generator=g) * 2 - 1

    b = {"I128": u(B, 3, 128, 128), "left_eye": u(B, 3, 40, 40), "right_eye": u(B, 3, 40, 40),
         "nose": u(B, 3, 32, 40), "mouth": u(B, 3, 32, 48), "z": u(B, 64), "frontal": u(B, 3, 128, 128),
         "frontal_left_eye": u(B, 3, 40, 40), "frontal_right_eye": u(B, 3, 40, 40),
         "frontal_nose": u(B, 3, 32, 40), "frontal_mouth": u(B, 3, 32, 48),
         "label": torch.randint(0, 347, (B,), generator=g)}
    cpu_train_step(PG, PD, b)
    t0 = time.perf_counter()
    for _ in range(iters):
        cpu_train_step(PG, PD, b)
    dt = (time.perf_counter() - t0) / iters
    return B / dt, dt, torch.get_num_threads()
