"""CPU baseline: the oracle's train steps on host cores (TEST INFRASTRUCTURE).

Used only by bench.py's cpu_baseline leg.  The same step as tp-gan_amd/tpgan_train.py (G
forward, D-step on [real; fake.detach()] + Adam on D, G-step through the updated D with the
config.py loss weights + Adam on G), restated with the functional oracle (aten CPU, float32),
and BASELINE configs[0] (GlobalPathway with zero local inputs + D on
its output, loss = mean D(fake) + L1, forward + backward of both; D_and_G_model.py:161-329,
409-435).  Timing follows §8d: one warm-up, then the median of `iters` steps.
"""
import statistics
import time

import torch
import torch.nn.functional as F

from . import tpgan_oracle as O

W = dict(weight_128=1.0, weight_pixelwise=1.0, weight_pixelwise_local=3.0, weight_symmetry=0.3, weight_adv_G=1e-3,
         weight_total_varation=1e-3, weight_cross_entropy=10.0)


def cpu_train_step(PG, PD, b, optG=None, optD=None):
    fake, pred, fused_fake, le, re, no, mo, _ = O.generator(PG, b["I128"], b["left_eye"], b["right_eye"], b["nose"],
                                                           b["mouth"], b["z"])
    B = fake.shape[0]
    d = O.discriminator(PD, torch.cat([b["frontal"], fake.detach()], 0))
    loss_D = d[B:].mean() - d[:B].mean()
    gD = torch.autograd.grad(loss_D, list(PD.values()))
    if optD is not None:
        for p, gr in zip(PD.values(), gD):
            p.grad = gr
        optD.step()
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
    if optG is not None:
        for p, gr in zip(PG.values(), gG):
            p.grad = gr
        optG.step()
    return float(loss_D.detach()), float(loss_G.detach()), gD, gG


def cpu_config1_step(PG, PD, b):
    """BASELINE configs[0]: global pathway (zero local inputs) + D, forward + backward."""
    fake, fc2 = O.global_only(PG, b["I128"], b["z"])
    loss = O.discriminator(PD, fake).mean() + (fake - b["frontal"]).abs().mean()
    grads = torch.autograd.grad(loss, list(PG.values()) + list(PD.values()))
    return float(loss.detach()), grads


def _batch(B, g):
    def u(*s):
        return torch.rand(*s, generator=g) * 2 - 1

    return {"I128": u(B, 3, 128, 128), "left_eye": u(B, 3, 40, 40), "right_eye": u(B, 3, 40, 40),
            "nose": u(B, 3, 32, 40), "mouth": u(B, 3, 32, 48), "z": u(B, 64), "frontal": u(B, 3, 128, 128),
            "frontal_left_eye": u(B, 3, 40, 40), "frontal_right_eye": u(B, 3, 40, 40),
            "frontal_nose": u(B, 3, 32, 40), "frontal_mouth": u(B, 3, 32, 48),
            "label": torch.randint(0, 347, (B,), generator=g)}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _median_time(fn, iters):
    fn()  # warm-up
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def time_cpu_step(B=32, iters=3, threads=None, seed=0, config1_batch=4):
    """{full step faces/s at B (with both Adam updates), config-1 faces/s at config1_batch,
    seconds per step of each, threads, CPU model}; one warm-up, median of `iters`."""
    if threads:
        torch.set_num_threads(threads)
    PG, PD = O.make_params(torch.float32, seed)
    for p in list(PG.values()) + list(PD.values()):
        p.requires_grad_(True)
    optG = torch.optim.Adam(list(PG.values()), lr=1e-4, betas=(0.5, 0.999))
    optD = torch.optim.Adam(list(PD.values()), lr=1e-4, betas=(0.5, 0.999))
    g = torch.Generator().manual_seed(seed)
    b = _batch(B, g)
    dt = _median_time(lambda: cpu_train_step(PG, PD, b, optG, optD), iters)
    out = {"full_fps": B / dt, "full_s": dt}
    if config1_batch:
        PG1 = {k: v for k, v in PG.items() if k.startswith("global_pathway.")}
        b1 = _batch(config1_batch, g)
        dt1 = _median_time(lambda: cpu_config1_step(PG1, PD, b1), iters)
        out.update(config1_fps=config1_batch / dt1, config1_s=dt1)
    out.update(threads=torch.get_num_threads(), cpu=cpu_model())
    return out
