"""Generate the committed golden fixtures by running the REFERENCE itself.

Run here (the reference is only present in the build container, never on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Recipe: stub torchvision (imported at D_and_G_model.py:14 and
UtilityMethods.py:9, never called on the hot path), then apply the three repairs
without which the reference cannot construct or run its models:

  R1  weight_initialization passes the module to kaiming_normal/xavier_normal
      (ModificationLayer.py:47,49,51)      -> initialise module.weight instead
  R2  _batchnorm_and_activation_layer appends activation=None into nn.Sequential
      (ModificationLayer.py:154)           -> drop None entries
  R3  GlobalPathway sizes dim128 = 72 but concatenates 75 channels
      (D_and_G_model.py:268-269 vs :323)   -> dim128 = 75, enhance_128 = 206, conv5 in 206

Weights are NOT taken from torch's RNG: every state_dict entry is overwritten with
oracle.det_init.det_param(prefix+key, shape), so fixtures are reproducible from names.
All reference runs are in float64.  Outputs go to tests/golden/*.npz (no pickles).
"""
import json
import os
import sys
import types

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle.det_init import det_input, det_param, det_uniform  # noqa: E402

REF = "/root/reference"


def import_reference():
    tv = types.ModuleType("torchvision")
    tvt = types.ModuleType("torchvision.transforms")
    tv.transforms = tvt
    sys.modules.setdefault("torchvision", tv)
    sys.modules.setdefault("torchvision.transforms", tvt)
    sys.path.insert(0, REF)
    import ModificationLayer as ML
    import D_and_G_model as DG

    # R1
    def _kaiming(module, a=0):
        torch.nn.init.kaiming_normal_(module.weight, a=a)

    def _xavier(module):
        torch.nn.init.xavier_normal_(module.weight)

    ML.kaiming_normal = _kaiming
    ML.xavier_normal = _xavier
    # R2
    _orig = ML._batchnorm_and_activation_layer

    def _bn_act(ch, act, bn):
        return [l for l in _orig(ch, act, bn) if l is not None]

    ML._batchnorm_and_activation_layer = _bn_act
    return ML, DG


def repair_global(DG, ML, gp):
    """R3."""
    nn = torch.nn
    gp.add_conv_and_deconv_128 = ML.ResidualBlock(75, kernel_size=7, activation=nn.LeakyReLU())
    gp.enhance_features_128 = ML.sequential(ML.ResidualBlock(206, kernel_size=5, activation=nn.LeakyReLU()))
    gp.conv5 = ML.sequential(
        ML.conv(206, 64, 5, 1, 2, "kaiming", nn.LeakyReLU(), False),
        ML.ResidualBlock(64, kernel_size=3, activation=nn.LeakyReLU()),
    )
    return gp


def load_det(module, prefix):
    sd = module.state_dict()
    new = {k: torch.from_numpy(det_param(prefix + k, v.shape)).to(v.dtype) for k, v in sd.items()}
    module.load_state_dict(new)


def t64(name, shape):
    return torch.from_numpy(det_input(name, shape))


def proj(name, shape):
    return torch.from_numpy(det_uniform("proj/" + name, int(np.prod(shape)))).reshape(shape)


def sample_idx(name, numel, k=16):
    u = det_uniform("sample/" + name, k)
    return np.floor((u + 1.0) * 0.5 * numel).astype(np.int64).clip(0, numel - 1)


def grad_summary(prefix, named):
    out = {}
    for k, g in named:
        g = g.detach().double().reshape(-1).numpy()
        idx = sample_idx(prefix + k, g.size)
        out[k] = np.concatenate([[np.sqrt((g * g).sum()), g.sum()], g[idx]])
    return out


# ----------------------------------------------------------------------------------
# per-op fixtures: the reference's own layer factories (ModificationLayer.py) + LocalFuser
# + the GlobalPathway maxout (D_and_G_model.py:214,290)
# ----------------------------------------------------------------------------------
def make_ops(ML, DG):
    nn = torch.nn
    L = nn.LeakyReLU
    cases = {
        # name: (factory, input shape)
        "conv_k3s1p1_leaky": (lambda: ML.conv(20, 24, 3, 1, 1, "kaiming", L(1e-2), False), (2, 20, 9, 11)),
        "conv_k3s2p1_leaky": (lambda: ML.conv(20, 24, 3, 2, 1, "kaiming", L(1e-2), False), (2, 20, 9, 11)),
        "conv_k5s2p2_leaky": (lambda: ML.conv(16, 16, 5, 2, 2, "kaiming", L(1e-2), False), (2, 16, 10, 9)),
        "conv_k5s1p2_leaky": (lambda: ML.conv(19, 13, 5, 1, 2, "kaiming", L(), False), (2, 19, 8, 7)),
        "conv_k7s1p3_leaky": (lambda: ML.conv(3, 18, 7, 1, 3, "kaiming", L(1e-2), False), (2, 3, 9, 10)),
        "conv_k1_noact": (lambda: ML.conv(20, 3, 1, 1, 0, None, None, False), (2, 20, 6, 5)),
        "conv_k3s1p1_noact_c1": (lambda: ML.conv(40, 1, 3, 1, 1, None, None, False), (2, 40, 4, 4)),
        "res_k3": (lambda: ML.ResidualBlock(20, activation=L()), (2, 20, 7, 6)),
        "res_k5_c27": (lambda: ML.ResidualBlock(27, kernel_size=5, activation=L()), (2, 27, 6, 6)),
        "res_k2_reflect": (lambda: ML.ResidualBlock(12, 12, 2, 1, padding=[1, 0, 1, 0], activation=L()), (2, 12, 5, 5)),
        "deconv_k3s2p1op1_relu": (lambda: ML.deconv(20, 12, 3, 2, 1, 1, "kaiming", nn.ReLU(), False), (2, 20, 5, 6)),
        "deconv_k3s4p0op1_relu": (lambda: ML.deconv(16, 8, 3, 4, 0, 1, "kaiming", nn.ReLU(), False), (2, 16, 4, 4)),
        "deconv_k8s1p0_relu": (lambda: ML.deconv(20, 8, 8, 1, 0, 0, "kaiming", nn.ReLU(), False), (2, 20, 1, 1)),
    }
    out = {}
    for name, (fac, shape) in cases.items():
        torch.manual_seed(0)
        m = fac().double()
        load_det(m, "op/%s/" % name)
        x = t64("op/%s/x" % name, shape).requires_grad_(True)
        y = m(x)
        gy = proj("op/%s/y" % name, tuple(y.shape))
        (y * gy).sum().backward()
        rec = {"x": x.detach().numpy(), "y": y.detach().numpy(), "gy": gy.numpy(), "dx": x.grad.numpy()}
        for k, p in m.named_parameters():  # parameter values are re-derived from det_param
            rec["g:" + k] = p.grad.numpy()
        out[name] = rec

    # LocalFuser (D_and_G_model.py:132-159): features with negatives so zero padding
    # wins some pixels (tie-break pinned through the gradient routing).
    fuser = DG.LocalFuser()
    shapes = {"le": (2, 5, 40, 40), "re": (2, 5, 40, 40), "nose": (2, 5, 32, 40), "mouth": (2, 5, 32, 48)}
    xs = {k: t64("op/fuser/" + k, s).requires_grad_(True) for k, s in shapes.items()}
    y = fuser(xs["le"], xs["re"], xs["nose"], xs["mouth"])
    gy = proj("op/fuser/y", tuple(y.shape))
    (y * gy).sum().backward()
    rec = {"y": y.detach().numpy(), "gy": gy.numpy()}
    for k in shapes:
        rec["x:" + k] = xs[k].detach().numpy()
        rec["dx:" + k] = xs[k].grad.numpy()
    out["fuser"] = rec

    # maxout fc2 = MaxPool1d(2,2) on view(B,-1,2) (D_and_G_model.py:214,290); exact ties
    # in half of the pairs pin the first-index tie-break.
    pool = torch.nn.MaxPool1d(2, 2, 0)
    x = t64("op/maxout/x", (3, 512))
    x[:, 1:256:2] = x[:, 0:256:2]
    x = x.clone().requires_grad_(True)
    y = pool(x.view(3, -1, 2)).view(3, -1)
    gy = proj("op/maxout/y", tuple(y.shape))
    (y * gy).sum().backward()
    out["maxout"] = {"x": x.detach().numpy(), "y": y.detach().numpy(), "gy": gy.numpy(), "dx": x.grad.numpy()}

    # Linear (fc1 / FeaturePredict.fc layer type, D_and_G_model.py:212,343)
    lin = torch.nn.Linear(96, 40).double()
    load_det(lin, "op/linear/")
    x = t64("op/linear/x", (4, 96)).requires_grad_(True)
    y = lin(x)
    gy = proj("op/linear/y", tuple(y.shape))
    (y * gy).sum().backward()
    out["linear"] = {"x": x.detach().numpy(), "y": y.detach().numpy(), "gy": gy.numpy(), "dx": x.grad.numpy(),
                     "g:weight": lin.weight.grad.numpy(), "g:bias": lin.bias.grad.numpy()}
    return out


G_OUT_NAMES = ["I128_fake", "encoder_predict", "fused_local_fake", "le_fake", "re_fake",
               "nose_fake", "mouth_fake", "fused_local_real"]
G_IN_SHAPES = {"I128": (3, 128, 128), "left_eye": (3, 40, 40), "right_eye": (3, 40, 40),
               "nose": (3, 32, 40), "mouth": (3, 32, 48), "z": (64,)}


def make_e2e(ML, DG, B=2):
    torch.manual_seed(0)
    G = DG.Generator(64, 347, use_batchnorm=False)
    repair_global(DG, ML, G.global_pathway)
    D = DG.Discriminator()
    G = G.double()
    D = D.double()
    load_det(G, "G/")
    load_det(D, "D/")
    keys = {"G": [(k, list(v.shape)) for k, v in G.state_dict().items()],
            "D": [(k, list(v.shape)) for k, v in D.state_dict().items()]}

    ins = {k: t64("e2e/" + k, (B,) + s).requires_grad_(True) for k, s in G_IN_SHAPES.items()}
    outs = G(ins["I128"], ins["left_eye"], ins["right_eye"], ins["nose"], ins["mouth"], ins["z"], False)
    loss = 0
    for name, o in zip(G_OUT_NAMES, outs):
        if name == "fused_local_real":
            continue  # no parameter dependence
        loss = loss + (o * proj("e2e/" + name, tuple(o.shape))).sum()
    d_fake = D(outs[0])
    loss = loss + (d_fake * proj("e2e/d_fake", tuple(d_fake.shape))).sum()
    loss.backward()
    rec = {}
    for name, o in zip(G_OUT_NAMES, outs):
        rec["out:" + name] = o.detach().numpy()
    rec["out:d_fake"] = d_fake.detach().numpy()
    for k, v in ins.items():
        rec["in:" + k] = v.detach().numpy()
        if v.grad is not None:
            rec["din:" + k] = v.grad.numpy()
    for k, v in grad_summary("G/", [(k, p.grad) for k, p in G.named_parameters()]).items():
        rec["gsum:G/" + k] = v
    for k, v in grad_summary("D/", [(k, p.grad) for k, p in D.named_parameters()]).items():
        rec["gsum:D/" + k] = v
    # D on the real input (config D(real) leg)
    D.zero_grad()
    d_real = D(ins["I128"].detach())
    rec["out:d_real"] = d_real.detach().numpy()
    return rec, keys


def main():
    torch.set_num_threads(os.cpu_count() or 8)
    ML, DG = import_reference()
    ops = make_ops(ML, DG)
    flat = {}
    for case, rec in ops.items():
        for k, v in rec.items():
            flat["%s|%s" % (case, k)] = np.asarray(v)
    np.savez_compressed(os.path.join(HERE, "ops_golden.npz"), **flat)
    print("ops fixtures:", len(ops))

    rec, keys = make_e2e(ML, DG)
    # large float tensors stored as float32 (the reference ran in float64; fp32 storage
    # keeps ~7 digits, far below the 1e-3 tolerance), summaries stay float64
    store = {}
    for k, v in rec.items():
        v = np.asarray(v)
        store[k] = v.astype(np.float32) if (v.size > 4096 and not k.startswith("gsum:")) else v
    np.savez_compressed(os.path.join(HERE, "e2e_golden.npz"), **store)
    with open(os.path.join(HERE, "state_dict_keys.json"), "w") as f:
        json.dump(keys, f)
    print("e2e: G keys", len(keys["G"]), "D keys", len(keys["D"]))


if __name__ == "__main__":
    main()
