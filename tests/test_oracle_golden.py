"""CPU: the oracle (oracle/tpgan_oracle.py) against the golden vectors produced by
running the reference itself (tests/golden/make_golden.py).  This pins the oracle that
the GPU parity tests and the CPU baseline rely on."""
import os
import sys

import numpy as np
import pytest
import torch

from _cases import case_arrays, golden, rel
from oracle import tpgan_oracle as O
from oracle.det_init import det_param, det_uniform

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

G_OUT = ["I128_fake", "encoder_predict", "fused_local_fake", "le_fake", "re_fake", "nose_fake", "mouth_fake",
         "fused_local_real"]


@pytest.fixture(scope="module")
def e2e_run():
    torch.set_num_threads(8)
    E = golden("e2e_golden.npz")
    PG, PD = O.make_params(torch.float64)
    for p in list(PG.values()) + list(PD.values()):
        p.requires_grad_(True)
    ins = {k: torch.from_numpy(E["in:" + k].astype(np.float64)).requires_grad_(True)
           for k in ["I128", "left_eye", "right_eye", "nose", "mouth", "z"]}
    outs = O.generator(PG, ins["I128"], ins["left_eye"], ins["right_eye"], ins["nose"], ins["mouth"], ins["z"])
    d = O.discriminator(PD, outs[0])
    loss = 0
    for n, o in zip(G_OUT, outs):
        if n != "fused_local_real":
            loss = loss + (o * torch.from_numpy(det_uniform("proj/e2e/" + n, o.numel())).reshape(o.shape)).sum()
    loss = loss + (d * torch.from_numpy(det_uniform("proj/e2e/d_fake", d.numel())).reshape(d.shape)).sum()
    loss.backward()
    return E, PG, PD, ins, outs, d


def test_oracle_generator_outputs(e2e_run):
    E, PG, PD, ins, outs, d = e2e_run
    for n, o in zip(G_OUT, outs):
        assert rel(o.detach(), E["out:" + n]) < 1e-6, n  # fixtures stored as fp32
    assert rel(d.detach(), E["out:d_fake"]) < 1e-6


def test_oracle_grad_summaries(e2e_run):
    E, PG, PD, ins, outs, d = e2e_run
    for pre, P in (("G", PG), ("D", PD)):
        for k, p in P.items():
            g = p.grad.detach().reshape(-1).numpy()
            ref = E["gsum:%s/%s" % (pre, k)]
            assert abs(np.sqrt((g * g).sum()) - ref[0]) <= 1e-8 * max(ref[0], 1.0), k
            u = det_uniform("sample/%s/%s" % (pre, k), 16)
            idx = np.floor((u + 1.0) * 0.5 * g.size).astype(np.int64).clip(0, g.size - 1)
            # float64 vs float64 with a different op order: observed <= 1e-7 of the largest sample
            assert np.abs(g[idx] - ref[2:]).max() <= 1e-6 * max(np.abs(ref[2:]).max(), 1e-30), k


def test_oracle_input_grads(e2e_run):
    E, PG, PD, ins, outs, d = e2e_run
    for k, v in ins.items():
        if "din:" + k in E.files:
            assert rel(v.grad, E["din:" + k]) < 1e-6, k


def _op_oracle(name, x, P):
    if name.startswith("conv_"):
        spec = {"conv_k3s1p1_leaky": (1, 1, "leaky"), "conv_k3s2p1_leaky": (2, 1, "leaky"),
                "conv_k5s2p2_leaky": (2, 2, "leaky"), "conv_k5s1p2_leaky": (1, 2, "leaky"),
                "conv_k7s1p3_leaky": (1, 3, "leaky"), "conv_k1_noact": (1, 0, None),
                "conv_k3s1p1_noact_c1": (1, 1, None)}[name]
        return O.conv(P, "", x, spec[0], spec[1], spec[2]) if False else O.conv({"k" + k: v for k, v in P.items()},
                                                                                   "k", x, spec[0], spec[1], spec[2])
    if name == "res_k3":
        return O.residual({"k." + k: v for k, v in P.items()}, "k", x, 3)
    if name == "res_k5_c27":
        return O.residual({"k." + k: v for k, v in P.items()}, "k", x, 5)
    if name == "res_k2_reflect":
        return O.residual({"k." + k: v for k, v in P.items()}, "k", x, 2, [1, 0, 1, 0])
    spec = {"deconv_k3s2p1op1_relu": (2, 1, 1), "deconv_k3s4p0op1_relu": (4, 0, 1), "deconv_k8s1p0_relu": (1, 0, 0)}
    s, p, op = spec[name]
    return O.deconv({"k" + k: v for k, v in P.items()}, "k", x, s, p, op)


OPS = ["conv_k3s1p1_leaky", "conv_k3s2p1_leaky", "conv_k5s2p2_leaky", "conv_k5s1p2_leaky", "conv_k7s1p3_leaky",
       "conv_k1_noact", "conv_k3s1p1_noact_c1", "res_k3", "res_k5_c27", "res_k2_reflect", "deconv_k3s2p1op1_relu",
       "deconv_k3s4p0op1_relu", "deconv_k8s1p0_relu"]


@pytest.mark.parametrize("name", OPS)
def test_oracle_ops(name):
    A = case_arrays(golden("ops_golden.npz"), name)
    P = {}
    for k in A:
        if k.startswith("g:"):
            key = k[2:]
            P["." + key if not name.startswith("res") else key] = None
    # parameter values re-derived from the generator's names
    params = {}
    for k in [k[2:] for k in A if k.startswith("g:")]:
        shape = A["g:" + k].shape
        params[k] = torch.from_numpy(det_param("op/%s/%s" % (name, k), shape)).requires_grad_(True)
    x = torch.from_numpy(A["x"]).requires_grad_(True)
    if name.startswith("res"):
        y = _op_oracle(name, x, params)
    else:
        y = _op_oracle(name, x, {"." + k: v for k, v in params.items()})
    assert rel(y.detach(), A["y"]) < 1e-12
    y.backward(torch.from_numpy(A["gy"]))
    assert rel(x.grad, A["dx"]) < 1e-12
    for k, p in params.items():
        assert rel(p.grad, A["g:" + k]) < 1e-12, k


def test_oracle_fuser():
    A = case_arrays(golden("ops_golden.npz"), "fuser")
    xs = [torch.from_numpy(A["x:" + k]).requires_grad_(True) for k in ("le", "re", "nose", "mouth")]
    y = O.local_fuser(*xs)
    np.testing.assert_array_equal(y.detach().numpy(), A["y"])
    y.backward(torch.from_numpy(A["gy"]))
    for k, t in zip(("le", "re", "nose", "mouth"), xs):
        np.testing.assert_array_equal(t.grad.numpy(), A["dx:" + k])


def test_oracle_maxout():
    A = case_arrays(golden("ops_golden.npz"), "maxout")
    x = torch.from_numpy(A["x"]).requires_grad_(True)
    y = torch.nn.functional.max_pool1d(x.view(3, -1, 2), 2, 2).view(3, -1)
    np.testing.assert_array_equal(y.detach().numpy(), A["y"])
    y.backward(torch.from_numpy(A["gy"]))
    np.testing.assert_array_equal(x.grad.numpy(), A["dx"])


# ---- identity-feature extractor oracle vs the reference's own MobileNetV2 run
def _mnv2_params(train=False):
    import torch
    F = golden("features_golden.npz")
    sys.path.insert(0, os.path.join(REPO, "tp-gan_amd"))
    import MobileNetV2 as MN  # product module: only for the state_dict key/shape listing
    from oracle.det_init import det_module_state
    m = MN.MobileNetV2()
    assert list(m.state_dict().keys()) == [str(k) for k in F["keys"]]
    st = det_module_state(m, "mnv2/")
    return F, {k: torch.from_numpy(np.asarray(v)).double() if np.asarray(v).dtype != np.int64
               else torch.from_numpy(np.asarray(v)) for k, v in st.items()}


def test_oracle_mobilenet_v2_eval():
    import torch
    from oracle import features_oracle as FO
    F, P = _mnv2_params()
    x = torch.from_numpy(F["in:x128"]).double()
    loc, cls, feats = FO.mobilenet_v2(P, x, training=False)
    assert rel(loc, F["eval:loc"]) < 1e-6
    assert rel(cls, F["eval:cls"]) < 1e-6
    assert rel(feats[0], F["eval:f0"]) < 1e-6
    assert rel(feats[1], F["eval:f1"]) < 1e-6
    x = torch.from_numpy(F["in:x256"]).double()
    loc, cls, feats = FO.mobilenet_v2(P, x, training=False)
    assert rel(loc, F["eval256:loc"]) < 1e-6 and rel(cls, F["eval256:cls"]) < 1e-6


def test_oracle_mobilenet_v2_train():
    import torch
    from oracle import features_oracle as FO
    F, P = _mnv2_params()
    x = torch.from_numpy(F["in:x128"]).double()
    loc, cls, feats = FO.mobilenet_v2(P, x, training=True)
    assert rel(loc, F["train:loc"]) < 1e-6
    assert rel(feats[1], F["train:f1"]) < 1e-6
    for k in F.files:
        if k.startswith("train:state:"):
            assert rel(P[k[len("train:state:"):]], F[k]) < 1e-9, k
