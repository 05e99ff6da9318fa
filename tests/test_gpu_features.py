"""GPU parity of the identity-feature extractors through the HIP
kernels: the product MobileNetV2 against the reference's own float64 run
(tests/golden/features_golden.npz, eval and train mode), ResNet-50 / repaired ResNet18
against the oracle restatement (parity unpinned: no reference source runs), and the new
ops one by one against aten on the CPU."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from _cases import golden, rel

pytestmark = pytest.mark.gpu


def _load_det(model, prefix):
    from oracle.det_init import det_module_state
    st = det_module_state(model, prefix)
    sd = model.state_dict()
    model.load_state_dict({k: torch.from_numpy(np.asarray(v)).to(sd[k].dtype) for k, v in st.items()})
    return st


def _gsum_check(G, tag, model, tol_norm=1e-2, tol_cat=1e-3):
    from oracle.det_init import det_uniform
    allg, allr = [], []
    worst = (0.0, None)
    # train-mode BatchNorm makes some gradients vanish analytically (a BN input's gradient
    # sums to zero per channel, so e.g. the beta of a BN feeding only BN'd convs gets
    # ~1e-16): norms are compared with a floor of 1e-4 x the largest tensor norm
    floor = 1e-4 * max(G["%s:gsum:%s" % (tag, k)][0] for k, _ in model.named_parameters())
    for k, p in model.named_parameters():
        ref = G["%s:gsum:%s" % (tag, k)]
        g = p.grad.detach().double().reshape(-1).cpu().numpy()
        u = det_uniform("sample/mnv2/%s/%s" % (tag, k), 16)
        idx = np.floor((u + 1.0) * 0.5 * g.size).astype(np.int64).clip(0, g.size - 1)
        e = abs(np.sqrt((g * g).sum()) - ref[0]) / max(ref[0], floor)
        if e > worst[0]:
            worst = (e, k)
        allg.append(g[idx])
        allr.append(ref[2:])
    assert worst[0] < tol_norm, worst
    assert rel(np.concatenate(allg), np.concatenate(allr)) < tol_cat


def _mnv2_run(gpu, train, dtype=torch.float32):
    import MobileNetV2 as MN
    import tpgan_ops
    G = golden("features_golden.npz")
    m = MN.MobileNetV2()
    _load_det(m, "mnv2/")
    m = m.to(gpu)
    m.train(train)
    tag = "train" if train else "eval"
    x = torch.from_numpy(G["in:x128"]).float().to(gpu).requires_grad_(True)
    feats = {}
    orig = m._backbone

    def spy(xx, stop_after_conv2=False):
        out, f = orig(xx)
        feats["f0"], feats["f1"] = f[0], f[1]
        return out, f

    m._backbone = spy
    with tpgan_ops.compute_dtype(dtype):
        loc, cls = m(x)
    outs = {"loc": loc, "cls": cls, "f0": feats["f0"], "f1": feats["f1"]}
    from oracle.det_init import det_uniform
    loss = 0
    for k, v in outs.items():
        pr = torch.from_numpy(det_uniform("proj/mnv2/%s/%s" % (tag, k), v.numel())).reshape(v.shape).float().to(gpu)
        loss = loss + (v.float() * pr).sum()
    loss.backward()
    torch.cuda.synchronize()
    return G, m, x, outs, tag


@pytest.mark.parametrize("train", [False, True])
def test_mobilenet_v2_fp32_vs_reference(gpu, train):
    G, m, x, outs, tag = _mnv2_run(gpu, train)
    for k, v in outs.items():
        assert tuple(v.shape) == G["%s:%s" % (tag, k)].shape, k
        assert rel(v.detach().float().cpu(), G["%s:%s" % (tag, k)]) < 1e-3, k
    tol_dx = 1e-3
    if train:  # fp32 floor of the batch-statistics backward (B=2, 4x4 maps): oracle in float32.
        # 5x, not 3x: the split-K / weight-gradient fp32 atomics make the HIP run's accumulation
        # order vary from run to run, and train-mode BN over 4x4 maps amplifies that rounding
        # noise (observed 2.5x..3.8x the oracle's own fp32 deviation across runs of one build)
        tol_dx = max(tol_dx, 5 * _mnv2_oracle_dx_floor(G))
    assert rel(x.grad.cpu(), G["%s:dx" % tag]) < tol_dx
    _gsum_check(G, tag, m, tol_cat=max(1e-3, tol_dx))
    if train:
        sd = m.state_dict()
        for k in G.files:
            if k.startswith("train:state:"):
                assert rel(sd[k[len("train:state:"):]].cpu(), G[k]) < 1e-4, k


def _mnv2_oracle_dx_floor(G):
    import MobileNetV2 as MN
    from oracle import features_oracle as FO
    from oracle.det_init import det_module_state, det_uniform
    P = {k: torch.from_numpy(np.asarray(v)).float() if np.asarray(v).dtype != np.int64 else torch.from_numpy(v)
         for k, v in det_module_state(MN.MobileNetV2(), "mnv2/").items()}
    x = torch.from_numpy(G["in:x128"]).float().requires_grad_(True)
    loc, cls, f = FO.mobilenet_v2(P, x, training=True)
    loss = 0
    for k, v in (("loc", loc), ("cls", cls), ("f0", f[0]), ("f1", f[1])):
        loss = loss + (v * torch.from_numpy(det_uniform("proj/mnv2/train/%s" % k, v.numel())).reshape(v.shape).float()).sum()
    loss.backward()
    return rel(x.grad.double(), G["train:dx"])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
def test_mobilenet_v2_bf16_eval(gpu, dtype):
    """16-bit MFMA / depthwise paths (bf16; fp16 = BASELINE configs[4]'s extractor dtype)."""
    G, m, x, outs, tag = _mnv2_run(gpu, False, dtype)
    for k, v in outs.items():
        assert rel(v.detach().float().cpu(), G["eval:%s" % k]) < 3e-2, k
    # the input gradient crosses 52 bf16 layers (each rounding activations and gradients
    # to 8 mantissa bits, ReLU6 masks flipping where bf16 moves a pre-activation across 0
    # or 6): measured 0.166 relative L2 — bound its direction instead of its exact value
    g, r = x.grad.cpu().double().reshape(-1), torch.from_numpy(G["eval:dx"]).double().reshape(-1)
    assert float(torch.dot(g, r) / (g.norm() * r.norm())) > 0.98


def test_mobilenet_v2_256(gpu):
    import MobileNetV2 as MN
    G = golden("features_golden.npz")
    m = MN.MobileNetV2()
    _load_det(m, "mnv2/")
    m = m.to(gpu).eval()
    with torch.no_grad():
        loc, cls = m(torch.from_numpy(G["in:x256"]).float().to(gpu))
    assert rel(loc.cpu(), G["eval256:loc"]) < 1e-3
    assert rel(cls.cpu(), G["eval256:cls"]) < 1e-3


def _oracle_params(model, prefix):
    st = {}
    from oracle.det_init import det_module_state
    for k, v in det_module_state(model, prefix).items():
        v = np.asarray(v)
        st[k] = torch.from_numpy(v).double() if v.dtype != np.int64 else torch.from_numpy(v)
    return st


@pytest.mark.parametrize("train", [False, True])
def test_resnet50_vs_oracle(gpu, train):
    """Build-defined ResNet-50: parity unpinned against the reference (none exists); the
    HIP path must match the aten restatement of the same network."""
    import ResNet as R
    from oracle import features_oracle as FO
    m = R.ResNet50(num_of_output_classes=10)
    _load_det(m, "rn50/")
    P = _oracle_params(m, "rn50/")
    m = m.to(gpu).train(train)
    xs = torch.from_numpy(__import__("oracle.det_init", fromlist=["x"]).det_input("rn50/x", (2, 3, 64, 64)))
    x = xs.float().to(gpu).requires_grad_(True)
    logits, feat = m(x)
    (logits.float().sum() + feat.float().square().sum()).backward()
    torch.cuda.synchronize()
    xr = xs.clone().requires_grad_(True)
    lr_, fr, _ = FO.resnet50(P, xr, training=train)
    (lr_.sum() + fr.square().sum()).backward()
    # fp32 floor: the same restatement in float32 (train-mode BN over 2x2 maps at B=2 is
    # ill-conditioned: its backward subtracts nearly equal batch means)
    P32 = {k: (v.float() if v.is_floating_point() else v) for k, v in _oracle_params(m, "rn50/").items()}
    x32 = xs.float().requires_grad_(True)
    l32, f32, _ = FO.resnet50(P32, x32, training=train)
    (l32.sum() + f32.square().sum()).backward()
    floor = rel(x32.grad.double(), xr.grad)
    assert rel(logits.detach().cpu(), lr_.detach()) < 1e-3
    assert rel(feat.detach().cpu(), fr.detach()) < 1e-3
    assert rel(x.grad.cpu(), xr.grad) < max(1e-3, 5 * floor), floor


def test_resnet18_repaired_vs_oracle(gpu):
    import ResNet as R
    from oracle import features_oracle as FO
    m = R.ResNet18(num_of_output_classes=7)
    _load_det(m, "rn18/")
    P = _oracle_params(m, "rn18/")
    m = m.to(gpu).eval()
    xs = torch.from_numpy(__import__("oracle.det_init", fromlist=["x"]).det_input("rn18/x", (2, 3, 64, 64)))
    with torch.no_grad():
        feats = m.extract_features(xs.float().to(gpu))
        out, fc0 = m(xs.float().to(gpu))
    ref_map, ref_feat = FO.resnet18_r4(P, xs, training=False)
    assert fc0 is None
    assert rel(feats[0].float().cpu(), ref_map) < 1e-3
    assert rel(feats[1].float().cpu(), ref_feat) < 1e-3
    ref_out = F.linear(ref_feat, P["FC.0.weight"], P["FC.0.bias"])
    assert rel(out.cpu(), ref_out) < 1e-3


# ------------------------------------------------------------------ single ops
@pytest.mark.parametrize("c,h,w,stride,dtype", [(24, 9, 11, 1, torch.float32), (40, 10, 7, 2, torch.float32),
                                                (96, 8, 8, 1, torch.bfloat16), (19, 6, 5, 2, torch.bfloat16)])
def test_dwconv_vs_aten(gpu, c, h, w, stride, dtype):
    import tpgan_ops
    g = torch.Generator().manual_seed(c + h)
    x = torch.randn(2, c, h, w, generator=g, dtype=torch.float64)
    wt = torch.randn(c, 1, 3, 3, generator=g, dtype=torch.float64) * 0.3
    b = torch.randn(c, generator=g, dtype=torch.float64) * 0.1
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, wt, b))
    yr = F.hardtanh(F.conv2d(xr, wr, br, stride, 1, groups=c), 0, 6)
    pr = torch.randn(yr.shape, generator=g, dtype=torch.float64)
    (yr * pr).sum().backward()
    xg, wg, bg = (t.float().to(gpu).requires_grad_(True) for t in (x, wt, b))
    with tpgan_ops.compute_dtype(dtype):
        y = tpgan_ops.dwconv2d(xg, wg, bg, (stride, stride), (1, 1), act=torch.nn.ReLU6())
    (y.float() * pr.float().to(gpu)).sum().backward()
    torch.cuda.synchronize()
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert rel(y.detach().float().cpu(), yr.detach()) < tol
    assert rel(xg.grad.cpu(), xr.grad) < tol * 4
    assert rel(wg.grad.cpu(), wr.grad) < tol * 4
    assert rel(bg.grad.cpu(), br.grad) < tol * 4


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_maxpool_avgpool_vs_aten(gpu, dtype):
    import tpgan_ops
    g = torch.Generator().manual_seed(7)
    x = torch.randperm(2 * 20 * 13 * 11, generator=g).reshape(2, 20, 13, 11).double() / 100.0  # distinct values
    x = x.to(dtype).double()  # bf16 rounding creates ties: both sides keep the first maximum in scan order
    xr = x.clone().requires_grad_(True)
    yr = F.max_pool2d(xr, 3, 2, 1)
    ar = xr.mean((2, 3), keepdim=True)
    pr = torch.randn(yr.shape, generator=g, dtype=torch.float64)
    pa = torch.randn(ar.shape, generator=g, dtype=torch.float64)
    ((yr * pr).sum() + (ar * pa).sum()).backward()
    xg = x.to(dtype).float().to(gpu).requires_grad_(True)
    with tpgan_ops.compute_dtype(dtype):
        y = tpgan_ops.maxpool2d(xg, 3, 2, 1)
        a = tpgan_ops.global_avgpool(xg)
    ((y.float() * pr.float().to(gpu)).sum() + (a.float() * pa.float().to(gpu)).sum()).backward()
    torch.cuda.synchronize()
    tol = 1e-6 if dtype == torch.float32 else 1e-2
    assert rel(y.detach().float().cpu(), yr.detach()) < tol
    assert rel(a.detach().float().cpu(), ar.detach()) < tol
    assert rel(xg.grad.cpu(), xr.grad) < tol * 10


def test_batchnorm_train_vs_aten(gpu):
    import tpgan_ops
    g = torch.Generator().manual_seed(9)
    bn = torch.nn.BatchNorm2d(37)
    with torch.no_grad():
        bn.weight.copy_(1 + 0.2 * torch.randn(37, generator=g))
        bn.bias.copy_(0.1 * torch.randn(37, generator=g))
    ref = torch.nn.BatchNorm2d(37).double()
    ref.load_state_dict(bn.state_dict())
    x = torch.randn(3, 37, 9, 7, generator=g, dtype=torch.float64) * 2 + 0.5
    xr = x.clone().requires_grad_(True)
    yr = F.relu6(ref(xr))
    pr = torch.randn(yr.shape, generator=g, dtype=torch.float64)
    (yr * pr).sum().backward()
    bng = bn.to(gpu).train()
    xg = x.float().to(gpu).requires_grad_(True)
    y = tpgan_ops.batchnorm_train(xg, bng, act=torch.nn.ReLU6())
    (y * pr.float().to(gpu)).sum().backward()
    torch.cuda.synchronize()
    assert rel(y.detach().cpu(), yr.detach()) < 1e-5
    assert rel(xg.grad.cpu(), xr.grad) < 1e-4
    assert rel(bng.weight.grad.cpu(), ref.weight.grad) < 1e-4
    assert rel(bng.bias.grad.cpu(), ref.bias.grad) < 1e-4
    assert rel(bng.running_mean.cpu(), ref.running_mean) < 1e-5
    assert rel(bng.running_var.cpu(), ref.running_var) < 1e-5
    assert int(bng.num_batches_tracked) == 1


@pytest.mark.parametrize("name", ["mobilenetv2", "resnet50"])
def test_identity_loss_in_train_step(gpu, name):
    """Config 3: the G step with the identity-preserving loss through a frozen extractor."""
    import D_and_G_model as DG
    import FeatureExtract as FE
    import tpgan_train
    ext = FE.FeatureExtractModel(name, 10).to(gpu)
    idl = FE.IdentityPreservingLoss(ext, torch.bfloat16)
    G = DG.Generator(64, 347, use_batchnorm=False).to(gpu)
    D = DG.Discriminator().to(gpu)
    tr = tpgan_train.TPGANTrainer(G, D, compute_dtype=torch.bfloat16, identity_fn=idl)
    b = tpgan_train.synthetic_batch(2, gpu, seed=3)
    out = tr.step(b)
    torch.cuda.synchronize()
    assert np.isfinite(float(out["loss_G"]))
    assert torch.isfinite(tr.fG.grad).all()
    assert all(p.grad is None for p in ext.parameters())
