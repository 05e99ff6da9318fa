"""CPU: host-side structure of the drop-in modules (no kernels run)."""
import json
import os

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _keys(m):
    return [[k, list(v.shape)] for k, v in m.state_dict().items()]


def test_state_dict_keys_match_reference():
    import D_and_G_model as DG
    ref = json.load(open(os.path.join(REPO, "tests", "golden", "state_dict_keys.json")))
    G = DG.Generator(64, 347, use_batchnorm=False)
    D = DG.Discriminator()
    assert _keys(G) == ref["G"]
    assert _keys(D) == ref["D"]
    assert sum(p.numel() for p in G.parameters()) == 137_764_238  # SURVEY.md §6 (with R3)
    assert sum(p.numel() for p in D.parameters()) == 13_354_625


def test_conv_weights_channels_last():
    import D_and_G_model as DG
    D = DG.Discriminator()
    for n, p in D.named_parameters():
        if p.dim() == 4:
            assert p.is_contiguous(memory_format=torch.channels_last), n


def test_fuser_placements_match_oracle():
    import D_and_G_model as DG
    from oracle.tpgan_oracle import FUSER_PADS
    for k, (l, r, t, b) in enumerate(FUSER_PADS):
        assert DG.LocalFuser.TOPS[k] == t and DG.LocalFuser.LEFTS[k] == l
        h, w = DG.LocalFuser.SIZES[k]
        assert t + h + b == 128 and l + w + r == 128


def test_factory_structure():
    import torch.nn as nn

    import ModificationLayer as ML
    c = ML.conv(8, 16, 3, 1, 1, "kaiming", nn.LeakyReLU(1e-2), False)
    assert c.out_channels == 16 and isinstance(c[0], nn.Conv2d) and isinstance(c[1], nn.LeakyReLU)
    c = ML.conv(8, 16, 2, 1, [1, 0, 1, 0], None, None, False)  # R2: no None module appended
    assert len(c) == 2 and isinstance(c[0], nn.ReflectionPad2d)
    r = ML.ResidualBlock(12, activation=nn.LeakyReLU())
    assert r.out_channels == 12 and len(r.shortcut) == 0 and r.padding == 1
    d = ML.deconv(8, 4, 3, 2, 1, 1, "kaiming", nn.ReLU(), False)
    assert d.out_channels == 4 and isinstance(d[0], nn.ConvTranspose2d)
    s = ML.sequential(c, r)
    assert s.out_channels == 12


def test_flat_params_binding_cpu():
    import D_and_G_model as DG
    import tpgan_train
    D = DG.Discriminator()
    before = {k: v.clone() for k, v in D.state_dict().items()}
    f = tpgan_train.FlatParams(D, torch.device("cpu"))
    after = D.state_dict()
    for k in before:
        assert torch.equal(before[k], after[k]), k
    assert f.data.numel() == sum(p.numel() for p in D.parameters())
    for p in D.parameters():
        assert p.grad is not None and p.grad.data_ptr() >= f.grad.data_ptr()
        if p.dim() == 4:
            assert p.is_contiguous(memory_format=torch.channels_last)
    f.grad.fill_(1.0)
    assert all(torch.all(p.grad == 1.0) for p in D.parameters())
    f.zero_grad()
    assert all(torch.all(p.grad == 0.0) for p in D.parameters())


def test_step_flops_match_survey():
    """Algorithmic FLOPs of G forward from the oracle graph (torch FlopCounterMode at
    B=1) equal SURVEY.md §6's 176.56 GF/face, which bench.py's per-step count builds on."""
    from torch.utils.flop_counter import FlopCounterMode

    from oracle import tpgan_oracle as O
    PG, PD = O.make_params(torch.float32)
    u = lambda *s: torch.rand(*s) * 2 - 1  # noqa: E731
    with torch.no_grad(), FlopCounterMode(display=False) as fc:
        out = O.generator(PG, u(1, 3, 128, 128), u(1, 3, 40, 40), u(1, 3, 40, 40), u(1, 3, 32, 40), u(1, 3, 32, 48),
                          u(1, 64))
    g = fc.get_total_flops() / 1e9
    assert abs(g - 176.56) < 0.5, g
    with torch.no_grad(), FlopCounterMode(display=False) as fc:
        O.discriminator(PD, out[0])
    assert abs(fc.get_total_flops() / 1e9 - 1.298) < 0.01


def test_tuning_file_roundtrip_and_old_keys(tmp_path):
    """weight-gradient tuning files written before the concurrency flag joined the
    cache key (18-field keys) load as whole-chip (flag 0) entries instead of never matching."""
    import tpgan_ops
    from tpgan_lib import FLAG_CONCURRENT, ConvDesc
    saved = dict(tpgan_ops.AUTOTUNE["cache"])
    try:
        d = ConvDesc()
        d.n, d.in_c, d.in_h, d.in_w, d.out_c, d.out_h, d.out_w, d.kh, d.kw = 32, 64, 40, 40, 64, 40, 40, 3, 3
        d.stride_h = d.stride_w = 1
        k0 = tpgan_ops._wgrad_key(d)
        d.flags = FLAG_CONCURRENT
        k1 = tpgan_ops._wgrad_key(d)
        assert len(k0[1]) == len(k1[1]) == tpgan_ops._WGRAD_KEY_LEN and k0 != k1
        tpgan_ops.AUTOTUNE["cache"].clear()
        tpgan_ops.AUTOTUNE["cache"][k1] = (7, 4)
        kd = ("dsplit", 1, tpgan_ops._desc_tuple(d) + (1, 2))  # (forward / input-gradient split picks)
        tpgan_ops.AUTOTUNE["cache"][kd] = (4, 2)
        p = str(tmp_path / "tune.json")
        tpgan_ops.save_tuning(p)
        old = str(tmp_path / "old.json")
        json.dump([[list(k0[1][:-1]), "wgrad", [12, 2]]], open(old, "w"))
        tpgan_ops.AUTOTUNE["cache"].clear()
        tpgan_ops.load_tuning(p)
        tpgan_ops.load_tuning(old)
        assert tpgan_ops.AUTOTUNE["cache"][k1] == (7, 4)
        assert tpgan_ops.AUTOTUNE["cache"][k0] == (12, 2)
        assert tpgan_ops.AUTOTUNE["cache"][kd] == (4, 2)
    finally:
        tpgan_ops.AUTOTUNE["cache"].clear()


def test_committed_tuning_caches_load():
    """The autotuner caches committed under profiles/ (bench.py --tune-file) load: every weight-
    gradient key has the current field count and every pick is an (algo, split) pair."""
    import glob
    import os
    import tpgan_ops
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                          "profiles", "r06", "tune_*.json")))
    assert files
    saved = dict(tpgan_ops.AUTOTUNE["cache"])
    try:
        for f in files:
            tpgan_ops.AUTOTUNE["cache"].clear()
            tpgan_ops.load_tuning(f)
            cache = tpgan_ops.AUTOTUNE["cache"]
            assert len(cache) > 50, f
            for k, v in cache.items():
                assert len(v) == 2 and all(isinstance(x, int) for x in v), (f, k, v)
                if k[0] == "wgrad":
                    assert len(k[1]) == tpgan_ops._WGRAD_KEY_LEN, (f, k)
    finally:
        tpgan_ops.AUTOTUNE["cache"].clear()
        tpgan_ops.AUTOTUNE["cache"].update(saved)
        tpgan_ops.AUTOTUNE["cache"].update(saved)
