"""GPU: pre-packed weight images (FlatParams-managed parameters, tpg_conv2d_pack_jobs +
tpg_pack_run) against the pack-inside-the-call path, bit for bit.

Both paths run the same kernel with the same plan, so they differ only in who wrote the bf16
weight image: the batched pack kernel (its item path for forward images, its LDS-transpose path
for input-gradient images) or the per-call pack.  The geometries include the channel counts
whose last 32-channel k-step holds <= 16 live channels (75, 206, 208, 80: the halo kernel's
paired steps, two taps per MFMA, tpg_halo.hip) -- the layers of D_and_G_model.py:257-279
(add_conv_and_deconv_128, enhance_features_128, conv5, enhance_features_64, add_conv_and_deconv_64).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

GEOMS = [  # (n, cin, h, w, cout, k)
    (2, 75, 24, 40, 75, 7),
    (2, 206, 16, 24, 206, 5),
    (1, 206, 20, 36, 64, 5),
    (2, 208, 16, 16, 208, 3),
    (2, 80, 20, 24, 80, 5),
    (2, 40, 12, 12, 48, 3),
    (2, 16, 8, 8, 8, 3),
]


@pytest.mark.parametrize("geom", GEOMS, ids=[str(g[1]) + "x" + str(g[5]) + "-" + str(i) for i, g in enumerate(GEOMS)])
def test_prepacked_equals_call_packed(gpu, geom):
    import tpgan_ops
    import tpgan_train
    n, cin, h, w, cout, k = geom
    gen = torch.Generator().manual_seed(cin * 31 + k)
    x0 = (torch.rand(n, cin, h, w, generator=gen) * 2 - 1)
    w0 = (torch.rand(cout, cin, k, k, generator=gen) * 2 - 1) * (1.0 / (cin * k * k) ** 0.5)
    b0 = torch.rand(cout, generator=gen) * 0.1
    gy0 = torch.rand(n, cout, h, w, generator=gen) * 2 - 1
    res = []
    for managed in (False, True):
        conv = torch.nn.Conv2d(cin, cout, k, padding=k // 2).to(gpu)
        with torch.no_grad():
            conv.weight.copy_(w0)
            conv.bias.copy_(b0)
        conv = conv.to(memory_format=torch.channels_last)
        if managed:  # (the parameters become views of one flat buffer: pre-packed images)
            flat = tpgan_train.FlatParams(conv, gpu)
        x = x0.to(gpu).contiguous(memory_format=torch.channels_last).requires_grad_(True)
        with tpgan_ops.compute_dtype(torch.bfloat16), tpgan_ops.deterministic():
            y = tpgan_ops.conv2d(x, conv.weight, conv.bias, pad=(k // 2,) * 4, act=torch.nn.LeakyReLU(0.01))
            y.backward(gy0.to(gpu).to(y.dtype))
        torch.cuda.synchronize()
        if managed:
            assert len(flat.pack_entries) >= 2, flat.pack_entries  # (forward and input-gradient images)
        res.append((y.detach().float().cpu(), x.grad.float().cpu()))
    (y0, dx0), (y1, dx1) = res
    assert torch.equal(y0, y1), float((y0 - y1).abs().max())
    assert torch.equal(dx0, dx1), float((dx0 - dx1).abs().max())
