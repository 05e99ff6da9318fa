"""GPU: the producer's activation backward moved into its consumer's input-gradient launch
(tpgan_ops.ActToken, desc.in_act).

A conv with an activation (reference ModificationLayer.py:54-123) whose output feeds one conv
alone -- a residual block's inner pair, a sequential chain (ModificationLayer.py:5-24,
233-302), D's layer chain (D_and_G_model.py:409-435) -- gets its masked gradient
g = gy * act'(y) from the consumer's epilogue instead of staging y beside gy itself.  The
result must be the same computation: with the links on and off, every gradient agrees -- bit
for bit in fp32 (the same fp32 product either way), within 16-bit rounding of the input
gradient in bf16 (once rounded instead of twice).  The consumer geometries cover every plan
the input gradient can take: the halo kernel with and without a k split (split-K epilogue
kernel), the tap-DMA pointwise kernel, stride-2 and transposed convs, the reflect-padded
fold and the full-kernel GEMM form (the last two through the in-place fallback pass)."""
import zlib

import pytest
import torch

from _cases import rel

pytestmark = pytest.mark.gpu

# consumer conv: (N, Cin, H, W, Cout, k, stride, pad, transposed, output_padding, reflect)
CONSUMERS = [
    (2, 64, 32, 32, 64, 3, 1, 1, False, 0, False),     # halo kernel, one tile per block
    (2, 206, 12, 10, 206, 5, 1, 2, False, 0, False),   # small map: k split + split-K epilogue
    (8, 512, 8, 8, 512, 3, 1, 1, False, 0, False),     # whole small images per block, k split
    (4, 128, 20, 20, 128, 3, 1, 1, False, 0, False),   # tap-DMA pointwise kernel (<= 256 ch)
    (3, 64, 17, 15, 128, 3, 2, 1, False, 0, False),    # stride-2 conv: dgrad parity classes
    (2, 96, 9, 9, 64, 3, 2, 1, True, 1, False),        # transposed: dgrad is a stride-2 conv
    (2, 64, 10, 10, 64, 2, 1, 0, False, 0, True),      # reflect 2x2: fold -> in-place pass
    (3, 64, 9, 7, 128, 1, 1, 0, False, 0, False),      # 1x1 on the pointwise kernel
    (2, 64, 8, 8, 40, 8, 1, 0, False, 0, False),       # full-kernel GEMM form -> in-place pass
]


def _chain(gpu, geom, dtype, act_prod, on):
    import tpgan_ops
    from tpgan_lib import PAD_REFLECT, PAD_ZERO
    (N, C, H, W, Cout, k, s, p, tr, op, refl) = geom
    gen = torch.Generator().manual_seed(zlib.crc32(repr(geom).encode()))
    x0 = torch.rand(N, 24, H, W, generator=gen) * 2 - 1
    w0 = (torch.rand(C, 24, 3, 3, generator=gen) * 2 - 1) * (3.0 / (24 * 9)) ** 0.5
    b0 = torch.rand(C, generator=gen) * 0.2 - 0.1
    wshape = (C, Cout, k, k) if tr else (Cout, C, k, k)
    w1 = (torch.rand(wshape, generator=gen) * 2 - 1) * (3.0 / (wshape[1] * k * k)) ** 0.5
    b1 = torch.rand(Cout, generator=gen) * 0.2 - 0.1
    cl = torch.channels_last
    x = x0.to(gpu).contiguous(memory_format=cl).requires_grad_(True)
    wa = w0.to(gpu).contiguous(memory_format=cl).requires_grad_(True)
    ba = b0.to(gpu).requires_grad_(True)
    wb = w1.to(gpu).contiguous(memory_format=cl).requires_grad_(True)
    bb = b1.to(gpu).requires_grad_(True)
    actp = {"leaky": torch.nn.LeakyReLU(0.01), "relu": torch.nn.ReLU()}[act_prod]
    prev = tpgan_ops.ACT_LINK["enabled"]
    tpgan_ops.ACT_LINK["enabled"] = on
    try:
        # (fp32: deterministic, so on == off bit for bit; bf16: the default mode, so the k-split
        # plans and their split-K epilogue launches run too)
        with tpgan_ops.compute_dtype(dtype), tpgan_ops.deterministic(dtype == torch.float32):
            h = tpgan_ops.conv2d(x, wa, ba, pad=(1, 1, 1, 1), act=actp)
            pad = (1, 0, 1, 0) if refl else (p, p, p, p)
            y = tpgan_ops.conv2d(h, wb, bb, stride=(s, s), pad=pad, pad_mode=PAD_REFLECT if refl else PAD_ZERO,
                                 act=torch.nn.LeakyReLU(0.01), transposed=tr, output_padding=(op, op),
                                 act_in_ok=True)
            gy = torch.cos(torch.arange(y.numel(), dtype=torch.float64) * 0.37).reshape(y.shape)
            y.backward(gy.to(gpu).to(y.dtype))
            torch.cuda.synchronize()
        # the link was taken exactly when it was on
        tok = getattr(h, "_tpg_act_tok", None)
        assert (tok is not None) == on and (tok is None or tok.pre is None)
    finally:
        tpgan_ops.ACT_LINK["enabled"] = prev
    return [t.grad.detach().float().cpu() for t in (x, wa, ba, wb, bb)]


@pytest.mark.parametrize("act_prod", ["leaky", "relu"])
@pytest.mark.parametrize("geom", CONSUMERS, ids=[str(i) for i in range(len(CONSUMERS))])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_link_matches_unlinked(gpu, geom, dtype, act_prod):
    _chain(gpu, geom, dtype, act_prod, True)  # (the first pass runs the autotuners)
    off = _chain(gpu, geom, dtype, act_prod, False)
    on = _chain(gpu, geom, dtype, act_prod, True)
    names = ("dx", "dW0", "db0", "dW1", "db1")
    for nm, a, b in zip(names, on, off):
        if dtype == torch.float32:
            assert torch.equal(a, b), (nm, rel(a, b))
        else:
            # the producer's g is rounded once (v * act') instead of twice (round(v) * act')
            assert rel(a, b) < 1e-2, (nm, rel(a, b))
    if dtype == torch.float32:  # the consumer's own weight gradient never sees the link
        assert torch.equal(on[3], off[3]) and torch.equal(on[4], off[4])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_link_through_residual_blocks(gpu, dtype):
    """conv -> ResidualBlock -> ResidualBlock as one sequential (the encoder's conv4 stage):
    the first block's first conv takes the whole gradient of the chain conv's output only
    because the block's GradLink carries the shortcut part into its launch (DX_ACCUM, then
    act'); the inner convs' links need no shortcut.  Links on == off."""
    import ModificationLayer as ML
    import tpgan_ops
    torch.manual_seed(7)
    L = torch.nn.LeakyReLU
    seq = ML.sequential(ML.conv(48, 64, 3, 2, 1, "kaiming", L(1e-2), False),
                        ML.ResidualBlock(64, 64, 3, 1, 1, "kaiming", L(1e-2)),
                        ML.ResidualBlock(64, 64, 3, 1, 1, "kaiming", L(1e-2))).to(gpu)
    for m in seq.modules():
        if hasattr(m, "weight") and m.weight is not None and m.weight.dim() == 4:
            m.weight.data = m.weight.data.contiguous(memory_format=torch.channels_last)
    x0 = (torch.rand(4, 48, 24, 24, device=gpu) * 2 - 1).contiguous(memory_format=torch.channels_last)
    res = {}
    for on in (True, False, True):
        tpgan_ops.ACT_LINK["enabled"] = on
        try:
            seq.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_(True)
            with tpgan_ops.compute_dtype(dtype), tpgan_ops.deterministic():
                y = seq(x)
                gy = torch.cos(torch.arange(y.numel(), device=gpu, dtype=torch.float32) * 0.11).reshape(y.shape)
                y.backward(gy.to(y.dtype))
            torch.cuda.synchronize()
            res[on] = [x.grad.float().cpu()] + [p.grad.float().cpu() for p in seq.parameters()]
        finally:
            tpgan_ops.ACT_LINK["enabled"] = True
    for a, b in zip(res[True], res[False]):
        if dtype == torch.float32:
            assert torch.equal(a, b), rel(a, b)
        else:
            assert rel(a, b) < 1e-2, rel(a, b)


def test_link_discriminator_bf16(gpu):
    """The whole Discriminator (stride-2 chain + residual blocks, D_and_G_model.py:409-435) in
    bf16 on a 2B batch: input and parameter gradients with links on vs off."""
    import D_and_G_model as DG
    import tpgan_ops
    torch.manual_seed(3)
    D = DG.Discriminator().to(gpu)
    x0 = torch.rand(4, 3, 128, 128, device=gpu) * 2 - 1
    res = {}
    for on in (True, False, True):
        tpgan_ops.ACT_LINK["enabled"] = on
        try:
            D.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_(True)
            with tpgan_ops.compute_dtype(torch.bfloat16), tpgan_ops.deterministic():
                D(x).float().mean().backward()
            torch.cuda.synchronize()
            res[on] = [x.grad.float().cpu()] + [p.grad.float().cpu() for p in D.parameters()]
        finally:
            tpgan_ops.ACT_LINK["enabled"] = True
    for a, b in zip(res[True], res[False]):
        assert rel(a, b) < 2e-2, rel(a, b)
