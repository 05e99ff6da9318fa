"""GPU: the fused G-step losses (tpg_losses.hip via tpgan_ops.image_losses / l1_means) against
their torch fp64 restatement on the CPU -- the same formulas tpgan_train._g_losses computed with
aten before (build-defined; weights config.py:59-82): values, gradients,
16-bit channels-last inputs with padded pixel rows, odd widths and one-row maps, and
bit-identical reruns (fixed-order reductions)."""
import pytest
import torch

from _cases import rel

pytestmark = pytest.mark.gpu


def _img_ref(x, r, wp, ws, wt):
    tv = (x[:, :, 1:, :] - x[:, :, :-1, :]).abs().mean() if x.shape[2] > 1 else x.new_zeros(())
    tv = tv + ((x[:, :, :, 1:] - x[:, :, :, :-1]).abs().mean() if x.shape[3] > 1 else x.new_zeros(()))
    return wp * (x - r).abs().mean() + ws * (x - x.flip(3)).abs().mean() + wt * tv


def _dev_input(x64, dtype, gpu, cl):
    t = x64.to(dtype).to(gpu)
    if cl:  # the conv output layout: channels last, pixel rows padded to 8 channels
        import tpgan_ops
        n, c, h, w = t.shape
        b = tpgan_ops.new_act(n, c, h, w, dtype, gpu)
        b.copy_(t)
        t = b
    return t


@pytest.mark.parametrize("shape", [(4, 3, 32, 32), (2, 3, 17, 13), (3, 2, 1, 9)], ids=["32", "odd", "1row"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_image_losses(gpu, shape, dtype):
    import tpgan_ops
    g = torch.Generator().manual_seed(11)
    x64 = torch.rand(shape, generator=g, dtype=torch.float64) * 2 - 1
    r64 = torch.rand(shape, generator=g, dtype=torch.float64) * 2 - 1
    wp, ws, wt = 1.7, 0.3, 1e-3
    x = _dev_input(x64, dtype, gpu, dtype != torch.float32).requires_grad_(True)
    r = r64.float().to(gpu)
    y = tpgan_ops.image_losses(x, r, wp, ws, wt)
    (y * 2.5).backward()
    xr = x.detach().double().cpu().requires_grad_(True)  # the same (rounded) input values
    yr = _img_ref(xr, r64.float().double(), wp, ws, wt)
    (yr * 2.5).backward()
    assert abs(y.item() - yr.item()) <= 1e-5 * abs(yr.item())
    assert rel(x.grad.double().cpu(), xr.grad) < (1e-6 if dtype == torch.float32 else 1e-2)
    y2 = tpgan_ops.image_losses(x.detach(), r, wp, ws, wt)
    assert torch.equal(y.detach(), y2)  # fixed-order reduction


def test_l1_means(gpu):
    import tpgan_ops
    g = torch.Generator().manual_seed(5)
    shapes = [(4, 3, 40, 40), (4, 3, 40, 40), (4, 3, 32, 40), (4, 3, 32, 48)]
    pairs, refs = [], []
    for s in shapes:
        a64 = torch.rand(s, generator=g, dtype=torch.float64) * 2 - 1
        b64 = torch.rand(s, generator=g, dtype=torch.float64) * 2 - 1
        a = _dev_input(a64, torch.bfloat16, gpu, True).requires_grad_(True)
        pairs.append((a, b64.float().to(gpu)))
        refs.append((a.detach().double().cpu().requires_grad_(True), b64.float().double()))
    wts = [0.25, 0.5, 0.75, 1.0]
    y = tpgan_ops.l1_means(pairs, wts)
    y.backward()
    yr = sum(w * (a - b).abs().mean() for w, (a, b) in zip(wts, refs))
    yr.backward()
    assert abs(y.item() - yr.item()) <= 1e-5 * abs(yr.item())
    for (a, _), (ar, _) in zip(pairs, refs):
        assert rel(a.grad.double().cpu(), ar.grad) < 1e-2
