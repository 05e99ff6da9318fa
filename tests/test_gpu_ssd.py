"""GPU: the SSD landmark head on the HIP kernels (tpg_ssd.hip) against the
reference's semantics.

MultiTaskLoss (MobileNetV2.py:342-534) and MultiTaskDecoder (:536-649) run on device tensors
through tpg_ssd_loss_fwd / _bwd / tpg_ssd_decode.  Checked against (a) the per-point loop
restatement oracle/multitask_oracle.py (assignment bit-exact, loss), (b) the Temp.py known
answer, and (c) the tensor form of tp-gan_amd/MobileNetV2.py on the CPU, fed the SAME torch.rand
background keys (the kernels take the caller's keys): labels and background draw identical,
loss and the location / logit gradients (torch autograd of the tensor form) to fp32 rounding."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tp-gan_amd")]

from oracle import multitask_oracle as O  # noqa: E402
from test_multitask import CP, KNOWN_LOSS, LP, LT  # noqa: E402


def _case(seed, B, n, spread=400.0):
    g = torch.Generator().manual_seed(seed)
    pred = torch.rand(B, n, 2, generator=g) * spread
    true = torch.rand(B, 8, generator=g) * spread
    cls = torch.randn(B, n, 5, generator=g) * 2
    return pred, cls, true


def test_ssd_known_answer(gpu):
    import MobileNetV2 as M
    torch.manual_seed(0)
    loss = M.MultiTaskLoss()(LP.to(gpu), CP.to(gpu), LT.to(gpu), (600, 800))
    assert float(loss) == pytest.approx(KNOWN_LOSS, rel=1e-6)
    dec = M.MultiTaskDecoder(nms_distance_threshold=30)(LP.to(gpu), CP.to(gpu))[0]
    assert len(dec) == 1
    c, s, p = dec[0]
    assert c == 1 and round(float(s), 4) == 0.5148 and [float(v) for v in p] == [370.0, 150.0]


@pytest.mark.parametrize("seed,n,ratio", [(1, 12, 0.1), (2, 40, 0.1), (3, 97, 0.25), (4, 394, 0.1), (5, 1540, 0.1)])
def test_ssd_assignment_vs_oracle(gpu, seed, n, ratio):
    import MobileNetV2 as M
    pred, cls, true = _case(seed, 1, n)
    lists, label = O.assign(O.as_lists(pred[0].double()), O.as_lists(true.view(4, 2).double()), ratio)
    m = M.MultiTaskLoss(distance_threshold_ratio=ratio)
    got_lists, got = m.get_positive_samples_and_classification_tensor(pred.to(gpu), true.to(gpu))
    assert got_lists == lists and got[0].cpu().tolist() == label


@pytest.mark.parametrize("seed,B,n,ratio_nb", [(11, 3, 394, 5.0), (12, 2, 1540, 0.5), (13, 4, 97, 1.0),
                                                (14, 1, 40, 5.0)])
def test_ssd_loss_and_grad_vs_tensor_form(gpu, seed, B, n, ratio_nb):
    """Same keys in both forms (torch.rand after the same seed): labels, background draw, loss
    and gradients agree; the draw path (more background than int(#positives * ratio_nb)) is
    exercised by the small ratio_nb cases."""
    import MobileNetV2 as M
    import tpgan_ops
    pred, cls, true = _case(seed, B, n)
    m = M.MultiTaskLoss(distance_threshold_ratio=0.1, ratio_non_background=ratio_nb)
    # tensor form on the CPU with the keys the HIP form draws on the device
    torch.manual_seed(7)
    keys = torch.rand(B, n, device=gpu)
    pc, cc = pred.clone().requires_grad_(True), cls.clone().requires_grad_(True)
    orig_rand = torch.rand
    try:
        torch.rand = lambda *s, **k: keys.cpu() if tuple(s[0] if len(s) == 1 else s) == (B, n) else orig_rand(*s, **k)
        ref = m(pc, cc, true, (480, 640))
    finally:
        torch.rand = orig_rand
    ref.backward()
    ph, ch = pred.to(gpu).requires_grad_(True), cls.to(gpu).requires_grad_(True)
    total, labels, sel, terms = tpgan_ops._SsdLoss.apply(ph, ch, true.to(gpu), keys, 640.0, 480.0, int(0.1 * n),
                                                         ratio_nb, m.alpha, m.beta)
    total.backward()
    torch.cuda.synchronize()
    _, ref_labels = m.get_positive_samples_and_classification_tensor(pred, true)  # (CPU: the tensor form)
    assert torch.equal(labels.cpu(), ref_labels)
    for b in range(B):  # the background draw: all, or int(#positives * ratio_nb) of them
        nbg = int((ref_labels[b] == -1).sum())
        cap = int((n - nbg) * ratio_nb)
        assert int(sel[b].sum()) == (nbg if nbg <= cap else cap)
        assert bool(((sel[b] == 1) <= (labels[b] == -1)).all().item())
    assert float(total) == pytest.approx(float(ref), rel=2e-5, abs=1e-6)
    assert torch.allclose(ph.grad.cpu(), pc.grad, rtol=1e-4, atol=1e-7), float((ph.grad.cpu() - pc.grad).abs().max())
    assert torch.allclose(ch.grad.cpu(), cc.grad, rtol=1e-4, atol=1e-7), float((ch.grad.cpu() - cc.grad).abs().max())


@pytest.mark.parametrize("seed,B,n,top_k,nms", [(21, 2, 394, 1, 20.0), (22, 3, 200, 5, 30.0), (23, 1, 1540, 8, 15.0)])
def test_ssd_decode_vs_oracle(gpu, seed, B, n, top_k, nms):
    import MobileNetV2 as M
    pred, cls, _ = _case(seed, B, n)
    cls = cls * 1.5
    got = M.MultiTaskDecoder(confidence_threshold=0.4, top_k=top_k, nms_distance_threshold=nms)(pred.to(gpu),
                                                                                                 cls.to(gpu))
    for b in range(B):
        want = O.decode(O.as_lists(pred[b].double()), O.as_lists(cls[b].double()), confidence_threshold=0.4,
                        top_k=top_k, nms_distance_threshold=nms)
        assert len(got[b]) == len(want), (b, len(got[b]), len(want))
        for (c, s, p), (wc, ws, wp) in zip(got[b], want):
            assert c == wc and float(s) == pytest.approx(ws, rel=1e-5) and [float(v) for v in p] == pytest.approx(wp)
