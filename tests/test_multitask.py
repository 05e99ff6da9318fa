"""SSD landmark pretraining pieces (reference MobileNetV2.py:252-649):
tp-gan_amd/MobileNetV2.py's batched MultiTaskLoss / MultiTaskDecoder / NMS against the
reference's known answer (Temp.py) and the per-point loop restatement
oracle/multitask_oracle.py on random cases."""
import os
import sys

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tp-gan_amd")]

from oracle import multitask_oracle as O  # noqa: E402

# Temp.py:8-19
LP = torch.tensor([[[1.0, 1.0], [420.0, 360.0], [370.0, 150.0], [180.0, 220.0], [330.0, 270.0], [290.0, 135.0],
                    [500.0, 380.0], [190.0, 400.0], [210.0, 420.0], [510.0, 70.0], [178.0, 321.0], [420.0, 110.0]]])
LT = torch.tensor([[0.0, 0.0, 150.0, 400.0, 350.0, 250.0, 300.0, 150.0]])
CP = torch.tensor([[[2.0, 1.0, 0.1, 0.5, 1.4], [1.0, 2.0, 0.1, 0.3, 1.1], [0.1, 2.0, 1.0, 0.4, 0.5],
                    [2.0, 0.1, 1.0, 0.7, 0.5], [1.0, 0.1, 1.4, 0.8, 2.0], [0.1, 1.0, 2.0, 0.6, 0.7],
                    [2.0, 1.0, 0.1, 0.9, 1.5], [1.0, 0.8, 0.1, 1.1, 2.0], [0.1, 1.2, 1.0, 2.0, 0.5],
                    [2.0, 0.1, 1.0, 1.3, 0.6], [1.0, 0.1, 2.0, 1.4, 1.6], [0.1, 1.0, 1.3, 1.5, 2.0]]])
KNOWN_LOSS = 0.8939134478569031  # SURVEY.md §4 [probe]: Temp.py's "Total Loss"


def _mods():
    import MobileNetV2 as M
    return M


def _known_answer(dev):
    M = _mods()
    torch.manual_seed(0)
    loss = M.MultiTaskLoss()(LP.to(dev), CP.to(dev), LT.to(dev), (600, 800))
    dec = M.MultiTaskDecoder(nms_distance_threshold=30)(LP.to(dev), CP.to(dev))[0]
    return float(loss), [(c, float(s), [float(v) for v in p]) for c, s, p in dec]


def test_temp_known_answer():
    loss, dec = _known_answer("cpu")
    assert loss == pytest.approx(KNOWN_LOSS, rel=1e-7)
    assert len(dec) == 1
    c, s, p = dec[0]
    assert c == 1 and round(s, 4) == 0.5148 and p == [370.0, 150.0]


def test_oracle_known_answer():
    loss = O.multitask_loss(O.as_lists(LP[0]), O.as_lists(CP[0]), O.as_lists(LT.view(4, 2)), (600, 800))
    assert loss == pytest.approx(KNOWN_LOSS, rel=1e-6)
    (c, s, p), = O.decode(O.as_lists(LP[0]), O.as_lists(CP[0]), nms_distance_threshold=30)
    assert c == 1 and round(s, 4) == 0.5148 and p == [370.0, 150.0]


def _case(seed, n, spread=400.0):
    g = torch.Generator().manual_seed(seed)
    pred = torch.rand(1, n, 2, generator=g, dtype=torch.float64) * spread
    true = torch.rand(1, 8, generator=g, dtype=torch.float64) * spread
    cls = torch.randn(1, n, 5, generator=g, dtype=torch.float64) * 2
    return pred, cls, true


@pytest.mark.parametrize("seed,n,ratio", [(1, 12, 0.1), (2, 40, 0.1), (3, 97, 0.25), (4, 200, 0.1), (5, 31, 0.5)])
def test_loss_vs_oracle(seed, n, ratio):
    M = _mods()
    pred, cls, true = _case(seed, n)
    lists, label = O.assign(O.as_lists(pred[0]), O.as_lists(true.view(4, 2)), ratio)
    nbg = label.count(-1)
    if nbg > int((n - nbg) * 5.0):
        pytest.skip("random background draw")
    ref = O.multitask_loss(O.as_lists(pred[0]), O.as_lists(cls[0]), O.as_lists(true.view(4, 2)), (480, 640),
                           ratio=ratio)
    mine_lists, mine_labels = M.MultiTaskLoss(distance_threshold_ratio=ratio).get_positive_samples_and_classification_tensor(pred, true)
    assert mine_lists == lists and mine_labels[0].tolist() == label
    got = float(M.MultiTaskLoss(distance_threshold_ratio=ratio)(pred, cls, true, (480, 640)))
    assert got == pytest.approx(ref, rel=1e-12, abs=1e-12)


def test_loss_batch_is_mean_of_images():
    M = _mods()
    cases = [_case(s, 50) for s in (11, 12, 13)]
    f = M.MultiTaskLoss()
    each = [float(f(p, c, t, (480, 640))) for p, c, t in cases]
    batched = float(f(torch.cat([c[0] for c in cases]), torch.cat([c[1] for c in cases]),
                      torch.cat([c[2] for c in cases]), (480, 640)))
    assert batched == pytest.approx(sum(each) / 3, rel=1e-12)


def test_background_draw_caps_samples():
    """Many background anchors: a uniform draw without replacement of int(5 x #positives)
    of them enters the background CE (the reference's torch.multinomial over equal weights,
    :501-507).  Checked through the draws' mean and variance against the finite-population
    values of a cap-sized sample."""
    M = _mods()
    n = 400
    pred = torch.rand(1, n, 2, generator=torch.Generator().manual_seed(7), dtype=torch.float64) * 600
    true = torch.tensor([[10.0, 10.0, 12.0, 12.0, 14.0, 14.0, 16.0, 16.0]], dtype=torch.float64)
    f = M.MultiTaskLoss(distance_threshold_ratio=0.01, alpha=0.0, beta=1.0)
    _, labels = f.get_positive_samples_and_classification_tensor(pred, true)
    lab = labels[0].tolist()
    npos = sum(1 for v in lab if v >= 0)
    cap = int(npos * 5.0)
    bgi = [i for i in range(n) if lab[i] < 0]
    assert 0 < cap < len(bgi)
    cls = torch.zeros(1, n, 5, dtype=torch.float64)
    cls[0, :, 0] = torch.arange(n, dtype=torch.float64) / 20  # background CE grows with the index
    logp = torch.log_softmax(cls[0], 1)
    ce_bg = torch.stack([-logp[i, 4] for i in bgi])
    pos_part = 0.0
    for l in range(4):
        idx = [i for i in range(n) if lab[i] == l]
        if idx:
            pos_part += float(torch.stack([-logp[i, l] for i in idx]).mean())
    draws = []
    for s in range(400):
        torch.manual_seed(s)
        draws.append(float(f(pred, cls, true, (600, 600))) - pos_part)
    d = torch.tensor(draws, dtype=torch.float64)
    N = len(bgi)
    var_pop = float(ce_bg.var(unbiased=False))
    var_mean = var_pop / cap * (N - cap) / (N - 1)  # variance of a cap-sized sample mean
    assert abs(float(d.mean()) - float(ce_bg.mean())) < 5 * (var_mean / len(draws)) ** 0.5
    assert 0.7 < float(d.var()) / var_mean < 1.4


def test_nms_vs_oracle():
    M = _mods()
    for seed in range(6):
        g = torch.Generator().manual_seed(100 + seed)
        pts = torch.rand(60, 2, generator=g, dtype=torch.float64) * 100
        sc = torch.rand(60, generator=g, dtype=torch.float64)
        ref = O.nms(O.as_lists(pts), sc.tolist(), 15.0)
        assert M._greedy_nms(pts, sc, 15.0).tolist() == ref
        assert M.MultiTaskDecoder(nms_distance_threshold=15.0).nms(pts, sc).tolist() == ref
        net = M.MobileNetV2.__new__(M.MobileNetV2)
        assert M.MobileNetV2.non_maximum_suppression(net, pts, sc, 15.0) == ref
    # R6: a round with exactly one survivor (the reference's 0-d index) keeps it
    pts = torch.tensor([[0.0, 0.0], [100.0, 0.0], [1.0, 0.0]])
    assert M._greedy_nms(pts, torch.tensor([0.9, 0.5, 0.8]), 5.0).tolist() == [0, 1]


@pytest.mark.parametrize("top_k", [1, 3])
def test_decoder_vs_oracle(top_k):
    M = _mods()
    for seed in range(4):
        pred, cls, _ = _case(200 + seed, 80)
        cls = cls * 2
        ref = O.decode(O.as_lists(pred[0]), O.as_lists(cls[0]), confidence_threshold=0.5, top_k=top_k,
                       nms_distance_threshold=40)
        got = M.MultiTaskDecoder(top_k=top_k, nms_distance_threshold=40)(pred, cls)[0]
        assert [(c, round(float(s), 12), [float(v) for v in p]) for c, s, p in got] == \
            [(c, round(s, 12), p) for c, s, p in ref]


def test_find_best_coordinates():
    M = _mods()
    g = torch.Generator().manual_seed(9)
    loc = torch.rand(1, 50, 10, generator=g, dtype=torch.float64) * 200
    cls = torch.rand(1, 50, 5, generator=g, dtype=torch.float64)
    net = M.MobileNetV2.__new__(M.MobileNetV2)
    out = M.MobileNetV2.find_best_coordinates(net, loc, cls, 15.0)
    for j, name in enumerate(("lefteye", "righteye", "nose", "leftmouth", "rightmouth")):
        keep = O.nms(O.as_lists(loc[0, :, 2 * j:2 * j + 2]), cls[0, :, j].tolist(), 15.0)
        assert torch.allclose(out[name], loc[0, keep, 2 * j:2 * j + 2].mean(0))


@pytest.mark.gpu
def test_known_answer_on_gpu(gpu):
    loss, dec = _known_answer(gpu)
    assert loss == pytest.approx(KNOWN_LOSS, rel=1e-6)
    c, s, p = dec[0]
    assert len(dec) == 1 and c == 1 and round(s, 4) == 0.5148 and p == [370.0, 150.0]
