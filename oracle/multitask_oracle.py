"""CPU restatement, per point with Python loops, of the reference's SSD landmark pieces
(MobileNetV2.py:252-649): greedy NMS, MultiTaskLoss target assignment + loss, and
MultiTaskDecoder — batch 1, as the reference runs them.

TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT.  Only tests/ may import this module, as the
checker of tp-gan_amd/MobileNetV2.py's batched tensor implementation.  Pinned by the
reference's own known answer (Temp.py: total loss 0.8939134478569031; decoder: class 1,
0.5148 at (370, 150)), see tests/test_multitask.py.  With the repairs R6
(a lone NMS survivor is kept) and R7 (a single background index is one sample); the
random background draw (:505) is not restated: callers keep #background <= the cap.
"""
import math

import torch


def nms(points, scores, threshold):
    """MobileNetV2.py:264-288 / :611-636: kept indices, best first."""
    order = sorted(range(len(scores)), key=lambda i: -float(scores[i]))
    keep = []
    while order:
        i = order[0]
        keep.append(i)
        px, py = float(points[i][0]), float(points[i][1])
        order = [j for j in order[1:]
                 if math.hypot(float(points[j][0]) - px, float(points[j][1]) - py) > threshold]
    return keep


def assign(pred, true, ratio):
    """MobileNetV2.py:372-443 for one image: pred [(x, y)] * n, true [(x, y)] * 4 ->
    (positive index lists per landmark, label per anchor or -1)."""
    n = len(pred)
    d = [[math.hypot(p[0] - t[0], p[1] - t[1]) for t in true] for p in pred]
    k = int(ratio * n)
    pos = []
    for l in range(4):
        col = sorted(d[i][l] for i in range(n))
        thr = max(col[:k])
        pos.append([i for i in range(n) if d[i][l] <= thr])
    best = [math.inf] * n
    label = [-1] * n
    for l in range(4):
        for i in pos[l]:
            if d[i][l] < best[i]:
                best[i] = d[i][l]
                label[i] = l
    lists = [[i for i in range(n) if label[i] == l] for l in range(4)]
    return lists, label


def _log_softmax(row):
    m = max(row)
    s = sum(math.exp(v - m) for v in row)
    return [v - m - math.log(s) for v in row]


def multitask_loss(pred, cls, true, image_size, alpha=30.0, beta=0.1, ratio=0.1, ratio_non_background=5.0):
    """MobileNetV2.py:445-534 for one image (float64 arithmetic)."""
    lists, label = assign(pred, true, ratio)
    h, w = image_size
    clamp = lambda v: min(max(v, 0.0), 1.0)  # noqa: E731
    pn = [(clamp(p[0] / w), clamp(p[1] / h)) for p in pred]
    tn = [(clamp(t[0] / w), clamp(t[1] / h)) for t in true]
    loc = 0.0
    for l, idx in enumerate(lists):
        if idx:
            loc += sum((pn[i][0] - tn[l][0]) ** 2 + (pn[i][1] - tn[l][1]) ** 2 for i in idx) / (2 * len(idx))
    bg = [i for i in range(len(pred)) if label[i] == -1]
    cap = int((len(pred) - len(bg)) * ratio_non_background)
    if len(bg) > cap:
        raise ValueError("background draw (random) not restated: keep #background <= %d" % cap)
    cl = 0.0
    if bg:
        cl += -sum(_log_softmax(cls[i])[4] for i in bg) / len(bg)
    for l, idx in enumerate(lists):
        if idx:
            cl += -sum(_log_softmax(cls[i])[l] for i in idx) / len(idx)
    return alpha * loc + beta * cl


def decode(points, cls, confidence_threshold=0.5, top_k=1, nms_distance_threshold=20):
    """MobileNetV2.py:551-597 for one image: [(class, score, (x, y))]."""
    probs = [[math.exp(v) for v in _log_softmax(row)] for row in cls]
    out = []
    for c in range(len(cls[0])):
        idx = [i for i in range(len(points)) if probs[i][c] > confidence_threshold]
        if not idx:
            continue
        pts = [points[i] for i in idx]
        sc = [probs[i][c] for i in idx]
        keep = nms(pts, sc, nms_distance_threshold)[:top_k]
        out.extend((c, sc[j], pts[j]) for j in keep)
    return out


def as_lists(t):
    return [list(map(float, r)) for r in torch.as_tensor(t).double().tolist()]
