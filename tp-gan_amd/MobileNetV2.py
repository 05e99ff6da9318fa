"""MobileNetV2 + SSD head (reference MobileNetV2.py:10-249), MI355X-native.

Class names, constructor / forward signatures, return tuples and state_dict keys are the
reference's.  Every conv runs on libtpgan_hip.so: the 1x1 expand / project and dense 3x3
convs on the MFMA conv family (tpgan_ops.conv2d), the depthwise 3x3 on tpg_dwconv2d, and
BatchNorm either folded into the conv (eval mode: one fused launch of conv + BN + ReLU6
[+ residual]) or as batch statistics with the activation fused (train mode).

Besides the reference API, `extract_features(x)` returns the identity features the
TP-GAN identity-preserving loss uses (a build choice: the reference
defines none): the input of the first SSD scale (bottleneck 12, 96 ch at H/16) and the
conv2 output (1280 ch at H/32), MobileNetV2.py:200-206.

The SSD landmark pretraining pieces are at the end: the model's
non_maximum_suppression / find_best_coordinates (:252-340) and MultiTaskLoss /
MultiTaskDecoder (:342-649), batched tensor ops on the predictions' device.
"""
import math

import torch
import torch.nn as nn

import tpgan_ops


class SSDHead(nn.Module):
    """Per-scale 3x3 location / classification convs (MobileNetV2.py:10-79)."""

    IN_CHANNELS = (96, 1280, 512, 256, 256, 128)
    ANCHORS = (4, 6, 6, 6, 6, 6)

    def __init__(self, num_of_out_classes=4):
        super(SSDHead, self).__init__()
        self.num_of_out_classes = num_of_out_classes
        self.num_of_out_location = 2
        self.location_layer = nn.ModuleList()
        self.classification_layer = nn.ModuleList()
        for cin, a in zip(self.IN_CHANNELS, self.ANCHORS):
            self.location_layer += [nn.Conv2d(cin, a * self.num_of_out_location, kernel_size=3, padding=1)]
            self.classification_layer += [nn.Conv2d(cin, a * self.num_of_out_classes, kernel_size=3, padding=1)]

    def forward(self, features):
        locations, classifications = [], []
        for idx, x in enumerate(features):
            loc = tpgan_ops.conv_bn_act(x, self.location_layer[idx], None, act=nn.ReLU())  # torch.relu (:64)
            loc = loc.permute(0, 2, 3, 1).contiguous()
            locations.append(loc.view(loc.size(0), -1, self.num_of_out_location))
            cls = tpgan_ops.conv_bn_act(x, self.classification_layer[idx], None)
            cls = cls.permute(0, 2, 3, 1).contiguous()
            classifications.append(cls.view(cls.size(0), -1, self.num_of_out_classes))
        return torch.cat(locations, 1), torch.cat(classifications, 1)


class InvertedResidual(nn.Module):
    """1x1 expand + BN + ReLU6, 3x3 depthwise + BN + ReLU6, 1x1 project + BN, identity
    shortcut when stride 1 and inp == oup (MobileNetV2.py:81-120).  The shortcut add is
    fused into the project conv's epilogue."""

    def __init__(self, inp, oup, stride=1, expand_ratio=6):
        super(InvertedResidual, self).__init__()
        self.stride = stride
        self.use_res_connect = self.stride == 1 and inp == oup
        hid = inp * expand_ratio
        self.conv = nn.Sequential(
            nn.Conv2d(inp, hid, 1, 1, 0, bias=False),
            nn.BatchNorm2d(hid),
            nn.ReLU6(inplace=True),
            nn.Conv2d(hid, hid, 3, stride, 1, groups=hid, bias=False),
            nn.BatchNorm2d(hid),
            nn.ReLU6(inplace=True),
            nn.Conv2d(hid, oup, 1, 1, 0, bias=False),
            nn.BatchNorm2d(oup),
        )

    def forward(self, x):
        c = self.conv
        h = tpgan_ops.conv_bn_act(x, c[0], c[1], act=c[2])
        h = tpgan_ops.conv_bn_act(h, c[3], c[4], act=c[5])
        if self.use_res_connect:
            if c[7].training:  # batch-statistics BN cannot take the residual in its epilogue
                return x + tpgan_ops.conv_bn_act(h, c[6], c[7])
            return tpgan_ops.conv_bn_act(h, c[6], c[7], residual=x)
        return tpgan_ops.conv_bn_act(h, c[6], c[7])


class MobileNetV2(nn.Module):
    """Backbone (17 inverted residuals) + extra layers + SSD head (MobileNetV2.py:122-249)."""

    def __init__(self):
        super(MobileNetV2, self).__init__()
        self.interverted_residual_setting = [
            [1, 16, 1, 1],
            [6, 24, 2, 2],
            [6, 32, 3, 2],
            [6, 64, 4, 2],
            [6, 96, 3, 1],
            [6, 160, 3, 2],
            [6, 320, 1, 1],
        ]
        self.conv1 = nn.Sequential(nn.Conv2d(3, 32, 3, 2, 1, bias=False), nn.BatchNorm2d(32), nn.ReLU6(inplace=True))
        input_channel = 32
        self.bottlenecks = nn.ModuleList()
        for t, c, n, s in self.interverted_residual_setting:
            for idx in range(n):
                self.bottlenecks.append(InvertedResidual(input_channel, c, s if idx == 0 else 1, t))
                input_channel = c
        self.conv2 = nn.Sequential(nn.Conv2d(320, 1280, 1, 1, 0, bias=False), nn.BatchNorm2d(1280),
                                   nn.ReLU6(inplace=True))
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.ssd_head = SSDHead(4 + 1)
        self.extra_layers = nn.ModuleList([
            nn.Conv2d(1280, 512, kernel_size=1),
            nn.Conv2d(512, 512, kernel_size=3, stride=2, padding=1),
            nn.Conv2d(512, 256, kernel_size=1),
            nn.Conv2d(256, 256, kernel_size=3, stride=2, padding=1),
            nn.Conv2d(256, 256, kernel_size=3, stride=2, padding=1),
            nn.Conv2d(256, 128, kernel_size=1),
            nn.Conv2d(128, 128, kernel_size=3, stride=2, padding=1),
        ])
        self._initialize_weights()
        for m in self.modules():  # channels-last master weights (the conv kernels' native layout)
            if isinstance(m, nn.Conv2d) and m.groups == 1:
                m.weight.data = m.weight.data.contiguous(memory_format=torch.channels_last)

    def _backbone(self, x, stop_after_conv2=False):
        features = []
        x = tpgan_ops.conv_bn_act(x, self.conv1[0], self.conv1[1], act=self.conv1[2])
        for idx, bottleneck in enumerate(self.bottlenecks):
            x = bottleneck(x)
            if idx == 12:
                features.append(x)
        x = tpgan_ops.conv_bn_act(x, self.conv2[0], self.conv2[1], act=self.conv2[2])
        features.append(x)
        return x, features

    def forward(self, x, use_dropout=False):
        """(locations (B, N, 2), classifications (B, N, 5)) as MobileNetV2.py:189-218."""
        x, features = self._backbone(x)
        for idx, extra_layer in enumerate(self.extra_layers):
            x = tpgan_ops.conv_bn_act(x, extra_layer, None)
            if idx in (1, 3, 4, 6):
                features.append(x)
        return self.ssd_head(features)

    def extract_features(self, x):
        """Identity features [bottleneck-12 output (96 ch, H/16), conv2 output (1280 ch, H/32)]."""
        return self._backbone(x)[1]

    def _initialize_weights(self):
        """MobileNetV2.py:220-249 (He normal over k*k*out for convs, BN to (1, 0))."""
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                n = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                m.weight.data.normal_(0, math.sqrt(2. / n))
                if m.bias is not None:
                    m.bias.data.zero_()
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()
            elif isinstance(m, nn.Linear):
                n = m.weight.size(1)
                m.weight.data.normal_(0, 0.01)
                m.bias.data.zero_()


# ---- SSD landmark pretraining: NMS, target assignment loss and decoder ----
# The reference (MobileNetV2.py:252-649) works on batch 1 with Python loops and .item() per
# point.  Here every step is a tensor op on the predictions' device over the whole batch:
# the distance matrix, per-landmark top-k thresholds and the nearest-landmark assignment of
# each anchor are masks, the losses are masked sums; only greedy NMS keeps a loop, one
# iteration per KEPT point (argmax of the remaining scores, then a vector suppression).
# Repairs of reference crashes (numbered after SURVEY.md §0.6's R1-R5):
#   R6  non_maximum_suppression (:285-286) indexes a 0-d tensor once exactly one point
#       survives a round (IndexError); here the lone survivor is simply kept.
#   R7  MultiTaskLoss (:507-510) squeezes a single background index to an int: index 0
#       is then skipped and any other single index raises; here it is one background sample.


def _greedy_nms(points, scores, threshold, max_keep=None):
    """Indices of `points` kept by greedy NMS, highest score first: take the best remaining
    point, drop every remaining point within `threshold` (Euclidean, <=), repeat."""
    keep = []
    if points.numel() == 0:
        return torch.zeros(0, dtype=torch.long, device=points.device)
    alive = torch.ones(points.shape[0], dtype=torch.bool, device=points.device)
    neg = torch.finfo(scores.dtype).min
    while bool(alive.any()) and (max_keep is None or len(keep) < max_keep):
        i = torch.where(alive, scores, torch.full_like(scores, neg)).argmax()
        keep.append(i)
        d = torch.linalg.vector_norm(points - points[i], dim=1)
        alive &= d > threshold
        alive[i] = False
    return torch.stack(keep) if keep else torch.zeros(0, dtype=torch.long, device=points.device)


def _mnv2_nms(self, points, scores, distance_threshold):
    """MobileNetV2.non_maximum_suppression (:252-288): kept indices (list), best first (R6)."""
    if points.numel() == 0:
        return []
    return [int(i) for i in _greedy_nms(points, scores, distance_threshold)]


def _mnv2_best_coordinates(self, locations, classifications, distance_threshold=15.0):
    """MobileNetV2.find_best_coordinates (:290-340): per landmark, the mean of the NMS
    survivors of batch element 0 (locations (B, N, 10), classifications (B, N, 5))."""
    names = ("lefteye", "righteye", "nose", "leftmouth", "rightmouth")
    out = {}
    for j, name in enumerate(names):
        pts = locations[0, :, 2 * j:2 * j + 2]
        keep = _greedy_nms(pts, classifications[0, :, j], distance_threshold)
        out[name] = pts[keep].mean(dim=0)
    return out


MobileNetV2.non_maximum_suppression = _mnv2_nms
MobileNetV2.find_best_coordinates = _mnv2_best_coordinates


class MultiTaskLoss(nn.Module):
    """SSD landmark loss (MobileNetV2.py:342-534): alpha * location MSE + beta * class CE.

    Target assignment per image: d = cdist(anchors, 4 landmarks); landmark l's positives are
    the anchors with d <= the k-th smallest distance to l (k = int(ratio * n)); an anchor
    positive for several landmarks takes the nearest (the first on ties), the rest are
    background (class 4).  Location loss: per landmark, the MSE between its positives and
    the landmark, both divided by (width, height) and clamped to [0, 1]; class loss: CE of
    the background samples (at most ratio_non_background x #positives, drawn uniformly
    without replacement when there are more) plus, per landmark, CE of its positives.  The
    reference takes batch 1; a batch here is the mean of the per-image losses.  `verbose`
    prints the reference's per-term lines (:488, 516, 527).

    Device tensors (fp32, <= 4096 anchors) run the HIP kernels (tpg_ssd_loss_fwd / _bwd: one
    block per image does the assignment, the background draw from the same torch.rand keys as
    the tensor form below, and the loss terms); CPU tensors -- the reference's own device in
    Pretrain.py on a host without a GPU, and Temp.py -- keep the tensor form."""

    def __init__(self, alpha=None, beta=None, distance_threshold_ratio=0.1, ratio_non_background=None,
                 verbose=False):
        super(MultiTaskLoss, self).__init__()
        from config import pretrain
        self.alpha = pretrain["loss"]["alpha"] if alpha is None else alpha
        self.beta = pretrain["loss"]["beta"] if beta is None else beta
        self.distance_threshold_ratio = distance_threshold_ratio
        self.ratio_non_background = (pretrain["loss"]["ratio_non_background"] if ratio_non_background is None
                                     else ratio_non_background)
        self.verbose = verbose

    def _hip(self, locations_pred):
        # (float64 device tensors keep the tensor form: the kernels compute in fp32)
        return locations_pred.is_cuda and locations_pred.shape[1] <= 4096 and locations_pred.dtype != torch.float64

    def get_positive_samples_and_classification_tensor(self, locations_pred, locations_true):
        """(positive index lists per landmark of image 0, labels (B, n) int: landmark or -1)."""
        B, n, _ = locations_pred.shape
        if self._hip(locations_pred):
            C = 5
            cls0 = torch.zeros(B, n, C, device=locations_pred.device)
            keys = torch.zeros(B, n, device=locations_pred.device)  # (no draw: only the labels are used)
            with torch.no_grad():
                k = int(self.distance_threshold_ratio * n)
                if k < 1:
                    raise ValueError("distance_threshold_ratio * anchors < 1: no positives can be chosen")
                _, labels, _, _ = tpgan_ops._SsdLoss.apply(locations_pred.detach(), cls0, locations_true, keys, 1.0, 1.0,
                                                           k, self.ratio_non_background, self.alpha, self.beta)
            lists = [torch.nonzero(labels[0] == l).flatten().tolist() for l in range(4)]
            return lists, labels
        true = locations_true.reshape(B, 4, 2).to(locations_pred.dtype)
        d = torch.cdist(locations_pred, true, p=2)                       # (B, n, 4)
        k = int(self.distance_threshold_ratio * n)
        if k < 1:
            raise ValueError("distance_threshold_ratio * anchors < 1: no positives can be chosen")
        thr = d.topk(k, dim=1, largest=False)[0].amax(dim=1, keepdim=True)  # (B, 1, 4)
        pos = d <= thr
        dm = torch.where(pos, d, torch.full_like(d, float("inf")))
        labels = torch.where(pos.any(dim=2), dm.argmin(dim=2), torch.full_like(dm[..., 0], -1, dtype=torch.long))
        lists = [torch.nonzero(labels[0] == l).flatten().tolist() for l in range(4)]
        return lists, labels.to(torch.int32)

    def forward(self, locations_pred, classifications_pred, locations_true, image_size):
        B, n, _ = locations_pred.shape
        if self._hip(locations_pred):
            total, labels, sel, terms = tpgan_ops.ssd_loss(locations_pred, classifications_pred, locations_true,
                                                           image_size, self.distance_threshold_ratio,
                                                           self.ratio_non_background, self.alpha, self.beta)
            if self.verbose:
                t = terms[0].tolist()
                for l in range(4):
                    if t[11 + l] > 0:
                        print("location loss %d               : %.4f * %s = %.4f" % (l, t[1 + l], self.alpha,
                                                                                     t[1 + l] * self.alpha))
                if t[10] > 0:
                    print("background classification loss: %.4f * %s = %.4f" % (t[9], self.beta, t[9] * self.beta))
                for l in range(4):
                    if t[11 + l] > 0:
                        print("classification loss %d         : %.4f * %s = %.4f" % (l, t[5 + l], self.beta,
                                                                                     t[5 + l] * self.beta))
            return total.to(locations_pred.dtype)
        _, labels = self.get_positive_samples_and_classification_tensor(locations_pred, locations_true)
        labels = labels.long()
        height, width = image_size
        size = torch.tensor([width, height], device=locations_pred.device, dtype=locations_pred.dtype)
        pred = torch.clamp(locations_pred / size, 0, 1)
        true = torch.clamp(locations_true.reshape(B, 4, 2).to(locations_pred.dtype) / size, 0, 1)
        onehot = labels.unsqueeze(2) == torch.arange(4, device=labels.device)       # (B, n, 4)
        cnt = onehot.sum(dim=1)                                                      # (B, 4)
        se = ((pred.unsqueeze(2) - true.unsqueeze(1)) ** 2).sum(dim=3)               # (B, n, 4)
        present = cnt > 0
        loc_l = torch.where(present, (se * onehot).sum(dim=1) / (2 * cnt.clamp(min=1)), torch.zeros_like(se[:, 0]))
        # background: all of them, or a uniform draw without replacement of
        # int(ratio * #positives) when there are more (random keys ranked among the background)
        bg = labels == -1
        nbg = bg.sum(dim=1, keepdim=True)
        cap = ((n - nbg).to(torch.float64) * self.ratio_non_background).floor().long()
        keys = torch.where(bg, torch.rand(bg.shape, device=bg.device), torch.full(bg.shape, 2.0, device=bg.device))
        rank = keys.argsort(dim=1).argsort(dim=1)
        sel = bg & ((nbg <= cap) | (rank < cap))
        cp = classifications_pred if classifications_pred.dtype in (torch.float32, torch.float64) \
            else classifications_pred.float()
        logp = torch.log_softmax(cp, dim=2)                                          # (B, n, C)
        nsel = sel.sum(dim=1)
        cls_bg = torch.where(nsel > 0, -(logp[..., 4] * sel).sum(dim=1) / nsel.clamp(min=1), torch.zeros_like(nsel,
                                                                                                       dtype=logp.dtype))
        ce_l = -(logp[..., :4] * onehot).sum(dim=1)                                  # (B, 4)
        cls_l = torch.where(present, ce_l / cnt.clamp(min=1), torch.zeros_like(ce_l))
        loc = loc_l.sum(dim=1)
        cls = cls_bg + cls_l.sum(dim=1)
        if self.verbose:
            for l in range(4):
                if bool(present[0, l]):
                    print("location loss %d               : %.4f * %s = %.4f" % (l, float(loc_l[0, l]), self.alpha,
                                                                                 float(loc_l[0, l]) * self.alpha))
            if int(nsel[0]):
                print("background classification loss: %.4f * %s = %.4f" % (float(cls_bg[0]), self.beta,
                                                                            float(cls_bg[0]) * self.beta))
            for l in range(4):
                if bool(present[0, l]):
                    print("classification loss %d         : %.4f * %s = %.4f" % (l, float(cls_l[0, l]), self.beta,
                                                                                 float(cls_l[0, l]) * self.beta))
        total = self.alpha * loc + self.beta * cls.to(loc.dtype)
        return total.mean()


class MultiTaskDecoder(nn.Module):
    """SSD landmark decoder (MobileNetV2.py:536-649): per image and class, the anchors whose
    softmax confidence exceeds confidence_threshold, greedy NMS at nms_distance_threshold
    pixels, at most top_k of them; a list per image of (class, score, point) tuples."""

    def __init__(self, confidence_threshold=0.5, top_k=1, nms_distance_threshold=20):
        super(MultiTaskDecoder, self).__init__()
        self.confidence_threshold = confidence_threshold
        self.top_k = top_k
        self.nms_distance_threshold = nms_distance_threshold

    def forward(self, locations, classifications):
        if (locations.is_cuda and locations.shape[1] <= 4096 and classifications.shape[2] >= 5 and
                locations.dtype != torch.float64):
            # (tpg_ssd_decode: one block per image and class; the kept points in score order)
            keep, score = tpgan_ops.ssd_decode(locations, classifications, self.confidence_threshold,
                                               self.nms_distance_threshold, self.top_k)
            keep, score = keep.cpu(), score.cpu()
            output = []
            for i in range(locations.shape[0]):
                results = []
                for c in range(classifications.shape[2]):
                    for r in range(self.top_k):
                        j = int(keep[i, c, r])
                        if j < 0:
                            break
                        results.append((c, score[i, c, r].to(locations.device), locations[i, j]))
                output.append(results)
            return output
        scores = torch.softmax(classifications, dim=-1)
        output = []
        for i in range(locations.shape[0]):
            results = []
            for c in range(scores.shape[2]):
                s = scores[i, :, c]
                mask = s > self.confidence_threshold
                if not bool(mask.any()):
                    continue
                pts, sc = locations[i][mask], s[mask]
                keep = _greedy_nms(pts, sc, self.nms_distance_threshold, max_keep=self.top_k)
                for j in keep:
                    results.append((c, sc[j], pts[j]))
            output.append(results)
        return output

    def nms(self, locations, scores):
        """Kept indices (tensor), best first (MobileNetV2.py:599-636)."""
        return _greedy_nms(locations, scores, self.nms_distance_threshold).cpu()

    def euclidean_distance(self, point1, points2):
        return torch.linalg.vector_norm(points2 - point1, dim=1)
