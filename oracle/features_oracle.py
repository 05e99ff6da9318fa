"""CPU restatement of the identity-feature extractors (functional, aten CPU ops).

TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT.  Only tests/ (and bench.py's cpu_baseline
leg) may use it, as the checker.

* mobilenet_v2(P, x, training) follows MobileNetV2.py:122-218 (+ SSDHead :10-79,
  InvertedResidual :81-120) and is pinned against tests/golden/features_golden.npz, which
  was produced by running the reference itself (tests/golden/make_golden_features.py).
* resnet50(P, x, training) restates the standard bottleneck ResNet-50 the build defines
  for BASELINE.json config 3 (no reference source exists: parity unpinned; it checks the
  HIP kernels against aten on the same architecture).
* resnet18_r4(P, x, training) restates the repaired reference ResNet18 (ResNet.py with
  R4a-d, see tp-gan_amd/ResNet.py): parity unpinned for the same reason.

P is a dict of tensors keyed by state_dict keys; BatchNorm in training mode uses batch
statistics and updates P's running statistics in place (momentum 0.1), as nn.BatchNorm2d.
"""
import torch
import torch.nn.functional as F

MNV2_SETTING = [[1, 16, 1, 1], [6, 24, 2, 2], [6, 32, 3, 2], [6, 64, 4, 2], [6, 96, 3, 1], [6, 160, 3, 2],
                [6, 320, 1, 1]]  # MobileNetV2.py:136-145


def _bn(P, key, x, training):
    return F.batch_norm(x, P[key + "running_mean"], P[key + "running_var"], P[key + "weight"], P[key + "bias"],
                        training=training, momentum=0.1, eps=1e-5)


def _relu6(x):
    return F.hardtanh(x, 0.0, 6.0)


def mobilenet_v2_backbone(P, x, training=False):
    """conv1 -> 17 inverted residuals -> conv2 (MobileNetV2.py:189-206); returns (x, features)."""
    x = _relu6(_bn(P, "conv1.1.", F.conv2d(x, P["conv1.0.weight"], None, 2, 1), training))
    features = []
    inp, idx = 32, 0
    for t, c, n, s in MNV2_SETTING:
        for i in range(n):
            stride = s if i == 0 else 1
            pre = "bottlenecks.%d.conv." % idx
            hid = inp * t
            h = _relu6(_bn(P, pre + "1.", F.conv2d(x, P[pre + "0.weight"]), training))
            h = _relu6(_bn(P, pre + "4.", F.conv2d(h, P[pre + "3.weight"], None, stride, 1, groups=hid), training))
            h = _bn(P, pre + "7.", F.conv2d(h, P[pre + "6.weight"]), training)
            x = x + h if (stride == 1 and inp == c) else h  # :117-120
            if idx == 12:
                features.append(x)
            inp = c
            idx += 1
    x = _relu6(_bn(P, "conv2.1.", F.conv2d(x, P["conv2.0.weight"]), training))
    features.append(x)
    return x, features


def mobilenet_v2(P, x, training=False):
    """(locations, classifications, features) of MobileNetV2.forward (:189-218)."""
    x, features = mobilenet_v2_backbone(P, x, training)
    extras = [(0, 1, 0), (1, 2, 1), (2, 1, 0), (3, 2, 1), (4, 2, 1), (5, 1, 0), (6, 2, 1)]  # :177-185
    for i, s, p in extras:
        x = F.conv2d(x, P["extra_layers.%d.weight" % i], P["extra_layers.%d.bias" % i], s, p)
        if i in (1, 3, 4, 6):
            features.append(x)
    locs, clss = [], []
    for i, f in enumerate(features):  # SSDHead.forward :56-79
        loc = F.conv2d(f, P["ssd_head.location_layer.%d.weight" % i], P["ssd_head.location_layer.%d.bias" % i], 1, 1)
        loc = torch.relu(loc.permute(0, 2, 3, 1).reshape(f.shape[0], -1, 2))
        cls = F.conv2d(f, P["ssd_head.classification_layer.%d.weight" % i],
                       P["ssd_head.classification_layer.%d.bias" % i], 1, 1)
        locs.append(loc)
        clss.append(cls.permute(0, 2, 3, 1).reshape(f.shape[0], -1, 5))
    return torch.cat(locs, 1), torch.cat(clss, 1), features[:2]


def resnet50_trunk(P, x, training=False):
    """Standard ResNet-50 trunk: (layer3 output, layer4 output)."""
    x = F.relu(_bn(P, "bn1.", F.conv2d(x, P["conv1.weight"], None, 2, 3), training))
    x = F.max_pool2d(x, 3, 2, 1)
    outs = []
    for li, (planes, blocks, stride) in enumerate(((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2))):
        for b in range(blocks):
            pre = "layer%d.%d." % (li + 1, b)
            s = stride if b == 0 else 1
            idt = x
            if pre + "downsample.0.weight" in P:
                idt = _bn(P, pre + "downsample.1.", F.conv2d(x, P[pre + "downsample.0.weight"], None, s), training)
            h = F.relu(_bn(P, pre + "bn1.", F.conv2d(x, P[pre + "conv1.weight"]), training))
            h = F.relu(_bn(P, pre + "bn2.", F.conv2d(h, P[pre + "conv2.weight"], None, s, 1), training))
            h = _bn(P, pre + "bn3.", F.conv2d(h, P[pre + "conv3.weight"]), training)
            x = F.relu(h + idt)
        outs.append(x)
    return outs[2], outs[3]


def resnet50(P, x, training=False):
    """(logits, pooled features, [layer3, pooled]) of ResNet.ResNet50."""
    x3, x4 = resnet50_trunk(P, x, training)
    feat = x4.mean((2, 3))
    return F.linear(feat, P["fc.weight"], P["fc.bias"]), feat, [x3, feat]


def resnet18_r4(P, x, training=False):
    """Repaired reference ResNet18 trunk (ResNet.py:20-53 with R4a-d): conv1 7x7/2 + BN + ReLU,
    max pool 3/2, three sections of two ModificationLayer.ResidualBlocks (3x3, stride 1,
    projection shortcut without BN when the channels change), global average pool, FC."""
    x = F.relu(_bn(P, "conv1.1.", F.conv2d(x, P["conv1.0.weight"], None, 2, 3), training))
    x = F.max_pool2d(x, 3, 2, 1)
    for s in range(3):
        for b in range(2):
            pre = "sections.%d.%d." % (s, b)
            short = x
            if pre + "shortcut.0.weight" in P:
                short = F.conv2d(x, P[pre + "shortcut.0.weight"], P[pre + "shortcut.0.bias"])
            h = F.relu(_bn(P, pre + "layers.0.1.", F.conv2d(x, P[pre + "layers.0.0.weight"], None, 1, 1), training))
            h = _bn(P, pre + "layers.1.1.", F.conv2d(h, P[pre + "layers.1.0.weight"], None, 1, 1), training)
            x = F.relu(h + short)
    feat = x.mean((2, 3))
    return x, feat
