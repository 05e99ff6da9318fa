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

The SSD landmark loss / decoder (MultiTaskLoss, MultiTaskDecoder, :342-649) belong to the
landmark pretraining loop and are not part of this module yet.
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
