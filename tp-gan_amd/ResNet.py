"""ResNet identity-feature extractors, MI355X-native.

ResNet18 keeps the reference's class name, constructor and forward signatures and
attribute names (`/root/reference/ResNet.py:5-126`: conv1, maxpool, sections, avgpool,
[FC0], dropout, FC; forward(x, use_dropout) -> (out, out_FC0)).  The reference cannot
construct or run it, so it is built with these repairs, and its numerics
are PARITY-UNPINNED (no reference output exists to pin them to):

  R4a  conv1: conv(3, 64, 7, 2, 3, "kaiming", activation, use_batchnorm) — the reference
       passes `activation` into the init slot and an unknown bias= keyword (:31)
  R4b  _build_blocks passes (in, out, kernel_size=3, stride) — the reference puts stride in
       the kernel_size slot (:75) — and every block after the first takes `out` channels
  R4c  a block whose channels change gets a projection shortcut (use_projection=True);
       the reference's identity shortcut cannot add 64 to 128 channels
  R4d  resnet18(fm_mult, **kw) is a plain function (the reference's is a self-less method
       passing [2,2,2,2] as num_of_output_classes, :121-126)

ResNet50 is build-defined: BASELINE.json config 3 names a "ResNet-50 identity loss" that
no reference file contains.  It is the standard bottleneck ResNet-50 (7x7/2 stem, 3x3/2
max pool, [3, 4, 6, 3] bottlenecks of expansion 4, projection on the first block of each
stage, stride on the 3x3) with torchvision's state_dict key names, so pretrained
checkpoints in that format load with load_state_dict.

All convs run on libtpgan_hip.so with BatchNorm folded (eval) or as batch statistics
(train), ReLU and the residual add fused into the conv epilogue; the stem max pool and the
global average pool are HIP kernels too.
"""
import copy

import torch
import torch.nn as nn

import tpgan_ops
from ModificationLayer import ResidualBlock, conv, linear


class ResNet18(nn.Module):
    def __init__(self, residualBlock=ResidualBlock, num_of_output_classes=1000, use_batchnorm=True,
                 feature_layer_dim_before_FC=None, activation=nn.ReLU(inplace=True), dropout_rate=0.0):
        super(ResNet18, self).__init__()
        self.use_batchnorm = use_batchnorm
        self.activation = activation
        self.feature_layer_dim_before_FC = feature_layer_dim_before_FC
        num_features = [64, 128, 256, 512]
        num_sections = [2, 2, 2, 2]
        self.conv1 = conv(3, num_features[0], 7, 2, 3, "kaiming", activation, use_batchnorm)  # R4a
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        sections = []
        for idx in range(len(num_sections) - 1):
            sections.append(self._build_blocks(residualBlock, num_features[idx], num_features[idx + 1], 1,
                                               num_sections[idx]))
        self.sections = nn.Sequential(*sections)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        if feature_layer_dim_before_FC is not None:
            self.FC0 = linear(num_features[-1], feature_layer_dim_before_FC, use_batchnorm=use_batchnorm)
        self.dropout = nn.Dropout(dropout_rate)
        fc_in = feature_layer_dim_before_FC if feature_layer_dim_before_FC is not None else num_features[-1]
        self.FC = linear(fc_in, num_of_output_classes, use_batchnorm=False)

    def _build_blocks(self, residualBlock, in_channels, out_channels, stride, num_of_residual_block):
        layers = []
        for i in range(num_of_residual_block):
            cin = in_channels if i == 0 else out_channels  # R4b
            layers.append(residualBlock(cin, out_channels, 3, stride, activation=copy.deepcopy(self.activation),
                                        use_projection=cin != out_channels,  # R4c
                                        use_batchnorm=self.use_batchnorm))
        return nn.Sequential(*layers)

    def _trunk(self, x):
        x = self.conv1(x)
        mp = self.maxpool
        x = tpgan_ops.maxpool2d(x, mp.kernel_size, mp.stride, mp.padding)
        return self.sections(x)

    def forward(self, x, use_dropout=False):
        x = tpgan_ops.global_avgpool(self._trunk(x))
        x = x.reshape(x.size(0), -1)
        out_FC0 = None
        if hasattr(self, "FC0"):
            x = self.FC0(x)
            out_FC0 = x
        if use_dropout:
            x = self.dropout(x)
        if isinstance(self.FC, nn.Linear):  # FeatureExtractModel swaps in a bare Linear (FeatureExtract.py:32)
            return tpgan_ops.linear(x, self.FC.weight, self.FC.bias), out_FC0
        return self.FC(x), out_FC0

    def extract_features(self, x):
        """Identity features [last section map, pooled vector]."""
        m = self._trunk(x)
        return [m, tpgan_ops.global_avgpool(m).reshape(m.size(0), -1)]


def resnet18(fm_mult=1.0, **kwargs):
    """R4d: ResNet18 factory (the reference's feature-map multiplier is not wired into the
    constructor, as in the reference)."""
    return ResNet18(ResidualBlock, **kwargs)


class Bottleneck(nn.Module):
    """1x1 -> 3x3 (stride) -> 1x1 x4 with BN, ReLU; projection shortcut when shapes change."""

    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super(Bottleneck, self).__init__()
        width = planes
        self.conv1 = nn.Conv2d(inplanes, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, planes * self.expansion, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x
        if self.downsample is not None:
            identity = tpgan_ops.conv_bn_act(x, self.downsample[0], self.downsample[1])
        h = tpgan_ops.conv_bn_act(x, self.conv1, self.bn1, act=self.relu)
        h = tpgan_ops.conv_bn_act(h, self.conv2, self.bn2, act=self.relu)
        if self.bn3.training:
            return torch.relu(tpgan_ops.conv_bn_act(h, self.conv3, self.bn3) + identity)
        return tpgan_ops.conv_bn_act(h, self.conv3, self.bn3, act=self.relu, residual=identity)


class ResNet50(nn.Module):
    """Standard ResNet-50 (build-defined; see the module docstring)."""

    def __init__(self, num_of_output_classes=1000, layers=(3, 4, 6, 3), dropout_rate=0.0):
        super(ResNet50, self).__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make_layer(64, layers[0])
        self.layer2 = self._make_layer(128, layers[1], stride=2)
        self.layer3 = self._make_layer(256, layers[2], stride=2)
        self.layer4 = self._make_layer(512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.dropout = nn.Dropout(dropout_rate)
        self.fc = nn.Linear(512 * Bottleneck.expansion, num_of_output_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
                m.weight.data = m.weight.data.contiguous(memory_format=torch.channels_last)
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _make_layer(self, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * Bottleneck.expansion:
            downsample = nn.Sequential(nn.Conv2d(self.inplanes, planes * Bottleneck.expansion, 1, stride, bias=False),
                                       nn.BatchNorm2d(planes * Bottleneck.expansion))
        layers = [Bottleneck(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * Bottleneck.expansion
        for _ in range(1, blocks):
            layers.append(Bottleneck(self.inplanes, planes))
        return nn.Sequential(*layers)

    def _trunk(self, x):
        x = tpgan_ops.conv_bn_act(x, self.conv1, self.bn1, act=self.relu)
        x = tpgan_ops.maxpool2d(x, self.maxpool.kernel_size, self.maxpool.stride, self.maxpool.padding)
        x = self.layer1(x)
        x = self.layer2(x)
        x3 = self.layer3(x)
        return x3, self.layer4(x3)

    def forward(self, x, use_dropout=False):
        """(logits, pooled 2048-d features) — the (out, out_FC0) shape of ResNet18.forward."""
        _, x4 = self._trunk(x)
        feat = tpgan_ops.global_avgpool(x4).reshape(x4.size(0), -1)
        h = self.dropout(feat) if use_dropout else feat
        return tpgan_ops.linear(h, self.fc.weight, self.fc.bias), feat

    def extract_features(self, x):
        """Identity features [layer3 map (1024 ch, H/16), pooled layer4 vector (2048)]."""
        x3, x4 = self._trunk(x)
        return [x3, tpgan_ops.global_avgpool(x4).reshape(x4.size(0), -1)]
