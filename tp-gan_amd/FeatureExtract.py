"""Identity-feature extractor wrapper (reference FeatureExtract.py:5-41), MI355X-native,
and the TP-GAN identity-preserving loss built on it.

FeatureExtractModel keeps the reference's constructor and forward.  The reference crashes
for both back-ends (ResNet18 cannot be built; MobileNetV2 has no `FC`
attribute for :35 to read); here:
  'resnet'      -> ResNet.ResNet18 (repairs R4, see ResNet.py), FC replaced by
                   nn.Linear(in_features, num_of_output_classes) as :32-33
  'resnet50'    -> ResNet.ResNet50 (build-defined, BASELINE.json config 3)
  'mobilenetv2' -> MobileNetV2.MobileNetV2; R5: the classifier of :36-39
                   (Dropout(0.2), Linear(1280, classes)) is attached as `FC` and applied
                   to the average-pooled conv2 features by classify(); forward() is the
                   backbone's own forward, as in the reference.
`use_pretrained` is accepted and unused, as in the reference (no weights are fetched).
"""
import torch
import torch.nn as nn

import tpgan_ops
from MobileNetV2 import MobileNetV2
from ResNet import ResNet18, ResNet50


class FeatureExtractModel(nn.Module):
    def __init__(self, base_model_name="resnet", num_of_output_classes=1000, use_pretrained=False, **kwargs):
        super(FeatureExtractModel, self).__init__()
        self.base_model_name = base_model_name.lower()
        self.num_of_output_classes = num_of_output_classes
        if self.base_model_name == "resnet":
            self.base_model = ResNet18(**kwargs)
            in_features = self.base_model.FC[0].in_features
            self.base_model.FC = nn.Linear(in_features, num_of_output_classes)
        elif self.base_model_name == "resnet50":
            self.base_model = ResNet50(num_of_output_classes=num_of_output_classes, **kwargs)
        elif self.base_model_name == "mobilenetv2":
            self.base_model = MobileNetV2(**kwargs)
            self.base_model.FC = nn.Sequential(nn.Dropout(p=0.2), nn.Linear(1280, num_of_output_classes))  # R5
        else:
            raise ValueError("FeatureExtractModel supports 'resnet', 'resnet50' or 'mobilenetv2'")

    def forward(self, x):
        return self.base_model(x)

    def classify(self, x, use_dropout=False):
        """MobileNetV2 back-end: logits of the R5 classifier over pooled conv2 features."""
        if self.base_model_name != "mobilenetv2":
            return self.base_model(x, use_dropout)[0]
        f = self.base_model.extract_features(x)[-1]
        h = tpgan_ops.global_avgpool(f).reshape(f.size(0), -1)
        drop, lin = self.base_model.FC
        if use_dropout:
            h = drop(h)
        return tpgan_ops.linear(h, lin.weight, lin.bias)

    def extract_features(self, x):
        return self.base_model.extract_features(x)


# (BATCH_REAL -- the real images riding in the fake images' extractor pass as one 2B batch --
# was built in round 4 and removed in round 6: measured slower than the real features on a side
# stream under G's forward, real_features_async)


class IdentityPreservingLoss(nn.Module):
    """L_ip of TP-GAN: sum over the extractor's identity features of the mean absolute
    difference between fake and real (config.py loss weight_identity_preserving = 30).
    The extractor is frozen (eval mode, no parameter gradients): the real features are
    computed without autograd, the fake ones with it, so the backward runs only input
    gradients through the HIP kernels into G."""

    def __init__(self, extractor, compute_dtype=torch.bfloat16):
        super(IdentityPreservingLoss, self).__init__()
        self.extractor = extractor.eval()
        for p in self.extractor.parameters():
            p.requires_grad_(False)
        self.compute_dtype = compute_dtype

    def real_features_async(self, real):
        """Start the real images' features (they do not depend on G) on a side HIP stream,
        planned for a share of the chip, so that they run under G's forward; the handle goes
        to forward(pre=...).  None when there is no GPU side stream to use."""
        if not (tpgan_ops.MULTISTREAM and real.is_cuda):
            return None
        main = torch.cuda.current_stream()
        # (a stream of its own: the weight-gradient side stream would queue behind this work)
        st = tpgan_ops.side_streams(real.device, 1, "identity")[0]
        st.wait_stream(main)
        with torch.cuda.stream(st), torch.no_grad(), tpgan_ops.compute_dtype(self.compute_dtype), \
                tpgan_ops.concurrent():
            fr = self.extractor.extract_features(real)
        return st, fr

    def forward(self, fake, real, pre=None):
        with tpgan_ops.compute_dtype(self.compute_dtype):
            if pre is not None:
                st, fr = pre
                main = torch.cuda.current_stream()
                # (the identity fork of tpgan_train runs this on the features' own stream: no
                # event wait of a stream on itself -- inside a graph capture that self-edge
                # crashed hipStreamEndCapture, gpurun r05ar / r06e)
                if main != st:
                    main.wait_stream(st)
                    for t in fr:
                        t.record_stream(main)
            else:
                with torch.no_grad():
                    fr = self.extractor.extract_features(real)
            ff = self.extractor.extract_features(fake)
        loss = 0.0
        for a, b in zip(ff, fr):
            loss = loss + (a.float() - b.float()).abs().mean()
        return loss
