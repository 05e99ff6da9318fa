"""TP-GAN generator and discriminator (reference D_and_G_model.py), MI355X-native.

Module names, constructor signatures, forward signatures / return tuples and state_dict
keys are the reference's (`/root/reference/D_and_G_model.py`).  Architecture = reference
+ repairs R1-R3; R3 sizes the 128-px fusion for the 75 channels the
forward actually concatenates (:323): dim128 = 75, enhance_features_128 = 206 channels,
conv5 input 206.

Every Conv2d / ConvTranspose2d / Linear / concat / LocalFuser max / maxout runs on the
HIP kernels of libtpgan_hip.so (tpgan_ops); there is no CPU path.
"""
import torch
import torch.nn as nn

import tpgan_ops
from ModificationLayer import *  # noqa: F401,F403  (conv, deconv, sequential, ResidualBlock, ...)
from ModificationLayer import ResidualBlock, conv, deconv, group_forward, sequential
from UtilityMethods import elementwise_multiply_and_cast_to_int as EMaC2I


class LocalPathway(nn.Module):
    """U-Net over one landmark patch (D_and_G_model.py:18-110): encoder 64/128/256/512,
    transposed-conv decoder with skip concats, 1x1 conv to RGB."""

    def __init__(self, use_batchnorm=True, feature_layer_dim=64, FM_multiplier=1.0):
        super(LocalPathway, self).__init__()
        n_FM_encoder = EMaC2I([64, 128, 256, 512], FM_multiplier)
        n_FM_decoder = EMaC2I([256, 128], FM_multiplier)
        L = nn.LeakyReLU
        self.conv0 = sequential(conv(3, n_FM_encoder[0], 3, 1, 1, "kaiming", L(1e-2), use_batchnorm),
                                ResidualBlock(n_FM_encoder[0], activation=L()))
        self.conv1 = sequential(conv(n_FM_encoder[0], n_FM_encoder[1], 3, 2, 1, "kaiming", L(1e-2), use_batchnorm),
                                ResidualBlock(n_FM_encoder[1], activation=L()))
        self.conv2 = sequential(conv(n_FM_encoder[1], n_FM_encoder[2], 3, 2, 1, "kaiming", L(1e-2), use_batchnorm),
                                ResidualBlock(n_FM_encoder[2], activation=L()))
        self.conv3 = sequential(conv(n_FM_encoder[2], n_FM_encoder[3], 3, 2, 1, "kaiming", L(1e-2), use_batchnorm),
                                ResidualBlock(n_FM_encoder[3], activation=L()))
        self.deconv0 = deconv(n_FM_encoder[3], n_FM_decoder[0], 3, 2, 1, 1, "kaiming", nn.ReLU(), use_batchnorm)
        self.after_select0 = sequential(
            conv(n_FM_decoder[0] + self.conv2.out_channels, n_FM_decoder[0], 3, 1, 1, "kaiming", L(), use_batchnorm),
            ResidualBlock(n_FM_decoder[0], activation=L()))
        self.deconv1 = deconv(self.after_select0.out_channels, n_FM_decoder[1], 3, 2, 1, 1, "kaiming", nn.ReLU(),
                              use_batchnorm)
        self.after_select1 = sequential(
            conv(n_FM_decoder[1] + self.conv1.out_channels, n_FM_decoder[1], 3, 1, 1, "kaiming", L(), use_batchnorm),
            ResidualBlock(n_FM_decoder[1], activation=L()))
        self.deconv2 = deconv(self.after_select1.out_channels, feature_layer_dim, 3, 2, 1, 1, "kaiming", nn.ReLU(),
                              use_batchnorm)
        self.after_select2 = sequential(
            conv(feature_layer_dim + self.conv0.out_channels, feature_layer_dim, 3, 1, 1, "kaiming", L(),
                 use_batchnorm),
            ResidualBlock(feature_layer_dim, activation=L()))
        self.local_img = conv(feature_layer_dim, 3, 1, 1, 0, None, None, False)

    def forward(self, x):
        conv0 = self.conv0(x)
        conv1 = self.conv1(conv0)
        conv2 = self.conv2(conv1)
        conv3 = self.conv3(conv2)
        deconv0 = self.deconv0(conv3)
        after_select0 = self.after_select0(tpgan_ops.cat([deconv0, conv2]), act_in_ok=True)
        deconv1 = self.deconv1(after_select0)
        after_select1 = self.after_select1(tpgan_ops.cat([deconv1, conv1]), act_in_ok=True)
        deconv2 = self.deconv2(after_select1)
        after_select2 = self.after_select2(tpgan_ops.cat([deconv2, conv0]))
        local_img = self.local_img(after_select2)
        assert local_img.shape == x.shape, "{} {}".format(local_img.shape, x.shape)
        return local_img, deconv2

    @staticmethod
    def forward_group(paths, xs):
        """[p.forward(x) for p, x in zip(paths, xs)] in lockstep: each layer of the four
        pathways runs as one grouped node (ModificationLayer.group_forward), one launch per
        kernel instead of one per patch."""
        G = group_forward
        cat = tpgan_ops.cat
        conv0 = G([p.conv0 for p in paths], xs)
        conv1 = G([p.conv1 for p in paths], conv0)
        conv2 = G([p.conv2 for p in paths], conv1)
        conv3 = G([p.conv3 for p in paths], conv2)
        deconv0 = G([p.deconv0 for p in paths], conv3)
        after_select0 = G([p.after_select0 for p in paths], [cat([a, b]) for a, b in zip(deconv0, conv2)],
                          act_in_ok=True)
        deconv1 = G([p.deconv1 for p in paths], after_select0)
        after_select1 = G([p.after_select1 for p in paths], [cat([a, b]) for a, b in zip(deconv1, conv1)],
                          act_in_ok=True)
        deconv2 = G([p.deconv2 for p in paths], after_select1)
        after_select2 = G([p.after_select2 for p in paths], [cat([a, b]) for a, b in zip(deconv2, conv0)])
        local_img = G([p.local_img for p in paths], after_select2)
        for img, x in zip(local_img, xs):
            assert img.shape == x.shape, "{} {}".format(img.shape, x.shape)
        return list(zip(local_img, deconv2))


class LocalFuser(nn.Module):
    """Zero-pad the four parts onto a 128x128 canvas and take the element-wise max
    (D_and_G_model.py:112-159).  Placements (top, left) follow the reference's pad
    arithmetic (:154-157); ties resolve to the first part, as torch.max does.

    img_size (build extension, BASELINE configs[4]; the reference is 128-only, :152): the
    patch sizes and the landmark centres of the 128 canvas scale by img_size / 128, and the
    placement keeps the reference's form centre - half - 1."""

    EYE_WIDTH, EYE_HEIGHT = 40, 40
    NOSE_WIDTH, NOSE_HEIGHT = 40, 32
    MOUTH_WIDTH, MOUTH_HEIGHT = 48, 32
    IMG_SIZE = 128
    # landmark centres (x, y) of the 128 canvas: left eye, right eye, nose, mouth (:154-157)
    CENTERS = ((39, 40), (86, 39), (64, 64), (65, 89))
    # (top, left) of left eye, right eye, nose, mouth
    TOPS = (40 - 20 - 1, 39 - 20 - 1, 64 - 16 - 1, 89 - 16 - 1)
    LEFTS = (39 - 20 - 1, 86 - 20 - 1, 64 - 20 - 1, 65 - 24 - 1)
    SIZES = ((40, 40), (40, 40), (32, 40), (32, 48))

    def __init__(self, img_size=128):
        super(LocalFuser, self).__init__()
        if img_size % 128:
            raise ValueError("LocalFuser: img_size must be a multiple of 128, got %d" % img_size)
        if img_size != 128:
            k = img_size // 128
            self.IMG_SIZE = img_size
            self.SIZES = tuple((h * k, w * k) for h, w in LocalFuser.SIZES)
            self.TOPS = tuple(cy * k - h * k // 2 - 1 for (cx, cy), (h, w) in zip(self.CENTERS, LocalFuser.SIZES))
            self.LEFTS = tuple(cx * k - w * k // 2 - 1 for (cx, cy), (h, w) in zip(self.CENTERS, LocalFuser.SIZES))

    def forward(self, f_left_eye, f_right_eye, f_nose, f_mouth):
        parts = (f_left_eye, f_right_eye, f_nose, f_mouth)
        for p, (h, w) in zip(parts, self.SIZES):
            if tuple(p.shape[2:]) != (h, w):
                raise RuntimeError("LocalFuser expects part of spatial size %dx%d, got %s" % (h, w, tuple(p.shape)))
        return tpgan_ops.local_fuse(parts, (self.IMG_SIZE, self.IMG_SIZE), self.TOPS, self.LEFTS)


class GlobalPathway(nn.Module):
    """Global encoder-decoder over the 128x128 face (D_and_G_model.py:161-329), R3 applied."""

    def __init__(self, zdim, local_feature_layer_dim=64, use_batchnorm=True, use_residual_block=True,
                 scaling_factor=1.0, FM_multiplier=1.0, img_size=128):
        super(GlobalPathway, self).__init__()
        # img_size (build extension, BASELINE configs[4]): the encoder ends at img_size / 16;
        # fc1 (:212, 512*8*8 inputs at 128) and the deconv_8 kernel (:218, 8 = the 8x8 map it
        # must produce) follow that size
        self.img_size = img_size
        e = img_size // 16
        n_FM_encoder = EMaC2I([64, 64, 128, 256, 512], FM_multiplier)
        n_FM_decoder = EMaC2I([64, 32, 16, 8], FM_multiplier)
        n_FM_decoder_enhance_features = EMaC2I([512, 256, 128, 64], FM_multiplier)
        n_FM_decoder_conv = EMaC2I([64, 32], FM_multiplier)
        L = nn.LeakyReLU
        self.zdim = zdim
        self.use_residual_block = use_residual_block
        sf = scaling_factor
        self.conv0 = sequential(conv(3, n_FM_encoder[0], 7, 1, 3, "kaiming", L(1e-2), use_batchnorm),
                                ResidualBlock(64, 64, 7, 1, 3, "kaiming", L(1e-2), scaling_factor=sf))
        self.conv1 = sequential(conv(n_FM_encoder[1], n_FM_encoder[1], 5, 2, 2, "kaiming", L(1e-2), use_batchnorm),
                                ResidualBlock(64, 64, 5, 1, 2, "kaiming", L(1e-2), scaling_factor=sf))
        self.conv2 = sequential(conv(n_FM_encoder[1], n_FM_encoder[2], 3, 2, 1, "kaiming", L(1e-2), use_batchnorm),
                                ResidualBlock(128, 128, 3, 1, 1, "kaiming", L(1e-2), scaling_factor=sf))
        self.conv3 = sequential(conv(n_FM_encoder[2], n_FM_encoder[3], 3, 2, 1, "kaiming", L(1e-2), use_batchnorm),
                                ResidualBlock(256, 256, 3, 1, 1, "kaiming", L(1e-2), is_bottleneck=False,
                                              scaling_factor=sf))
        self.conv4 = sequential(conv(n_FM_encoder[3], n_FM_encoder[4], 3, 2, 1, "kaiming", L(1e-2), use_batchnorm),
                                *[ResidualBlock(512, 512, 3, 1, 1, "kaiming", L(1e-2), is_bottleneck=False,
                                                scaling_factor=sf) for i in range(4)])
        self.fc1 = nn.Linear(n_FM_encoder[4] * e * e, 512)
        self.fc2 = nn.MaxPool1d(2, 2, 0)
        self.deconv_8 = deconv(256 + self.zdim, n_FM_decoder[0], e, 1, 0, 0, "kaiming", nn.ReLU(), use_batchnorm)
        self.deconv_32 = deconv(n_FM_decoder[0], n_FM_decoder[1], 3, 4, 0, 1, "kaiming", nn.ReLU(), use_batchnorm)
        self.deconv_64 = deconv(n_FM_decoder[1], n_FM_decoder[2], 3, 2, 1, 1, "kaiming", nn.ReLU(), use_batchnorm)
        self.deconv_128 = deconv(n_FM_decoder[2], n_FM_decoder[3], 3, 2, 1, 1, "kaiming", nn.ReLU(), use_batchnorm)
        dim8 = self.deconv_8.out_channels + self.conv4.out_channels
        self.add_conv_and_deconv_8 = ResidualBlock(dim8, dim8, 2, 1, padding=[1, 0, 1, 0], activation=L())
        self.enhance_features_8 = sequential(
            *[ResidualBlock(dim8, dim8, 2, 1, padding=[1, 0, 1, 0], activation=L()) for i in range(2)])
        self.upsample_16 = deconv(self.enhance_features_8.out_channels, n_FM_decoder_enhance_features[0], 3, 2, 1, 1,
                                  "kaiming", nn.ReLU(), use_batchnorm)
        dim16 = self.conv3.out_channels
        self.add_conv_and_deconv_16 = ResidualBlock(dim16, activation=L())
        self.enhance_features_16 = sequential(
            *[ResidualBlock(self.upsample_16.out_channels + self.add_conv_and_deconv_16.out_channels, activation=L())
              for i in range(2)])
        self.upsample_32 = deconv(self.enhance_features_16.out_channels, n_FM_decoder_enhance_features[1], 3, 2, 1, 1,
                                  "kaiming", nn.ReLU(), use_batchnorm)
        dim32 = self.conv2.out_channels + self.deconv_32.out_channels
        self.add_conv_and_deconv_32 = ResidualBlock(dim32, activation=L())
        self.enhance_features_32 = sequential(
            *[ResidualBlock(self.upsample_32.out_channels + self.add_conv_and_deconv_32.out_channels, activation=L())
              for i in range(2)])
        self.upsample_64 = deconv(self.enhance_features_32.out_channels, n_FM_decoder_enhance_features[2], 3, 2, 1, 1,
                                  "kaiming", nn.ReLU(), use_batchnorm)
        dim64 = self.conv1.out_channels + self.deconv_64.out_channels
        self.add_conv_and_deconv_64 = ResidualBlock(dim64, kernel_size=5, activation=L())
        self.enhance_features_64 = sequential(
            *[ResidualBlock(self.upsample_64.out_channels + self.add_conv_and_deconv_64.out_channels, activation=L())
              for i in range(2)])
        self.upsample_128 = deconv(self.enhance_features_64.out_channels, n_FM_decoder_enhance_features[3], 3, 2, 1,
                                   1, "kaiming", nn.ReLU(), use_batchnorm)
        # R3: the forward concatenates [deconv_128, conv0, I128] = 8 + 64 + 3 channels (:323)
        dim128 = self.deconv_128.out_channels + self.conv0.out_channels + 3
        self.add_conv_and_deconv_128 = ResidualBlock(dim128, kernel_size=7, activation=L())
        self.enhance_features_128 = sequential(
            *[ResidualBlock(self.upsample_128.out_channels + self.add_conv_and_deconv_128.out_channels +
                            local_feature_layer_dim + 3, kernel_size=5, activation=L())])
        self.conv5 = sequential(
            conv(self.enhance_features_128.out_channels, n_FM_decoder_conv[0], 5, 1, 2, "kaiming", L(),
                 use_batchnorm),
            ResidualBlock(n_FM_decoder_conv[0], kernel_size=3, activation=L()))
        self.conv6 = conv(n_FM_decoder_conv[0], n_FM_decoder_conv[1], 3, 1, 1, "kaiming", L(), use_batchnorm)
        self.decoded_img128 = conv(n_FM_decoder_conv[1], 3, 3, 1, 1, None, activation=None)

    def forward(self, I128, local_fake_image, local_feature, z):
        return self.decode_128(self.encode(I128, z), local_fake_image, local_feature)

    def encode(self, I128, z):
        """Everything that does not depend on the local pathways (:283-320): the encoder,
        fc1/fc2, the decoder up to upsample_128 and add_conv_and_deconv_128."""
        cat = tpgan_ops.cat
        conv0 = self.conv0(I128)
        conv1 = self.conv1(conv0)
        conv2 = self.conv2(conv1)
        conv3 = self.conv3(conv2)
        conv4 = self.conv4(conv3)
        B = conv4.shape[0]
        # fc1 on the NCHW flattening of conv4 (:289) = an 8x8 full-kernel conv on the NHWC map
        fc1 = tpgan_ops.linear(conv4, self.fc1.weight, self.fc1.bias)
        fc2 = tpgan_ops.maxout2(fc1)  # self.fc2 = MaxPool1d(2, 2) on view(B, -1, 2) (:290)
        deconv_8 = self.deconv_8(cat([fc2.view(B, -1, 1, 1), z.view(B, -1, 1, 1)]))
        deconv_32 = self.deconv_32(deconv_8)
        deconv_64 = self.deconv_64(deconv_32)
        deconv_128 = self.deconv_128(deconv_64)
        add_conv_and_deconv_8 = self.add_conv_and_deconv_8(cat([deconv_8, conv4]))
        enhance_features_8 = self.enhance_features_8(add_conv_and_deconv_8, act_in_ok=True)
        assert enhance_features_8.shape[2] == self.img_size // 16  # :301
        upsample_16 = self.upsample_16(enhance_features_8, act_in_ok=True)
        add_conv_and_deconv_16 = self.add_conv_and_deconv_16(conv3)
        enhance_features_16 = self.enhance_features_16(cat([upsample_16, add_conv_and_deconv_16]),
                                                       act_in_ok=True)
        assert enhance_features_16.shape[2] == self.img_size // 8  # :308
        upsample_32 = self.upsample_32(enhance_features_16, act_in_ok=True)
        add_conv_and_deconv_32 = self.add_conv_and_deconv_32(cat([deconv_32, conv2]))
        enhance_features_32 = self.enhance_features_32(cat([upsample_32, add_conv_and_deconv_32]),
                                                       act_in_ok=True)
        upsample_64 = self.upsample_64(enhance_features_32, act_in_ok=True)
        add_conv_and_deconv_64 = self.add_conv_and_deconv_64(cat([deconv_64, conv1]))
        enhance_features_64 = self.enhance_features_64(cat([upsample_64, add_conv_and_deconv_64]),
                                                       act_in_ok=True)
        upsample_128 = self.upsample_128(enhance_features_64, act_in_ok=True)
        add_conv_and_deconv_128 = self.add_conv_and_deconv_128(cat([deconv_128, conv0, I128]),
                                                               act_in_ok=True)
        return upsample_128, add_conv_and_deconv_128, fc2

    def decode_128(self, enc, local_fake_image, local_feature):
        """The 128-px fusion with the local features (:321-329).  (act_in_ok: each of these
        outputs feeds the next module alone, so its consumer applies its activation backward,
        tpgan_ops.ActToken; likewise in encode() for the decoder's enhance -> upsample chain.)"""
        cat = tpgan_ops.cat
        upsample_128, add_conv_and_deconv_128, fc2 = enc
        enhance_features_128 = self.enhance_features_128(
            cat([upsample_128, add_conv_and_deconv_128, local_feature, local_fake_image]), act_in_ok=True)
        conv5 = self.conv5(enhance_features_128, act_in_ok=True)
        conv6 = self.conv6(conv5, act_in_ok=True)
        decoded_img128 = self.decoded_img128(conv6, act_in_ok=True)
        return decoded_img128, fc2


class FeaturePredict(nn.Module):
    """Dropout(0.3) + Linear(256 -> num_classes) on the maxout features (:331-348)."""

    def __init__(self, num_classes, global_feature_layer_dim=256, dropout=0.3):
        super(FeaturePredict, self).__init__()
        self.dropout = nn.Dropout(p=dropout)
        self.fc = nn.Linear(global_feature_layer_dim, num_classes)

    def forward(self, x, use_dropout):
        if use_dropout:
            x = self.dropout(x)
        return tpgan_ops.linear(x, self.fc.weight, self.fc.bias)


class Generator(nn.Module):
    """Four LocalPathways, three LocalFuser calls, the GlobalPathway and FeaturePredict;
    forward returns the reference's 8-tuple (D_and_G_model.py:350-407)."""

    def __init__(self, zdim, num_classes, use_batchnorm=True, use_residual_block=True, img_size=128):
        super(Generator, self).__init__()
        self.img_size = img_size  # build extension (BASELINE configs[4]: 256); the reference is 128-only
        self.local_pathway_left_eye = LocalPathway(use_batchnorm=use_batchnorm)
        self.local_pathway_right_eye = LocalPathway(use_batchnorm=use_batchnorm)
        self.local_pathway_nose = LocalPathway(use_batchnorm=use_batchnorm)
        self.local_pathway_mouth = LocalPathway(use_batchnorm=use_batchnorm)
        self.global_pathway = GlobalPathway(zdim, use_batchnorm=use_batchnorm, use_residual_block=use_residual_block,
                                            img_size=img_size)
        self.local_fuser = LocalFuser(img_size)
        self.feature_predict = FeaturePredict(num_classes)
        self._groupable = None

    def forward(self, I128, left_eye, right_eye, nose, mouth, z, use_dropout):
        paths = (self.local_pathway_left_eye, self.local_pathway_right_eye, self.local_pathway_nose,
                 self.local_pathway_mouth)
        patches = (left_eye, right_eye, nose, mouth)
        fused = None
        if self._groupable is None:
            # lockstep grouping fuses conv + bias + activation layers only: with BatchNorm
            # (use_batchnorm=True, the reference default) group_forward would run the members
            # one by one on one stream, so those pathways keep one stream each instead
            self._groupable = not any(isinstance(m, nn.BatchNorm2d) for p in paths for m in p.modules())
        if tpgan_ops.GROUP["enabled"] and I128.is_cuda and self._groupable:
            # the four local pathways in lockstep on one side stream (one grouped launch per
            # layer and kernel), concurrently with the global pathway's local-independent part
            # The three LocalFuser calls run on that stream too, so their backward does (autograd
            # replays a node on its forward's stream): on the main stream the fuser backward was
            # enqueued behind the whole global backward and held the local backward there
            # (29.58 / 29.61 vs 29.78 / 29.71 ms/step, gpurun r06g).  (Creating the local nodes
            # after the global encoder's, so that autograd -- latest-created first -- enqueues the
            # local backward as soon as its gradients exist, ran it beside the global backward
            # but measured 29.75 / 29.80 vs 29.54 / 29.63: the chip is already busy, r06h.)
            main = torch.cuda.current_stream()
            st = tpgan_ops.side_streams(I128.device, 1, "local")[0] if tpgan_ops.MULTISTREAM else main
            st.wait_stream(main)
            with torch.cuda.stream(st), tpgan_ops.concurrent(tpgan_ops.MULTISTREAM):
                outs = LocalPathway.forward_group(paths, patches)
                fused = self._fuse(outs, patches)
            enc = self.global_pathway.encode(I128, z)
            if st is not main:
                main.wait_stream(st)
                for t in [t for o in outs for t in o] + list(fused):
                    t.record_stream(main)
        elif tpgan_ops.MULTISTREAM and I128.is_cuda:
            # The four local pathways (small maps: kernels that fill few CUs) run on their
            # own HIP streams, concurrently with the global pathway's local-independent part
            # on the current stream; autograd replays each op's backward on its forward
            # stream, so the backward overlaps the same way.
            main = torch.cuda.current_stream()
            side = tpgan_ops.side_streams(I128.device, 4, "local")
            outs = []
            for st, path, x in zip(side, paths, patches):
                st.wait_stream(main)
                with torch.cuda.stream(st), tpgan_ops.concurrent():
                    outs.append(path(x))
            enc = self.global_pathway.encode(I128, z)
            for st, (img, feat) in zip(side, outs):
                main.wait_stream(st)
                img.record_stream(main)
                feat.record_stream(main)
        else:
            outs = [path(x) for path, x in zip(paths, patches)]
            enc = self.global_pathway.encode(I128, z)
        if fused is None:
            fused = self._fuse(outs, patches)
        ((left_eye_fake_image, _), (right_eye_fake_image, _), (nose_fake_image, _), (mouth_fake_image, _)) = outs
        fused_local_feature, fused_local_fake_image, fused_local_origin_4_part = fused
        I128_fake, encoder_feature = self.global_pathway.decode_128(enc, fused_local_fake_image, fused_local_feature)
        encoder_predict = self.feature_predict(encoder_feature, use_dropout)
        return (I128_fake, encoder_predict, fused_local_fake_image, left_eye_fake_image, right_eye_fake_image,
                nose_fake_image, mouth_fake_image, fused_local_origin_4_part)


    def _fuse(self, outs, patches):
        """The three LocalFuser calls of the reference (D_and_G_model.py:395-398): the local
        features, the local fake images, the real patches."""
        ((le_img, le_feat), (re_img, re_feat), (no_img, no_feat), (mo_img, mo_feat)) = outs
        return (self.local_fuser(le_feat, re_feat, no_feat, mo_feat), self.local_fuser(le_img, re_img, no_img, mo_img),
                self.local_fuser(*patches))


class Discriminator(nn.Module):
    """5x [3x3 s2 conv + LeakyReLU], ResidualBlocks after stages 4 and 5, 3x3 conv to one
    channel: a B x 1 x H/32 x W/32 patch map (D_and_G_model.py:409-435)."""

    def __init__(self, use_batchnorm=False, FM_multiplier=1.0):
        super(Discriminator, self).__init__()
        layers = []
        n_Fmap = EMaC2I([3, 64, 128, 256, 512, 512], FM_multiplier)
        for i in range(len(n_Fmap) - 1):
            layers.append(conv(n_Fmap[i], n_Fmap[i + 1], 3, 2, 1, "kaiming", nn.LeakyReLU(1e-2), use_batchnorm))
            if i >= 3:
                layers.append(ResidualBlock(n_Fmap[i + 1], activation=nn.LeakyReLU()))
        layers.append(conv(n_Fmap[-1], 1, kernel_size=3, stride=1, padding=1, init=None, activation=None))
        self.model = sequential(*layers)

    def forward(self, x):
        return self.model(x)
