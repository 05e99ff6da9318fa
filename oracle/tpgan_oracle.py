"""CPU restatement of the TP-GAN hot path (reference + repairs R1-R3), functional form.

TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT.  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import this module, and only as a checker / the
CPU baseline.  The shipped path (tp-gan_amd/) never imports or calls it.

Pinned against golden vectors produced by running the reference itself
(tests/golden/make_golden.py -> tests/golden/{ops,e2e}_golden.npz); see
tests/test_oracle_golden.py.

Every function is a pure function of a flat parameter dict whose keys are the
reference's state_dict keys (e.g. "global_pathway.conv0.0.0.weight"), computed with
aten CPU ops (F.conv2d / F.conv_transpose2d / F.linear) in whatever dtype the
parameters carry (float64 for fixtures, float32 for the CPU baseline).
"""
import torch
import torch.nn.functional as F

SLOPE = 0.01  # nn.LeakyReLU() default and nn.LeakyReLU(1e-2) everywhere in the hot path


def _act(x, act):
    if act == "leaky":
        return F.leaky_relu(x, SLOPE)
    if act == "relu":
        return F.relu(x)
    return x


def conv(P, key, x, stride=1, padding=0, act="leaky"):
    """ModificationLayer.conv (ModificationLayer.py:54-123): [ReflectionPad2d if padding is
    a 4-list (:83-96)] -> Conv2d(bias=True since BN is off, :98-101) -> activation (:119,
    R2 drops a None activation).  `key` is the Sequential prefix; the Conv2d sits at
    index 1 when a reflection pad occupies index 0."""
    if isinstance(padding, (list, tuple)) and len(padding) == 4:
        x = F.pad(x, tuple(padding), mode="reflect")
        w, b = P[key + ".1.weight"], P[key + ".1.bias"]
        y = F.conv2d(x, w, b, stride, 0)
    else:
        w, b = P[key + ".0.weight"], P[key + ".0.bias"]
        y = F.conv2d(x, w, b, stride, padding)
    return _act(y, act)


def deconv(P, key, x, stride, padding, output_padding, act="relu"):
    """ModificationLayer.deconv (ModificationLayer.py:158-202): ConvTranspose2d + ReLU."""
    y = F.conv_transpose2d(x, P[key + ".0.weight"], P[key + ".0.bias"], stride, padding, output_padding)
    return _act(y, act)


def residual(P, key, x, k=3, padding=None, scale=1.0):
    """ModificationLayer.ResidualBlock (ModificationLayer.py:233-302), non-bottleneck:
    out = act(conv_b(act(conv_a(x))) + scale * x).  The shortcut is always identity
    because :283 tests the argument use_projection, not self.use_projection (:281).
    Padding defaults to (k-1)//2 (:271); conv_b has no activation (:294, R2)."""
    pad = (k - 1) // 2 if padding is None else padding
    h = conv(P, key + ".layers.0", x, 1, pad, "leaky")
    h = conv(P, key + ".layers.1", h, 1, pad, None)
    return F.leaky_relu(h + scale * x, SLOPE)


def local_pathway(P, key, x):
    """LocalPathway.forward (D_and_G_model.py:84-110); channel plan :43-81."""
    c0 = residual(P, key + ".conv0.1", conv(P, key + ".conv0.0", x, 1, 1))
    c1 = residual(P, key + ".conv1.1", conv(P, key + ".conv1.0", c0, 2, 1))
    c2 = residual(P, key + ".conv2.1", conv(P, key + ".conv2.0", c1, 2, 1))
    c3 = residual(P, key + ".conv3.1", conv(P, key + ".conv3.0", c2, 2, 1))
    d0 = deconv(P, key + ".deconv0", c3, 2, 1, 1)
    a0 = residual(P, key + ".after_select0.1", conv(P, key + ".after_select0.0", torch.cat([d0, c2], 1), 1, 1))
    d1 = deconv(P, key + ".deconv1", a0, 2, 1, 1)
    a1 = residual(P, key + ".after_select1.1", conv(P, key + ".after_select1.0", torch.cat([d1, c1], 1), 1, 1))
    d2 = deconv(P, key + ".deconv2", a1, 2, 1, 1)
    a2 = residual(P, key + ".after_select2.1", conv(P, key + ".after_select2.0", torch.cat([d2, c0], 1), 1, 1))
    img = conv(P, key + ".local_img", a2, 1, 0, None)
    assert img.shape == x.shape  # :108
    return img, d2


# LocalFuser zero-pad placements (l, r, t, b) on a 128x128 canvas, D_and_G_model.py:148-157
FUSER_PADS = (
    (39 - 20 - 1, 128 - (39 + 20 - 1), 40 - 20 - 1, 128 - (40 + 20 - 1)),  # left eye 40x40
    (86 - 20 - 1, 128 - (86 + 20 - 1), 39 - 20 - 1, 128 - (39 + 20 - 1)),  # right eye 40x40
    (64 - 20 - 1, 128 - (64 + 20 - 1), 64 - 16 - 1, 128 - (64 + 16 - 1)),  # nose W40 H32
    (65 - 24 - 1, 128 - (65 + 24 - 1), 89 - 16 - 1, 128 - (89 + 16 - 1)),  # mouth W48 H32
)


def fuser_pads(img_size=128):
    """FUSER_PADS at 128; at k*128 (build extension for BASELINE configs[4], no reference
    counterpart) the landmark centres and patch sizes scale by k, placement centre - half - 1."""
    if img_size == 128:
        return FUSER_PADS
    k = img_size // 128
    out = []
    for (cx, cy), (h, w) in zip(((39, 40), (86, 39), (64, 64), (65, 89)), ((40, 40), (40, 40), (32, 40), (32, 48))):
        top, left = cy * k - h * k // 2 - 1, cx * k - w * k // 2 - 1
        out.append((left, img_size - left - w * k, top, img_size - top - h * k))
    return tuple(out)


def local_fuser(le, re, nose, mouth):
    """LocalFuser.forward (D_and_G_model.py:132-159): zero-pad to 128x128, max over the
    stack (first index wins ties, so padding zeros of an earlier patch win over a
    negative value of a later one).  The canvas is 128 * (eye height / 40)."""
    pads = fuser_pads(128 * le.shape[2] // 40)
    xs = [F.pad(t, p) for t, p in zip((le, re, nose, mouth), pads)]
    return torch.max(torch.stack(xs, 0), 0)[0]


def global_pathway(P, key, I128, local_fake, local_feat, z):
    """GlobalPathway.forward (D_and_G_model.py:281-329) with repair R3 (dim128 = 75)."""
    k = key + "."
    c0 = residual(P, k + "conv0.1", conv(P, k + "conv0.0", I128, 1, 3), 7, 3)
    c1 = residual(P, k + "conv1.1", conv(P, k + "conv1.0", c0, 2, 2), 5, 2)
    c2 = residual(P, k + "conv2.1", conv(P, k + "conv2.0", c1, 2, 1), 3, 1)
    c3 = residual(P, k + "conv3.1", conv(P, k + "conv3.0", c2, 2, 1), 3, 1)
    c4 = conv(P, k + "conv4.0", c3, 2, 1)
    for i in range(1, 5):  # 4 ResidualBlocks (:209)
        c4 = residual(P, k + "conv4.%d" % i, c4, 3, 1)
    B = c4.shape[0]
    fc1 = F.linear(c4.reshape(B, -1), P[k + "fc1.weight"], P[k + "fc1.bias"])  # :289
    fc2 = F.max_pool1d(fc1.view(B, -1, 2), 2, 2).view(B, -1)  # maxout :214,:290
    d8 = deconv(P, k + "deconv_8", torch.cat([fc2, z], 1).view(B, -1, 1, 1), 1, 0, 0)  # :293
    d32 = deconv(P, k + "deconv_32", d8, 4, 0, 1)
    d64 = deconv(P, k + "deconv_64", d32, 2, 1, 1)
    d128 = deconv(P, k + "deconv_128", d64, 2, 1, 1)
    rp = [1, 0, 1, 0]  # ReflectionPad2d(l=1,r=0,t=1,b=0) 2x2 convs (:235,:237)
    a8 = residual(P, k + "add_conv_and_deconv_8", torch.cat([d8, c4], 1), 2, rp)
    e8 = a8
    for i in range(2):
        e8 = residual(P, k + "enhance_features_8.%d" % i, e8, 2, rp)
    u16 = deconv(P, k + "upsample_16", e8, 2, 1, 1)
    a16 = residual(P, k + "add_conv_and_deconv_16", c3)
    e16 = torch.cat([u16, a16], 1)
    for i in range(2):
        e16 = residual(P, k + "enhance_features_16.%d" % i, e16)
    u32 = deconv(P, k + "upsample_32", e16, 2, 1, 1)
    a32 = residual(P, k + "add_conv_and_deconv_32", torch.cat([d32, c2], 1))
    e32 = torch.cat([u32, a32], 1)
    for i in range(2):
        e32 = residual(P, k + "enhance_features_32.%d" % i, e32)
    u64 = deconv(P, k + "upsample_64", e32, 2, 1, 1)
    a64 = residual(P, k + "add_conv_and_deconv_64", torch.cat([d64, c1], 1), 5)
    e64 = torch.cat([u64, a64], 1)
    for i in range(2):
        e64 = residual(P, k + "enhance_features_64.%d" % i, e64)
    u128 = deconv(P, k + "upsample_128", e64, 2, 1, 1)
    a128 = residual(P, k + "add_conv_and_deconv_128", torch.cat([d128, c0, I128], 1), 7)  # R3: 75 ch
    e128 = residual(P, k + "enhance_features_128.0",
                    torch.cat([u128, a128, local_feat, local_fake], 1), 5)  # R3: 206 ch
    c5 = residual(P, k + "conv5.1", conv(P, k + "conv5.0", e128, 1, 2), 3)
    c6 = conv(P, k + "conv6", c5, 1, 1)
    img = conv(P, k + "decoded_img128", c6, 1, 1, None)
    return img, fc2


def generator(P, I128, left_eye, right_eye, nose, mouth, z, use_dropout=False):
    """Generator.forward (D_and_G_model.py:374-407) -> the reference's 8-tuple."""
    le_img, le_f = local_pathway(P, "local_pathway_left_eye", left_eye)
    re_img, re_f = local_pathway(P, "local_pathway_right_eye", right_eye)
    no_img, no_f = local_pathway(P, "local_pathway_nose", nose)
    mo_img, mo_f = local_pathway(P, "local_pathway_mouth", mouth)
    fused_feat = local_fuser(le_f, re_f, no_f, mo_f)
    fused_fake = local_fuser(le_img, re_img, no_img, mo_img)
    fused_real = local_fuser(left_eye, right_eye, nose, mouth)
    fake, fc2 = global_pathway(P, "global_pathway", I128, fused_fake, fused_feat, z)
    if use_dropout:
        fc2 = F.dropout(fc2, 0.3, True)
    pred = F.linear(fc2, P["feature_predict.fc.weight"], P["feature_predict.fc.bias"])  # :344-348
    return fake, pred, fused_fake, le_img, re_img, no_img, mo_img, fused_real


def global_only(P, I128, z):
    """BASELINE config 1: GlobalPathway with zero local inputs."""
    B = I128.shape[0]
    lf = torch.zeros(B, 3, 128, 128, dtype=I128.dtype)
    lfeat = torch.zeros(B, 64, 128, 128, dtype=I128.dtype)
    return global_pathway(P, "global_pathway", I128, lf, lfeat, z)


def discriminator(P, x):
    """Discriminator.forward (D_and_G_model.py:409-435): 5x [3x3 s2 conv + LeakyReLU],
    ResidualBlocks after stages 4 and 5, then a 3x3 conv to one channel."""
    chans = [3, 64, 128, 256, 512, 512]
    idx = 0
    for i in range(5):
        x = conv(P, "model.%d" % idx, x, 2, 1)
        idx += 1
        if i >= 3:
            x = residual(P, "model.%d" % idx, x)
            idx += 1
    return conv(P, "model.%d" % idx, x, 1, 1, None)


def g_param_shapes():
    """Reference state_dict (key, shape) list for Generator(64, 347) with R3, in order."""
    import json
    import os
    p = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                     "state_dict_keys.json")
    with open(p) as f:
        keys = json.load(f)
    return keys["G"], keys["D"]


def make_params(dtype=torch.float64, seed=0, img_size=128):
    """Deterministic G and D parameter dicts (oracle.det_init).  img_size 256: fc1 takes
    512*16*16 inputs and deconv_8 has a 16x16 kernel (build extension, BASELINE configs[4])."""
    from .det_init import det_param
    gk, dk = g_param_shapes()
    if img_size != 128:
        e = img_size // 16
        fix = {"global_pathway.fc1.weight": [512, 512 * e * e],
               "global_pathway.deconv_8.0.weight": [320, 64, e, e]}
        gk = [(k, fix.get(k, s)) for k, s in gk]
    PG = {k: torch.from_numpy(det_param("G/" + k, s, seed)).to(dtype) for k, s in gk}
    PD = {k: torch.from_numpy(det_param("D/" + k, s, seed)).to(dtype) for k, s in dk}
    return PG, PD
