"""Layer factories of the reference (ModificationLayer.py), MI355X-native.

Same names, signatures, module trees and state_dict keys as the reference
(`/root/reference/ModificationLayer.py`), with the two construction/forward defects the
reference cannot run with repaired:
  R1  weight_initialization initialises `module.weight` (reference passes the module to
      kaiming_normal, ModificationLayer.py:47,49,51)
  R2  a None activation is not appended to nn.Sequential (ModificationLayer.py:154)

The returned containers are nn.Sequential subclasses whose forward does not walk the
children: the Conv2d / ConvTranspose2d + bias + activation (+ the ResidualBlock's
residual add and its ReflectionPad2d) run as one fused HIP call (tpgan_ops.conv2d).
Convolution weights are kept channels-last (logical shape unchanged), which is the
layout the HIP weight-gradient kernel accumulates into.
"""
import torch
import torch.nn as nn

import tpgan_ops
from tpgan_lib import PAD_REFLECT, PAD_ZERO

_CL = torch.channels_last


def _channels_last_(m):
    if getattr(m, "weight", None) is not None and m.weight.dim() == 4:
        m.weight.data = m.weight.data.contiguous(memory_format=_CL)
    return m


def sequential(*kargs):
    """nn.Sequential with `.out_channels` taken from the last layer that has
    out_channels / out_features (ModificationLayer.py:5-24)."""
    seq = _FusedSequential(*kargs)
    for layer in reversed(kargs):
        if hasattr(layer, "out_channels"):
            seq.out_channels = layer.out_channels
            break
        if hasattr(layer, "out_features"):
            seq.out_channels = layer.out_features
            break
    return seq


def weight_initialization(weight, init, activation):
    """Kaiming (a = LeakyReLU negative slope, 0 for ReLU) or Xavier normal init
    (ModificationLayer.py:26-52).  R1: accepts the layer module or its weight tensor."""
    if init is None:
        return
    w = weight.weight if isinstance(weight, nn.Module) else weight
    if init == "kaiming":
        a = activation.negative_slope if hasattr(activation, "negative_slope") else 0
        nn.init.kaiming_normal_(w, a=a)
    elif init == "xavier":
        nn.init.xavier_normal_(w)


class _FusedSequential(nn.Sequential):
    """nn.Sequential whose forward fuses [ReflectionPad2d] Conv2d|ConvTranspose2d [act]
    into one HIP call; any other layout (BatchNorm, pre-activation, Sigmoid/Tanh)
    runs its extra modules with torch around the fused conv."""

    def _parts(self):
        mods = list(self._modules.values())
        pad = None
        if mods and isinstance(mods[0], nn.ReflectionPad2d):
            pad = mods[0]
            mods = mods[1:]
        if (mods and isinstance(mods[0], (nn.Conv2d, nn.ConvTranspose2d)) and
                (len(mods) == 1 or (len(mods) == 2 and tpgan_ops.act_code(mods[1]) is not None))):
            return pad, mods[0], (mods[1] if len(mods) == 2 else None)
        return None

    def forward(self, x, residual=None, res_scale=1.0, post_act=None, link_res=None, link_dx=None, act_in_ok=False):
        """act_in_ok: the caller's promise that x is consumed by this module alone, so the
        first conv may apply x's producer activation backward (tpgan_ops.ActToken)."""
        parts = self._parts()
        if parts is not None:
            pad, layer, act = parts
            if residual is not None:
                if act is not None:
                    raise RuntimeError("residual fusion expects a conv without activation")
                act = post_act
            return _apply_conv(layer, x, pad, act, residual, res_scale, link_res, link_dx, act_in_ok)
        if residual is not None:
            raise RuntimeError("residual fusion needs a [pad] conv [act] sequence")
        return _generic_forward(self, x, act_in_ok)


def _conv_geom_args(layer, pad_mod):
    kh, kw = layer.kernel_size
    stride = tuple(layer.stride)
    if isinstance(layer, nn.ConvTranspose2d):
        ph, pw = layer.padding
        return dict(stride=stride, pad=(ph, ph, pw, pw), pad_mode=PAD_ZERO, transposed=True,
                    output_padding=tuple(layer.output_padding))
    if pad_mod is not None:
        l, r, t, b = pad_mod.padding  # ReflectionPad2d stores (left, right, top, bottom)
        ph, pw = layer.padding
        if ph or pw:
            raise NotImplementedError("reflection padding plus Conv2d padding")
        return dict(stride=stride, pad=(t, b, l, r), pad_mode=PAD_REFLECT)
    if layer.padding_mode != "zeros":
        raise NotImplementedError("padding_mode %s" % layer.padding_mode)
    ph, pw = layer.padding
    return dict(stride=stride, pad=(ph, ph, pw, pw), pad_mode=PAD_ZERO)


def _apply_conv(layer, x, pad_mod, act, residual=None, res_scale=1.0, link_res=None, link_dx=None, act_in_ok=False):
    if tuple(layer.dilation) != (1, 1) or layer.groups != 1:
        raise NotImplementedError("dilated / grouped convolution")
    if (isinstance(layer, nn.Conv2d) and layer.in_channels <= 4 and residual is None and link_dx is None and
            pad_mod is None and layer.padding_mode == "zeros" and layer.kernel_size != (1, 1)):
        # thin input: taps folded into channels (tpgan_ops.conv2d_folded)
        ph, pw = layer.padding
        y = tpgan_ops.conv2d_folded(x, layer.weight, layer.bias, tuple(layer.stride), (ph, ph, pw, pw), act)
        if y is not None:
            return y
    return tpgan_ops.conv2d(x, layer.weight, layer.bias, act=act, residual=residual, res_scale=res_scale,
                            link_res=link_res, link_dx=link_dx, act_in_ok=act_in_ok, **_conv_geom_args(layer, pad_mod))


def _conv_call(layer, x, pad_mod, act, residual=None, res_scale=1.0, link_res=None, link_dx=None, act_in_ok=False):
    """tpgan_ops.conv2d keyword arguments of _apply_conv's call, or None where it would not
    call conv2d (dilated / grouped convs)."""
    if tuple(layer.dilation) != (1, 1) or layer.groups != 1:
        return None
    if (isinstance(layer, nn.Conv2d) and layer.in_channels <= 4 and residual is None and link_dx is None and
            pad_mod is None and layer.padding_mode == "zeros" and layer.kernel_size != (1, 1)):
        ph, pw = layer.padding
        a = tpgan_ops.folded_args(x, layer.weight, tuple(layer.stride), (ph, ph, pw, pw))
        if a is not None:
            a.update(bias=layer.bias, act=act)
            return a
    return dict(x=x, weight=layer.weight, bias=layer.bias, act=act, residual=residual, res_scale=res_scale,
                link_res=link_res, link_dx=link_dx, act_in_ok=act_in_ok, **_conv_geom_args(layer, pad_mod))


def group_forward(mods, xs, act_in_ok=False):
    """mods[k](xs[k]) for same-structured modules (the four LocalPathways' copies of one
    layer), in lockstep: each fused conv of the structure runs as ONE grouped node over all k
    (tpgan_ops.conv2d_group: one launch per kernel position instead of one per module).
    Structures it does not know run module by module.  act_in_ok as in
    _FusedSequential.forward (the same promise for every member)."""
    m0 = mods[0]
    if all(isinstance(m, _FusedSequential) for m in mods):
        parts = [m._parts() for m in mods]
        if all(p is not None for p in parts):
            return _group_fused(mods, xs, act_in_ok=act_in_ok)
        kids = [list(m._modules.values()) for m in mods]
        if (all(p is None for p in parts) and all(len(k) == len(kids[0]) for k in kids) and
                all(isinstance(c, (_FusedSequential, ResidualBlock)) for c in kids[0])):
            for i in range(len(kids[0])):
                xs = group_forward([k[i] for k in kids], xs, act_in_ok=act_in_ok if i == 0 else True)
            return xs
    elif all(isinstance(m, ResidualBlock) for m in mods) and all(type(m) is type(m0) for m in mods):
        out = _group_resblock(mods, xs, act_in_ok)
        if out is not None:
            return out
    return [m(x, act_in_ok=act_in_ok) if isinstance(m, (_FusedSequential, ResidualBlock)) else m(x)
            for m, x in zip(mods, xs)]


def _group_fused(seqs, xs, residuals=None, res_scales=None, post_acts=None, links_res=None, links_dx=None,
                 act_in_ok=False):
    n = len(seqs)
    calls = []
    for k, (seq, x) in enumerate(zip(seqs, xs)):
        pad, layer, act = seq._parts()
        residual = residuals[k] if residuals is not None else None
        if residual is not None:
            if act is not None:
                raise RuntimeError("residual fusion expects a conv without activation")
            act = post_acts[k]
        c = _conv_call(layer, x, pad, act, residual, res_scales[k] if res_scales is not None else 1.0,
                       links_res[k] if links_res is not None else None, links_dx[k] if links_dx is not None else None,
                       act_in_ok)
        if c is None:
            return [seq(x, residual=(residuals[k] if residuals is not None else None),
                        res_scale=(res_scales[k] if res_scales is not None else 1.0),
                        post_act=(post_acts[k] if post_acts is not None else None),
                        link_res=(links_res[k] if links_res is not None else None),
                        link_dx=(links_dx[k] if links_dx is not None else None), act_in_ok=act_in_ok)
                    for k, (seq, x) in enumerate(zip(seqs, xs))]
        calls.append(c)
    assert len(calls) == n
    return tpgan_ops.conv2d_group(calls)


def _group_resblock(blocks, xs, act_in_ok=False):
    """ResidualBlock.forward over the group; None where the block is not the fused form."""
    b0 = blocks[0]
    layers = [list(b.layers) for b in blocks]
    if (len(layers[0]) < 2 or any(len(b.shortcut._modules) for b in blocks) or
            tpgan_ops.act_code(b0.activation) is None or
            any(l[-1]._parts() is None or any(m._parts() is None for m in l[:-1]) for l in layers)):
        return None
    links = None
    if tpgan_ops.RES_LINK["enabled"] and torch.is_grad_enabled() and all(_link_ok(l[0]) for l in layers):
        links = [tpgan_ops.GradLink() for _ in blocks]
    h = xs
    for i in range(len(layers[0]) - 1):
        h = _group_fused([l[i] for l in layers], h, links_dx=links if i == 0 else None,
                         act_in_ok=(act_in_ok and links is not None) if i == 0 else True)
    return _group_fused([l[-1] for l in layers], h, residuals=xs, res_scales=[b.scaling_factor for b in blocks],
                        post_acts=[b.activation for b in blocks], links_res=links, act_in_ok=True)


def _link_ok(seq):
    """seq is a fused [conv] [act] whose input gradient can take a parked gradient (GradLink)."""
    parts = seq._parts() if isinstance(seq, _FusedSequential) else None
    if parts is None or parts[0] is not None or not isinstance(parts[1], nn.Conv2d):
        return False
    layer = parts[1]
    return layer.padding_mode == "zeros" and layer.kernel_size[0] * layer.kernel_size[1] <= 49


def _generic_forward(seq, x, act_in_ok=False):
    mods = list(seq._modules.values())
    i = 0
    pad = None
    # a chain of fused modules: each one's output is consumed by the next alone (ActToken)
    chain_ok = act_in_ok
    while i < len(mods):
        m = mods[i]
        if isinstance(m, (_FusedSequential, ResidualBlock)):
            x = m(x, act_in_ok=chain_ok)
            chain_ok = True
            i += 1
            continue
        chain_ok = False
        if isinstance(m, nn.ReflectionPad2d) and i + 1 < len(mods) and isinstance(mods[i + 1], nn.Conv2d):
            pad = m
            i += 1
            continue
        if (isinstance(m, nn.Conv2d) and pad is None and i + 1 < len(mods) and
                isinstance(mods[i + 1], nn.BatchNorm2d)):
            # Conv2d -> BatchNorm2d [-> act]: BN folded (eval) or batch statistics (train)
            act = None
            if i + 2 < len(mods) and tpgan_ops.act_code(mods[i + 2]) is not None and mods[i + 2] is not None:
                act = mods[i + 2]
            x = tpgan_ops.conv_bn_act(x, m, mods[i + 1], act)
            i += 3 if act is not None else 2
            continue
        if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)):
            act = None
            if i + 1 < len(mods) and tpgan_ops.act_code(mods[i + 1]) is not None and mods[i + 1] is not None:
                act = mods[i + 1]
                i += 1
            x = _apply_conv(m, x, pad, act)
            pad = None
        elif isinstance(m, nn.Linear):
            bn = None
            if i + 1 < len(mods) and isinstance(mods[i + 1], nn.BatchNorm1d):
                bn = mods[i + 1]
                i += 1
            act = None
            if i + 1 < len(mods) and tpgan_ops.act_code(mods[i + 1]) is not None:
                act = mods[i + 1]
                i += 1
            x = tpgan_ops.linear(x, m.weight, m.bias, act=act) if bn is None else \
                tpgan_ops.linear_bn_act(x, m, bn, act)
        else:
            x = m(x)
        i += 1
    return x


def conv(in_channels, out_channels, kernel_size, stride=1, padding=0, init="kaiming", activation=nn.ReLU(),
         use_batchnorm=False, pre_activation=False):
    """[ReflectionPad2d when padding is a 4-list] + Conv2d(bias = not use_batchnorm)
    + [BatchNorm2d] + activation (ModificationLayer.py:54-123)."""
    layers = []
    if type(padding) == type(list()):
        assert len(padding) != 3
        if len(padding) == 4:
            layers.append(nn.ReflectionPad2d(padding))
            padding = 0
    bias = not use_batchnorm
    conv_layer = nn.Conv2d(in_channels, out_channels, kernel_size, stride, padding, bias=bias)
    weight_initialization(conv_layer, init, activation)
    _channels_last_(conv_layer)
    layers.append(conv_layer)
    if pre_activation:
        layers = _batchnorm_and_activation_layer(in_channels, activation, use_batchnorm) + layers
    else:
        layers += _batchnorm_and_activation_layer(out_channels, activation, use_batchnorm)
    seq = _FusedSequential(*layers)
    seq.out_channels = out_channels
    return seq


def _batchnorm_and_activation_layer(specific_channels, activation, use_batchnorm):
    """[BatchNorm2d, activation] (or activation first for Sigmoid/Tanh), skipping a None
    activation (R2; ModificationLayer.py:125-156)."""
    return_layers = []
    nonlinear_activations = (nn.Sigmoid, nn.Tanh)
    if use_batchnorm:
        if isinstance(activation, nonlinear_activations):
            return_layers.append(activation)
            return_layers.append(nn.BatchNorm2d(specific_channels))
        else:
            return_layers.append(nn.BatchNorm2d(specific_channels))
            if activation is not None:
                return_layers.append(activation)
    elif activation is not None:
        return_layers.append(activation)
    return return_layers


def deconv(in_channels, out_channels, kernel_size, stride=1, padding=0, output_padding=0, init="kaiming",
           activation=nn.ReLU(), use_batchnorm=False, pre_activation=False):
    """ConvTranspose2d + [BatchNorm2d] + activation (ModificationLayer.py:158-202)."""
    layers = []
    bias = not use_batchnorm
    deconv_layer = nn.ConvTranspose2d(in_channels, out_channels, kernel_size, stride, padding, output_padding,
                                      bias=bias)
    weight_initialization(deconv_layer, init, activation)
    _channels_last_(deconv_layer)
    layers.append(deconv_layer)
    if pre_activation:
        layers = _batchnorm_and_activation_layer(in_channels, activation, use_batchnorm) + layers
    else:
        layers += _batchnorm_and_activation_layer(out_channels, activation, use_batchnorm)
    seq = _FusedSequential(*layers)
    seq.out_channels = out_channels
    return seq


def linear(in_channels, out_channels, activation=None, use_batchnorm=False):
    """Linear + [BatchNorm1d] + [activation] (ModificationLayer.py:204-231)."""
    layers = [nn.Linear(in_channels, out_channels, bias=not use_batchnorm)]
    if use_batchnorm:
        layers.append(nn.BatchNorm1d(out_channels))
    if activation is not None:
        layers.append(activation)
    return _FusedSequential(*layers)


class ResidualBlock(nn.Module):
    """out = act(layers(x) + scaling_factor * shortcut(x)) (ModificationLayer.py:233-302).

    As in the reference, the shortcut is a projection only when the *argument*
    use_projection is True (:283 tests the argument, not self.use_projection of :281),
    so every block built by the TP-GAN models has an identity shortcut.  The second conv
    of the main path, the residual add and the activation run as one fused HIP call."""

    def __init__(self, in_channels, out_channels=None, kernel_size=3, stride=1, padding=None, weight_init="kaiming",
                 activation=nn.ReLU(), is_bottleneck=False, use_projection=False, scaling_factor=1.0,
                 is_inplace_of_activation=False, use_batchnorm=False):
        super(ResidualBlock, self).__init__()
        self.out_channels = in_channels // stride if out_channels is None else out_channels
        self.padding = (1 if is_inplace_of_activation else (kernel_size - 1) // 2) if padding is None else padding
        if is_inplace_of_activation and (activation is nn.ReLU or isinstance(activation, nn.ReLU)):
            self.activation = nn.ReLU(inplace=True)
        else:
            self.activation = activation
        self.use_projection = use_projection
        self.scaling_factor = scaling_factor
        convs = []
        self.use_projection = use_projection or (stride != 1 or in_channels != out_channels)
        self.shortcut = conv(in_channels, out_channels, 1, stride, 0, weight_init, None, False) \
            if use_projection else nn.Sequential()
        if is_bottleneck:
            convs.append(conv(in_channels, in_channels // 2, 1, 1, 0, weight_init, self.activation, use_batchnorm,
                              False))
            convs.append(conv(in_channels // 2, self.out_channels // 2, kernel_size, stride, (kernel_size - 1) // 2,
                              weight_init, self.activation, use_batchnorm, False))
            convs.append(conv(self.out_channels // 2, self.out_channels, 1, 1, 0, None, None, use_batchnorm, False))
        else:
            convs.append(conv(in_channels, in_channels, kernel_size, 1, self.padding, weight_init, self.activation,
                              use_batchnorm, False))
            convs.append(conv(in_channels, self.out_channels, kernel_size, 1, self.padding, None, None, use_batchnorm,
                              False))
        self.layers = nn.Sequential(*convs)

    def forward(self, x, act_in_ok=False):
        """act_in_ok: x is consumed by this block alone (see _FusedSequential.forward)."""
        short = self.shortcut(x) if len(self.shortcut._modules) else x
        h = x
        layers = list(self.layers)
        last = self.layers[-1]
        fused_last = tpgan_ops.act_code(self.activation) is not None and last._parts() is not None
        # identity shortcut: the shortcut gradient is added inside the first conv's input-
        # gradient launch instead of by autograd (tpgan_ops.GradLink)
        link = (tpgan_ops.GradLink() if tpgan_ops.RES_LINK["enabled"] and fused_last and short is x and len(layers) >= 2 and _link_ok(layers[0])
                and torch.is_grad_enabled() else None)
        # ActToken: the first conv sees the whole gradient of x only when the link carries the
        # shortcut's part into its launch; the inner convs' inputs are this block's own
        for i, m in enumerate(layers[:-1]):
            if i == 0:
                h = m(h, link_dx=link, act_in_ok=act_in_ok and link is not None) if link is not None else m(h)
            else:
                h = m(h, act_in_ok=True)
        if fused_last:
            return last(h, residual=short, res_scale=self.scaling_factor, post_act=self.activation, link_res=link,
                        act_in_ok=len(layers) >= 2)
        lm = list(last._modules.values())
        if (tpgan_ops.act_code(self.activation) is not None and len(lm) == 2 and isinstance(lm[0], nn.Conv2d) and
                isinstance(lm[1], nn.BatchNorm2d) and not lm[1].training):
            # conv -> eval BN, + shortcut, activation: one fused launch (BN folded)
            return tpgan_ops.conv_bn_act(h, lm[0], lm[1], act=self.activation, residual=short,
                                         res_scale=self.scaling_factor)
        out = last(h) + self.scaling_factor * short
        return self.activation(out) if self.activation is not None else out
