"""ctypes binding of libtpgan_hip.so (C-ABI in include/tpgan.h).

This is the boundary a maintainer of the reference would bind: plain
pointers, strides and a hipStream_t, no torch types.  torch is used only to own device
memory and to name the current HIP stream.

The library is loaded lazily and loudly: there is no CPU fallback.  If the .so is
missing, or no ROCm device is visible, every op raises RuntimeError.
"""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libtpgan_hip.so")
if os.environ.get("TPG_LIB_PATH"):  # A/B builds of the same library (tools/ only)
    LIB_PATH = os.environ["TPG_LIB_PATH"]

TPG_F32, TPG_BF16, TPG_F16 = 0, 1, 2
ACT_NONE, ACT_RELU, ACT_LEAKY, ACT_RELU6 = 0, 1, 2, 3
SSD_TERMS, SSD_MAXN = 16, 4096  # (include/tpgan.h TPG_SSD_TERMS / TPG_SSD_MAXN)
PAD_ZERO, PAD_REFLECT = 0, 1
OP_FWD, OP_BWD_DATA, OP_BWD_FILTER = 0, 1, 2


class TpgTensor(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("dtype", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("stride", ctypes.c_int64 * 4)]


class ConvDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "n", "in_c", "in_h", "in_w", "out_c", "out_h", "out_w", "kh", "kw", "stride_h", "stride_w",
        "pad_t", "pad_b", "pad_l", "pad_r", "pad_mode", "transposed", "dtype", "act")] + [
        ("slope", ctypes.c_float), ("res_scale", ctypes.c_float), ("ksplit", ctypes.c_int32),
        ("algo", ctypes.c_int32), ("flags", ctypes.c_int32), ("data_ksplit", ctypes.c_int32),
        ("data_algo", ctypes.c_int32), ("in_act", ctypes.c_int32), ("in_slope", ctypes.c_float)]


class L1Seg(ctypes.Structure):  # tpg_l1_seg
    _fields_ = [("n", ctypes.c_int32), ("c", ctypes.c_int32), ("h", ctypes.c_int32), ("w", ctypes.c_int32),
                ("a", TpgTensor), ("b", TpgTensor), ("da", TpgTensor), ("weight", ctypes.c_float)]


L1_MAX_SEGS = 8

FLAG_WPACKED = 1
FLAG_CONCURRENT = 2
FLAG_DX_ACCUM = 4


EXPORTS = {
    "tpg_conv2d_workspace": (ctypes.c_size_t, [ctypes.POINTER(ConvDesc), ctypes.c_int32]),
    "tpg_conv2d_fwd": (ctypes.c_int32, [ctypes.POINTER(ConvDesc), TpgTensor, TpgTensor, ctypes.c_void_p, TpgTensor,
                                        TpgTensor, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "tpg_conv2d_bwd_data": (ctypes.c_int32, [ctypes.POINTER(ConvDesc), TpgTensor, TpgTensor, TpgTensor,
                                             ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "tpg_conv2d_bwd_filter": (ctypes.c_int32, [ctypes.POINTER(ConvDesc), TpgTensor, TpgTensor, TpgTensor,
                                               ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "tpg_conv2d_bwd": (ctypes.c_int32, [ctypes.POINTER(ConvDesc), TpgTensor, TpgTensor, TpgTensor, TpgTensor,
                                        TpgTensor, TpgTensor, TpgTensor, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_size_t, ctypes.c_void_p]),
    "tpg_act_bwd": (ctypes.c_int32, [ctypes.c_int32] * 5 + [ctypes.c_float, TpgTensor, TpgTensor, TpgTensor,
                                                             ctypes.c_void_p, ctypes.c_void_p]),
    "tpg_copy4d": (ctypes.c_int32, [ctypes.c_int32] * 4 + [TpgTensor, TpgTensor, ctypes.c_void_p]),
    "tpg_fold_taps": (ctypes.c_int32, [ctypes.c_int32] * 12 + [TpgTensor, TpgTensor, ctypes.c_int32, ctypes.c_void_p]),
    "tpg_local_fuse_fwd": (ctypes.c_int32, [ctypes.c_int32] * 4 + [ctypes.POINTER(TpgTensor)] +
                           [ctypes.POINTER(ctypes.c_int32)] * 4 + [TpgTensor, ctypes.c_void_p, ctypes.c_void_p]),
    "tpg_local_fuse_bwd": (ctypes.c_int32, [ctypes.c_int32] * 4 + [TpgTensor, ctypes.c_void_p,
                                                                   ctypes.POINTER(TpgTensor)] +
                           [ctypes.POINTER(ctypes.c_int32)] * 4 + [ctypes.c_void_p]),
    "tpg_maxout2_fwd": (ctypes.c_int32, [ctypes.c_int32, ctypes.c_int32, TpgTensor, TpgTensor, ctypes.c_void_p,
                                         ctypes.c_void_p]),
    "tpg_maxout2_bwd": (ctypes.c_int32, [ctypes.c_int32, ctypes.c_int32, TpgTensor, ctypes.c_void_p, TpgTensor,
                                         ctypes.c_void_p]),
    "tpg_adam": (ctypes.c_int32, [ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_void_p] + [ctypes.c_float] * 5 + [ctypes.c_int32, ctypes.c_float,
                                                                              ctypes.c_void_p, ctypes.c_void_p]),
    "tpg_grad_check": (ctypes.c_int32, [ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "tpg_dwconv2d_fwd": (ctypes.c_int32, [ctypes.POINTER(ConvDesc), TpgTensor, TpgTensor, ctypes.c_void_p, TpgTensor,
                                          TpgTensor, ctypes.c_void_p]),
    "tpg_dwconv2d_bwd_data": (ctypes.c_int32, [ctypes.POINTER(ConvDesc), TpgTensor, TpgTensor, TpgTensor,
                                               ctypes.c_void_p]),
    "tpg_dwconv2d_bwd_filter": (ctypes.c_int32, [ctypes.POINTER(ConvDesc), TpgTensor, TpgTensor, TpgTensor,
                                                 ctypes.c_void_p]),
    "tpg_maxpool2d_fwd": (ctypes.c_int32, [ctypes.c_int32] * 9 + [TpgTensor, TpgTensor, ctypes.c_void_p,
                                                                  ctypes.c_void_p]),
    "tpg_maxpool2d_bwd": (ctypes.c_int32, [ctypes.c_int32] * 9 + [TpgTensor, ctypes.c_void_p, TpgTensor,
                                                                  ctypes.c_void_p]),
    "tpg_avgpool_fwd": (ctypes.c_int32, [ctypes.c_int32] * 4 + [TpgTensor, TpgTensor, ctypes.c_void_p]),
    "tpg_avgpool_bwd": (ctypes.c_int32, [ctypes.c_int32] * 4 + [TpgTensor, TpgTensor, ctypes.c_void_p]),
    "tpg_bn_fold": (ctypes.c_int32, [ctypes.c_int32] * 4 + [TpgTensor] + [ctypes.c_void_p] * 5 +
                    [ctypes.c_float, TpgTensor, ctypes.c_void_p, ctypes.c_void_p]),
    "tpg_bn_train_fwd": (ctypes.c_int32, [ctypes.c_int32] * 4 + [TpgTensor] + [ctypes.c_void_p] * 4 +
                         [ctypes.c_float, ctypes.c_float, ctypes.c_int32, ctypes.c_float, TpgTensor] +
                         [ctypes.c_void_p] * 4),
    "tpg_bn_train_bwd": (ctypes.c_int32, [ctypes.c_int32] * 5 + [ctypes.c_float, TpgTensor, TpgTensor, TpgTensor] +
                         [ctypes.c_void_p] * 3 + [TpgTensor] + [ctypes.c_void_p] * 4),
    "tpg_conv2d_packed_bytes": (ctypes.c_size_t, [ctypes.POINTER(ConvDesc), ctypes.c_int32]),
    "tpg_pack_job_bytes": (ctypes.c_size_t, []),
    "tpg_conv2d_pack_jobs": (ctypes.c_int32, [ctypes.POINTER(ConvDesc), ctypes.c_int32, TpgTensor, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_int32]),
    "tpg_pack_prepare": (ctypes.c_int64, [ctypes.c_void_p, ctypes.c_int32]),
    "tpg_pack_run": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p]),
    "tpg_landmark_boxes": (ctypes.c_int32, [ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "tpg_crop_normalize": (ctypes.c_int32, [ctypes.c_int32] * 4 + [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64),
                                                                   ctypes.c_int32, ctypes.POINTER(TpgTensor),
                                                                   ctypes.POINTER(ctypes.c_int32),
                                                                   ctypes.POINTER(ctypes.c_int32), ctypes.c_void_p,
                                                                   ctypes.c_int32, ctypes.c_void_p]),
    "tpg_loss_workspace": (ctypes.c_size_t, []),
    "tpg_image_losses_fwd": (ctypes.c_int32, [ctypes.c_int32] * 4 + [TpgTensor, TpgTensor] + [ctypes.c_float] * 3 +
                             [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]),
    "tpg_image_losses_bwd": (ctypes.c_int32, [ctypes.c_int32] * 4 + [TpgTensor, TpgTensor] + [ctypes.c_float] * 3 +
                             [ctypes.c_void_p, TpgTensor, ctypes.c_void_p]),
    "tpg_l1_set_fwd": (ctypes.c_int32, [ctypes.c_int32, ctypes.POINTER(L1Seg), ctypes.c_void_p, ctypes.c_size_t,
                                        ctypes.c_void_p, ctypes.c_void_p]),
    "tpg_l1_set_bwd": (ctypes.c_int32, [ctypes.c_int32, ctypes.POINTER(L1Seg), ctypes.c_void_p, ctypes.c_void_p]),
    "tpg_ssd_loss_fwd": (ctypes.c_int32, [ctypes.c_int32] * 3 + [ctypes.c_void_p] * 3 + [ctypes.c_float] * 2 +
                         [ctypes.c_int32, ctypes.c_double, ctypes.c_float, ctypes.c_float] + [ctypes.c_void_p] * 5),
    "tpg_ssd_loss_bwd": (ctypes.c_int32, [ctypes.c_int32] * 3 + [ctypes.c_void_p] * 3 + [ctypes.c_float] * 4 +
                         [ctypes.c_void_p] * 7),
    "tpg_ssd_decode": (ctypes.c_int32, [ctypes.c_int32] * 3 + [ctypes.c_void_p] * 2 + [ctypes.c_float] * 2 +
                       [ctypes.c_int32] + [ctypes.c_void_p] * 3),
    "tpg_set_deterministic": (None, [ctypes.c_int32]),
    "tpg_group_begin": (None, []),
    "tpg_group_member": (None, []),
    "tpg_group_end": (ctypes.c_int32, []),
    "tpg_get_deterministic": (ctypes.c_int32, []),
    "tpg_version": (ctypes.c_char_p, []),
    "tpg_last_error": (ctypes.c_char_p, []),
}

_lib = None


def load(require_gpu=True):
    """Load libtpgan_hip.so (the HIP runtime it links is the one torch already loaded)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("libtpgan_hip.so not built (%s): run `make -C tp-gan_amd` or "
                           "__graft_entry__.build()" % LIB_PATH)
    if require_gpu and not torch.cuda.is_available():
        raise RuntimeError("tpgan HIP ops need a ROCm GPU; none is visible (there is no CPU fallback)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in EXPORTS.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def check(rc):
    if rc != 0:
        raise RuntimeError("tpgan HIP op failed (%d): %s" % (rc, _lib.tpg_last_error().decode()))


def dtype_code(dt):
    if dt == torch.float32:
        return TPG_F32
    if dt == torch.bfloat16:
        return TPG_BF16
    if dt == torch.float16:
        return TPG_F16
    raise TypeError("tpgan ops support float32, bfloat16 and float16, got %s" % dt)


def dtype_from_code(code):
    return {TPG_BF16: torch.bfloat16, TPG_F16: torch.float16}.get(code, torch.float32)


def tt(t):
    """TpgTensor for a torch tensor of rank <= 4 (logical NCHW; missing dims get stride 0)."""
    if t is None:
        return TpgTensor()
    if not t.is_cuda:
        raise RuntimeError("tpgan ops need device tensors (got a %s tensor)" % t.device)
    s = list(t.stride()) + [0] * (4 - t.dim())
    d = TpgTensor()
    d.data = t.data_ptr()
    d.dtype = dtype_code(t.dtype)
    for i in range(4):
        d.stride[i] = s[i]
    return d


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr():
    """The current HIP stream of the current device (the raw accessor skips
    torch.cuda.current_stream()'s Stream object and device-index resolution: ~10 us per op
    of host time, measured with tools/host_profile.py)."""
    if _raw_stream is not None:
        return ctypes.c_void_p(_raw_stream(torch._C._cuda_getDevice()))
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
