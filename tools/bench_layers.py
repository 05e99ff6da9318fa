"""Per-layer kernel timing (bf16) for the dominant TP-GAN conv shapes at bs32.

    python tools/bench_layers.py [--iters 20] [--only NAME]

For each shape: forward (act + optional residual), input gradient and weight gradient
through the C-ABI, timed with HIP events on the launching stream, reported as
algorithmic TFLOP/s and fraction of the 2.5 PF dense bf16 MFMA peak.
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tp-gan_amd"))

import torch  # noqa: E402

import tpgan_ops as T  # noqa: E402
from tpgan_lib import ACT_LEAKY, ACT_NONE, ACT_RELU, FLAG_DX_ACCUM, OP_BWD_DATA, OP_FWD, check, load, stream_ptr, tt  # noqa: E402

# name: (N, Cin, H, W, Cout, k, stride, pad, transposed, output_padding, act, residual)
SHAPES = {
    "enhance_128": (32, 206, 128, 128, 206, 5, 1, 2, False, 0, ACT_LEAKY, True),
    "e128_nores": (32, 206, 128, 128, 206, 5, 1, 2, False, 0, ACT_LEAKY, False),
    "e128_plain": (32, 206, 128, 128, 206, 5, 1, 2, False, 0, ACT_NONE, False),
    "add_128": (32, 75, 128, 128, 75, 7, 1, 3, False, 0, ACT_LEAKY, True),
    "conv0_res": (32, 64, 128, 128, 64, 7, 1, 3, False, 0, ACT_LEAKY, True),
    "conv5_0": (32, 206, 128, 128, 64, 5, 1, 2, False, 0, ACT_LEAKY, False),
    "conv5_res": (32, 64, 128, 128, 64, 3, 1, 1, False, 0, ACT_LEAKY, True),
    "conv6": (32, 64, 128, 128, 32, 3, 1, 1, False, 0, ACT_LEAKY, False),
    "enhance_64": (32, 208, 64, 64, 208, 3, 1, 1, False, 0, ACT_LEAKY, True),
    "add_64": (32, 80, 64, 64, 80, 5, 1, 2, False, 0, ACT_LEAKY, True),
    "enhance_32": (32, 416, 32, 32, 416, 3, 1, 1, False, 0, ACT_LEAKY, True),
    "enhance_16": (32, 768, 16, 16, 768, 3, 1, 1, False, 0, ACT_LEAKY, True),
    "up_128": (32, 208, 64, 64, 64, 3, 2, 1, True, 1, ACT_RELU, False),
    "enh_8": (32, 576, 8, 8, 576, 2, 1, 0, False, 0, ACT_LEAKY, True),
    "conv4_res": (32, 512, 8, 8, 512, 3, 1, 1, False, 0, ACT_LEAKY, True),
    "local_5": (32, 512, 5, 5, 512, 3, 1, 1, False, 0, ACT_LEAKY, True),
    "local_10": (32, 256, 10, 10, 256, 3, 1, 1, False, 0, ACT_LEAKY, True),
    "local_20": (32, 128, 20, 20, 128, 3, 1, 1, False, 0, ACT_LEAKY, True),
    "local_40": (32, 64, 40, 40, 64, 3, 1, 1, False, 0, ACT_LEAKY, True),
    "conv4_s2": (32, 256, 16, 16, 512, 3, 2, 1, False, 0, ACT_LEAKY, False),
    "conv1_s2": (32, 64, 128, 128, 64, 5, 2, 2, False, 0, ACT_LEAKY, False),
    "conv2_s2": (32, 64, 64, 64, 128, 3, 2, 1, False, 0, ACT_LEAKY, False),
    "conv3_s2": (32, 128, 32, 32, 256, 3, 2, 1, False, 0, ACT_LEAKY, False),
    "d_conv1_s2": (64, 64, 64, 64, 128, 3, 2, 1, False, 0, ACT_LEAKY, False),
    "local_s2": (32, 256, 10, 10, 512, 3, 2, 1, False, 0, ACT_LEAKY, False),
    "local_up": (32, 512, 5, 5, 256, 3, 2, 1, True, 1, ACT_RELU, False),
    "up_16": (32, 576, 8, 8, 512, 3, 2, 1, True, 1, ACT_RELU, False),
    "up_64": (32, 416, 32, 32, 128, 3, 2, 1, True, 1, ACT_RELU, False),
    "first_7x7": (32, 3, 128, 128, 64, 7, 1, 3, False, 0, ACT_LEAKY, False),
    "dec_img": (32, 32, 128, 128, 3, 3, 1, 1, False, 0, ACT_NONE, False),
    "d_first": (64, 3, 128, 128, 64, 3, 2, 1, False, 0, ACT_LEAKY, False),
    "up_32": (32, 768, 16, 16, 256, 3, 2, 1, True, 1, ACT_RELU, False),
    # tiny layers (D_and_G_model.py:212 fc1, :220 deconv_32, :222 deconv_128, :81 local_img)
    "fc1": (32, 32768, 1, 1, 512, 1, 1, 0, False, 0, ACT_NONE, False),
    "deconv_32": (32, 64, 8, 8, 32, 3, 4, 0, True, 1, ACT_RELU, False),
    "deconv_128": (32, 16, 64, 64, 8, 3, 2, 1, True, 1, ACT_RELU, False),
    "local_img": (32, 64, 40, 40, 3, 1, 1, 0, False, 0, ACT_NONE, False),
    "local_fold": (32, 27, 40, 40, 64, 1, 1, 0, False, 0, ACT_LEAKY, False),
}
# ResNet-50 identity extractor (configs[2], ResNet.py Bottleneck; BN folded: bias + ReLU) on the
# 128 x 128 G output, bs32: one line per distinct shape, with its count per forward pass
R50 = {
    "r50_conv1": ((32, 3, 128, 128, 64, 7, 2, 3, False, 0, ACT_RELU, False), 1),
    "r50_l1_a0": ((32, 64, 32, 32, 64, 1, 1, 0, False, 0, ACT_RELU, False), 1),
    "r50_l1_a": ((32, 256, 32, 32, 64, 1, 1, 0, False, 0, ACT_RELU, False), 2),
    "r50_l1_b": ((32, 64, 32, 32, 64, 3, 1, 1, False, 0, ACT_RELU, False), 3),
    "r50_l1_c": ((32, 64, 32, 32, 256, 1, 1, 0, False, 0, ACT_RELU, True), 4),
    "r50_l2_a0": ((32, 256, 32, 32, 128, 1, 1, 0, False, 0, ACT_RELU, False), 1),
    "r50_l2_b0": ((32, 128, 32, 32, 128, 3, 2, 1, False, 0, ACT_RELU, False), 1),
    "r50_l2_ds": ((32, 256, 32, 32, 512, 1, 2, 0, False, 0, ACT_NONE, False), 1),
    "r50_l2_a": ((32, 512, 16, 16, 128, 1, 1, 0, False, 0, ACT_RELU, False), 3),
    "r50_l2_b": ((32, 128, 16, 16, 128, 3, 1, 1, False, 0, ACT_RELU, False), 3),
    "r50_l2_c": ((32, 128, 16, 16, 512, 1, 1, 0, False, 0, ACT_RELU, True), 4),
    "r50_l3_a0": ((32, 512, 16, 16, 256, 1, 1, 0, False, 0, ACT_RELU, False), 1),
    "r50_l3_b0": ((32, 256, 16, 16, 256, 3, 2, 1, False, 0, ACT_RELU, False), 1),
    "r50_l3_ds": ((32, 512, 16, 16, 1024, 1, 2, 0, False, 0, ACT_NONE, False), 1),
    "r50_l3_a": ((32, 1024, 8, 8, 256, 1, 1, 0, False, 0, ACT_RELU, False), 5),
    "r50_l3_b": ((32, 256, 8, 8, 256, 3, 1, 1, False, 0, ACT_RELU, False), 5),
    "r50_l3_c": ((32, 256, 8, 8, 1024, 1, 1, 0, False, 0, ACT_RELU, True), 6),
    "r50_l4_a0": ((32, 1024, 8, 8, 512, 1, 1, 0, False, 0, ACT_RELU, False), 1),
    "r50_l4_b0": ((32, 512, 8, 8, 512, 3, 2, 1, False, 0, ACT_RELU, False), 1),
    "r50_l4_ds": ((32, 1024, 8, 8, 2048, 1, 2, 0, False, 0, ACT_NONE, False), 1),
    "r50_l4_a": ((32, 2048, 4, 4, 512, 1, 1, 0, False, 0, ACT_RELU, False), 2),
    "r50_l4_b": ((32, 512, 4, 4, 512, 3, 1, 1, False, 0, ACT_RELU, False), 2),
    "r50_l4_c": ((32, 512, 4, 4, 2048, 1, 1, 0, False, 0, ACT_RELU, True), 3),
}


def flops(s):
    N, Cin, H, W, Cout, k, st, p, tr, op, act, res = s
    if tr:
        return 2 * N * H * W * Cin * Cout * k * k
    OH = (H + 2 * p - k) // st + 1
    OW = (W + 2 * p - k) // st + 1
    return 2 * N * OH * OW * Cout * Cin * k * k


def timed(fn, iters, graph):
    """ms per call of fn over iters back-to-back calls.  graph: the calls are captured into one
    HIP graph and replayed, so the time is the GPU's alone (eagerly, ctypes issue of a short
    kernel -- ~20 us -- outruns the kernel and the loop measures the host)."""
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if graph:
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(iters):
                fn()
        gr.replay()
        torch.cuda.synchronize()
        e0.record()
        gr.replay()
        e1.record()
    else:
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


SWEEP = {"algos": tuple(range(1, 13)), "ks": (1, 2, 4, 8, 16, 32, 64)}  # (--wg-sweep candidates)


def run(name, s, iters, passes, sweep=False, wg_algo=0, graph=False, dsplits=(), dalgo=0):
    lib = load()
    dev = torch.device("cuda", 0)
    N, Cin, H, W, Cout, k, st, p, tr, op, act, use_res = s
    dt = torch.bfloat16
    geom = T.ConvGeom(k, k, (st, st), (p, p, p, p), 0, tr, (op, op))
    OH, OW = geom.out_hw(H, W)
    x = T.new_act(N, Cin, H, W, dt, dev)
    x.normal_()
    w = torch.randn((Cin, Cout, k, k) if tr else (Cout, Cin, k, k), device=dev) * 0.05
    w = w.contiguous(memory_format=torch.channels_last)
    b = torch.zeros(Cout, device=dev)
    y = T.new_act(N, Cout, OH, OW, dt, dev)
    res = T.new_act(N, Cout, OH, OW, dt, dev).normal_() if use_res else None
    g = T.new_act(N, Cout, OH, OW, dt, dev).normal_()
    gy = T.new_act(N, Cout, OH, OW, dt, dev).normal_()
    dx = T.new_act(N, Cin, H, W, dt, dev)
    dw = torch.zeros_like(w)
    d = geom.desc(N, Cin, H, W, Cout, OH, OW, dt, act, 0.01, 1.0)
    d.data_algo = dalgo  # (0: the planner's rule; 1 halo, 2 pointwise tap-DMA kernel)
    wd = geom.desc(N, Cin, H, W, Cout, OH, OW, dt, act, 0.01, 1.0)
    wd.algo, wd.ksplit = wg_algo  # ((0, 0): the library's untuned default)
    if wg_algo == (0, 0) and T.AUTOTUNE["cache"]:  # --tune-file: the step's own pick for this shape
        wd.algo, wd.ksplit = T.AUTOTUNE["cache"].get(T._wgrad_key(wd), (0, 0))
    gd = geom.desc(N, Cin, H, W, Cout, OH, OW, dt, act, 0.01, 1.0)  # fused backward, input gradient only
    # the step's input-gradient modes since round 5 (act links): gy arrives premasked, the
    # epilogue applies the producer's act'(x) (desc.in_act) or adds into the parked shortcut
    # gradient (TPG_FLAG_DX_ACCUM) -- enhance_128's two dgrads per step are one of each
    xd = geom.desc(N, Cin, H, W, Cout, OH, OW, dt, ACT_NONE, 0.01, 1.0)
    xd.in_act, xd.in_slope = ACT_LEAKY, 0.01
    ad = geom.desc(N, Cin, H, W, Cout, OH, OW, dt, ACT_NONE, 0.01, 1.0)
    ad.flags |= FLAG_DX_ACCUM
    wsf = torch.empty(lib.tpg_conv2d_workspace(ctypes.byref(d), OP_FWD), dtype=torch.uint8, device=dev)
    wsd = torch.empty(lib.tpg_conv2d_workspace(ctypes.byref(d), OP_BWD_DATA), dtype=torch.uint8, device=dev)
    calls = {
        "fwd": lambda: check(lib.tpg_conv2d_fwd(ctypes.byref(d), tt(x), tt(w), b.data_ptr() if act else None,
                                                tt(res), tt(y), wsf.data_ptr(), wsf.numel(), stream_ptr())),
        "dgrad": lambda: check(lib.tpg_conv2d_bwd_data(ctypes.byref(d), tt(g), tt(w), tt(dx), wsd.data_ptr(),
                                                       wsd.numel(), stream_ptr())),
        "wgrad": lambda: check(lib.tpg_conv2d_bwd_filter(ctypes.byref(wd), tt(x), tt(g), tt(dw), None, 0,
                                                         stream_ptr())),
        # the step's fused backward without the weight gradient: g = gy * act'(y) staged in the
        # input gradient's halo (masked mode) where the geometry allows
        "bwd": lambda: check(lib.tpg_conv2d_bwd(ctypes.byref(gd), tt(x), tt(w), tt(y), tt(gy), tt(g), tt(dx),
                                                tt(None), None, wsd.data_ptr(), wsd.numel(), stream_ptr())),
        "dgxa": lambda: check(lib.tpg_conv2d_bwd(ctypes.byref(xd), tt(x), tt(w), tt(None), tt(gy), tt(None), tt(dx),
                                                 tt(None), None, wsd.data_ptr(), wsd.numel(), stream_ptr())),
        "dgacc": lambda: check(lib.tpg_conv2d_bwd(ctypes.byref(ad), tt(x), tt(w), tt(None), tt(gy), tt(None), tt(dx),
                                                  tt(None), None, wsd.data_ptr(), wsd.numel(), stream_ptr())),
    }
    f = flops(s)
    if sweep:  # every weight-gradient (algo, pixel split) the tuner would try
        res = []
        for algo in SWEEP["algos"]:
            for ks in SWEEP["ks"]:
                d.algo, d.ksplit = algo, ks
                rc = lib.tpg_conv2d_bwd_filter(ctypes.byref(d), tt(x), tt(g), tt(dw), None, 0, stream_ptr())
                if rc:
                    break
                ms = timed(lambda: lib.tpg_conv2d_bwd_filter(ctypes.byref(d), tt(x), tt(g), tt(dw), None, 0,
                                                              stream_ptr()), iters, graph)
                res.append((ms, algo, ks))
        d.algo, d.ksplit = 0, 0
        res.sort()
        print("%-12s wgrad sweep best: %s" % (name, "  ".join("a%d/k%d %.3f ms %.0f TF/s" % (a_, k_, ms, f / ms / 1e9)
                                                          for ms, a_, k_ in res[:6])), flush=True)
        return
    out = []
    for kind, fn in calls.items():
        if kind not in passes:
            continue
        for _ in range(3):
            fn()
        ms = timed(fn, iters, graph)
        tf = f / (ms * 1e-3) / 1e12
        out.append("%s %.3f ms %.0f TF/s (%.1f%%)" % (kind, ms, tf, 100 * tf / 2500))
        if dsplits and kind in ("fwd", "dgrad"):  # forced forward / input-gradient k splits (desc.data_ksplit)
            op = OP_FWD if kind == "fwd" else OP_BWD_DATA
            alt = []
            for ks in dsplits:
                d.data_ksplit = ks
                nb = lib.tpg_conv2d_workspace(ctypes.byref(d), op)
                wsk = torch.empty(nb, dtype=torch.uint8, device=dev)
                if kind == "fwd":
                    fk = lambda: check(lib.tpg_conv2d_fwd(ctypes.byref(d), tt(x), tt(w), b.data_ptr() if act else None,
                                                          tt(res), tt(y), wsk.data_ptr(), wsk.numel(), stream_ptr()))
                else:
                    fk = lambda: check(lib.tpg_conv2d_bwd_data(ctypes.byref(d), tt(g), tt(w), tt(dx), wsk.data_ptr(),
                                                               wsk.numel(), stream_ptr()))
                fk()
                alt.append("%d:%.3f" % (ks, timed(fk, iters, graph)))
            d.data_ksplit = 0
            out.append("splits " + " ".join(alt))
    print("%-12s %6.1f GF | %s" % (name, f / 1e9, " | ".join(out)), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default=None)
    ap.add_argument("--passes", default="fwd,dgrad,wgrad")
    ap.add_argument("--wg-sweep", action="store_true", help="time every weight-gradient algo / pixel split")
    ap.add_argument("--wg-algo", default="",
                    help="weight-gradient algo[/pixel splits] per shape, e.g. enhance_128=12/1,add_128=7")
    ap.add_argument("--sweep-algos", default="", help="--wg-sweep: these algos only, e.g. 7,12")
    ap.add_argument("--sweep-ks", default="", help="--wg-sweep: these pixel splits, e.g. 16,24,29,32")
    ap.add_argument("--graph", action="store_true", help="time graph replays (GPU time of short kernels)")
    ap.add_argument("--r50", action="store_true", help="the ResNet-50 identity extractor's shapes (configs[2])")
    ap.add_argument("--dsplits", default="", help="also time forced fwd / dgrad k splits, e.g. 1,2,4,8")
    ap.add_argument("--dalgo", type=int, default=0, help="forward / input-gradient kernel (desc.data_algo)")
    ap.add_argument("--tune-file", default=None,
                    help="weight-gradient picks saved by a train step (bench.py with TPG_TUNE_DUMP=path)")
    a = ap.parse_args()
    if a.sweep_algos:
        SWEEP["algos"] = tuple(int(v) for v in a.sweep_algos.split(","))
    if a.sweep_ks:
        SWEEP["ks"] = tuple(int(v) for v in a.sweep_ks.split(","))
    if a.tune_file:
        T.load_tuning(a.tune_file)
    shapes = {k: v[0] for k, v in R50.items()} if a.r50 else SHAPES
    ds = tuple(int(v) for v in a.dsplits.split(",") if v)
    for name, s in shapes.items():
        if a.only and name not in a.only.split(","):
            continue
        algos = dict(kv.split("=") for kv in a.wg_algo.split(",") if kv)
        al = algos.get(name, "0").split("/")
        run(name, s, a.iters, a.passes.split(","), a.wg_sweep, (int(al[0]), int(al[1]) if len(al) > 1 else 0),
            a.graph, ds, a.dalgo)


if __name__ == "__main__":
    main()
