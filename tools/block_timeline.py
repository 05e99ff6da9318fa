"""Where a small-map conv kernel's time goes, block by block (ablation build only).

    make -C tp-gan_amd ablate ABL_SRCS="tpg_halo tpg_pw tpg_wgrad2" VARIANT=-DTPG_BLOCK_TIMING ADIR=abl/tl
    TPG_LIB_PATH=tp-gan_amd/abl/tl/libtpgan_hip.so python tools/block_timeline.py \
        --only conv4_res,local_10 --passes fwd,dgrad,wgrad [--dalgo 2] [--dsplit 4]

Thread 0 of every halo / pointwise / wgrad2 block stores s_memrealtime (100 MHz, one clock for the whole
chip) at entry (t0), before the main loop (t1), after it (t2) and after the epilogue (t3).  Per
launch: the kernel span (first t0 to last t3), the spread of block start times (dispatch ramp),
and the per-block prologue / main loop / epilogue durations, in microseconds.
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tp-gan_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))

import torch  # noqa: E402

import tpgan_ops as T  # noqa: E402
from bench_layers import SHAPES  # noqa: E402
from tpgan_lib import ACT_LEAKY, OP_BWD_DATA, OP_FWD, check, load, stream_ptr, tt  # noqa: E402

CAP = 1 << 16  # blocks


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * (len(v) - 1) + 0.5))]


def run(name, s, passes, dalgo, dsplit, buf, lib):
    dev = torch.device("cuda", 0)
    N, Cin, H, W, Cout, k, st, p, tr, op, act, use_res = s
    dt = torch.bfloat16
    geom = T.ConvGeom(k, k, (st, st), (p, p, p, p), 0, tr, (op, op))
    OH, OW = geom.out_hw(H, W)
    x = T.new_act(N, Cin, H, W, dt, dev).normal_()
    w = (torch.randn((Cin, Cout, k, k) if tr else (Cout, Cin, k, k), device=dev) * 0.05).contiguous(
        memory_format=torch.channels_last)
    b = torch.zeros(Cout, device=dev)
    y = T.new_act(N, Cout, OH, OW, dt, dev)
    res = T.new_act(N, Cout, OH, OW, dt, dev).normal_() if use_res else None
    g = T.new_act(N, Cout, OH, OW, dt, dev).normal_()
    dx = T.new_act(N, Cin, H, W, dt, dev)
    d = geom.desc(N, Cin, H, W, Cout, OH, OW, dt, act, 0.01, 1.0)
    d.data_algo, d.data_ksplit = dalgo, dsplit
    wsf = torch.empty(lib.tpg_conv2d_workspace(ctypes.byref(d), OP_FWD), dtype=torch.uint8, device=dev)
    wsd = torch.empty(lib.tpg_conv2d_workspace(ctypes.byref(d), OP_BWD_DATA), dtype=torch.uint8, device=dev)
    dw = torch.zeros_like(w)
    wd = geom.desc(N, Cin, H, W, Cout, OH, OW, dt, act, 0.01, 1.0)
    if T.AUTOTUNE["cache"]:  # --tune-file: the step's own weight-gradient pick for this shape
        wd.algo, wd.ksplit = T.AUTOTUNE["cache"].get(T._wgrad_key(wd), (0, 0))
    calls = {
        "wgrad": lambda: check(lib.tpg_conv2d_bwd_filter(ctypes.byref(wd), tt(x), tt(g), tt(dw), None, 0,
                                                         stream_ptr())),
        "fwd": lambda: check(lib.tpg_conv2d_fwd(ctypes.byref(d), tt(x), tt(w), b.data_ptr() if act else None,
                                                tt(res), tt(y), wsf.data_ptr(), wsf.numel(), stream_ptr())),
        "dgrad": lambda: check(lib.tpg_conv2d_bwd_data(ctypes.byref(d), tt(g), tt(w), tt(dx), wsd.data_ptr(),
                                                       wsd.numel(), stream_ptr())),
    }
    for kind in passes:
        fn = calls[kind]
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        call_us = e0.elapsed_time(e1) * 1e3
        buf.zero_()
        torch.cuda.synchronize()
        fn()
        torch.cuda.synchronize()
        t8 = buf.view(-1, 8).cpu()
        t8 = t8[t8[:, 0] != 0].double() * 0.01  # 100 MHz ticks -> us
        t = t8[:, :4]
        if t.numel() == 0:
            print("%-10s %-5s no instrumented blocks" % (name, kind), flush=True)
            continue
        T0 = t[:, 0].min().item()
        span = t[:, 3].max().item() - T0
        start = (t[:, 0] - T0).tolist()
        pro = (t[:, 1] - t[:, 0]).tolist()
        loop = (t[:, 2] - t[:, 1]).tolist()
        epi = (t[:, 3] - t[:, 2]).tolist()
        first_end = t[:, 3].min().item() - T0
        late = sum(1 for v in start if v > first_end)
        print("%-10s %-5s algo %d ks %d | call %.1f us  span %.1f  blocks %d (started after the first ended: %d) | "
              "start p50 %.1f p90 %.1f max %.1f | prologue %.1f/%.1f  loop %.1f/%.1f  epilogue %.1f/%.1f (mean/max)"
              % (name, kind, dalgo, dsplit, call_us, span, t.shape[0], late, pct(start, .5), pct(start, .9),
                 max(start), sum(pro) / len(pro), max(pro), sum(loop) / len(loop), max(loop),
                 sum(epi) / len(epi), max(epi)), flush=True)
        x = t8[(t8[:, 4] != 0) & (t8[:, 5] != 0) & (t8[:, 6] != 0)]
        if x.shape[0]:  # halo epilogue: to the table/barrier (4), pass 0 parked (5), pass 0 finished (6)
            m = lambda a, b: ((x[:, b] - x[:, a]).mean().item())  # noqa: E731
            print("%-10s %-5s   halo epilogue: start->4 %.1f  4->park0 %.1f  park0->fin0 %.1f  fin0->end %.1f"
                  % (name, kind, m(2, 4), m(4, 5), m(5, 6), m(6, 3)), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", required=True)
    ap.add_argument("--passes", default="fwd,dgrad")
    ap.add_argument("--dalgo", default="0", help="comma list of desc.data_algo values")
    ap.add_argument("--dsplit", default="0", help="comma list of desc.data_ksplit values")
    ap.add_argument("--tune-file", default=None, help="weight-gradient picks saved by a train step (TPG_TUNE_DUMP)")
    a = ap.parse_args()
    lib = load()
    if not (hasattr(lib, "tpg_abl_tl_pw") and hasattr(lib, "tpg_abl_tl_halo")):
        raise SystemExit("needs the -DTPG_BLOCK_TIMING ablation build (TPG_LIB_PATH)")
    if a.tune_file:
        T.load_tuning(a.tune_file)
    buf = torch.zeros(CAP * 8, dtype=torch.int64, device="cuda")
    for f in [getattr(lib, n) for n in ("tpg_abl_tl_pw", "tpg_abl_tl_halo", "tpg_abl_tl_wgrad2") if hasattr(lib, n)]:
        f.argtypes = [ctypes.c_void_p]
        assert f(buf.data_ptr()) == 0
    for name in a.only.split(","):
        for al in (int(v) for v in a.dalgo.split(",")):
            for ks in (int(v) for v in a.dsplit.split(",")):
                run(name, SHAPES[name], a.passes.split(","), al, ks, buf, lib)


if __name__ == "__main__":
    main()
