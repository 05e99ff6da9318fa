"""Autograd ops over libtpgan_hip.so — what the reference's torch.nn layers call into.

Activation layout: every activation produced here is a logical NCHW tensor whose memory
is channels-last with the pixel stride rounded up to 8 elements (16-byte rows for bf16),
i.e. a channel slice of an [N, H, W, ceil8(C)] buffer.  Consumers accept any strides
with channel stride 1; anything else (e.g. the user's NCHW fp32 images) is converted on
the device by tpg_copy4d.

Compute dtype: float32 by default (the reference's precision; MFMA f32 path), or
bfloat16 / float16 inside `with compute_dtype(torch.bfloat16)` (or torch.float16): the 16-bit MFMA
paths, fp32 accumulate.
Master weights and their gradients stay float32.
"""
import contextlib
import ctypes
import os
import weakref

import torch

from tpgan_lib import (ACT_LEAKY, ACT_NONE, ACT_RELU, ACT_RELU6, FLAG_CONCURRENT, FLAG_DX_ACCUM, FLAG_WPACKED, OP_BWD_DATA, OP_FWD,
                       PAD_REFLECT,
                       PAD_ZERO, SSD_TERMS, TPG_BF16, TPG_F32, ConvDesc, TpgTensor, check, dtype_code, dtype_from_code,
                       load, stream_ptr, tt)

_DTYPE = [torch.float32]

# Algorithmic FLOPs (2 * MAC of every conv / conv-transpose / linear) issued since the
# last reset, split by pass; bench.py divides by faces for the roofline figure.
FLOPS = {"fwd": 0, "dgrad": 0, "wgrad": 0}


def reset_flops():
    for k in FLOPS:
        FLOPS[k] = 0


# Optional in-step timing probe for one conv shape (bench.py roofline): when
# PROBE["match"](desc, pass) is true the HIP call is bracketed by HIP events on the
# current stream (the stream the kernels are launched on).
PROBE = {"match": None, "events": []}


def _probe_begin(d, which):
    m = PROBE["match"]
    if m is None or not m(d, which):
        return None
    e0 = torch.cuda.Event(enable_timing=True)
    e0.record()
    return e0


def _probe_end(e0, d, which="", work=None):
    if e0 is not None:
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        if work is None:
            work = _conv_flops(d) if which != "actb" else 6 * d.n * d.out_h * d.out_w * d.out_c  # bytes for act'
        PROBE["events"].append((e0, e1, work, which, desc_key(d)))


def desc_key(d):
    """Short human-readable shape of a conv descriptor (per-layer traces)."""
    return "%s%dx%d s%d n%d %dx%dx%d->%dx%dx%d" % ("T" if d.transposed else "", d.kh, d.kw, d.stride_h, d.n,
                                                 d.in_c, d.in_h, d.in_w, d.out_c, d.out_h, d.out_w)


def _conv_flops(d):
    if d.transposed:
        return 2 * d.n * d.in_h * d.in_w * d.in_c * d.out_c * d.kh * d.kw
    return 2 * d.n * d.out_h * d.out_w * d.out_c * d.in_c * d.kh * d.kw


@contextlib.contextmanager
def compute_dtype(dt):
    _DTYPE.append(dt)
    try:
        yield
    finally:
        _DTYPE.pop()


def get_compute_dtype():
    return _DTYPE[-1]


@contextlib.contextmanager
def deterministic(on=True):
    """Fixed-order reductions in every HIP op inside the block (tpg_set_deterministic):
    bit-identical reruns, for parity tests; slower."""
    lib = load()
    prev = lib.tpg_get_deterministic()
    lib.tpg_set_deterministic(1 if on else 0)
    try:
        yield
    finally:
        lib.tpg_set_deterministic(prev)


# Run the Generator's four local pathways on side streams (D_and_G_model.Generator).
MULTISTREAM = True
# Ops created inside `concurrent()` carry TPG_FLAG_CONCURRENT: their grids are planned for a
# share of the chip (the side-stream local pathways), forward and backward.
_CONCURRENT = [False]
CONCURRENT_HINT = {"enabled": True}


@contextlib.contextmanager
def concurrent(on=True):
    _CONCURRENT.append(bool(on) and CONCURRENT_HINT["enabled"])
    try:
        yield
    finally:
        _CONCURRENT.pop()
_SIDE = {}

def side_streams(device, n, tag=""):
    """n persistent side HIP streams of `device` (created once per (n, tag): users that may
    be in flight at the same time ask with different tags)."""
    key = (torch.device(device).index, n, tag)
    if key not in _SIDE:
        prio = SIDE_PRIORITY.get(tag, 0)
        _SIDE[key] = [torch.cuda.Stream(device=device, priority=prio) for _ in range(n)]
    return _SIDE[key]


# HIP stream priorities of the side streams (lower = higher priority).  (High priority for the
# local pathways measured 36.13 vs 35.90-35.95 ms/step in round 3: default priority.)
SIDE_PRIORITY = {"local": 0}


_ROCTX = [None]


def _roctx():
    if _ROCTX[0] is None:
        lib = False
        for name in ("libroctx64.so.4", "libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                break
            except (OSError, AttributeError):
                lib = False
        _ROCTX[0] = lib
    return _ROCTX[0]


@contextlib.contextmanager
def roctx_range(name):
    """A roctx range (SURVEY.md §5 tracing: G-fwd / D-step / G-step / all-reduce), shown by
    `rocprofv3 --marker-trace`; a no-op when libroctx64 is absent."""
    lib = _roctx()
    if lib:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib:
            lib.roctxRangePop()


def _ceil8(c):
    return (c + 7) // 8 * 8


def new_act(n, c, h, w, dtype, device):
    """Logical [n, c, h, w] view of a channels-last buffer with pixel stride ceil8(c)."""
    buf = torch.empty((n, h, w, _ceil8(c)), dtype=dtype, device=device)
    return buf.permute(0, 3, 1, 2)[:, :c]


def is_cl(t):
    return t.dim() == 4 and (t.stride(1) == 1 or t.shape[1] == 1)


def to_cl(x, dtype):
    """x as a channels-last activation of `dtype` (no copy when it already is one)."""
    if x.dim() != 4:
        raise ValueError("expected a 4-D tensor, got shape %s" % (tuple(x.shape),))
    if x.dtype == dtype and x.stride(1) == 1:
        return x
    lib = load()
    y = new_act(*x.shape, dtype=dtype, device=x.device)
    n, c, h, w = x.shape
    check(lib.tpg_copy4d(n, c, h, w, tt(x), tt(y), stream_ptr()))
    return y


def _fix_c1(t):
    """A C == 1 tensor may report any channel stride; make it 1 for the kernels."""
    if t.shape[1] == 1 and t.stride(1) != 1:
        return t.as_strided(t.shape, (t.stride(0), 1, t.stride(2), t.stride(3)))
    return t


def act_code(act):
    """(code, slope) for an activation module instance (or None)."""
    if act is None:
        return ACT_NONE, 0.0
    if isinstance(act, torch.nn.LeakyReLU):
        return ACT_LEAKY, float(act.negative_slope)
    if isinstance(act, torch.nn.ReLU6):
        return ACT_RELU6, 0.0
    if isinstance(act, torch.nn.ReLU):
        return ACT_RELU, 0.0
    return None


class ConvGeom:
    """Static geometry of one Conv2d / ConvTranspose2d call."""

    __slots__ = ("kh", "kw", "sh", "sw", "pt", "pb", "pl", "pr", "pad_mode", "transposed", "oph", "opw")

    def __init__(self, kh, kw, stride=(1, 1), pad=(0, 0, 0, 0), pad_mode=PAD_ZERO, transposed=False,
                 output_padding=(0, 0)):
        self.kh, self.kw = kh, kw
        self.sh, self.sw = stride
        self.pt, self.pb, self.pl, self.pr = pad
        self.pad_mode = pad_mode
        self.transposed = transposed
        self.oph, self.opw = output_padding

    def out_hw(self, h, w):
        if self.transposed:
            return ((h - 1) * self.sh - self.pt - self.pb + self.kh + self.oph,
                    (w - 1) * self.sw - self.pl - self.pr + self.kw + self.opw)
        return ((h + self.pt + self.pb - self.kh) // self.sh + 1, (w + self.pl + self.pr - self.kw) // self.sw + 1)

    def desc(self, n, cin, h, w, cout, oh, ow, dtype, act, slope, res_scale):
        d = ConvDesc()
        d.n, d.in_c, d.in_h, d.in_w = n, cin, h, w
        d.out_c, d.out_h, d.out_w = cout, oh, ow
        d.kh, d.kw, d.stride_h, d.stride_w = self.kh, self.kw, self.sh, self.sw
        d.pad_t, d.pad_b, d.pad_l, d.pad_r = self.pt, self.pb, self.pl, self.pr
        d.pad_mode = self.pad_mode
        d.transposed = 1 if self.transposed else 0
        d.dtype = dtype_code(dtype)
        d.act = act
        d.slope = slope
        d.res_scale = res_scale
        d.ksplit = 0
        d.flags = FLAG_CONCURRENT if _CONCURRENT[-1] else 0
        return d


# Weight-gradient autotuning: the tile (desc.algo 1..5) and pixel split (desc.ksplit) of
# tpg_conv2d_bwd_filter are chosen per shape on first use by timing every candidate into a
# scratch gradient (HIP events, device synchronised around each trial, so only during
# warm-up).  bf16 only; the cache can be saved / loaded as JSON for reproducible runs.
# frozen: shapes first seen now take the planner's default plan instead of being timed (a
# trainer closes the tuning window after its first steps, so a later new shape -- a partial
# last batch -- does not stop the device for a tuning sweep in the middle of training)
AUTOTUNE = {"enabled": True, "cache": {}, "trials": 0, "frozen": False}
# (adding the library's own split for each tile, which fills whole rounds of the chip and won
# several isolated trials, measured 36.22-36.26 vs 36.10-36.14 ms/step in round 3)
_WG_SPLITS = (1, 2, 4, 8, 16, 32, 64)
# between the powers of two: the 128 x 32 row-halo tile of enhance_128 (70 tiles) fills the
# chip's 512 resident blocks best at 36 splits -- 1.381 vs 1.405 ms at 32 (tools/bench_layers.py
# --wg-sweep, gpurun r06n); 3 / 6 / 12 for the one-round small-map grids (162 tiles x 3 = 1.9
# rounds of 256 instead of 1.3 at 2).  False: powers of two; "small" False: without 3 / 6 / 12 (A/B)
WG_SPLITS_EXTRA = {"enabled": True, "small": True}
_WG_SPLITS_X = (1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 36, 48, 64)


def _desc_tuple(d):
    return (d.n, d.in_c, d.in_h, d.in_w, d.out_c, d.out_h, d.out_w, d.kh, d.kw, d.stride_h, d.stride_w,
            d.pad_t, d.pad_b, d.pad_l, d.pad_r, d.pad_mode, d.transposed, d.dtype)


def save_tuning(path):
    """Write the autotuner's picks: weight-gradient keys as [shape, "wgrad", pick], forward /
    input-gradient split keys as [shape, "dsplit:<op>", pick]."""
    import json
    rows = []
    for k, v in AUTOTUNE["cache"].items():
        if k[0] == "dsplit":
            rows.append([list(k[2]), "dsplit:%d" % k[1], list(v)])
        else:
            rows.append([list(k[1]), k[0], list(v)])
    with open(path, "w") as f:
        json.dump(rows, f)


_WGRAD_KEY_LEN = 19  # _desc_tuple (18 fields) + the concurrency flag


def load_tuning(path):
    """Load a save_tuning file.  Files written before the concurrency flag joined the key
    (18-field keys) are upgraded: their entries were tuned for the whole chip (flag 0)."""
    import json
    with open(path) as f:
        for key, op, v in json.load(f):
            key = tuple(key)
            if op.startswith("dsplit:"):
                AUTOTUNE["cache"][("dsplit", int(op.split(":")[1]), key)] = tuple(v)
                continue
            if len(key) == _WGRAD_KEY_LEN - 1:
                key = key + (0,)
            elif len(key) != _WGRAD_KEY_LEN:
                raise ValueError("tuning file %s: key of %d fields, expected %d" % (path, len(key), _WGRAD_KEY_LEN))
            AUTOTUNE["cache"][(op, key)] = tuple(v)


def _wgrad_key(d):
    return ("wgrad", _desc_tuple(d) + (int(d.flags & FLAG_CONCURRENT),))


_TUNE_GRAPH = True
_TUNE_REPS = 4
_TUNE_STREAMS = {}


def _tune_stream():
    dev = torch.cuda.current_device()
    s = _TUNE_STREAMS.get(dev)
    if s is None:
        s = _TUNE_STREAMS[dev] = torch.cuda.Stream(dev)
    return s


def _time_wgrad(lib, d, x, g, scratch):
    """GPU times (ms) of one tpg_conv2d_bwd_filter candidate.  Default: _TUNE_REPS launches
    captured into one HIP graph, replayed twice, the second replay timed -- the GPU's time
    alone.  (Eager event pairs around one launch also time the host's ~20 us ctypes issue of
    the launch, comparable to a small layer's whole weight gradient, so candidates a few us
    apart were ranked by host jitter; _TUNE_GRAPH = False restores that timing for A/B.)"""
    if not _TUNE_GRAPH:
        ms = []
        for rep in range(2):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            check(lib.tpg_conv2d_bwd_filter(ctypes.byref(d), tt(x), tt(g), tt(scratch), None, 0, stream_ptr()))
            e1.record()
            e1.synchronize()
            ms.append(e0.elapsed_time(e1))
        return ms
    # (capture_begin on a stream of our own rather than torch.cuda.graph(), whose entry runs
    # gc.collect() + empty_cache() -- thousands of trials; thread-local capture: the tuner
    # runs on autograd's device thread)
    gr = torch.cuda.CUDAGraph()
    cs = _tune_stream()
    cs.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cs):
        gr.capture_begin(capture_error_mode="thread_local")
        try:
            for _ in range(_TUNE_REPS):
                check(lib.tpg_conv2d_bwd_filter(ctypes.byref(d), tt(x), tt(g), tt(scratch), None, 0, stream_ptr()))
        finally:
            gr.capture_end()
    gr.replay()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    gr.replay()
    e1.record()
    e1.synchronize()
    t = e0.elapsed_time(e1) / _TUNE_REPS
    del gr
    return [t]


# Forward / input-gradient k-split autotuning (desc.data_ksplit): the planner splits the k-steps
# of a small grid (< 256 blocks) over more blocks and finishes with a split-K epilogue launch; on
# the small maps a shape's best split -- or none, which drops the epilogue launch -- is timed on
# first use like the weight gradient's tile (graph replays of the candidate launches).
# Measured (profiles/r04/data_split_tuner.txt): configs[1] re-picks 8 of 90 shapes, step unchanged
# (33.33 vs 33.33 ms interleaved); configs[2]'s ResNet-50 layers gain 38.36 -> 37.93 ms/step.
_DATA_SPLITS = (0, 1, 2, 4, 8, 16)
_DATA_ALGOS = (1, 2)  # desc.data_algo: the halo-tiled kernel, the tap-DMA pointwise kernel
# log: a list to append (op, shape, {split: ms}, pick) to; margin: a candidate replaces the
# planner's plan when it takes less than margin x the plan's time (0.97: 30.68 / 30.56 against
# 30.77 / 31.00 ms/step with round 4's 0.9, alternating bench runs, gpurun r05at)
DATA_TUNE = {"enabled": True, "log": None, "margin": 0.97}
_DATA_SPLIT_WS_CAP = 256 << 20


def _time_launches(fn, reps=_TUNE_REPS):
    """GPU ms per call of fn (a launch on the current stream), from a replayed HIP graph."""
    gr = torch.cuda.CUDAGraph()
    cs = _tune_stream()
    cs.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cs):
        gr.capture_begin(capture_error_mode="thread_local")
        try:
            for _ in range(reps):
                fn()
        finally:
            gr.capture_end()
    gr.replay()  # (replays run on the current stream)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    gr.replay()
    e1.record()
    e1.synchronize()
    t = e0.elapsed_time(e1) / reps
    del gr
    return t


def _tuned_data_split(lib, d, op, device, launch):
    """(data_ksplit, data_algo) for this (op, shape): on first use the planner's own plan and
    every (kernel, split) candidate are timed through launch(ws) with the descriptor set (a
    workspace sized for it); a candidate replaces the planner's plan when it is faster by
    DATA_TUNE["margin"] (0.97: 3 %).  That margin is within one trial's noise, so the plan and
    the best candidate are timed a second time and each keeps its faster trial before the
    comparison.  Returns the pick (also left in d.data_ksplit / d.data_algo)."""
    d.data_ksplit, d.data_algo = 0, 0
    if not (AUTOTUNE["enabled"] and DATA_TUNE["enabled"]) or d.dtype == TPG_F32 or lib.tpg_get_deterministic():
        return (0, 0)
    key = ("dsplit", op, _desc_tuple(d) + (int(d.flags & FLAG_CONCURRENT), d.act))
    hit = AUTOTUNE["cache"].get(key)
    if hit is not None:
        d.data_ksplit, d.data_algo = hit
        return hit
    if torch.cuda.is_current_stream_capturing() or AUTOTUNE["frozen"]:
        return (0, 0)
    times = {}
    torch.cuda.synchronize()
    for cand in [(0, 0)] + [(ks, al) for al in _DATA_ALGOS for ks in _DATA_SPLITS]:
        d.data_ksplit, d.data_algo = cand
        if cand[0] > 1 and lib.tpg_conv2d_workspace(ctypes.byref(d), op) > _DATA_SPLIT_WS_CAP:
            continue  # (a split this large never won; its partials would not fit L2 / MALL anyway)
        ws = _ws(lib, d, op, device)
        rc = launch(ws)
        if rc:
            continue
        times[cand] = _time_launches(lambda: check(launch(ws)))
        AUTOTUNE["trials"] += 1
    best = (0, 0)
    if times:
        kbest = min(times, key=times.get)
        if kbest != (0, 0) and (0, 0) in times:
            for cand in ((0, 0), kbest):  # (second trial of the two contenders)
                d.data_ksplit, d.data_algo = cand
                ws = _ws(lib, d, op, device)
                times[cand] = min(times[cand], _time_launches(lambda: check(launch(ws))))
        if (0, 0) not in times or times[kbest] < DATA_TUNE["margin"] * times[(0, 0)]:
            best = kbest
    torch.cuda.synchronize()
    AUTOTUNE["cache"][key] = best
    if DATA_TUNE["log"] is not None:
        DATA_TUNE["log"].append((op, _desc_tuple(d)[:8], times, best))
    d.data_ksplit, d.data_algo = best
    return best


def _tuned_wgrad(lib, d, x, g, dwv):
    """(algo, ksplit) for this weight-gradient shape, tuning it on first use (pixel splits
    capped at 16 for ops planned for a share of the chip)."""
    key = _wgrad_key(d)
    hit = AUTOTUNE["cache"].get(key)
    if hit is not None:
        return hit
    if not AUTOTUNE["enabled"] or d.dtype == TPG_F32 or AUTOTUNE["frozen"]:
        return (0, 0)
    scratch = torch.empty_strided(dwv.shape, dwv.stride(), dtype=torch.float32, device=dwv.device)
    npix = d.n * (d.in_h * d.in_w if d.transposed else d.out_h * d.out_w)
    nkt = (npix + 63) // 64
    best, best_ms = (0, 0), None
    torch.cuda.synchronize()
    for algo in range(1, 13):
        for ks in (_WG_SPLITS if not WG_SPLITS_EXTRA["enabled"] else
                   _WG_SPLITS_X if WG_SPLITS_EXTRA["small"] else tuple(k for k in _WG_SPLITS_X if k not in (3, 6, 12))):
            if ks > nkt or (ks > 16 and (d.flags & FLAG_CONCURRENT)):
                break
            d.algo, d.ksplit = algo, ks
            rc = lib.tpg_conv2d_bwd_filter(ctypes.byref(d), tt(x), tt(g), tt(scratch), None, 0, stream_ptr())
            if rc == -30:  # algos 6..12 (row / image-halo kernel) do not cover this shape
                break
            check(rc)
            ms = _time_wgrad(lib, d, x, g, scratch)
            AUTOTUNE["trials"] += 1
            if not ms:
                break
            t = min(ms)
            if best_ms is None or t < best_ms:
                best, best_ms = (algo, ks), t
    d.algo, d.ksplit = 0, 0
    torch.cuda.synchronize()
    AUTOTUNE["cache"][key] = best
    return best


# ---- pre-packed weights (FlatParams-managed parameters) --------------------------------
# A conv's fp32 master weight is converted to the kernels' bf16 tile order once per weight
# update instead of inside every fwd / dgrad call: each (parameter, op, shape) gets a
# persistent packed image; FlatParams.adam() repacks every image of its network with ONE
# batched launch (tpg_pack_run) right after the Adam launch.
PACK = {"enabled": True}


class _PackEntry:
    __slots__ = ("buf", "jobs", "njobs", "dev", "nblocks", "epoch")


def _pack_entry(flat, key, d, op, w):
    lib = load()
    e = flat.pack_entries.get(key)
    if e is not None:
        return e
    nb = lib.tpg_conv2d_packed_bytes(ctypes.byref(d), op)
    if nb == 0:
        flat.pack_entries[key] = None
        return None
    jb = lib.tpg_pack_job_bytes()
    e = _PackEntry()
    e.buf = torch.empty(nb, dtype=torch.uint8, device=w.device)
    host = ctypes.create_string_buffer(jb * 64)
    n = lib.tpg_conv2d_pack_jobs(ctypes.byref(d), op, tt(w), e.buf.data_ptr(), host, 64)
    if n < 0:
        check(n)
    e.jobs = host.raw[:jb * n]
    e.njobs = n
    single = ctypes.create_string_buffer(e.jobs, len(e.jobs))
    e.nblocks = lib.tpg_pack_prepare(single, n)
    e.dev = torch.frombuffer(bytearray(single.raw), dtype=torch.uint8).to(w.device)
    e.epoch = -1
    flat.pack_entries[key] = e
    flat.pack_table = None  # the batched tables must be rebuilt
    flat.pack_version = getattr(flat, "pack_version", 0) + 1
    return e


def _packed_weight(param, d, op, w):
    """The packed image of w for (d, op) if param is FlatParams-managed, packing it now if
    it was not packed since the last update; None otherwise."""
    flat = getattr(param, "_tpg_flat", None)
    if flat is None or not PACK["enabled"] or d.dtype == TPG_F32 or w.dtype != torch.float32:
        return None
    key = (op, _desc_tuple(d), w.data_ptr(), tuple(w.stride()))
    e = _pack_entry(flat, key, d, op, w)
    if e is None:
        return None
    if e.epoch != flat.epoch:
        if e.njobs:
            check(load().tpg_pack_run(e.dev.data_ptr(), e.njobs, e.nblocks, stream_ptr()))
        e.epoch = flat.epoch
    return e.buf


def repack(flat):
    """Re-pack every weight image of `flat` in one launch (after its parameters changed)."""
    entries = [e for e in flat.pack_entries.values() if e is not None and e.njobs]
    if not entries:
        return
    lib = load()
    if flat.pack_table is None:
        raw = b"".join(e.jobs for e in entries)
        n = sum(e.njobs for e in entries)
        host = ctypes.create_string_buffer(raw, len(raw))
        nblocks = lib.tpg_pack_prepare(host, n)
        flat.pack_table = (torch.frombuffer(bytearray(host.raw), dtype=torch.uint8).to(flat.data.device), n, nblocks)
    dev, n, nblocks = flat.pack_table
    check(lib.tpg_pack_run(dev.data_ptr(), n, nblocks, stream_ptr()))
    for e in entries:
        e.epoch = flat.epoch


def _packed_tt(buf, dtype=TPG_BF16):
    t = TpgTensor()
    t.data = buf.data_ptr()
    t.dtype = dtype  # (a packed image is flagged by the descriptor; the field is informational)
    return t


def _run_maybe_packed(fn_packed, fn_plain, d, pk):
    """Call with the packed image (desc flag set); fall back to packing inside the call
    when the tensors need a different plan (-21)."""
    if pk is not None:
        base = d.flags
        d.flags = base | FLAG_WPACKED
        rc = fn_packed()
        d.flags = base
        if rc != -21:
            check(rc)
            return
    check(fn_plain())


_WS_BYTES = {}  # (op, descriptor) -> workspace bytes: the C planner runs once per shape, not per call


def _ws(lib, desc, op, device):
    key = ((op, desc.flags, desc.algo, desc.ksplit, desc.data_ksplit, desc.data_algo, lib.tpg_get_deterministic()) +
           _desc_tuple(desc))
    nb = _WS_BYTES.get(key)
    if nb is None:
        nb = lib.tpg_conv2d_workspace(ctypes.byref(desc), op)
        if nb == 0:
            check(-1)
        _WS_BYTES[key] = nb
    return torch.empty(nb, dtype=torch.uint8, device=device)


def _conv_act_forward(ctx, x, weight, bias, residual, geom, act, slope, res_scale, wparam, link_res=None, link_dx=None,
                      keep=None, links=None):
    """_ConvAct's forward on any ctx with save_for_backward (a _MemberCtx inside a grouped
    node); keep: a list that holds every temporary a deferred (grouped) launch still reads."""
    lib = load()
    dtype = get_compute_dtype()
    ctx.in_dtype = x.dtype
    x = _fix_c1(to_cl(x, dtype))
    n, cin, h, w = x.shape
    if geom.transposed:
        cin_w, cout = weight.shape[0], weight.shape[1]
    else:
        cout, cin_w = weight.shape[0], weight.shape[1]
    if cin_w != cin:
        raise RuntimeError("expected input with %d channels, got %d" % (cin_w, cin))
    oh, ow = geom.out_hw(h, w)
    y = new_act(n, cout, oh, ow, dtype, x.device)
    res = None
    if residual is not None:
        res = _fix_c1(to_cl(residual, dtype))
        if tuple(res.shape) != (n, cout, oh, ow):
            raise RuntimeError("residual shape %s != output %s" % (tuple(res.shape), (n, cout, oh, ow)))
    d = geom.desc(n, cin, h, w, cout, oh, ow, dtype, act, slope, res_scale)
    wv = weight if weight.dtype == torch.float32 else weight.float()
    pk = _packed_weight(wparam if wparam is not None else weight, d, OP_FWD, wv)
    bptr = bias.data_ptr() if bias is not None else None
    if keep is None:
        def launch(ws_):
            if pk is not None:
                d.flags = d.flags | FLAG_WPACKED
                try:
                    return lib.tpg_conv2d_fwd(ctypes.byref(d), tt(x), _packed_tt(pk), bptr, tt(res), tt(_fix_c1(y)),
                                              ws_.data_ptr(), ws_.numel(), stream_ptr())
                finally:
                    d.flags = d.flags & ~FLAG_WPACKED
            return lib.tpg_conv2d_fwd(ctypes.byref(d), tt(x), tt(wv), bptr, tt(res), tt(_fix_c1(y)), ws_.data_ptr(),
                                      ws_.numel(), stream_ptr())
        _tuned_data_split(lib, d, OP_FWD, x.device, launch)
    ws = _ws(lib, d, OP_FWD, x.device)
    FLOPS["fwd"] += _conv_flops(d)
    e0 = _probe_begin(d, "fwd")
    _run_maybe_packed(
        lambda: lib.tpg_conv2d_fwd(ctypes.byref(d), tt(x), _packed_tt(pk), bptr, tt(res), tt(_fix_c1(y)),
                                   ws.data_ptr(), ws.numel(), stream_ptr()),
        lambda: lib.tpg_conv2d_fwd(ctypes.byref(d), tt(x), tt(wv), bptr, tt(res), tt(_fix_c1(y)),
                                   ws.data_ptr(), ws.numel(), stream_ptr()), d, pk)
    _probe_end(e0, d, "fwd")
    if keep is not None:
        keep += [ws, res, wv]
    ctx.save_for_backward(x, weight, y)
    ctx.geom, ctx.act, ctx.slope, ctx.res_scale = geom, act, slope, res_scale
    ctx.has_bias, ctx.has_res = bias is not None, residual is not None
    ctx.d = d
    ctx.wparam = wparam if wparam is not None else weight
    ctx.bparam = bias
    ctx.res_dtype = residual.dtype if residual is not None else None
    ctx.x_dtype = x.dtype
    ctx.link_res, ctx.link_dx = link_res, link_dx
    ctx.act_in, ctx.act_out = links if links is not None else (None, None)
    return y


class _ConvAct(torch.autograd.Function):
    """y = act(conv(x, w) + b [+ res_scale * residual]) with a HIP forward, input gradient,
    weight gradient and a fused activation'/bias-gradient pass (backward reads only the
    saved input and output, never the pre-activation)."""

    @staticmethod
    def forward(ctx, x, weight, bias, residual, geom, act, slope, res_scale, wparam, link_res=None, link_dx=None,
                links=None):
        return _conv_act_forward(ctx, x, weight, bias, residual, geom, act, slope, res_scale, wparam, link_res,
                                 link_dx, links=links)

    @staticmethod
    def backward(ctx, gy):
        if torch.is_grad_enabled():  # create_graph=True (WGAN-GP): differentiable backward
            _act_out_taken(ctx, gy, allowed=False)
            return tuple(_conv_act_backward_graph(ctx, gy)) + (None, None, None)
        if FUSED_BWD["enabled"]:
            return _conv_act_backward_fused(ctx, gy) + (None, None, None)
        _act_out_taken(ctx, gy, allowed=False)
        return _ConvAct._backward_three_calls(ctx, gy) + (None, None, None)

    @staticmethod
    def _backward_three_calls(ctx, gy):
        lib = load()
        x, weight, y = ctx.saved_tensors
        d = ctx.d
        d.data_ksplit, d.data_algo = 0, 0  # (the forward's pick)
        dtype = y.dtype
        n, cout, oh, ow = y.shape
        g = new_act(n, cout, oh, ow, dtype, y.device)
        dbias = None
        fused_b = False
        if ctx.has_bias and ctx.needs_input_grad[2]:
            fused_b = _fused_target(ctx.bparam) is not None
            dbias = ctx.bparam.grad if fused_b else torch.zeros(cout, dtype=torch.float32, device=y.device)
        e0 = _probe_begin(d, "actb")
        check(lib.tpg_act_bwd(n, cout, oh, ow, ctx.act, ctx.slope, tt(gy), tt(y), tt(_fix_c1(g)),
                              dbias.data_ptr() if dbias is not None else None, stream_ptr()))
        _probe_end(e0, d, "actb")
        if fused_b:
            dbias = None  # accumulated straight into bias.grad
            _grad_ready(ctx.bparam)
        g = _fix_c1(g)
        dx = dw = dres = None
        wv = weight if weight.dtype == torch.float32 else weight.float()
        if ctx.needs_input_grad[0]:
            dx = new_act(*x.shape, dtype=dtype, device=x.device)
            ws = _ws(lib, d, OP_BWD_DATA, x.device)
            FLOPS["dgrad"] += _conv_flops(d)
            e0 = _probe_begin(d, "dgrad")
            pk = _packed_weight(ctx.wparam, d, OP_BWD_DATA, wv)
            _run_maybe_packed(
                lambda: lib.tpg_conv2d_bwd_data(ctypes.byref(d), tt(g), _packed_tt(pk), tt(_fix_c1(dx)), ws.data_ptr(),
                                                ws.numel(), stream_ptr()),
                lambda: lib.tpg_conv2d_bwd_data(ctypes.byref(d), tt(g), tt(wv), tt(_fix_c1(dx)), ws.data_ptr(),
                                                ws.numel(), stream_ptr()), d, pk)
            _probe_end(e0, d, "dgrad")
            if dx.dtype != ctx.in_dtype:
                dx = dx.to(ctx.in_dtype)
        if ctx.needs_input_grad[1]:
            tgt = _fused_target(ctx.wparam)
            if tgt is not None:  # dW accumulates straight into the flat gradient buffer
                dw = None
                dwv = _grad_view(tgt, weight, ctx.wparam)
            else:
                dw = torch.zeros(weight.shape, dtype=torch.float32, device=weight.device)
                if weight.dim() == 4 and weight.is_contiguous(memory_format=torch.channels_last):
                    dw = dw.contiguous(memory_format=torch.channels_last)
                dwv = dw
            FLOPS["wgrad"] += _conv_flops(d)
            algo, ks = _tuned_wgrad(lib, d, x, g, dwv)
            d.algo, d.ksplit = algo, ks
            e0 = _probe_begin(d, "wgrad")
            check(lib.tpg_conv2d_bwd_filter(ctypes.byref(d), tt(x), tt(g), tt(dwv), None, 0, stream_ptr()))
            _probe_end(e0, d, "wgrad")
            d.algo, d.ksplit = 0, 0
            if dw is None:
                _grad_ready(ctx.wparam)
            if dw is not None and dw.dtype != weight.dtype:
                dw = dw.to(weight.dtype)
        if ctx.has_res and ctx.needs_input_grad[3]:
            dres = g if ctx.res_scale == 1.0 else g * ctx.res_scale
            if dres.dtype != ctx.res_dtype:
                dres = dres.to(ctx.res_dtype)
        return dx, dw, dbias, dres, None, None, None, None, None


# Fused per-layer backward (tpg_conv2d_bwd): one C-ABI call per layer instead of
# act_bwd + bwd_data + bwd_filter; for stride-1 "same" convs the activation' is applied in
# the input-gradient kernel's halo staging and the bias gradient rides on the weight-gradient
# kernel.  FUSED_BWD["enabled"] = False restores the three-call path (A/B, tests).
FUSED_BWD = {"enabled": True}


def _deferred_read(what):
    raise RuntimeError("grouped backward: %s would read a gradient whose launch is still deferred" % what)


def _conv_act_backward_fused(ctx, gy, keep=None):
    """keep (grouped node, inside tpg_group_begin / end): the launches are deferred, so every
    temporary they use is appended to keep, and nothing may read their outputs here."""
    grouped = keep is not None
    lib = load()
    x, weight, y = ctx.saved_tensors
    d = ctx.d
    dtype = y.dtype
    n, cout, oh, ow = y.shape
    need_dx, need_dw = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
    need_db = ctx.has_bias and ctx.needs_input_grad[2]
    gy = _fix_c1(gy)
    # ActToken (producer side): the consumer's input-gradient launch already applied this conv's
    # act', so gy IS g -- the backward runs as that of the un-activated conv
    act_eff = ACT_NONE if _act_out_taken(ctx, gy) else ctx.act
    es = 4 if dtype == torch.float32 else 2
    g_is_gy = (act_eff == ACT_NONE and gy.dtype == dtype and gy.dim() == 4 and gy.stride(1) == 1 and
               gy.data_ptr() % 16 == 0 and all((gy.stride(i) * es) % 16 == 0 for i in (0, 2, 3)))
    g = gy if g_is_gy else _fix_c1(new_act(n, cout, oh, ow, dtype, y.device))
    dbias = None
    fused_b = False
    if need_db:
        fused_b = _fused_target(ctx.bparam) is not None
        dbias = ctx.bparam.grad if fused_b else torch.zeros(cout, dtype=torch.float32, device=y.device)
    # a residual block's parked shortcut gradient (GradLink): accumulated by the dgrad launch
    acc = None
    if ctx.link_dx is not None and ctx.link_dx.g is not None:
        acc, ctx.link_dx.g = ctx.link_dx.g, None
    if need_dx and acc is not None and tuple(acc.shape) == tuple(x.shape) and acc.dtype == dtype:
        dx = acc  # dgrad is added into the parked buffer in place
        acc = None
        d.flags = d.flags | FLAG_DX_ACCUM
    else:
        dx = new_act(*x.shape, dtype=dtype, device=x.device) if need_dx else None
    # ActToken (consumer side): x is the activated output of a conv whose only gradient is this
    # launch's dx (+ the parked shortcut gradient, when the residual block's link carried it in):
    # the launch leaves dx * act_x'(x) for that producer (desc.in_act)
    tok_in = ctx.act_in
    fuse_in = (tok_in is not None and ACT_LINK["enabled"] and need_dx and acc is None and
               (ctx.link_dx is None or bool(d.flags & FLAG_DX_ACCUM)))
    d.act = act_eff
    if fuse_in:
        d.in_act, d.in_slope = tok_in.act, tok_in.slope
    try:
        out = _conv_act_backward_fused_body(ctx, gy, keep, lib, x, weight, y, d, dtype, n, cout, oh, ow, need_dx, need_dw,
                                            g_is_gy, g, dbias, fused_b, acc, dx, act_eff)
    finally:
        d.act = ctx.act
        d.in_act, d.in_slope = ACT_NONE, 0.0
    if fuse_in and out[0] is not None:
        tok_in.take(out[0])
    return out


def _conv_act_backward_fused_body(ctx, gy, keep, lib, x, weight, y, d, dtype, n, cout, oh, ow, need_dx, need_dw,
                                  g_is_gy, g, dbias, fused_b, acc, dx, act_eff):
    grouped = keep is not None
    dw = dwv = None
    if need_dw:
        tgt = _fused_target(ctx.wparam)
        if tgt is not None:  # dW accumulates straight into the flat gradient buffer
            dwv = _grad_view(tgt, weight, ctx.wparam)
        else:
            dw = torch.zeros(weight.shape, dtype=torch.float32, device=weight.device)
            if weight.dim() == 4 and weight.is_contiguous(memory_format=torch.channels_last):
                dw = dw.contiguous(memory_format=torch.channels_last)
            dwv = dw
    wv = weight if weight.dtype == torch.float32 else weight.float()
    d.data_ksplit, d.data_algo = 0, 0  # (ctx.d carries the forward's pick)
    pk = _packed_weight(ctx.wparam, d, OP_BWD_DATA, wv) if need_dx else None
    if need_dx and not grouped:
        # the input-gradient launch's k split, tuned on first use into scratch g / dx (the real
        # dx may hold a parked shortcut gradient it accumulates into)
        sc = []

        def launch(ws_):
            if not sc:
                sc.extend([_fix_c1(new_act(n, cout, oh, ow, dtype, y.device)), _fix_c1(new_act(*x.shape, dtype=dtype,
                                                                                               device=x.device))])
            if pk is not None:
                d.flags = d.flags | FLAG_WPACKED
            try:
                return lib.tpg_conv2d_bwd(ctypes.byref(d), tt(x), _packed_tt(pk) if pk is not None else tt(wv), tt(y),
                                          tt(gy), tt(gy if g_is_gy else sc[0]), tt(sc[1]), tt(None), None,
                                          ws_.data_ptr(), ws_.numel(), stream_ptr())
            finally:
                d.flags = d.flags & ~FLAG_WPACKED
        _tuned_data_split(lib, d, OP_BWD_DATA, x.device, launch)
        del sc
    ws = _ws(lib, d, OP_BWD_DATA, x.device) if need_dx else None
    wsp, wsn = (ws.data_ptr(), ws.numel()) if ws is not None else (None, 0)
    # the weight-gradient tile / split is autotuned on a shape's first call, which needs g:
    # that call runs the fused op without dW, tunes on its g, then runs the weight gradient
    key = _wgrad_key(d)
    tune_first = (need_dw and AUTOTUNE["enabled"] and d.dtype != TPG_F32 and key not in AUTOTUNE["cache"] and
                  not grouped)
    if need_dw and not tune_first:
        d.algo, d.ksplit = AUTOTUNE["cache"].get(key, (0, 0))
    if need_dx:
        FLOPS["dgrad"] += _conv_flops(d)
    if need_dw:
        FLOPS["wgrad"] += _conv_flops(d)
    fx = _fix_c1(dx) if dx is not None else None
    dwt = dwv if (need_dw and not tune_first) else None
    bptr = dbias.data_ptr() if dbias is not None else None
    # probing the weight gradient (bench.py roofline, tools/trace_step.py): the same two calls
    # as the side-stream split, both on this stream, events around the second -- the kernels
    # and their order on the stream are the fused call's (input gradient, then weight gradient)
    # (only where dW and the bias go into the flat buffers: a local dw buffer would otherwise be
    # dropped below.  A parked residual gradient is fine here: both calls stay on this stream,
    # ahead of the first conv's in-place write of it)
    probe_w = (not grouped and dwt is not None and dw is None and (dbias is None or fused_b) and
               not ctx.geom.transposed and PROBE["match"] is not None and PROBE["match"](d, "wgrad") and
               not torch.cuda.is_current_stream_capturing())
    split = probe_w
    e0 = _probe_begin(d, "bwd")
    _run_maybe_packed(
        lambda: lib.tpg_conv2d_bwd(ctypes.byref(d), tt(x), _packed_tt(pk), tt(y), tt(gy), tt(g), tt(fx),
                                   tt(None if split else dwt), None if split else bptr, wsp, wsn, stream_ptr()),
        lambda: lib.tpg_conv2d_bwd(ctypes.byref(d), tt(x), tt(wv), tt(y), tt(gy), tt(g), tt(fx),
                                   tt(None if split else dwt), None if split else bptr, wsp, wsn, stream_ptr()), d, pk)
    _probe_end(e0, d, "bwd", _conv_flops(d) * (int(bool(need_dx)) + int(bool(need_dw and not tune_first and not split))))
    d.flags = d.flags & ~FLAG_DX_ACCUM
    if grouped:
        keep += [ws, g, gy, wv]
    if split:
        gt = gy if g_is_gy else g  # (g now holds act'(y) * gy: the second call takes it as is)
        d2 = _plain_desc(d)
        d2.algo, d2.ksplit = d.algo, d.ksplit
        ew = _probe_begin(d, "wgrad")
        check(lib.tpg_conv2d_bwd(ctypes.byref(d2), tt(x), tt(None), tt(None), tt(gt), tt(gt), tt(None), tt(dwt),
                                 bptr, None, 0, stream_ptr()))
        _probe_end(ew, d, "wgrad")
        if fused_b:
            _grad_ready(ctx.bparam)
        _grad_ready(ctx.wparam)
        fused_b = False
        dbias = None  # (accumulated into the flat buffer by the second call)
        dw = None
        need_dw = False
    if acc is not None and dx is not None:  # (not accumulated in the launch: shape / dtype mismatch)
        if grouped:
            _deferred_read("the parked shortcut gradient's add")
        dx = dx + acc
    if tune_first:
        algo, ks = _tuned_wgrad(lib, d, x, g, dwv)
        d.algo, d.ksplit = algo, ks
        check(lib.tpg_conv2d_bwd_filter(ctypes.byref(d), tt(x), tt(g), tt(dwv), None, 0, stream_ptr()))
    d.algo, d.ksplit = 0, 0
    if fused_b:
        dbias = None  # accumulated straight into bias.grad
        _grad_ready(ctx.bparam)
    if need_dw:
        if dw is None:
            _grad_ready(ctx.wparam)
        elif dw.dtype != weight.dtype:
            if grouped:
                _deferred_read("a weight-gradient dtype cast")
            dw = dw.to(weight.dtype)
    if dx is not None and dx.dtype != ctx.in_dtype:
        if grouped:
            _deferred_read("an input-gradient dtype cast")
        dx = dx.to(ctx.in_dtype)
    dres = None
    if ctx.has_res and ctx.needs_input_grad[3]:
        dres = g if ctx.res_scale == 1.0 else g * ctx.res_scale
        # (gy itself only when it is the ActToken consumer's input gradient: then this backward
        # owns it, and the first conv may accumulate into it in place)
        if ctx.link_res is not None and (dres is not gy or act_eff == ACT_NONE and ctx.act != ACT_NONE) and \
                dres.dtype == dtype:
            # park it for the block's first conv (its input-gradient launch adds it)
            ctx.link_res.g = dres
            dres = None
        elif dres.dtype != ctx.res_dtype:
            if grouped:
                _deferred_read("a residual-gradient dtype cast")
            dres = dres.to(ctx.res_dtype)
    if grouped and dres is not None and dres is not g and dres is not gy:
        _deferred_read("the scaled residual gradient")
    return dx, dw, dbias, dres, None, None, None, None, None


# ---- double backward (WGAN-GP): the backward of _ConvAct written as
# autograd Functions whose own backwards are the same three HIP ops, so
# torch.autograd.grad(..., create_graph=True) followed by .backward() runs entirely on
# the conv kernels:
#   g  = act'(y) * gy                (linear in gy; the mask is piecewise constant)
#   dx = dgrad(g, w)      d/dg: fwd(., w)      d/dw: wgrad(., g)
#   dw = wgrad(x, g)      d/dx: dgrad(g, .)    d/dg: fwd(x, .)
#   y' = fwd(x, w)        d/dx: dgrad(., w)    d/dw: wgrad(x, .)
def _plain_desc(d):
    e = ConvDesc()
    ctypes.memmove(ctypes.byref(e), ctypes.byref(d), ctypes.sizeof(ConvDesc))
    e.act, e.slope, e.res_scale, e.ksplit, e.algo, e.data_ksplit, e.data_algo = ACT_NONE, 0.0, 1.0, 0, 0, 0, 0
    e.in_act, e.in_slope = ACT_NONE, 0.0
    return e


class _ActMask(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gy, y, act, slope):
        lib = load()
        n, c, h, w = y.shape
        g = new_act(n, c, h, w, y.dtype, y.device)
        check(lib.tpg_act_bwd(n, c, h, w, act, slope, tt(_fix_c1(to_cl(gy, y.dtype))), tt(y), tt(_fix_c1(g)), None,
                              stream_ptr()))
        ctx.save_for_backward(y)
        ctx.act, ctx.slope = act, slope
        return _fix_c1(g)

    @staticmethod
    def backward(ctx, dg):
        (y,) = ctx.saved_tensors
        return _ActMask.apply(dg, y, ctx.act, ctx.slope), None, None, None


# (wp: the FlatParams parameter w is (a view of), when w is a layer's weight -- its pre-packed
# images then serve these launches as they serve the first-order ones, instead of a pack launch
# per call; None for a weight GRADIENT in the weight slot of the second-order terms)
class _ConvFwdPlain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, d, wp=None):
        lib = load()
        x = _fix_c1(to_cl(x, dtype_from_code(d.dtype)))
        y = new_act(d.n, d.out_c, d.out_h, d.out_w, x.dtype, x.device)
        ws = _ws(lib, d, OP_FWD, x.device)
        FLOPS["fwd"] += _conv_flops(d)
        wv = w.float()
        pk = _packed_weight(wp, d, OP_FWD, wv) if wp is not None else None
        _run_maybe_packed(
            lambda: lib.tpg_conv2d_fwd(ctypes.byref(d), tt(x), _packed_tt(pk), None, TpgTensor(), tt(_fix_c1(y)),
                                       ws.data_ptr(), ws.numel(), stream_ptr()),
            lambda: lib.tpg_conv2d_fwd(ctypes.byref(d), tt(x), tt(wv), None, TpgTensor(), tt(_fix_c1(y)),
                                       ws.data_ptr(), ws.numel(), stream_ptr()), d, pk)
        ctx.save_for_backward(x, w)
        ctx.d = d
        ctx.wp = wp
        return _fix_c1(y)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx = _ConvDgrad.apply(dy, w, ctx.d, ctx.wp) if ctx.needs_input_grad[0] else None
        dw = _ConvWgrad.apply(x, dy, ctx.d) if ctx.needs_input_grad[1] else None
        return dx, dw, None, None


class _ConvDgrad(torch.autograd.Function):
    @staticmethod
    def forward(ctx, g, w, d, wp=None):
        lib = load()
        g = _fix_c1(to_cl(g, dtype_from_code(d.dtype)))
        dx = new_act(d.n, d.in_c, d.in_h, d.in_w, g.dtype, g.device)
        ws = _ws(lib, d, OP_BWD_DATA, g.device)
        FLOPS["dgrad"] += _conv_flops(d)
        wv = w.float()
        pk = _packed_weight(wp, d, OP_BWD_DATA, wv) if wp is not None else None
        _run_maybe_packed(
            lambda: lib.tpg_conv2d_bwd_data(ctypes.byref(d), tt(g), _packed_tt(pk), tt(_fix_c1(dx)), ws.data_ptr(),
                                            ws.numel(), stream_ptr()),
            lambda: lib.tpg_conv2d_bwd_data(ctypes.byref(d), tt(g), tt(wv), tt(_fix_c1(dx)), ws.data_ptr(),
                                            ws.numel(), stream_ptr()), d, pk)
        ctx.save_for_backward(g, w)
        ctx.d = d
        ctx.wp = wp
        return _fix_c1(dx)

    @staticmethod
    def backward(ctx, ddx):
        g, w = ctx.saved_tensors
        dg = _ConvFwdPlain.apply(ddx, w, ctx.d, ctx.wp) if ctx.needs_input_grad[0] else None
        dw = _ConvWgrad.apply(ddx, g, ctx.d) if ctx.needs_input_grad[1] else None
        return dg, dw, None, None


class _ConvWgrad(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g, d):
        lib = load()
        dt = dtype_from_code(d.dtype)
        x = _fix_c1(to_cl(x, dt))
        g = _fix_c1(to_cl(g, dt))
        if d.transposed:
            shape = (d.in_c, d.out_c, d.kh, d.kw)
        else:
            shape = (d.out_c, d.in_c, d.kh, d.kw)
        dw = torch.zeros(shape, dtype=torch.float32, device=x.device).contiguous(memory_format=torch.channels_last)
        FLOPS["wgrad"] += _conv_flops(d)
        check(lib.tpg_conv2d_bwd_filter(ctypes.byref(d), tt(x), tt(g), tt(dw), None, 0, stream_ptr()))
        ctx.save_for_backward(x, g)
        ctx.d = d
        return dw

    @staticmethod
    def backward(ctx, ddw):
        x, g = ctx.saved_tensors
        dx = _ConvDgrad.apply(g, ddw, ctx.d) if ctx.needs_input_grad[0] else None
        dg = _ConvFwdPlain.apply(x, ddw, ctx.d) if ctx.needs_input_grad[1] else None
        return dx, dg, None


def _conv_act_backward_graph(ctx, gy):
    x, weight, y = ctx.saved_tensors
    wp = ctx.wparam
    if wp is not None and weight is not wp and wp.requires_grad:
        # a view of the parameter (tap-folded / reshaped weight): the same view taken again now,
        # so that it is connected to the parameter even when the forward ran with the parameter
        # frozen (the WGAN-GP first-order pass; the old view then has no gradient edge)
        weight = wp.as_strided(weight.shape, weight.stride(), weight.storage_offset())
    d = _plain_desc(ctx.d)
    g = _ActMask.apply(gy, y, ctx.d.act, ctx.d.slope)
    dx = dw = dbias = dres = None
    if ctx.needs_input_grad[0]:
        dx = _ConvDgrad.apply(g, weight, d, wp)
        if dx.dtype != ctx.in_dtype:
            dx = dx.to(ctx.in_dtype)
    if ctx.needs_input_grad[1]:
        dw = _ConvWgrad.apply(x, g, d)
        if tuple(dw.shape) != tuple(weight.shape):
            dw = dw.reshape(weight.shape)
    if ctx.has_bias and ctx.needs_input_grad[2]:
        dbias = g.float().sum((0, 2, 3))
    if ctx.has_res and ctx.needs_input_grad[3]:
        dres = g if ctx.res_scale == 1.0 else g * ctx.res_scale
        if dres.dtype != ctx.res_dtype:
            dres = dres.to(ctx.res_dtype)
    return dx, dw, dbias, dres, None, None, None, None, None


# Data-parallel overlap (tpgan_train.OverlappedGradSync): called once the last kernel that
# accumulates a fused parameter gradient has been enqueued on the current stream.
GRAD_READY_HOOK = [None]


_READY_DEFER = [None]  # inside a grouped backward: the launches are deferred, so are their ready marks


def _grad_ready(p):
    if _READY_DEFER[-1] is not None:
        _READY_DEFER[-1].append(p)
        return
    h = GRAD_READY_HOOK[0]
    if h is not None:
        h(p)


def _grad_view(tgt, weight, wparam):
    """The flat-gradient view matching `weight`, a view (reshape / tap-folded as_strided) of
    the parameter wparam: FlatParams lays p.grad out exactly like p.data."""
    if tgt.shape == weight.shape and tgt.stride() == weight.stride():
        return tgt
    return tgt.as_strided(weight.shape, weight.stride(),
                          tgt.storage_offset() + weight.storage_offset() - wparam.storage_offset())


def _fused_target(p):
    """p.grad when p opted into in-place gradient accumulation (FlatParams sets
    p._tpg_fused_grad): the HIP kernels then add into the flat fp32 gradient buffer
    directly instead of returning a fresh gradient for autograd to add.  Valid for
    .backward() use (the train step); torch.autograd.grad callers must not opt in."""
    if p is None or not getattr(p, "_tpg_fused_grad", False):
        return None
    gr = p.grad
    if gr is None or gr.dtype != torch.float32:
        return None
    return gr


def conv2d(x, weight, bias=None, stride=(1, 1), pad=(0, 0, 0, 0), pad_mode=PAD_ZERO, act=None, residual=None,
           res_scale=1.0, transposed=False, output_padding=(0, 0), wparam=None, link_res=None, link_dx=None,
           act_in_ok=False):
    """Functional entry: act is an activation module (LeakyReLU / ReLU) or None.  link_res /
    link_dx: a GradLink shared by a residual block's last conv (residual = the block input)
    and its first conv (input = the block input), see GradLink.  act_in_ok: the caller's
    promise that x is consumed by this conv alone (with link_dx: and by the shortcut whose
    gradient the link carries into this conv's input gradient) -- see ActToken."""
    code = act_code(act)
    if code is None:
        raise ValueError("activation %r cannot be fused" % (act,))
    kh, kw = weight.shape[2], weight.shape[3]
    geom = ConvGeom(kh, kw, stride, pad, pad_mode, transposed, output_padding)
    links = _act_links(x, code, act_in_ok)
    y = _ConvAct.apply(x, weight, bias, residual, geom, code[0], code[1], float(res_scale), wparam, link_res,
                       link_dx, links)
    _set_act_token(links, y)
    return y


def _act_links(x, code, act_in_ok):
    """(token of x to apply in this conv's input gradient, token of this conv's output), or None."""
    if not (ACT_LINK["enabled"] and torch.is_grad_enabled()):
        return None
    tok_in = getattr(x, "_tpg_act_tok", None) if act_in_ok else None
    if tok_in is not None and (tok_in.y is None or tok_in.y() is not x or x.dtype != get_compute_dtype() or
                               tok_in.version != x._version):
        # (converted on the way in: the gradient would pass through the conversion; or x was
        # modified in place since the producer wrote it, e.g. x.add_(c): act'(x) would then not
        # be the producer's act'(y))
        tok_in = None
    tok_out = ActToken(code[0], code[1]) if code[0] != ACT_NONE else None
    return (tok_in, tok_out)


def _set_act_token(links, y):
    if links is not None and links[1] is not None:
        links[1].y = weakref.ref(y)
        links[1].version = y._version
        y._tpg_act_tok = links[1]


class ActToken(object):
    """The producer's activation backward, moved into its consumer's input-gradient launch.

    A fused conv with an activation (ModificationLayer.py:54-123 conv(): Conv2d + LeakyReLU /
    ReLU) saves its output y; its backward would stage g = gy * act'(y) -- reading y a second
    time as a halo beside gy (the masked input gradient) or in a separate activation-backward
    pass.  When y is consumed by ONE conv alone (a residual block's inner conv pair, a chain of
    sequential layers, ModificationLayer.py:5-24, 233-302; D_and_G_model.py:409-435), that
    consumer's input-gradient launch already produces the whole gradient of y at its own
    output pixels, and it reads y there (y is its input x): its epilogue writes
    dx * act'(x) (desc.in_act), and the producer's backward takes that as g.

    The producer creates the token (act, slope, its output y); the consumer's caller asserts
    exclusivity (conv2d(act_in_ok=True)); the consumer's backward sets `pre` to the gradient
    it wrote; the producer's backward checks that the gradient it received is that tensor.
    Every path that does not apply it (double backward, three-call mode, a consumer whose
    shortcut gradient went through autograd) leaves `pre` unset, and the producer masks as
    before."""
    __slots__ = ("act", "slope", "pre", "y", "version")

    def __init__(self, act, slope):
        # (y: a weak reference -- the output carries the token, a strong one would be a cycle;
        # version: y._version when the producer returned it)
        self.act, self.slope, self.pre, self.y, self.version = act, slope, None, None, None

    def take(self, dx):
        """The consumer wrote dx = its input gradient * act'(x)."""
        self.pre = dx


# (Concat links -- a CatToken carrying per-channel-segment slopes of a concat's producers into
# the consuming conv's epilogue, desc.in_act = TPG_ACT_CHANNEL -- were built in round 5 and
# removed in round 6: measured slower on the train step, 33.40 vs 32.87 ms/step, since the
# producers then read their gradients as strided channel slices of the concat's.)


ACT_LINK = {"enabled": True}  # (A/B, tests: off = every conv masks its own gradient)


@contextlib.contextmanager
def act_links(on=True):
    """Enable / disable ActToken links for the convs run inside (the WGAN-GP forward of
    D(x_hat) disables them: its saved outputs also feed the double backward)."""
    prev = ACT_LINK["enabled"]
    ACT_LINK["enabled"] = bool(on)
    try:
        yield
    finally:
        ACT_LINK["enabled"] = prev


def _act_out_taken(ctx, gy, allowed=True):
    """True when the consumer of this conv's output already applied its act' (ActToken)."""
    tok = getattr(ctx, "act_out", None)
    if tok is None or tok.pre is None:
        return False
    pre, tok.pre = tok.pre, None
    if not allowed:
        raise RuntimeError("ActToken: a linked consumer applied act' but this backward cannot take it")
    if pre.data_ptr() != gy.data_ptr() or tuple(pre.shape) != tuple(gy.shape):
        raise RuntimeError("ActToken: the output gradient of a linked conv is not its consumer's input gradient "
                           "alone (another consumer's gradient was summed in): act_in_ok was asserted wrongly")
    return True


# ---- launch groups: one node for the same layer of several independent networks (the four
# LocalPathways, D_and_G_model.py:18-110), whose forward and backward each run inside one
# tpg_group_begin / tpg_group_end scope: every kernel position becomes ONE grid over all members
# instead of one small launch per patch.  GROUP["enabled"] = False: per-member _ConvAct nodes.
GROUP = {"enabled": True}


class _MemberCtx(object):
    """Stands in for a _ConvAct ctx inside a grouped node."""

    def save_for_backward(self, *t):
        self.saved = t


class _ConvActGroup(torch.autograd.Function):
    """n _ConvAct calls on independent inputs as one autograd node (see GROUP)."""

    @staticmethod
    def forward(ctx, specs, *flat):
        lib = load()
        keep, subs, outs = [], [], []
        lib.tpg_group_begin()
        try:
            for m, sp in enumerate(specs):
                x, w, b, r = flat[4 * m:4 * m + 4]
                lib.tpg_group_member()
                sc = _MemberCtx()
                outs.append(_conv_act_forward(sc, x, w, b, r, *sp[:7], keep=keep, links=sp[7]))
                subs.append(sc)
        finally:
            rc = lib.tpg_group_end()
        check(rc)
        saved = []
        for sc in subs:
            saved += list(sc.saved)
            sc.saved = None
        ctx.subs = subs
        ctx.save_for_backward(*saved)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gys):
        saved = ctx.saved_tensors
        for m, sc in enumerate(ctx.subs):
            sc.saved_tensors = saved[3 * m:3 * m + 3]
            sc.needs_input_grad = tuple(ctx.needs_input_grad[1 + 4 * m:5 + 4 * m]) + (False,) * 5
        grads = []
        if torch.is_grad_enabled():  # create_graph (WGAN-GP): members one by one, differentiable
            for sc, gy in zip(ctx.subs, gys):
                _act_out_taken(sc, gy, allowed=False)  # (as _ConvAct.backward: no linked act' here)
                grads += list(_conv_act_backward_graph(sc, gy)[:4])
        elif FUSED_BWD["enabled"]:
            lib = load()
            keep, ready = [], []
            lib.tpg_group_begin()
            _READY_DEFER.append(ready)
            try:
                for sc, gy in zip(ctx.subs, gys):
                    lib.tpg_group_member()
                    grads += list(_conv_act_backward_fused(sc, gy, keep=keep)[:4])
            finally:
                _READY_DEFER.pop()
                rc = lib.tpg_group_end()
            check(rc)
            for p in ready:  # (their accumulating launches are enqueued now)
                _grad_ready(p)
        else:
            for sc, gy in zip(ctx.subs, gys):
                _act_out_taken(sc, gy, allowed=False)
                grads += list(_ConvAct._backward_three_calls(sc, gy)[:4])
        for sc in ctx.subs:
            sc.saved_tensors = None
        return (None,) + tuple(grads)


def conv2d_group(calls):
    """conv2d over several independent problems as one grouped node; calls = list of dicts of
    conv2d's keyword arguments (x, weight required).  Returns the list of outputs."""
    if not GROUP["enabled"] or len(calls) < 2:
        return [conv2d(**c) for c in calls]
    specs, flat = [], []
    for c in calls:
        code = act_code(c.get("act"))
        if code is None:
            raise ValueError("activation %r cannot be fused" % (c.get("act"),))
        weight = c["weight"]
        geom = ConvGeom(weight.shape[2], weight.shape[3], c.get("stride", (1, 1)), c.get("pad", (0, 0, 0, 0)),
                        c.get("pad_mode", PAD_ZERO), c.get("transposed", False), c.get("output_padding", (0, 0)))
        specs.append((geom, code[0], code[1], float(c.get("res_scale", 1.0)), c.get("wparam"), c.get("link_res"),
                      c.get("link_dx"), _act_links(c["x"], code, c.get("act_in_ok", False))))
        flat += [c["x"], weight, c.get("bias"), c.get("residual")]
    outs = list(_ConvActGroup.apply(specs, *flat))
    for sp, y in zip(specs, outs):
        _set_act_token(sp[7], y)
    return outs


RES_LINK = {"enabled": True}  # (A/B, tests: off = autograd sums it)


class _FoldTaps(torch.autograd.Function):
    """tpg_fold_taps: an FH x FW tap window folded into channels (see conv2d_folded)."""

    @staticmethod
    def forward(ctx, x, fh, fw, sh, sw, pt, pl, oh, ow):
        lib = load()
        dtype = get_compute_dtype()
        n, c, h, w = x.shape
        y = new_act(n, fh * fw * c, oh, ow, dtype, x.device)
        check(lib.tpg_fold_taps(n, c, h, w, fh, fw, sh, sw, pt, pl, oh, ow, tt(x), tt(y), 0, stream_ptr()))
        ctx.geo = (n, c, h, w, fh, fw, sh, sw, pt, pl, oh, ow)
        ctx.x_dtype = x.dtype
        return y

    @staticmethod
    def backward(ctx, gy):
        # (differentiable under create_graph, WGAN-GP: the unfold's own backward is the fold)
        return (_UnfoldTaps.apply(gy, ctx.geo, ctx.x_dtype),) + (None,) * 8


class _UnfoldTaps(torch.autograd.Function):
    """The fold's backward: dx = the sum over every folded copy (linear; its backward is the fold)."""

    @staticmethod
    def forward(ctx, gy, geo, x_dtype):
        n, c, h, w, fh, fw, sh, sw, pt, pl, oh, ow = geo
        ctx.geo = geo
        dx = new_act(n, c, h, w, x_dtype, gy.device)
        check(load().tpg_fold_taps(n, c, h, w, fh, fw, sh, sw, pt, pl, oh, ow, tt(dx), tt(gy), 1, stream_ptr()))
        return dx

    @staticmethod
    def backward(ctx, g):
        n, c, h, w, fh, fw, sh, sw, pt, pl, oh, ow = ctx.geo
        return _FoldTaps.apply(g, fh, fw, sh, sw, pt, pl, oh, ow), None, None


FOLD = {"enabled": True}


def folded_args(x, weight, stride, pad):
    """conv2d keyword arguments (x, weight, pad, wparam) of the tap-folded form of a zero-padded
    Conv2d on a thin input (the 3-channel images; reference ModificationLayer.py:54-123 conv()
    at D_and_G_model.py:33,193,415): all KHxKW taps folded (KH*KW*C <= 32: one 32-channel MFMA
    k-step, a 1x1 conv) or, at stride 1, the KW horizontal taps (a KHx1 conv on KW*C channels)
    -- instead of KH*KW k-steps with 3 live channels of 32.  The weight is a strided view of
    the same channels-last memory ([co][ky][kx][c] is also [co][(ky*KW+kx)*C+c]), so its
    gradient accumulates in place.  None when the shape is not covered."""
    if not FOLD["enabled"] or not x.is_cuda or weight.dim() != 4:
        return None
    co, c, kh, kw = weight.shape
    if weight.stride() != (kh * kw * c, 1, kw * c, c):  # (channels-last weights only)
        return None
    n, _, h, w = x.shape
    sh, sw = stride
    pt, pb, pl, pr = pad
    oh, ow = (h + pt + pb - kh) // sh + 1, (w + pl + pr - kw) // sw + 1
    if kh * kw * c <= 32:
        xf = _FoldTaps.apply(x, kh, kw, sh, sw, pt, pl, oh, ow)
        wf = weight.as_strided((co, kh * kw * c, 1, 1), (kh * kw * c, 1, kh * kw * c, kh * kw * c))
        return dict(x=xf, weight=wf, wparam=weight)
    if sh == 1 and sw == 1 and kw * c <= 32:
        xf = _FoldTaps.apply(x, 1, kw, 1, 1, 0, pl, h, ow)
        wf = weight.as_strided((co, kw * c, kh, 1), (kh * kw * c, 1, kw * c, kw * c))
        return dict(x=xf, weight=wf, pad=(pt, pb, 0, 0), wparam=weight)
    return None


def conv2d_folded(x, weight, bias, stride, pad, act):
    """conv2d on the tap-folded form (folded_args); None when the shape is not covered."""
    a = folded_args(x, weight, stride, pad)
    if a is None:
        return None
    return conv2d(bias=bias, act=act, **a)


class GradLink(object):
    """Hand-off of a residual block's shortcut gradient (ModificationLayer.ResidualBlock,
    reference ModificationLayer.py:233-302).  The block input x feeds both the first conv and,
    as the residual, the last one, so autograd would sum two gradients of x with a separate
    add.  Instead the last conv's fused backward parks its residual gradient here (returning
    None for it) and the first conv's input-gradient launch adds it in its epilogue
    (TPG_FLAG_DX_ACCUM: dx = dgrad + parked gradient, written into the parked buffer).  The
    first conv's backward always runs after the last conv's (it needs its output gradient);
    the double-backward and three-call paths leave the link unused."""
    __slots__ = ("g",)

    def __init__(self):
        self.g = None

    @staticmethod
    def accepts(geom):
        """Geometries whose input-gradient launch can accumulate (zero padding, no GEMM form)."""
        return geom.pad_mode == PAD_ZERO and not geom.transposed and geom.kh * geom.kw <= 49


class _FlattenNCHW(torch.autograd.Function):
    """[B, C, H, W] channels-last map -> [B, C*H*W, 1, 1] in NCHW flattening order (the
    reference's view(B, -1) before fc1, D_and_G_model.py:289); the backward hands the
    gradient back channels-last."""

    @staticmethod
    def forward(ctx, x):
        b, c, h, w = x.shape
        ctx.shape = (b, c, h, w)
        return x.contiguous().view(b, c * h * w, 1, 1)

    @staticmethod
    def backward(ctx, g):
        b, c, h, w = ctx.shape
        return to_cl(g.reshape(b, c, h, w), g.dtype)


# fc1 (a Linear on an NCHW-flattened map): as a 1x1 conv on the flattened activation instead
# of an HxW full-kernel conv on the channels-last map, so its weight gradient walks the weight
# in its own (NCHW) order -- coalesced rows instead of 4-byte accesses 256 B apart (the
# full-kernel form's weight-gradient launch took 0.34 ms for 67 MB)
LINEAR_FLAT = {"enabled": True}


def linear(x, weight, bias=None, act=None, image_hw=None):
    """nn.Linear on [B, K] (or a [B, C, H, W] map flattened in NCHW order, fc1 at
    D_and_G_model.py:289); returns [B, out]."""
    out_f, in_f = weight.shape
    if x.dim() == 4 and LINEAR_FLAT["enabled"] and x.is_cuda:
        b = x.shape[0]
        xf = _FlattenNCHW.apply(to_cl(x, get_compute_dtype()))
        y = conv2d(xf, weight.view(out_f, in_f, 1, 1), bias, act=act, wparam=weight)
    elif x.dim() == 4:
        b, c, h, w = x.shape
        w4 = weight.view(out_f, c, h, w)
        y = conv2d(x, w4, bias, act=act, wparam=weight)
    else:
        b = x.shape[0]
        w4 = weight.view(out_f, in_f, 1, 1)
        y = conv2d(x.reshape(b, in_f, 1, 1), w4, bias, act=act, wparam=weight)
    return y.reshape(b, out_f)


class _Cat(torch.autograd.Function):
    """torch.cat(dim=1) into one channels-last buffer; the backward is free channel views."""

    @staticmethod
    def forward(ctx, *xs):
        lib = load()
        dtype = get_compute_dtype()
        n, _, h, w = xs[0].shape
        ctot = sum(t.shape[1] for t in xs)
        out = new_act(n, ctot, h, w, dtype, xs[0].device)
        off = 0
        sizes = []
        for t in xs:
            c = t.shape[1]
            if t.shape[0] != n or t.shape[2] != h or t.shape[3] != w:
                raise RuntimeError("Sizes of tensors must match except in dimension 1")
            check(lib.tpg_copy4d(n, c, h, w, tt(t), tt(out[:, off:off + c]), stream_ptr()))
            sizes.append(c)
            off += c
        ctx.sizes = sizes
        ctx.dtypes = [t.dtype for t in xs]
        return out

    @staticmethod
    def backward(ctx, gy):
        outs = []
        off = 0
        for c, dt in zip(ctx.sizes, ctx.dtypes):
            gv = gy[:, off:off + c]
            outs.append(gv if gv.dtype == dt else gv.to(dt))
            off += c
        return tuple(outs)


def cat(xs):
    """torch.cat(xs, 1) into one channels-last buffer."""
    return _Cat.apply(*xs)


# ---- fused G-step image losses (tpg_losses.hip; tpgan_train._g_losses): one partial-sum and one
# final launch forward, one launch backward, instead of ~100 aten launches on the critical path
_LOSS_WS = {}


def _loss_ws(device):
    """The losses' partial-sum scratch (one per device; every loss launch is on the step's own
    stream, in order)."""
    ws = _LOSS_WS.get(device)
    if ws is None:
        ws = _LOSS_WS[device] = torch.empty(load().tpg_loss_workspace() // 4, dtype=torch.float32, device=device)
    return ws


def _grad_like(x):
    n, c, h, w = x.shape
    return new_act(n, c, h, w, x.dtype, x.device) if is_cl(x) else torch.empty_like(x, memory_format=torch.contiguous_format)


class _ImageLosses(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, r, w_pix, w_sym, w_tv):
        lib = load()
        n, c, h, w = x.shape
        if tuple(r.shape) != tuple(x.shape):
            raise RuntimeError("image_losses: target %s != %s" % (tuple(r.shape), tuple(x.shape)))
        ws = _loss_ws(x.device)
        out = torch.empty((), dtype=torch.float32, device=x.device)
        check(lib.tpg_image_losses_fwd(n, c, h, w, tt(x), tt(r), w_pix, w_sym, w_tv, ws.data_ptr(), ws.numel() * 4,
                                       out.data_ptr(), stream_ptr()))
        ctx.save_for_backward(x, r)
        ctx.wts = (w_pix, w_sym, w_tv)
        return out

    @staticmethod
    def backward(ctx, g):
        x, r = ctx.saved_tensors
        n, c, h, w = x.shape
        g = g.float().contiguous()
        dx = _grad_like(x)
        check(load().tpg_image_losses_bwd(n, c, h, w, tt(x), tt(r), *ctx.wts, g.data_ptr(), tt(dx), stream_ptr()))
        return dx, None, None, None, None


def image_losses(x, target, w_pix, w_sym, w_tv):
    """w_pix * mean|x - target| + w_sym * mean|x - flip_W(x)| + w_tv * (mean |vertical| + mean
    |horizontal| neighbour differences of x), as one fp32 scalar (the G step's pixel,
    symmetry and total-variation terms, tpgan_train._g_losses).  Gradients flow to x only: a
    target that requires grad is refused rather than silently left without one."""
    if target.requires_grad and torch.is_grad_enabled():
        raise ValueError("image_losses: the target must not require grad (no gradient is computed for it)")
    return _ImageLosses.apply(x, target, float(w_pix), float(w_sym), float(w_tv))


class _L1Set(torch.autograd.Function):
    @staticmethod
    def forward(ctx, weights, *ts):
        from tpgan_lib import L1Seg
        lib = load()
        nseg = len(weights)
        segs = (L1Seg * nseg)()
        for k in range(nseg):
            a, b = ts[2 * k], ts[2 * k + 1]
            if tuple(a.shape) != tuple(b.shape) or a.dim() != 4:
                raise RuntimeError("l1_means: pair %d shapes %s / %s" % (k, tuple(a.shape), tuple(b.shape)))
            segs[k].n, segs[k].c, segs[k].h, segs[k].w = a.shape
            segs[k].a, segs[k].b, segs[k].weight = tt(a), tt(b), float(weights[k])
        ws = _loss_ws(ts[0].device)
        out = torch.empty((), dtype=torch.float32, device=ts[0].device)
        check(lib.tpg_l1_set_fwd(nseg, segs, ws.data_ptr(), ws.numel() * 4, out.data_ptr(), stream_ptr()))
        ctx.save_for_backward(*ts)
        ctx.weights = weights
        return out

    @staticmethod
    def backward(ctx, g):
        from tpgan_lib import L1Seg
        ts = ctx.saved_tensors
        nseg = len(ctx.weights)
        segs = (L1Seg * nseg)()
        grads = [None] * len(ts)
        for k in range(nseg):
            a, b = ts[2 * k], ts[2 * k + 1]
            segs[k].n, segs[k].c, segs[k].h, segs[k].w = a.shape
            segs[k].a, segs[k].b, segs[k].weight = tt(a), tt(b), float(ctx.weights[k])
            if ctx.needs_input_grad[1 + 2 * k]:
                grads[2 * k] = _grad_like(a)
                segs[k].da = tt(grads[2 * k])
        g = g.float().contiguous()
        check(load().tpg_l1_set_bwd(nseg, segs, g.data_ptr(), stream_ptr()))
        return (None,) + tuple(grads)


def l1_means(pairs, weights):
    """sum_i weights[i] * mean|a_i - b_i| over up to 8 (a_i, b_i) pairs of 4-D tensors, one fp32
    scalar; gradients flow to the a_i (the G step's local-pathway pixel terms)."""
    from tpgan_lib import L1_MAX_SEGS
    if not 1 <= len(pairs) <= L1_MAX_SEGS or len(weights) != len(pairs):
        raise ValueError("l1_means: 1..%d pairs with one weight each" % L1_MAX_SEGS)
    if torch.is_grad_enabled() and any(b.requires_grad for _, b in pairs):
        raise ValueError("l1_means: the b_i must not require grad (gradients flow to the a_i only)")
    return _L1Set.apply(tuple(float(w) for w in weights), *[t for p in pairs for t in p])


class _LocalFuse(torch.autograd.Function):
    @staticmethod
    def forward(ctx, geom, *parts):
        lib = load()
        dtype = get_compute_dtype()
        out_h, out_w, tops, lefts = geom
        n, c = parts[0].shape[:2]
        y = new_act(n, c, out_h, out_w, dtype, parts[0].device)
        amax = torch.empty((n, out_h, out_w, c), dtype=torch.uint8, device=parts[0].device)
        arr = (TpgTensor * 4)(*[tt(p) for p in parts])
        ph = (ctypes.c_int32 * 4)(*[p.shape[2] for p in parts])
        pw = (ctypes.c_int32 * 4)(*[p.shape[3] for p in parts])
        top = (ctypes.c_int32 * 4)(*tops)
        left = (ctypes.c_int32 * 4)(*lefts)
        check(lib.tpg_local_fuse_fwd(n, c, out_h, out_w, arr, ph, pw, top, left, tt(_fix_c1(y)), amax.data_ptr(),
                                     stream_ptr()))
        ctx.save_for_backward(amax)
        ctx.geom = geom
        ctx.shapes = [tuple(p.shape) for p in parts]
        ctx.dtypes = [p.dtype for p in parts]
        return y

    @staticmethod
    def backward(ctx, gy):
        lib = load()
        (amax,) = ctx.saved_tensors
        out_h, out_w, tops, lefts = ctx.geom
        grads = []
        tts = []
        for i, (shp, dt) in enumerate(zip(ctx.shapes, ctx.dtypes)):
            if ctx.needs_input_grad[1 + i]:
                gdt = dt if dt in (torch.float32, torch.bfloat16, torch.float16) else torch.float32
                gi = new_act(*shp, dtype=gdt, device=gy.device)
                grads.append(gi)
                tts.append(tt(_fix_c1(gi)))
            else:
                grads.append(None)
                tts.append(TpgTensor())
        if any(gr is not None for gr in grads):
            n, c = ctx.shapes[0][:2]
            arr = (TpgTensor * 4)(*tts)
            ph = (ctypes.c_int32 * 4)(*[s[2] for s in ctx.shapes])
            pw = (ctypes.c_int32 * 4)(*[s[3] for s in ctx.shapes])
            check(lib.tpg_local_fuse_bwd(n, c, out_h, out_w, tt(gy), amax.data_ptr(), arr, ph, pw,
                                         (ctypes.c_int32 * 4)(*tops), (ctypes.c_int32 * 4)(*lefts), stream_ptr()))
        return (None,) + tuple(grads)


def local_fuse(parts, out_hw, tops, lefts):
    return _LocalFuse.apply((out_hw[0], out_hw[1], tuple(tops), tuple(lefts)), *parts)


class _Maxout2(torch.autograd.Function):
    """fc2: MaxPool1d(2, 2) over pairs of fc1 features (D_and_G_model.py:214,290)."""

    @staticmethod
    def forward(ctx, x):
        lib = load()
        b, k = x.shape
        m = k // 2
        y = torch.empty((b, m), dtype=x.dtype, device=x.device)
        amax = torch.empty((b, m), dtype=torch.uint8, device=x.device)
        check(lib.tpg_maxout2_fwd(b, m, tt(x), tt(y), amax.data_ptr(), stream_ptr()))
        ctx.save_for_backward(amax)
        ctx.shape = (b, k)
        ctx.dtype = x.dtype
        return y

    @staticmethod
    def backward(ctx, gy):
        lib = load()
        (amax,) = ctx.saved_tensors
        b, k = ctx.shape
        dx = torch.empty((b, k), dtype=ctx.dtype, device=gy.device)
        check(lib.tpg_maxout2_bwd(b, k // 2, tt(gy), amax.data_ptr(), tt(dx), stream_ptr()))
        return dx


def maxout2(x):
    return _Maxout2.apply(x)


def grad_check(grad, state):
    """state[3] := 1 if grad holds an inf / NaN (the next adam_step on `state` then skips)."""
    check(load().tpg_grad_check(grad.numel(), grad.data_ptr(), state.data_ptr(), stream_ptr()))


def adam_advance(state, beta1, beta2):
    """Advance the device step counter in `state` (and its bias corrections) without updating
    anything: the per-step call of an optimizer whose buckets then run adam_slice."""
    lib = load()
    check(lib.tpg_adam(0, None, None, None, None, 0.0, beta1, beta2, 0.0, 0.0, 0, 1.0, state.data_ptr(),
                       stream_ptr()))


def adam_slice(param, grad, exp_avg, exp_avg_sq, off, n, lr, beta1, beta2, eps, weight_decay, state, grad_scale=1.0):
    """Adam on elements [off, off + n) of the flat buffers under the step adam_advance set."""
    lib = load()
    check(lib.tpg_adam(n, param.data_ptr() + 4 * off, grad.data_ptr() + 4 * off, exp_avg.data_ptr() + 4 * off,
                       exp_avg_sq.data_ptr() + 4 * off, lr, beta1, beta2, eps, weight_decay, -1, grad_scale,
                       state.data_ptr(), stream_ptr()))


def repack_range(flat, off, n, epoch):
    """Re-pack, in one launch on the current stream, the weight images of the parameters that
    lie in elements [off, off + n) of flat.data, marking them packed at `epoch`."""
    cache = getattr(flat, "range_packs", None)
    if cache is None or cache[0] != flat.pack_version:
        cache = flat.range_packs = (flat.pack_version, {})
    hit = cache[1].get((off, n))
    lib = load()
    if hit is None:
        base = flat.data.data_ptr()
        entries = [e for k, e in flat.pack_entries.items()
                   if e is not None and e.njobs and off <= (k[2] - base) // 4 < off + n]
        if entries:
            raw = b"".join(e.jobs for e in entries)
            nj = sum(e.njobs for e in entries)
            host = ctypes.create_string_buffer(raw, len(raw))
            nblocks = lib.tpg_pack_prepare(host, nj)
            hit = (entries, torch.frombuffer(bytearray(host.raw), dtype=torch.uint8).to(flat.data.device), nj, nblocks)
        else:
            hit = (entries, None, 0, 0)
        cache[1][(off, n)] = hit
    entries, dev, nj, nblocks = hit
    if nj:
        check(lib.tpg_pack_run(dev.data_ptr(), nj, nblocks, stream_ptr()))
    for e in entries:
        e.epoch = epoch


def adam_step(param, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay, state, step=0, grad_scale=1.0):
    """In-place Adam on flat fp32 buffers (torch.optim.Adam semantics).  `state` is a device
    float32[4] {step, bias corrections, skip flag}; step=0 advances its counter on the device
    (graph-safe); a set skip flag (grad_check) leaves everything untouched."""
    lib = load()
    check(lib.tpg_adam(param.numel(), param.data_ptr(), grad.data_ptr(), exp_avg.data_ptr(), exp_avg_sq.data_ptr(),
                       lr, beta1, beta2, eps, weight_decay, int(step), grad_scale, state.data_ptr(), stream_ptr()))


# ---------------------------------------------------------------------------------------
# Identity-feature extractor ops (MobileNetV2.py, ResNet.py): depthwise conv, BatchNorm
# (eval: folded into the conv; train: batch statistics), max / average pooling.
# ---------------------------------------------------------------------------------------
def _dw_desc(n, c, h, w, oh, ow, kh, kw, stride, pad, dtype, act, slope, res_scale):
    d = ConvDesc()
    d.n, d.in_c, d.in_h, d.in_w = n, c, h, w
    d.out_c, d.out_h, d.out_w = c, oh, ow
    d.kh, d.kw, d.stride_h, d.stride_w = kh, kw, stride[0], stride[1]
    d.pad_t, d.pad_b, d.pad_l, d.pad_r = pad[0], pad[0], pad[1], pad[1]
    d.dtype = dtype_code(dtype)
    d.act, d.slope, d.res_scale = act, slope, res_scale
    return d


class _DWConv(torch.autograd.Function):
    """Depthwise Conv2d (groups = C) + bias [+ residual] + activation (MobileNetV2.py:105-107)."""

    @staticmethod
    def forward(ctx, x, weight, bias, residual, stride, pad, act, slope, res_scale):
        lib = load()
        dtype = get_compute_dtype()
        x = to_cl(x, dtype)
        n, c, h, w = x.shape
        kh, kw = weight.shape[2], weight.shape[3]
        if weight.shape[0] != c or weight.shape[1] != 1:
            raise RuntimeError("depthwise weight %s does not match %d channels" % (tuple(weight.shape), c))
        oh = (h + 2 * pad[0] - kh) // stride[0] + 1
        ow = (w + 2 * pad[1] - kw) // stride[1] + 1
        y = new_act(n, c, oh, ow, dtype, x.device)
        res = to_cl(residual, dtype) if residual is not None else None
        d = _dw_desc(n, c, h, w, oh, ow, kh, kw, stride, pad, dtype, act, slope, res_scale)
        wv = weight if weight.dtype == torch.float32 else weight.float()
        FLOPS["fwd"] += 2 * n * oh * ow * c * kh * kw
        check(lib.tpg_dwconv2d_fwd(ctypes.byref(d), tt(x), tt(wv), bias.data_ptr() if bias is not None else None,
                                   tt(res), tt(y), stream_ptr()))
        ctx.save_for_backward(x, wv, y)
        ctx.d = d
        ctx.has_bias, ctx.has_res = bias is not None, residual is not None
        ctx.in_dtype = ctx.res_dtype = None
        ctx.wdtype = weight.dtype
        return y

    @staticmethod
    def backward(ctx, gy):
        lib = load()
        x, wv, y = ctx.saved_tensors
        d = ctx.d
        n, c, oh, ow = y.shape
        g = new_act(n, c, oh, ow, y.dtype, y.device)
        dbias = torch.zeros(c, dtype=torch.float32, device=y.device) \
            if (ctx.has_bias and ctx.needs_input_grad[2]) else None
        check(lib.tpg_act_bwd(n, c, oh, ow, d.act, d.slope, tt(to_cl(gy, y.dtype)), tt(y), tt(g),
                              dbias.data_ptr() if dbias is not None else None, stream_ptr()))
        dx = dw = dres = None
        if ctx.needs_input_grad[0]:
            dx = new_act(*x.shape, dtype=x.dtype, device=x.device)
            FLOPS["dgrad"] += 2 * n * oh * ow * c * d.kh * d.kw
            check(lib.tpg_dwconv2d_bwd_data(ctypes.byref(d), tt(g), tt(wv), tt(dx), stream_ptr()))
        if ctx.needs_input_grad[1]:
            dw = torch.zeros(wv.shape, dtype=torch.float32, device=wv.device)
            FLOPS["wgrad"] += 2 * n * oh * ow * c * d.kh * d.kw
            check(lib.tpg_dwconv2d_bwd_filter(ctypes.byref(d), tt(x), tt(g), tt(dw), stream_ptr()))
            if ctx.wdtype != torch.float32:
                dw = dw.to(ctx.wdtype)
        if ctx.has_res and ctx.needs_input_grad[3]:
            dres = g if d.res_scale == 1.0 else g * d.res_scale
        return dx, dw, dbias, dres, None, None, None, None, None


def dwconv2d(x, weight, bias=None, stride=(1, 1), pad=(0, 0), act=None, residual=None, res_scale=1.0):
    code = act_code(act)
    if code is None:
        raise ValueError("activation %r cannot be fused" % (act,))
    return _DWConv.apply(x, weight, bias, residual, tuple(stride), tuple(pad), code[0], code[1], float(res_scale))


def bn_fold(weight, bias, bn):
    """Eval-mode BatchNorm2d folded into the preceding conv: (w * g / sqrt(v + eps),
    (b - m) * g / sqrt(v + eps) + beta).  HIP kernel (tpg_bn_fold) when nothing needs a
    gradient; differentiable aten form (parameter-sized, a few elements per channel)
    when the conv weight or the BN affine parameters are trained in eval mode."""
    gamma = bn.weight if bn.affine else torch.ones_like(bn.running_mean)
    beta = bn.bias if bn.affine else torch.zeros_like(bn.running_mean)
    needs = torch.is_grad_enabled() and (weight.requires_grad or gamma.requires_grad or beta.requires_grad or
                                         (bias is not None and bias.requires_grad))
    if needs:
        sc = gamma / torch.sqrt(bn.running_var + bn.eps)
        wf = weight * sc.view(-1, 1, 1, 1)
        bf = ((bias if bias is not None else 0.0) - bn.running_mean) * sc + beta
        return wf, bf
    lib = load()
    co, ci, kh, kw = weight.shape
    wf = torch.empty_strided(weight.shape, weight.stride(), dtype=torch.float32, device=weight.device)
    bf = torch.empty(co, dtype=torch.float32, device=weight.device)
    wv = weight.detach() if weight.dtype == torch.float32 else weight.detach().float()
    with torch.no_grad():
        check(lib.tpg_bn_fold(co, ci, kh, kw, tt(wv), bias.data_ptr() if bias is not None else None,
                              gamma.detach().float().data_ptr(), beta.detach().float().data_ptr(),
                              bn.running_mean.data_ptr(), bn.running_var.data_ptr(), float(bn.eps), tt(wf),
                              bf.data_ptr(), stream_ptr()))
    return wf, bf


_FOLD_CACHE = True


class _FrozenPack:
    """Packed-image holder (the FlatParams fields _packed_weight reads) for a folded weight
    that never changes: its epoch stays 0, so each (op, shape) image is packed once."""

    def __init__(self):
        self.pack_entries = {}
        self.pack_table = None
        self.epoch = 0


def _frozen_fold(conv, bn):
    """bn_fold for an eval-mode conv + BN.  When nothing needs a gradient (the frozen
    identity extractors, FeatureExtract.py), the folded (w, b) are computed once and kept
    on the conv module -- refolded only when one of the source tensors was replaced or
    modified in place (data pointers and version counters) -- and the folded weight
    carries a _FrozenPack, so its packed bf16/fp16 images are built once too.  (Folding and
    packing every call cost 106 + 162 launches per configs[2] step.)"""
    gamma = bn.weight if bn.affine else None
    beta = bn.bias if bn.affine else None
    srcs = [t for t in (conv.weight, conv.bias, gamma, beta) if t is not None]
    if (torch.is_grad_enabled() and any(t.requires_grad for t in srcs)) or not _FOLD_CACHE:
        return bn_fold(conv.weight, conv.bias, bn)
    if torch.cuda.is_current_stream_capturing():
        c = getattr(conv, "_tpg_folded", None)  # (no host-side cache fill inside a capture)
        return (c[1], c[2]) if c is not None else bn_fold(conv.weight, conv.bias, bn)
    key = (float(bn.eps),) + tuple((t.data_ptr(), t._version) for t in srcs + [bn.running_mean, bn.running_var])
    c = getattr(conv, "_tpg_folded", None)
    if c is not None and c[0] == key:
        return c[1], c[2]
    w, b = bn_fold(conv.weight, conv.bias, bn)
    w._tpg_flat = _FrozenPack()
    conv._tpg_folded = (key, w, b)
    return w, b


def _pix_dense(t):
    """t itself when its channels-last rows are pixel-dense with a 16-byte pixel stride
    (what the batch-statistics kernels walk), else a packed copy."""
    n, c, h, w = t.shape
    ps = t.stride(3)
    if (t.stride(1) == 1 and ps % 8 == 0 and ps >= _ceil8(c) and t.stride(2) == ps * w and
            t.stride(0) == ps * w * h and t.data_ptr() % 16 == 0):
        return t
    out = new_act(n, c, h, w, t.dtype, t.device)
    check(load().tpg_copy4d(n, c, h, w, tt(t), tt(out), stream_ptr()))
    return out


class _BNTrain(torch.autograd.Function):
    """Training-mode BatchNorm2d + activation (batch statistics, running stats updated)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, bn, act, slope):
        lib = load()
        dtype = get_compute_dtype()
        x = _pix_dense(to_cl(x, dtype))
        n, c, h, w = x.shape
        y = new_act(n, c, h, w, dtype, x.device)
        mean = torch.empty(c, dtype=torch.float32, device=x.device)
        invstd = torch.empty_like(mean)
        ws = torch.empty(2 * c, dtype=torch.float32, device=x.device)
        rm = bn.running_mean if bn.track_running_stats else None
        rv = bn.running_var if bn.track_running_stats else None
        mom = 0.1 if bn.momentum is None else float(bn.momentum)
        check(lib.tpg_bn_train_fwd(n, c, h, w, tt(x), gamma.detach().float().data_ptr(),
                                   beta.detach().float().data_ptr(), rm.data_ptr() if rm is not None else None,
                                   rv.data_ptr() if rv is not None else None, mom, float(bn.eps), act, slope, tt(y),
                                   mean.data_ptr(), invstd.data_ptr(), ws.data_ptr(), stream_ptr()))
        if bn.track_running_stats:
            bn.num_batches_tracked.add_(1)
        ctx.save_for_backward(x, y, gamma, mean, invstd)
        ctx.act, ctx.slope = act, slope
        return y

    @staticmethod
    def backward(ctx, gy):
        lib = load()
        x, y, gamma, mean, invstd = ctx.saved_tensors
        n, c, h, w = x.shape
        gy = _pix_dense(to_cl(gy, y.dtype))
        dx = new_act(n, c, h, w, x.dtype, x.device) if ctx.needs_input_grad[0] else None
        dgamma = torch.zeros(c, dtype=torch.float32, device=x.device) if ctx.needs_input_grad[1] else None
        dbeta = torch.zeros(c, dtype=torch.float32, device=x.device) if ctx.needs_input_grad[2] else None
        ws = torch.empty(2 * c, dtype=torch.float32, device=x.device)
        check(lib.tpg_bn_train_bwd(n, c, h, w, ctx.act, ctx.slope, tt(gy), tt(y), tt(x),
                                   gamma.detach().float().data_ptr(), mean.data_ptr(), invstd.data_ptr(), tt(dx),
                                   dgamma.data_ptr() if dgamma is not None else None,
                                   dbeta.data_ptr() if dbeta is not None else None, ws.data_ptr(), stream_ptr()))
        if dgamma is not None and gamma.dtype != torch.float32:
            dgamma = dgamma.to(gamma.dtype)
        return dx, dgamma, dbeta, None, None, None


def batchnorm_train(x, bn, act=None):
    code = act_code(act)
    if code is None:
        raise ValueError("activation %r cannot be fused" % (act,))
    gamma = bn.weight if bn.affine else torch.ones_like(bn.running_mean)
    beta = bn.bias if bn.affine else torch.zeros_like(bn.running_mean)
    return _BNTrain.apply(x, gamma, beta, bn, code[0], code[1])


def conv_bn_act(x, conv, bn, act=None, residual=None, res_scale=1.0):
    """Conv2d (dense or depthwise) -> BatchNorm2d -> activation [+ residual before the
    activation] as HIP calls: eval mode folds BN into the conv (one fused launch),
    train mode runs the conv then the batch-statistics BN with the activation fused."""
    dw = conv.groups != 1
    if dw and conv.groups != conv.in_channels:
        raise NotImplementedError("grouped convolution other than depthwise")
    ph, pw = conv.padding
    if bn is None or not bn.training:
        if bn is not None:
            w, b = _frozen_fold(conv, bn)
        else:
            w, b = conv.weight, conv.bias
        if dw:
            return dwconv2d(x, w, b, conv.stride, (ph, pw), act=act, residual=residual, res_scale=res_scale)
        return conv2d(x, w, b, stride=tuple(conv.stride), pad=(ph, ph, pw, pw), act=act, residual=residual,
                      res_scale=res_scale)
    if residual is not None:
        raise NotImplementedError("residual inside a training-mode conv-BN block")
    if dw:
        h = dwconv2d(x, conv.weight, conv.bias, conv.stride, (ph, pw))
    else:
        h = conv2d(x, conv.weight, conv.bias, stride=tuple(conv.stride), pad=(ph, ph, pw, pw))
    return batchnorm_train(h, bn, act)


class _MaxPool2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        lib = load()
        x = to_cl(x, get_compute_dtype())
        n, c, h, w = x.shape
        oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
        y = new_act(n, c, oh, ow, x.dtype, x.device)
        amax = torch.empty((n, oh, ow, c), dtype=torch.uint8, device=x.device)
        check(lib.tpg_maxpool2d_fwd(n, c, h, w, k, s, p, oh, ow, tt(x), tt(y), amax.data_ptr(), stream_ptr()))
        ctx.save_for_backward(amax)
        ctx.geo = (n, c, h, w, k, s, p, oh, ow)
        ctx.dtype = x.dtype
        return y

    @staticmethod
    def backward(ctx, gy):
        lib = load()
        (amax,) = ctx.saved_tensors
        n, c, h, w, k, s, p, oh, ow = ctx.geo
        dx = new_act(n, c, h, w, ctx.dtype, gy.device)
        check(lib.tpg_maxpool2d_bwd(n, c, h, w, k, s, p, oh, ow, tt(to_cl(gy, ctx.dtype)), amax.data_ptr(), tt(dx),
                                    stream_ptr()))
        return dx, None, None, None


def maxpool2d(x, kernel_size, stride, padding):
    return _MaxPool2d.apply(x, int(kernel_size), int(stride), int(padding))


class _AvgPool(torch.autograd.Function):
    """AdaptiveAvgPool2d(1): [n, c, h, w] -> [n, c, 1, 1]."""

    @staticmethod
    def forward(ctx, x):
        lib = load()
        x = to_cl(x, get_compute_dtype())
        n, c, h, w = x.shape
        y = new_act(n, c, 1, 1, x.dtype, x.device)
        check(lib.tpg_avgpool_fwd(n, c, h, w, tt(x), tt(y), stream_ptr()))
        ctx.geo = (n, c, h, w)
        ctx.dtype = x.dtype
        return y

    @staticmethod
    def backward(ctx, gy):
        lib = load()
        n, c, h, w = ctx.geo
        dx = new_act(n, c, h, w, ctx.dtype, gy.device)
        gy = to_cl(gy.reshape(n, c, 1, 1), ctx.dtype)
        check(lib.tpg_avgpool_bwd(n, c, h, w, tt(gy), tt(dx), stream_ptr()))
        return dx


def global_avgpool(x):
    return _AvgPool.apply(x)


def linear_bn_act(x, lin, bn, act=None):
    """Linear -> BatchNorm1d [-> act] (ModificationLayer.linear with use_batchnorm,
    ModificationLayer.py:204-231) as a 1x1 conv on [B, in, 1, 1] with the BN folded (eval)
    or as batch statistics over the batch (train)."""
    b = x.shape[0]
    out_f, in_f = lin.weight.shape
    x4 = x.reshape(b, in_f, 1, 1)
    w4 = lin.weight.view(out_f, in_f, 1, 1)
    if not bn.training:
        wf, bf = bn_fold(w4, lin.bias, bn)
        y = conv2d(x4, wf, bf, act=act)
    else:
        y = batchnorm_train(conv2d(x4, w4, lin.bias), bn, act)
    return y.reshape(b, out_f)


# ---- SSD landmark head of the MobileNetV2 pretraining (MobileNetV2.py:342-649; tpg_ssd.hip):
# MultiTaskLoss / MultiTaskDecoder on device tensors.  The background draw's uniform keys are
# torch.rand of the caller's generator state, the same draw as MobileNetV2.MultiTaskLoss's aten
# form, so the two forms select the same background anchors.
class _SsdLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, cls, truth, keys, width, height, k, ratio_nb, alpha, beta):
        lib = load()
        B, n, C = cls.shape
        pred = pred.float().contiguous()
        cls = cls.float().contiguous()
        truth = truth.reshape(B, 8).float().contiguous()
        keys = keys.float().contiguous()
        labels = torch.empty(B, n, dtype=torch.int32, device=pred.device)
        sel = torch.empty(B, n, dtype=torch.uint8, device=pred.device)
        terms = torch.empty(B, SSD_TERMS, dtype=torch.float32, device=pred.device)
        check(lib.tpg_ssd_loss_fwd(B, n, C, pred.data_ptr(), cls.data_ptr(), truth.data_ptr(), float(width),
                                   float(height), int(k), float(ratio_nb), float(alpha), float(beta),
                                   keys.data_ptr(), labels.data_ptr(), sel.data_ptr(), terms.data_ptr(), stream_ptr()))
        ctx.save_for_backward(pred, cls, truth, labels, sel, terms)
        ctx.cfg = (float(width), float(height), float(alpha), float(beta))
        ctx.mark_non_differentiable(labels, sel, terms)
        return terms[:, 0].mean(), labels, sel, terms

    @staticmethod
    def backward(ctx, g, _gl, _gs, _gt):
        lib = load()
        pred, cls, truth, labels, sel, terms = ctx.saved_tensors
        B, n, C = cls.shape
        width, height, alpha, beta = ctx.cfg
        gout = g.reshape(1).float().contiguous()
        dloc = torch.empty_like(pred)
        dcls = torch.empty_like(cls)
        check(lib.tpg_ssd_loss_bwd(B, n, C, pred.data_ptr(), cls.data_ptr(), truth.data_ptr(), width, height, alpha,
                                   beta, labels.data_ptr(), sel.data_ptr(), terms.data_ptr(), gout.data_ptr(),
                                   dloc.data_ptr(), dcls.data_ptr(), stream_ptr()))
        return dloc, dcls, None, None, None, None, None, None, None, None


def ssd_loss(pred, cls, truth, image_size, ratio, ratio_nb, alpha, beta):
    """(mean over images of alpha * loc + beta * cls, labels (B, n) int32, background draw (B, n)
    u8, per-image terms (B, 16): tpg_ssd_loss_fwd's layout)."""
    height, width = image_size
    keys = torch.rand(pred.shape[0], pred.shape[1], device=pred.device)
    k = int(ratio * pred.shape[1])  # (MobileNetV2.py:393, in double precision as there)
    return _SsdLoss.apply(pred, cls, truth, keys, width, height, k, ratio_nb, alpha, beta)


def ssd_decode(loc, cls, conf, nms_thr, top_k):
    """(keep (B, C, top_k) anchor indices or -1, score (B, C, top_k)) of tpg_ssd_decode."""
    lib = load()
    B, n, C = cls.shape
    loc = loc.float().contiguous()
    cls = cls.float().contiguous()
    keep = torch.empty(B, C, top_k, dtype=torch.int32, device=loc.device)
    score = torch.empty(B, C, top_k, dtype=torch.float32, device=loc.device)
    check(lib.tpg_ssd_decode(B, n, C, loc.data_ptr(), cls.data_ptr(), float(conf), float(nms_thr), int(top_k),
                             keep.data_ptr(), score.data_ptr(), stream_ptr()))
    return keep, score
