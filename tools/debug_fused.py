"""Localise a non-deterministic-mode backward difference for one test_gpu_ops GEOMS entry."""
import os
import sys
import zlib
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tp-gan_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
import tpgan_ops  # noqa: E402
from _cases import rel  # noqa: E402

geom = eval(sys.argv[1]) if len(sys.argv) > 1 else (3, 40, 10, 10, 72, 3, 1, 1, False, 0, "leaky", False, False)
dtype = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}[sys.argv[2] if len(sys.argv) > 2 else "f32"]
(N, Cin, H, W, Cout, k, s, p, tr, op, act, use_res, refl) = geom
assert not tr and not refl and not use_res
gen = torch.Generator().manual_seed(zlib.crc32(repr(geom).encode()) + 1)
x0 = torch.rand(N, Cin, H, W, generator=gen) * 2 - 1
w0 = (torch.rand(Cout, Cin, k, k, generator=gen) * 2 - 1) * (3.0 / (Cin * k * k)) ** 0.5
b0 = torch.rand(Cout, generator=gen) * 0.2 - 0.1
dev = torch.device("cuda", 0)
actm = {"leaky": torch.nn.LeakyReLU(0.01), "relu": torch.nn.ReLU(), None: None}[act]

x64, w64, b64 = (t.double().requires_grad_(True) for t in (x0, w0, b0))
y64 = F.conv2d(x64, w64, b64, s, p)
y64 = actm(y64) if actm is not None else y64
gy64 = torch.from_numpy(np.cos(np.arange(y64.numel(), dtype=np.float64) * 0.37).reshape(y64.shape))
y64.backward(gy64)


def run(tag, fused, det):
    x = x0.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    w = w0.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    b = b0.to(dev).requires_grad_(True)
    tpgan_ops.FUSED_BWD["enabled"] = fused
    with tpgan_ops.compute_dtype(dtype), tpgan_ops.deterministic(det):
        y = tpgan_ops.conv2d(x, w, b, stride=(s, s), pad=(p, p, p, p), act=actm)
        y.backward(gy64.to(dev).to(y.dtype))
        torch.cuda.synchronize()
    tpgan_ops.FUSED_BWD["enabled"] = True
    dx = x.grad.double().cpu()
    e = (dx - x64.grad).abs()
    idx = np.unravel_index(int(e.argmax()), e.shape)
    bad = (e > 1e-3 * x64.grad.abs().max()).nonzero()
    print("%-28s dx %.3g dw %.3g db %.3g  max|e| %.3g at %s  n_bad %d" % (
        tag, rel(dx, x64.grad), rel(w.grad.cpu(), w64.grad), rel(b.grad.cpu(), b64.grad), float(e.max()),
        tuple(int(i) for i in idx), len(bad)))
    if len(bad):
        for col, nm in enumerate("nchw"):
            print("   bad %s values:" % nm, sorted(set(bad[:, col].tolist()))[:40])


run("three-call det", False, True)
run("fused det", True, True)
run("three-call nondet", False, False)
run("fused nondet", True, False)
run("fused nondet (tuned)", True, False)
os.environ["TPG_NO_MASKED_DGRAD"] = "1"
run("fused nondet, no mask", True, False)
