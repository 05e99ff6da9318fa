"""Which backward path gets res_k5_c27's layers.0 bias gradient wrong (bf16)?"""
import os
import sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tp-gan_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402
from _cases import case_arrays, golden, load_det, op_cases, rel  # noqa: E402
import ModificationLayer as ML  # noqa: E402
import tpgan_ops  # noqa: E402

npz = golden("ops_golden.npz")
name = sys.argv[1] if len(sys.argv) > 1 else "res_k5_c27"
arrs = case_arrays(npz, name)
dev = torch.device("cuda", 0)
print("x", arrs["x"].shape)


def run(tag, dtype=torch.bfloat16):
    m = op_cases(ML)[name]()
    load_det(m, "op/%s/" % name, torch.float32)
    m = m.to(dev)
    x = torch.from_numpy(arrs["x"]).float().to(dev).requires_grad_(True)
    with tpgan_ops.compute_dtype(dtype):
        y = m(x)
    gy = torch.from_numpy(arrs["gy"]).to(dev).to(y.dtype)
    (y.float() * gy.float()).sum().backward()
    torch.cuda.synchronize()
    errs = {k: rel(p.grad.cpu(), arrs["g:" + k]) for k, p in m.named_parameters()}
    print(tag, "dx %.3g" % rel(x.grad.float().cpu(), arrs["dx"]), " ".join("%s %.3g" % kv for kv in errs.items()))


run("default")
run("default-again (tuned)")
tpgan_ops.FUSED_BWD["enabled"] = False
run("three-call")
tpgan_ops.FUSED_BWD["enabled"] = True
tpgan_ops.AUTOTUNE["enabled"] = False
tpgan_ops.AUTOTUNE["cache"].clear()
run("fused, no autotune")
with tpgan_ops.deterministic():
    run("fused, det")
run("fused fp32", torch.float32)
