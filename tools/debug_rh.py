"""Row-halo weight gradient (algo 6) vs fp64 per tap over a few shapes (debug aid)."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tp-gan_amd")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def main():
    import tpgan_ops as T
    from tpgan_lib import check, load, stream_ptr, tt
    lib = load()
    dev = torch.device("cuda", 0)
    gen = torch.Generator().manual_seed(0)
    for (N, Cin, H, W, Cout, k, p) in [(1, 75, 4, 128, 75, 7, 3), (1, 75, 4, 64, 75, 7, 3), (1, 64, 4, 128, 64, 5, 2),
                                       (1, 64, 4, 64, 64, 7, 3), (1, 64, 2, 64, 64, 3, 1), (1, 64, 1, 128, 64, 3, 1)]:
        geo = T.ConvGeom(k, k, (1, 1), (p, p, p, p))
        x64 = (torch.rand(N, Cin, H, W, generator=gen, dtype=torch.float64) * 2 - 1).bfloat16().double()
        g64 = (torch.rand(N, Cout, H, W, generator=gen, dtype=torch.float64) * 2 - 1).bfloat16().double()
        w64 = torch.zeros((Cout, Cin, k, k), dtype=torch.float64, requires_grad=True)
        F.conv2d(x64, w64, None, 1, p).backward(g64)
        ref = w64.grad
        x = T.new_act(N, Cin, H, W, torch.bfloat16, dev)
        x.copy_(x64.to(dev))
        g = T.new_act(N, Cout, H, W, torch.bfloat16, dev)
        g.copy_(g64.to(dev))
        d = geo.desc(N, Cin, H, W, Cout, H, W, torch.bfloat16, 0, 0.0, 1.0)
        dw = torch.zeros((Cout, Cin, k, k), device=dev).contiguous(memory_format=torch.channels_last)
        d.algo, d.ksplit = 6, 1
        check(lib.tpg_conv2d_bwd_filter(ctypes.byref(d), tt(x), tt(g), tt(dw), None, 0, stream_ptr()))
        torch.cuda.synchronize()
        err = (dw.cpu().double() - ref).abs()
        print((N, Cin, H, W, Cout, k, p), "rel %.2e" % float((dw.cpu().double() - ref).norm() / ref.norm()))
        print("  per r:", " ".join("%.1e" % float(err[:, :, r].max()) for r in range(k)))
        print("  per s:", " ".join("%.1e" % float(err[:, :, :, s].max()) for s in range(k)))
        bad = (err > 1e-3 * ref.abs().max()).nonzero()
        if len(bad):
            print("  bad a range", int(bad[:, 0].min()), int(bad[:, 0].max()), "b range", int(bad[:, 1].min()),
                  int(bad[:, 1].max()), "count", len(bad))


if __name__ == "__main__":
    main()
