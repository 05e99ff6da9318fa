"""Library GEMM (hipBLASLt through torch.matmul, bf16) on the ResNet-50 1x1-conv shapes of the
configs[2] identity extractor, graph-replay timed, beside this library's conv kernel for the same
shape (tools/bench_layers.py --r50 prints the latter).  A measurement tool: decides whether the
small 1x1 layers belong on a library GEMM.

    python tools/probe_gemm.py
"""
import torch

# (name, M = pixels, K = in channels, N = out channels)
SHAPES = [("l1_a0", 32768, 64, 64), ("l1_a", 32768, 256, 64), ("l1_c", 32768, 64, 256), ("l2_a", 8192, 512, 128),
          ("l2_c", 8192, 128, 512), ("l3_a", 2048, 1024, 256), ("l3_c", 2048, 256, 1024), ("l4_a", 512, 2048, 512),
          ("l4_c", 512, 512, 2048), ("fc1", 32, 32768, 512)]


def timed(fn, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    dev = torch.device("cuda", 0)
    for name, M, K, N in SHAPES:
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        b = torch.randn(N, device=dev, dtype=torch.bfloat16)
        r = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        gy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        t_mm = timed(lambda: torch.matmul(x, w.t(), out=out))
        t_addmm = timed(lambda: torch.addmm(b, x, w.t(), out=out))
        t_res = timed(lambda: torch.addmm(r, x, w.t(), out=out))
        t_dg = timed(lambda: torch.matmul(gy, w, out=dx))
        fl = 2.0 * M * N * K
        print("%-6s M %5d K %5d N %5d  %.2f GF | mm %.1f us (%.0f TF/s) | +bias %.1f us | +residual %.1f us | dgrad %.1f us"
              % (name, M, K, N, fl / 1e9, t_mm, fl / t_mm / 1e6, t_addmm, t_res, t_dg), flush=True)


if __name__ == "__main__":
    main()
