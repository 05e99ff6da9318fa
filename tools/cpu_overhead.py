"""Is the train step launch-bound?  For each step: synchronize, time the Python call that
enqueues the whole step (host time), then synchronize and time the rest (GPU drain).
If the enqueue time approaches the step time the GPU is waiting on the host."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tp-gan_amd")]
import torch  # noqa: E402


def main():
    import D_and_G_model as DG
    import tpgan_train
    dev = torch.device("cuda", 0)
    G = DG.Generator(64, 347, use_batchnorm=False).to(dev)
    D = DG.Discriminator().to(dev)
    tr = tpgan_train.TPGANTrainer(G, D, compute_dtype=torch.bfloat16)
    b = tpgan_train.synthetic_batch(32, dev)
    for _ in range(4):
        tr.step(b)
    torch.cuda.synchronize()
    enq, tot = [], []
    for _ in range(8):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        c0 = time.process_time()
        tr.step(b)
        t1 = time.perf_counter()
        c1 = time.process_time()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        enq.append((t1 - t0, c1 - c0))
        tot.append(t2 - t0)
    n = len(tot)
    print("step wall %.2f ms | host enqueue wall %.2f ms | host CPU (all threads) %.2f ms | drain after enqueue %.2f ms"
          % (1e3 * sum(tot) / n, 1e3 * sum(e[0] for e in enq) / n, 1e3 * sum(e[1] for e in enq) / n,
             1e3 * (sum(tot) - sum(e[0] for e in enq)) / n))


if __name__ == "__main__":
    main()
