"""GPU, world_size 2 on ONE device (two processes sharing cuda:0, gloo over CUDA tensors):
the data-parallel train step with the bucketed, backward-overlapped G all-reduce
(tpgan_train.OverlappedGradSync) keeps the replicas bit-identical, issues buckets during
the backward, and learns the same bucket layout on both ranks.  (RCCL needs one device
per rank; the 8-GPU RCCL run is the driver's scaling bench.)"""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path[:0] = [REPO, os.path.join(REPO, "tp-gan_amd")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import D_and_G_model as DG
        import tpgan_train
        dev = torch.device("cuda", 0)
        torch.manual_seed(10 + rank)  # different init per rank: the broadcast must unify it
        G = DG.Generator(64, 347, use_batchnorm=False).to(dev)
        D = DG.Discriminator().to(dev)
        tr = tpgan_train.TPGANTrainer(G, D, compute_dtype=torch.bfloat16, bucket_mb=16.0)
        b = tpgan_train.synthetic_batch(2, dev, seed=100 + rank)
        issued_early = []
        orig_finish = tr.gsync.finish

        def finish():
            issued_early.append(tr.gsync.next)  # buckets already issued when backward returned
            return orig_finish()

        tr.gsync.finish = finish
        for _ in range(3):
            tr.step(b)
        torch.cuda.synchronize()
        sums = torch.stack([tr.fG.data.double().sum(), tr.fD.data.double().sum(),
                            tr.fG.data.double().square().sum()]).cpu()
        q.put((rank, sums.tolist(), issued_early, len(tr.gsync.buckets), list(tr.fG.offsets[:50]),
               tr.gsync.order_learned))
    except Exception as e:
        q.put((rank, repr(e), [], 0, [], False))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_dp_overlap_two_ranks_one_gpu(gpu):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=280) for _ in range(world)])
    for p in procs:
        p.join(60)
    (r0, s0, e0, nb0, off0, l0), (r1, s1, e1, nb1, off1, l1) = res
    assert isinstance(s0, list) and isinstance(s1, list), (s0, s1)
    assert s0 == s1  # identical replicas after 3 steps
    assert nb0 == nb1 and nb0 > 10 and l0 and l1
    assert off0 == off1
    assert max(e0) > 0 and max(e1) > 0  # some buckets went out while the backward was running
