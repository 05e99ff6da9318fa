"""CPU, world_size 2 over gloo: the data-parallel pieces of the train step
(tpgan_train.GradSync + FlatParams): rank-0 parameter broadcast and the gradient
all-reduce whose 1/world average is folded into the optimizer's grad_scale."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path.insert(0, os.path.join(REPO, "tp-gan_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import D_and_G_model as DG
        import tpgan_train
        torch.manual_seed(100 + rank)  # different init per rank
        D = DG.Discriminator()
        flat = tpgan_train.FlatParams(D, torch.device("cpu"))
        sync = tpgan_train.GradSync()
        sync.broadcast(flat)
        # after the broadcast every rank holds rank 0's parameters (module views included)
        ref = flat.data.clone()
        dist.broadcast(ref, 0)
        p0 = next(D.parameters())  # channels-last conv weight: physical order [a][kh][kw][b]
        ok_bcast = torch.equal(ref, flat.data) and torch.equal(p0.data.permute(0, 2, 3, 1).reshape(-1),
                                                                 flat.data[:p0.numel()])
        flat.grad.copy_(torch.arange(flat.grad.numel(), dtype=torch.float32) * (rank + 1))
        sync.allreduce(flat)
        expect = torch.arange(flat.grad.numel(), dtype=torch.float32) * sum(r + 1 for r in range(world))
        ok_reduce = torch.allclose(flat.grad, expect) and sync.grad_scale == 1.0 / world
        # grads seen through the parameter views are the reduced ones
        ok_view = torch.equal(p0.grad.permute(0, 2, 3, 1).reshape(-1), expect[:p0.numel()])
        q.put((rank, ok_bcast, ok_reduce, ok_view, sync.world))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_dp_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(60)
    for rank, ok_b, ok_r, ok_v, w in res:
        assert w == world
        assert ok_b, "broadcast rank %d" % rank
        assert ok_r, "allreduce rank %d" % rank
        assert ok_v


def _worker_overlap(rank, world, port, q):
    sys.path.insert(0, os.path.join(REPO, "tp-gan_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import D_and_G_model as DG
        import tpgan_ops
        import tpgan_train
        torch.manual_seed(5)
        D = DG.Discriminator()
        flat = tpgan_train.FlatParams(D, torch.device("cpu"))
        sync = tpgan_train.OverlappedGradSync(flat, bucket_mb=2.0)  # several buckets
        names = [n for n, _ in D.named_parameters()]
        before = {n: p.detach().clone() for n, p in D.named_parameters()}
        results = []
        for step in range(2):
            flat.grad.zero_()
            sync.begin()
            params = list(D.parameters())
            # ranks report gradients in different orders; one parameter never reports
            order = list(range(len(params))) if rank == 0 else list(reversed(range(len(params))))
            for i in order:
                p = params[i]
                p.grad.copy_(torch.full_like(p, float(rank + 1) * (i + 1)))
                if i != 3:
                    tpgan_ops.GRAD_READY_HOOK[0](p)
            nb = len(sync.buckets)
            sync.finish()
            ok = all(torch.allclose(p.grad, torch.full_like(p, 3.0 * (i + 1))) for i, p in enumerate(D.parameters()))
            results.append((ok, nb))
        same_values = all(torch.equal(before[n], p.detach()) for n, p in zip(names, D.parameters()))
        q.put((rank, results, list(sync.flat.offsets), same_values, tpgan_ops.GRAD_READY_HOOK[0] is None))
    except Exception as e:  # report instead of leaving the parent waiting on the queue
        q.put((rank, [(False, repr(e))], [], False, False))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_overlapped_bucket_sync_gloo_world2():
    """OverlappedGradSync: buckets issued in index order whatever order the gradients
    complete in (ranks differ on purpose), unreported parameters flushed by finish(), the
    learned layout (rank 0's completion order) identical on both ranks and value-preserving."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_overlap, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)])
    for p in procs:
        p.join(60)
    for rank, results, offsets, same, unhooked in res:
        assert all(ok for ok, _ in results), (rank, results)
        assert results[0][1] > 2
        assert same and unhooked
    assert res[0][2] == res[1][2]


def _worker_overlap_opt(rank, world, port, q):
    sys.path.insert(0, os.path.join(REPO, "tp-gan_amd"))
    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import D_and_G_model as DG
        import tpgan_ops
        import tpgan_train
        torch.manual_seed(5)
        D = DG.Discriminator()
        flat = tpgan_train.FlatParams(D, torch.device("cpu"))
        calls = []

        def opt(off, n):  # the bucket's gradients must already be the reduced ones
            calls.append((off, n, bool(torch.all(flat.grad[off:off + n] == float(sum(range(1, world + 1)))))))

        sync = tpgan_train.OverlappedGradSync(flat, bucket_mb=2.0, optimizer=opt)
        results = []
        for step in range(2):
            calls.clear()
            flat.grad.zero_()
            sync.begin()
            params = list(D.parameters())
            order = list(range(len(params))) if rank == 0 else list(reversed(range(len(params))))
            for i in order:
                p = params[i]
                p.grad.fill_(float(rank + 1))
                if i != 3:
                    tpgan_ops.GRAD_READY_HOOK[0](p)
            sync.finish()
            cover = torch.zeros(flat.grad.numel(), dtype=torch.int32)
            for off, n, _ in calls:
                cover[off:off + n] += 1
            results.append((bool(torch.all(cover == 1)), all(c[2] for c in calls), len(calls), sync.updated))
        q.put((rank, results))
    except Exception as e:
        q.put((rank, [(False, repr(e), 0, False)]))
        raise
    finally:
        if world > 1:
            dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [1, 2])
def test_overlapped_optimizer_buckets(world):
    """OverlappedGradSync(optimizer=...): every element of the flat buffer is handed to the
    optimizer exactly once per step, bucket by bucket, each bucket only after its all-reduce
    (world 2: the values seen are the summed ones) -- before and after the step-1 relayout;
    world 1 runs the same bucketed update with no process group."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_overlap_opt, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(60)
    for rank, results in res:
        for once, reduced, ncalls, updated in results:
            assert once and reduced and updated, (rank, results)
            assert ncalls > 2
