"""GPU: bench.py's own data-parallel launch path, rehearsed on ONE device.

The driver's 8-GPU scaling run launches `python -m torch.distributed.run --nproc-per-node N
bench.py --gpus N ...` over RCCL; this test runs that same command line with 2 processes that
share cuda:0 over gloo (`--dist-backend gloo`: RCCL needs one device per rank), so the env
parsing, process-group init, device mapping, barrier + max-over-ranks timing, bucketed
overlapped all-reduces and the real_ahead D(real) pass have executed before the
driver's run.  The launcher is a child process started by this one (nothing re-execs).
Reference: single-device `Pretrain.py:111`."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


ARGS = ["--gpus", "2", "--steps", "2", "--warmup", "2", "--batch", "2", "--no-cpu-baseline", "--dist-backend", "gloo"]


def _rank_env():
    return {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}


@pytest.mark.timeout(400)
def test_bench_gpus_flag_alone_launches_two_ranks(gpu):
    """the driver's command shape, `bench.py --gpus N` with no launcher in
    front, must run N ranks (bench.py starts torch.distributed.run as its child)."""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + ARGS, cwd=REPO, env=_rank_env(),
                       capture_output=True, text=True, timeout=380)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 4
    assert out["dp"]["backend"] == "gloo" and out["value"] > 0


@pytest.mark.timeout(400)
def test_bench_torchrun_two_ranks_one_gpu(gpu):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py")] + ARGS
    env = dict(_rank_env(), MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=380)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]  # rank 0 alone prints
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["scaling"] == "weak"
    assert out["config"]["global_batch"] == 4 and out["config"]["parallelism"] == "dp2"
    assert out["value"] > 0 and out["ms_per_step"] > 0
    # the roofline object names the probed enhance_features_128 kernel with the most time per step,
    # and the forward / input-gradient / weight-gradient probes are all listed
    kern = out["roofline_kernels"]
    assert sorted(k["pass"] for k in kern) == ["bwd", "fwd", "wgrad"], kern
    assert out["roofline"]["pass"] == kern[0]["pass"]
    assert kern[0]["ms_per_step"] == max(k["ms_per_step"] for k in kern)
    assert all(0 < k["frac"] < 1 for k in kern), kern
    dp = out["dp"]
    assert dp["backend"] == "gloo"
    # every step after the first reuses the D(real) pass the previous one ran under G's tail
    assert dp["real_ahead_reused"] >= 2, dp
    assert dp["g_buckets"] > 1 and dp["d_buckets"] >= 1 and dp["bucket_order_learned"], dp
    # what the first 8-GPU run needs to show where scaling is lost -- bucket
    # counts and bytes of both exchanges, and the communication time the compute stream waited for
    b = dp["buckets"]
    assert b["G"]["buckets"] == dp["g_buckets"] and b["D"]["buckets"] == dp["d_buckets"], b
    assert b["G"]["bytes"] == dp["g_bucket_bytes"] > 500e6 and b["D"]["bytes"] == dp["d_bucket_bytes"] > 50e6, b
    assert b["G"]["min_bucket_bytes"] <= b["G"]["max_bucket_bytes"] and b["G"]["overlapped"], b
    ex = dp["exposed_comm_ms_per_step"]
    assert ex["steps"] == 2, ex
    assert ex["G"] >= 0 and ex["D"] >= 0 and abs(ex["total"] - ex["G"] - ex["D"]) < 1e-3, ex
    # (gloo on one shared GPU: the host-side waits are real, so some exposure is measured)
    assert ex["total"] > 0, ex
    assert dp["overlap_optimizer"] is False
