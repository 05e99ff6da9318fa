"""CPU: bench.py's rank launch and its refusal to misreport.

`python bench.py --gpus N` with no launcher in front starts `torch.distributed.run` with N
ranks itself, as a child process; under a launcher every rank checks --gpus == WORLD_SIZE and,
with nccl, that the node has a GPU per local rank.  These run without a GPU: each exits before
anything touches a device.  The GPU half (two ranks over gloo on one MI355X, with no launcher in
front) is tests/test_gpu_bench_dp.py.  Reference: single-device `Pretrain.py:111`."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def test_argv_gpus_and_launcher_cmd():
    sys.path.insert(0, REPO)
    import importlib
    bench = importlib.import_module("bench")
    assert bench.argv_gpus(["--steps", "3"]) is None
    assert bench.argv_gpus(["--gpus", "8", "--steps", "3"]) == 8
    assert bench.argv_gpus(["--steps", "3", "--gpus=4"]) == 4
    cmd = bench.launcher_cmd(["--gpus", "8", "--steps", "3"], 8, 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    i = cmd.index("--nproc-per-node")
    assert cmd[i + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and cmd[cmd.index("--master-port") + 1] == "29511"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"] and cmd[-5] == os.path.abspath(BENCH)
    # a rank (WORLD_SIZE set) or --gpus 1 never launches
    old = os.environ.get("WORLD_SIZE")
    os.environ["WORLD_SIZE"] = "2"
    try:
        assert bench.launch_ranks(["--gpus", "2"]) is None
    finally:
        if old is None:
            del os.environ["WORLD_SIZE"]
        else:
            os.environ["WORLD_SIZE"] = old
    assert bench.launch_ranks(["--gpus", "1"]) is None


def test_gpus_mismatch_exits_nonzero():
    # one rank (WORLD_SIZE=1) told it is one of 2 GPUs: n_gpus would be misreported
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--no-cpu-baseline"], cwd=REPO,
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode != 0
    assert "--gpus 2 but this run has 1 rank" in r.stderr, r.stderr[-2000:]
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_gpus_launches_ranks_and_nccl_needs_a_device_each():
    # no launcher in front: bench.py starts 2 ranks under torch.distributed.run; with nccl each
    # rank refuses to share a device (this container has none), and the parent returns non-zero
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--no-cpu-baseline"], cwd=REPO, env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "2 ranks on this node but 0 visible GPU(s)" in r.stderr, r.stderr[-3000:]
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
