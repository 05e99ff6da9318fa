"""TP-GAN G+D train-step benchmark (BASELINE.json metric: faces/sec at 128x128, bs32/GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

`--gpus N` (N > 1) without a launcher starts the second form itself, as a child process, and
exits with its code; under a launcher every rank checks that --gpus equals WORLD_SIZE, and
with nccl that the node has a GPU per local rank.

Workload = BASELINE.json configs[1]: full two-pathway Generator (global + 4 local
pathways) + Discriminator train step, 128x128, bs32 per GPU, bf16 activations / MFMA
with fp32 accumulate and fp32 master weights, synthetic Multi-PIE-shaped data resident in
HBM, random-init weights.  Data parallel over N GPUs (one process per GPU, RCCL
all-reduce of G and D gradients): per-GPU batch fixed, so scaling is weak.

Rank 0 prints one JSON line.  `roofline` is for the dominant kernel: of the 5x5 206->206
enhance_features_128 convolution's forward, input-gradient and weight-gradient kernels (each
timed with HIP events around its launches on the launching stream during the timed steps), the
one with the most time per step; `roofline_kernels` lists all three.  `cpu_baseline` times the
CPU oracle restatement (oracle/cpu_step.py, "port") on the host cores on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "tp-gan_amd"))
sys.path.insert(0, REPO)


def argv_gpus(argv):
    """The --gpus value of a command line, read before argparse (and before torch is imported);
    None when absent."""
    for i, a in enumerate(argv):
        if a == "--gpus" and i + 1 < len(argv):
            return int(argv[i + 1])
        if a.startswith("--gpus="):
            return int(a.split("=", 1)[1])
    return None


def launcher_cmd(argv, n, port):
    """The torch.distributed.run command that starts n ranks of this script, one per GPU."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def launch_ranks(argv):
    """`bench.py --gpus N` (N > 1) with no launcher in front: start N ranks under
    torch.distributed.run as a CHILD process (never an exec -- nothing here has touched the GPU or
    imported torch), pass its output through (rank 0 prints the JSON line) and return its exit
    code.  None when this process is itself a rank (WORLD_SIZE set) or N <= 1."""
    n = argv_gpus(argv)
    if n is None or n <= 1 or "WORLD_SIZE" in os.environ:
        return None
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.call(launcher_cmd(argv, n, port), env=env)


if __name__ == "__main__":
    _rc = launch_ranks(sys.argv[1:])
    if _rc is not None:
        sys.exit(_rc)

# Launch mode: one process (N = 1) replays the whole step as a hipGraph by default (r05ac, same
# box: 30.39 / 30.46 vs 31.10 / 30.97 ms/step eager); data-parallel ranks run eager, where each
# gradient bucket's all-reduce overlaps the rest of the backward (graph replays would issue the
# whole-network exchange between phase graphs, exposed).  --eager / --graph force either.
GRAPH_DEFAULT = int(os.environ.get("WORLD_SIZE", "1")) == 1 and "--eager" not in sys.argv
if "--graph" in sys.argv or GRAPH_DEFAULT:
    # hipGraph replay that keeps the side-stream branches concurrent: without packet capture
    # the runtime launches independent graph branches on up to 8 streams (with it, every node
    # goes to the launch stream in topological order: 39.6 vs 37.0 ms/step).  Read by the HIP
    # runtime at initialisation, so set before torch touches the GPU.
    os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
    os.environ.setdefault("DEBUG_HIP_FORCE_GRAPH_QUEUES", "8")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 / fp16 MFMA (MI355X_MICROARCH.md, chip table; fp32 mode: same denominator)
PEAK_HBM_GBS = 8000.0
PROBED = ("fwd", "bwd", "wgrad")
PASS_KERNEL = {"fwd": "halo_kernel forward",
               "bwd": "halo_kernel input gradient (gy arrives premasked by the consumer's epilogue; its own epilogue "
                      "applies the producer's act' (in_act) or accumulates into the parked shortcut gradient)",
               "wgrad": "wgrad_rh_kernel weight gradient (+ bias)"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs = ranks (one process each).  N > 1 without a launcher: bench.py starts "
                         "torch.distributed.run itself; under a launcher it must equal WORLD_SIZE")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, choices=[2, 3, 5], default=2,
                    help="BASELINE.json configs[n-1]: 2 = full G+D step, 128x128, bs32, bf16 (the headline); "
                         "3 = 2 + ResNet-50 identity loss; 5 = 256x256, bs16/GPU, fp16 MFMA, MobileNetV2 identity")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--img-size", type=int, default=None)
    ap.add_argument("--dtype", choices=["bf16", "fp16", "fp32"], default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="CPU baseline threads (default: OMP_NUM_THREADS, i.e. this process's CPU share -- 16 "
                         "on the GPU box, whose os.cpu_count() reports the whole host -- else os.cpu_count())")
    ap.add_argument("--cpu-iters", type=int, default=3)
    ap.add_argument("--cpu-batch", type=int, default=32)
    ap.add_argument("--graph", action="store_true",
                    help="replay the step as hipGraph(s) with packet capture off and 8 graph queues, so the "
                         "side-stream branches stay concurrent (the default at N = 1; at N > 1 one graph per "
                         "phase with the all-reduces between them)")
    ap.add_argument("--eager", action="store_true", help="launch the step eagerly (the default at N > 1)")
    ap.add_argument("--segmented", action="store_true", help="one hipGraph per step phase even at world 1")
    ap.add_argument("--probe-steps", type=int, default=2)
    ap.add_argument("--identity", choices=["none", "resnet50", "mobilenetv2"], default=None,
                    help="identity-preserving loss extractor in the G step (BASELINE configs[2]: resnet50)")
    ap.add_argument("--gp", action="store_true", help="WGAN-GP in the D step (double backward through D)")
    ap.add_argument("--tune-file", default=None,
                    help="start from a saved autotuner cache (tpgan_ops.save_tuning / TPG_TUNE_DUMP); shapes "
                         "it lacks are tuned in the warm-up as usual")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI, the product; gloo: the "
                         "one-GPU rehearsal of this launch path in tests/test_gpu_bench_dp.py)")
    a = ap.parse_args()
    dflt = {2: (32, 128, "bf16", "none"), 3: (32, 128, "bf16", "resnet50"), 5: (16, 256, "fp16", "mobilenetv2")}
    b, im, dt, ident = dflt[a.config]
    a.batch = a.batch or b
    a.img_size = a.img_size or im
    a.dtype = a.dtype or dt
    a.identity = a.identity or ident
    return a


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # the JSON line's n_gpus is the world size: a --gpus that disagrees with the ranks actually
    # started would misreport, so it is an error (checked before anything touches the GPU)
    if args.gpus is not None and args.gpus != world:
        sys.exit("bench.py: --gpus %d but this run has %d rank(s) (WORLD_SIZE=%s)"
                 % (args.gpus, world, os.environ.get("WORLD_SIZE", "unset")))
    # one process per GPU.  RCCL needs a device per rank: with nccl, fewer devices than local
    # ranks is an error; only the gloo rehearsal of this path (two ranks on one GPU,
    # tests/test_gpu_bench_dp.py) shares a device
    # (device_count does not initialise HIP: nothing GPU-side happens before the process group)
    ndev_seen = torch.cuda.device_count()
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if world > 1 and args.dist_backend == "nccl" and ndev_seen < local_world:
        sys.exit("bench.py: rank %d: %d ranks on this node but %d visible GPU(s); RCCL needs one device per rank"
                 % (rank, local_world, ndev_seen))
    ndev = max(ndev_seen, 1)
    dev = torch.device("cuda", local % ndev)
    if world > 1:
        torch.cuda.set_device(dev)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    torch.manual_seed(1234)
    import D_and_G_model as DG
    import tpgan_ops
    import tpgan_train
    from config import G as GCFG

    cdt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[args.dtype]
    S = args.img_size
    G = DG.Generator(GCFG["zdim"], GCFG["num_classes"], use_batchnorm=False, img_size=S).to(dev)
    D = DG.Discriminator().to(dev)
    identity_fn = None
    if args.identity != "none":
        import FeatureExtract as FE
        ext = FE.FeatureExtractModel(args.identity, 347).to(dev)
        identity_fn = FE.IdentityPreservingLoss(ext, cdt)
    trainer = tpgan_train.TPGANTrainer(G, D, lr=1e-4, compute_dtype=cdt, identity_fn=identity_fn,
                                       gradient_penalty=args.gp)
    B = args.batch
    batch = tpgan_train.synthetic_batch(B, dev, seed=1000 + rank, img_size=S)

    # dominant-kernel probes: enhance_features_128 (206 -> 206, 5x5, at the full face size), its
    # forward, input gradient (the fused backward's first call: round 5 act links) and weight
    # gradient -- the step's three largest kernels; `roofline` reports the one with the most
    # time per step (profiles/r04/kernel_trace_summary.txt: the weight gradient)
    def match(d, which):
        return which in PROBED and d.in_c == 206 and d.out_c == 206 and d.kh == 5 and d.in_h == S

    # warm-up (autotunes the weight-gradient tiles), one eager step counted for the
    # algorithmic FLOPs, then the step is captured as hipGraph(s)
    # (next_b: the next step's batch -- here the same resident one -- so that, data-parallel,
    # its D(real) pass runs under the G all-reduce tail)
    if args.tune_file:
        tpgan_ops.load_tuning(args.tune_file)
    for _ in range(max(args.warmup - 1, 0)):
        trainer.step(batch, next_b=batch)
    tpgan_ops.reset_flops()
    trainer.step(batch, next_b=batch)
    flops_step = sum(tpgan_ops.FLOPS.values())
    if os.environ.get("TPG_TUNE_DUMP") and rank == 0:  # the weight-gradient tiles the autotuner picked
        tpgan_ops.save_tuning(os.environ["TPG_TUNE_DUMP"])
    torch.cuda.synchronize()
    graphed = args.graph or (world == 1 and not args.eager)
    capture_error = None
    if graphed:
        try:
            trainer.capture(batch, warmup=1, segmented=args.segmented or None)
            trainer.step_graphed()
        except RuntimeError as e:  # (a capture the runtime refuses: the eager step is the same work)
            if args.graph:
                raise
            # reported in the JSON line (config.capture_error), so a capture regression is visible
            capture_error = "%s: %s" % (type(e).__name__, str(e)[:400])
            print("bench: graph capture failed (%s), timing eager steps" % e, file=sys.stderr, flush=True)
            torch.cuda.synchronize()
            trainer.reset_capture()
            graphed = False
    if graphed:
        run = trainer.step_graphed
    else:
        def run():
            return trainer.step(batch, next_b=batch)

    if not graphed:
        tpgan_ops.PROBE["match"] = match
        tpgan_ops.PROBE["events"] = []
    if world > 1:
        trainer.comm_timing = True  # exposed-communication events around each exchange (timed steps only)
        trainer.comm_events = []
        dist.barrier()
    torch.cuda.synchronize()
    # per-step HIP events on the launching stream (every step ends on it: side streams join)
    marks = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    marks[0].record()
    for i in range(args.steps):
        run()
        marks[i + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed.item())
    exposed = None
    if world > 1:
        trainer.comm_timing = False
        exposed = trainer.exposed_comm_ms()
        # max over ranks, like the step time (the slowest rank's wait is the one that costs)
        ex = torch.tensor([exposed["G"], exposed["D"]], dtype=torch.float64, device=dev)
        dist.all_reduce(ex, op=dist.ReduceOp.MAX)
        exposed["G"], exposed["D"] = float(ex[0]), float(ex[1])
    ms_per_step = elapsed / args.steps * 1e3
    faces = world * B * args.steps / elapsed
    step_ms = sorted(marks[i].elapsed_time(marks[i + 1]) for i in range(args.steps))
    step_med = step_ms[len(step_ms) // 2] if len(step_ms) % 2 else 0.5 * (step_ms[len(step_ms) // 2 - 1] +
                                                                          step_ms[len(step_ms) // 2])

    # dominant-kernel probe: HIP events around each launch on its launch stream.  Graph
    # nodes cannot be bracketed, so with graphs the probe runs eager steps right after the
    # timed region (same kernel, same shapes); eager runs probe the timed steps themselves.
    if graphed:
        tpgan_ops.PROBE["match"] = match
        tpgan_ops.PROBE["events"] = []
    for _ in range(args.probe_steps if graphed else 0):
        trainer.step(batch)
    torch.cuda.synchronize()
    tpgan_ops.PROBE["match"] = None
    evs = tpgan_ops.PROBE["events"]
    per = {}
    for e0, e1, work, which, _ in evs:
        r = per.setdefault(which, {"ms": 0.0, "n": 0, "flops": work})
        r["ms"] += e0.elapsed_time(e1)
        r["n"] += 1
    n_steps = args.probe_steps if graphed else args.steps
    kern = []
    for which, r in per.items():
        avg = r["ms"] / r["n"]
        ach = r["flops"] / (avg * 1e-3) / 1e12
        kern.append({"pass": which, "kernel": PASS_KERNEL.get(which, which), "achieved": round(ach, 2),
                     "frac": round(ach / PEAK_BF16_TFLOPS, 4), "avg_launch_ms": round(avg, 4), "launches": r["n"],
                     "ms_per_step": round(r["ms"] / max(n_steps, 1), 4), "flops_per_launch": r["flops"]})
    kern.sort(key=lambda k: -k["ms_per_step"])
    top = kern[0] if kern else {"pass": "fwd", "achieved": 0.0, "avg_launch_ms": 0.0, "launches": 0,
                                "flops_per_launch": 0, "ms_per_step": 0.0}
    k_ms, k_flops, achieved = top["avg_launch_ms"], top["flops_per_launch"], top["achieved"]

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    cpu = None
    if not args.no_cpu_baseline and world == 1:
        # the fixture-pinned CPU restatement (aten fp32) on the host cores, the
        # headline workload (full step incl. both Adam updates) at its batch and BASELINE
        # configs[0] at B=4, each one warm-up + median of --cpu-iters
        from oracle.cpu_step import time_cpu_step
        cb = min(B, args.cpu_batch) if args.img_size == 128 else 0
        if cb:
            threads = args.cpu_threads or int(os.environ.get("OMP_NUM_THREADS") or 0) or os.cpu_count()
            r = time_cpu_step(B=cb, iters=args.cpu_iters, threads=threads)
            cpu = {"value": round(r["full_fps"], 4), "unit": "faces/s", "cores": r["threads"], "threads": r["threads"],
                   "host_cpu_count": os.cpu_count(),
                   "cores_meaning": "threads this process used (its CPU share on the box: OMP_NUM_THREADS, else "
                                    "os.cpu_count()), not the host's core count (host_cpu_count)",
                   "kind": "port", "cpu_model": r["cpu"],
                   "sample": "oracle/cpu_step.py full G+D train step incl. both Adam updates, 128x128, B=%d, fp32 "
                             "aten CPU, 1 warm-up + median of %d steps (%.2f s/step)" % (cb, args.cpu_iters,
                                                                                        r["full_s"]),
                   "config1": {"value": round(r["config1_fps"], 4), "unit": "faces/s",
                               "sample": "BASELINE configs[0]: global pathway + D fwd+bwd, B=4, median of %d "
                                         "(%.2f s/step)" % (args.cpu_iters, r["config1_s"])}}

    # HBM bytes per launch of each probed kernel from the committed rocprofv3 PMC passes
    # (tools/pmc_summary.py: FETCH_SIZE x2 gfx950 correction + WRITE_SIZE), or null
    def pmc_traffic(which):
        path = os.path.join(REPO, "profiles", "pmc_enhance128_%s.json" % which)
        if not (os.path.exists(path) and args.config == 2 and S == 128 and args.dtype == "bf16" and B == 32):
            return None, None
        with open(path) as f:
            pj = json.load(f)
        return int(pj["traffic_bytes"]), (
            "profiles/pmc_enhance128_%s.json: rocprofv3 --pmc FETCH_SIZE (x2, calibrated) + WRITE_SIZE (exact, "
            "calibrated), median over that pass's dispatches of tools/bench_layers.py enhance_128; algorithmic %d B"
            % (which, int(pj.get("algorithmic_bytes", 0))))
    for k in kern:
        k["traffic"], _ = pmc_traffic(k["pass"])
    traffic, traffic_src = pmc_traffic(top["pass"])
    workload = "BASELINE configs[1]: full two-pathway G (global + 4 local) + D train step, 128x128, bf16"
    ext_name = {"resnet50": "ResNet-50", "mobilenetv2": "MobileNetV2"}.get(args.identity)
    if args.config == 5:
        workload = ("BASELINE configs[4]: full two-pathway G + D train step, %dx%d, %s MFMA, %s identity-preserving "
                    "loss, bs%d/GPU (G generalised to 256: LocalFuser placements and fc1 / deconv_8 sizes scale; "
                    "parity unpinned at 256 for G)" % (S, S, args.dtype, ext_name or "no", B))
    elif args.identity != "none":
        workload = ("BASELINE configs[2]: configs[1] + %s identity-preserving loss (frozen extractor, eval BN) "
                    "in the G step" % ext_name)
    if args.config != 5 and (S != 128 or args.dtype != "bf16"):
        workload += " [overridden: %dx%d, %s]" % (S, S, args.dtype)
    if args.gp:
        workload += " + WGAN-GP (double backward through D)"
    out = {
        "metric": "faces/sec (G+D train step) at 128x128 bs32, 1/2/4/8 MI355X; % MFMA roofline",
        "value": round(faces, 2),
        "unit": "faces/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "ms_per_step_median": round(step_med, 3),
        "step_ms_events": {"min": round(step_ms[0], 3), "median": round(step_med, 3), "max": round(step_ms[-1], 3),
                           "n": len(step_ms), "source": "HIP events between consecutive steps on the launch stream"},
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (U[-1,1] Multi-PIE-shaped batch resident in HBM; random-init weights)",
        "config": {"workload": workload, "global_batch": B * world, "per_gpu_batch": B,
                   "parallelism": "dp%d" % world,
                   "launch": ("eager" + (" (graph capture failed)" if capture_error else "")) if not graphed
                   else ("hipGraph x3 (per phase)" if (world > 1 or args.segmented) else "hipGraph (whole step)"),
                   "capture_error": capture_error, "tune_file": args.tune_file},
        "roofline": {"bound": "mfma", "achieved": round(achieved, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / PEAK_BF16_TFLOPS, 4), "traffic": traffic,
                     "traffic_source": traffic_src,
                     "kernel": "tpg %s, enhance_features_128 (206->206, 5x5, %dx%d, bs%d, +residual, LeakyReLU, %s)"
                               % (PASS_KERNEL.get(top["pass"], top["pass"]), S, S, B, args.dtype),
                     "pass": top["pass"], "flops_per_launch": k_flops, "avg_launch_ms": round(k_ms, 4),
                     "launches": top["launches"], "ms_per_step": top["ms_per_step"],
                     "timing": ("HIP events on the launch stream, eager probe steps after the timed graph replays"
                                if graphed else "HIP events on the launch stream over the timed steps"),
                     "selection": "the probed enhance_features_128 kernel with the most time per step"},
        "roofline_kernels": kern,
        "step_mfma": {"algorithmic_tflop_per_step": round(flops_step / 1e12, 4),
                      "gflop_per_face": round(flops_step / B / 1e9, 2),
                      "achieved_tflops": round(flops_step / (ms_per_step * 1e-3) / 1e12, 2),
                      "frac_of_peak": round(flops_step / (ms_per_step * 1e-3) / 1e12 / PEAK_BF16_TFLOPS, 4)},
        "cpu_baseline": cpu,
    }
    if world > 1:
        bst = trainer.bucket_stats()
        n_ex = max(exposed["steps"], 1)
        out["dp"] = {"backend": args.dist_backend, "devices": ndev,
                     "real_ahead_reused": trainer.real_ahead_used,
                     "g_buckets": bst["G"]["buckets"], "d_buckets": bst["D"]["buckets"],
                     "g_bucket_bytes": bst["G"]["bytes"], "d_bucket_bytes": bst["D"]["bytes"],
                     "buckets": bst,
                     "exposed_comm_ms_per_step": {
                         "G": round(exposed["G"] / n_ex, 4), "D": round(exposed["D"] / n_ex, 4),
                         "total": round((exposed["G"] + exposed["D"]) / n_ex, 4), "steps": exposed["steps"],
                         "source": "HIP events on the compute stream around each gradient exchange (bucket tail "
                                   "wait + any un-overlapped all-reduce), max over ranks"},
                     "overlap_optimizer": trainer.overlap_optimizer,
                     "bucket_order_learned": bool(trainer.gsync is not None and trainer.gsync.order_learned)}
    print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
