"""The G+D train step of TP-GAN (build-defined: the reference has no GAN loop).

The reference stops at the models (`D_and_G_model.py`) and the loss weights
(`config.py:71-82`, marked provisional at :48); SURVEY.md §3C / §8f1 define the step this
module implements:

  1. G forward (Generator.forward, D_and_G_model.py:374-407)
  2. D-step: D on [real ; fake.detach()] as one 2B batch, WGAN critic loss
     mean D(fake) - mean D(real) (+ weight_gradient_penalty * GP when enabled), backward,
     gradient all-reduce (data parallel), Adam
  3. G-step: D frozen (UtilityMethods.set_requires_grad, :43-56), D(fake),
     L = w_pix*L1(fake, frontal) + w_local*mean L1(local fakes, local targets)
       + w_sym*L1(fake, mirror(fake)) - w_adv*mean D(fake) + w_tv*TV(fake)
       + w_ce*CE(encoder_predict, label) [+ w_id*identity]
     backward through D into G, gradient all-reduce, Adam
  (config.loss weight_128 multiplies the 128-px pixel term; weight_64/weight_32 have no
  producer because decoded_img32/64 are commented out in the reference, :254,:263.)

Parameters of G and D live in one flat fp32 buffer each (params are views), so the
optimizer is one HIP Adam launch per network and the data-parallel exchange is one
RCCL all-reduce per network (torch.distributed, backend "nccl" = RCCL over xGMI).
"""
import gc
import os
import weakref

import torch
import torch.distributed as dist
import torch.nn.functional as F

import tpgan_ops
from config import loss as LOSS_W
from UtilityMethods import set_requires_grad


class FlatParams:
    """All parameters of `module` as views into one fp32 buffer, grads likewise."""

    def __init__(self, module, device):
        self.params = [p for p in module.parameters()]
        total = sum(p.numel() for p in self.params)
        self.data = torch.zeros(total, dtype=torch.float32, device=device)
        self.grad = torch.zeros(total, dtype=torch.float32, device=device)
        self.exp_avg = torch.zeros_like(self.data)
        self.exp_avg_sq = torch.zeros_like(self.data)
        self.adam_state = torch.zeros(4, dtype=torch.float32, device=device)  # {step, bias corrections}
        self.step = 0             # host count of adam() calls; adam_state[0] (device) is the optimizer's
        self.skipped = torch.zeros((), dtype=torch.float32, device=device)  # fp16 steps skipped as non-finite
        self.epoch = 0            # bumped by every optimizer update (pre-packed weight images follow it)
        self.layout_version = 0   # bumped by relayout(): captured hipGraphs hold the old buffers
        self.pack_entries = {}    # tpgan_ops pre-packed weight images of this network's convs
        self.pack_table = None
        self.pack_version = 0     # bumped whenever pack_entries change (per-bucket pack tables follow it)
        self.offsets = []
        off = 0
        for p in self.params:
            n = p.numel()
            self.offsets.append(off)
            self._bind(p, off, n)
            off += n

    def relayout(self, order):
        """Re-place the parameters in the flat buffers in `order` (a permutation of
        parameter indices): values, gradients and Adam moments move with them and every
        parameter / .grad view is re-bound."""
        assert sorted(order) == list(range(len(self.params)))
        bufs = [self.data, self.grad, self.exp_avg, self.exp_avg_sq]
        new = [torch.empty_like(b) for b in bufs]
        offsets = [0] * len(self.params)
        off = 0
        for i in order:
            n = self.params[i].numel()
            for b, nb in zip(bufs, new):
                nb[off:off + n].copy_(b[self.offsets[i]:self.offsets[i] + n])
            offsets[i] = off
            off += n
        self.data, self.grad, self.exp_avg, self.exp_avg_sq = new
        self.offsets = offsets
        self.layout_version += 1
        self.pack_entries = {}  # weights moved: packed images are rebuilt on next use
        self.pack_table = None
        self.pack_version += 1
        for i, p in enumerate(self.params):
            n = p.numel()
            p.data = self._view(self.data, p, offsets[i], n)
            p.grad = self._view(self.grad, p, offsets[i], n)

    def _view(self, buf, p, off, n):
        flat = buf[off:off + n]
        if p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last) and not p.is_contiguous():
            a, b, h, w = p.shape
            return flat.view(a, h, w, b).permute(0, 3, 1, 2)
        return flat.view(p.shape)

    def _bind(self, p, off, n):
        v = self._view(self.data, p, off, n)
        v.copy_(p.data)
        p.data = v
        p.grad = self._view(self.grad, p, off, n)
        p._tpg_fused_grad = True  # HIP weight/bias gradients add straight into self.grad
        p._tpg_flat = self

    def zero_grad(self):
        self.grad.zero_()

    def adam(self, lr, betas=(0.5, 0.999), eps=1e-8, weight_decay=0.0, grad_scale=1.0, check_finite=False):
        """One Adam update of the whole network (one launch).  check_finite (the loss-scaled
        fp16 step): an inf / NaN anywhere in the gradients skips the update on the device --
        parameters, moments and the step counter stay as they were (last_step_skipped())."""
        self.step += 1
        if check_finite:
            tpgan_ops.grad_check(self.grad, self.adam_state)
        # (Adam fused with the weight-image repack was built in round 5 and removed in round 6:
        # bit-identical but slower, G 1.084 + 0.341 ms against 0.652 + 0.509 ms isolated --
        # the images' 16-byte chunks gather 8 channels from 8 master rows, so one of the two
        # streams scatters whichever order the fused kernel walks)
        tpgan_ops.adam_step(self.data, self.grad, self.exp_avg, self.exp_avg_sq, lr, betas[0], betas[1], eps,
                            weight_decay, self.adam_state, 0, grad_scale)
        if check_finite:  # (on the device: no synchronisation; skipped_steps() reads it)
            self.skipped.add_(self.adam_state[3].ne(0).float())
        self.epoch += 1
        tpgan_ops.repack(self)

    def skipped_steps(self):
        """Updates skipped for non-finite gradients so far (synchronises).  A run whose static
        loss scale keeps overflowing stops learning; this is the signal.  The step counter that
        drives Adam's bias correction is adam_state[0], which a skipped update leaves alone
        (self.step counts adam() calls, skipped or not)."""
        return int(self.skipped.item())

    # ---- the same update bucket by bucket (OverlappedGradSync's optimizer): adam_begin once per
    # step on the launching stream, adam_bucket per bucket on the communication stream as its
    # gradients complete (under the rest of the backward), adam_end when all have been issued.
    def adam_begin(self, betas=(0.5, 0.999)):
        self.step += 1
        tpgan_ops.adam_advance(self.adam_state, betas[0], betas[1])

    def adam_bucket(self, off, n, lr, betas=(0.5, 0.999), eps=1e-8, weight_decay=0.0, grad_scale=1.0):
        tpgan_ops.adam_slice(self.data, self.grad, self.exp_avg, self.exp_avg_sq, off, n, lr, betas[0], betas[1], eps,
                             weight_decay, self.adam_state, grad_scale)
        tpgan_ops.repack_range(self, off, n, self.epoch + 1)  # (the images of these parameters, at the new epoch)

    def adam_end(self):
        self.epoch += 1  # (images outside every bucket range keep the old epoch: re-packed on next use)

    def last_step_skipped(self):
        """True when the last adam(check_finite=True) found non-finite gradients (synchronises)."""
        return float(self.adam_state[3]) != 0.0

    # ---- checkpoint: torch.optim.Adam's state_dict format, so the files of
    # UtilityMethods.save_optimizer (UtilityMethods.py:78-103) load into either optimizer.
    def optimizer_state_dict(self, lr, betas=(0.5, 0.999), eps=1e-8, weight_decay=0.0):
        # the device counter advances inside graph replays: it, not self.step, is the truth
        step = int(round(float(self.adam_state[0].item())))
        state = {}
        for i, p in enumerate(self.params):
            o, n = self.offsets[i], p.numel()
            state[i] = {"step": torch.tensor(float(step)),
                        "exp_avg": self._view(self.exp_avg, p, o, n).detach().cpu().contiguous().clone(),
                        "exp_avg_sq": self._view(self.exp_avg_sq, p, o, n).detach().cpu().contiguous().clone()}
        group = {"lr": lr, "betas": tuple(betas), "eps": eps, "weight_decay": weight_decay, "amsgrad": False,
                 "maximize": False, "foreach": None, "capturable": False, "differentiable": False, "fused": None,
                 "params": list(range(len(self.params)))}
        return {"state": state, "param_groups": [group]}

    def check_optimizer_state_dict(self, sd):
        """Validate an Adam state_dict against this network without touching any state;
        returns (step, stored hyperparameters {lr, betas, eps, weight_decay})."""
        st = sd["state"]
        steps = {int(round(float(v["step"]))) for v in st.values()} or {0}
        if len(steps) != 1:
            raise ValueError("optimizer state: parameters at different step counts %s" % sorted(steps))
        for i, v in st.items():
            if not (0 <= int(i) < len(self.params)):
                raise ValueError("optimizer state: parameter index %s out of range" % (i,))
            p = self.params[int(i)]
            for k in ("exp_avg", "exp_avg_sq"):
                if tuple(v[k].shape) != tuple(p.shape):
                    raise ValueError("optimizer state %d/%s: shape %s, parameter %s" %
                                     (int(i), k, tuple(v[k].shape), tuple(p.shape)))
        groups = sd.get("param_groups") or [{}]
        g = groups[0]
        hp = {k: (tuple(g[k]) if k == "betas" else g[k]) for k in ("lr", "betas", "eps", "weight_decay") if k in g}
        return steps.pop(), hp

    def load_optimizer_state_dict(self, sd):
        """Restore Adam moments and the step count (per parameter, so a checkpoint written
        before a bucket relayout loads after it).  Missing entries mean zero moments.  Returns
        the stored hyperparameters {lr, betas, eps, weight_decay} (param_groups[0]); the
        caller compares them with its own (TPGANTrainer.load_checkpoint).  Everything is
        validated before any state changes."""
        step, hp = self.check_optimizer_state_dict(sd)
        st = sd["state"]
        with torch.no_grad():
            self.exp_avg.zero_()
            self.exp_avg_sq.zero_()
            for i, p in enumerate(self.params):
                if i not in st:
                    continue
                o, n = self.offsets[i], p.numel()
                for k, buf in (("exp_avg", self.exp_avg), ("exp_avg_sq", self.exp_avg_sq)):
                    self._view(buf, p, o, n).copy_(st[i][k])
            self.adam_state.zero_()
            self.adam_state[0] = float(step)  # the next launch advances it and recomputes the corrections
        self.step = step
        return hp

    def weights_loaded(self):
        """After parameter values were overwritten in place (load_state_dict): rebuild the packed images."""
        self.epoch += 1
        tpgan_ops.repack(self)


class GradSync:
    """Data-parallel exchange of one FlatParams: parameters broadcast from
    rank 0 once, gradients summed with one all-reduce per network per step (RCCL over
    xGMI with backend "nccl"; gloo on CPU for tests).  The 1/world average is folded into
    the optimizer's grad_scale, so no extra pass over the gradients is made."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1

    def broadcast(self, flat):
        if self.world > 1:
            dist.broadcast(flat.data, 0, group=self.group)

    def allreduce(self, flat):
        if self.world > 1:
            dist.all_reduce(flat.grad, group=self.group)

    @property
    def grad_scale(self):
        return 1.0 / self.world


class OverlappedGradSync(GradSync):
    """Bucketed gradient all-reduce overlapped with the backward.

    The flat gradient buffer is cut into parameter-aligned buckets of ~bucket_mb.  During
    the backward every fused HIP weight/bias-gradient launch reports its parameter
    (tpgan_ops.GRAD_READY_HOOK); when all parameters of a bucket are in, an event is
    recorded on each producing stream and the bucket's RCCL all-reduce is issued on a
    communication stream that waits on those events — while the backward of the
    remaining layers keeps the compute streams busy.  Buckets are issued strictly in
    index order (a bucket that completes early waits for its predecessors), so every rank
    issues the same collective sequence regardless of timing.  finish() issues what is
    left (parameters that reported nothing are complete once backward() has returned)
    and makes the current stream wait for all of them.

    After the first step the parameters are re-laid out in the order rank 0 observed
    their gradients completing (broadcast, so all ranks agree), which turns "bucket k is
    ready" into "the k-th stretch of the backward is done" — DDP's bucket rebuild."""

    def __init__(self, flat, group=None, bucket_mb=32.0, count_accumulate=False, optimizer=None):
        super(OverlappedGradSync, self).__init__(group)
        self.flat = flat
        # optimizer(off, n): enqueue the update of flat[off:off + n] on the current stream; each
        # bucket's update runs on the communication stream right behind its all-reduce (world 1:
        # behind its producers' events), i.e. under the remaining backward
        self.optimizer = optimizer
        self.updated = False  # set by finish(): this step's update was issued bucket by bucket
        self.bucket_bytes = int(bucket_mb * 2 ** 20)
        self.active = False
        self.order_learned = False
        # count_accumulate (WGAN-GP's D): a parameter receives several gradient contributions in
        # one backward (the fused HIP weight gradient, then autograd's accumulation of the double
        # backward's); each is counted (the fused path's report, a post-accumulate-grad hook) and
        # the parameter is ready at the count the first step observed -- that step issues its
        # buckets only at finish()
        self.count_accumulate = count_accumulate
        self.expected = None
        if count_accumulate:
            for p in flat.params:
                if p.requires_grad:
                    p.register_post_accumulate_grad_hook(self._ready)
        self._build()

    def _build(self):
        f = self.flat
        self.index = {id(p): i for i, p in enumerate(f.params)}
        self.buckets = []  # (offset, numel, [param indices])
        cur, start, size = [], None, 0
        # walk the buffer from its end (the last-laid-out parameters finish first)
        for i in sorted(range(len(f.params)), key=lambda j: f.offsets[j], reverse=True):
            off, n = f.offsets[i], f.params[i].numel()
            if cur and (size + n) * 4 > self.bucket_bytes:
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(i)
            size += n
        if cur:
            self.buckets.append(cur)
        self.bucket_of = {}
        self.spans = []
        for b, idxs in enumerate(self.buckets):
            lo = min(f.offsets[i] for i in idxs)
            hi = max(f.offsets[i] + f.params[i].numel() for i in idxs)
            assert hi - lo == sum(f.params[i].numel() for i in idxs), "bucket must be contiguous"
            self.spans.append((lo, hi - lo))
            for i in idxs:
                self.bucket_of[i] = b

    def begin(self):
        if self.world == 1 and self.optimizer is None:
            return
        self.active = True
        self.updated = False
        if self.expected is not None:  # parameters that get no gradient at all count as done
            self.pending = [sum(1 for i in idxs if self.expected[i] > 0) for idxs in self.buckets]
        else:
            self.pending = [len(idxs) for idxs in self.buckets]
        self.seen = set()
        self.counts = [0] * len(self.flat.params)
        self.last_seq = [-1] * len(self.flat.params)
        self.next = 0
        self.works = []
        self.order = []
        self.events = [[] for _ in self.buckets]
        cuda = self.flat.grad.is_cuda
        if cuda and not hasattr(self, "comm"):
            self.comm = torch.cuda.Stream(device=self.flat.grad.device)
        tpgan_ops.GRAD_READY_HOOK[0] = self._ready

    def _ready(self, p):
        if not self.active:
            return
        i = self.index.get(id(p))
        if i is None or (i in self.seen and not self.count_accumulate):
            return
        b = self.bucket_of[i]
        if self.flat.grad.is_cuda:  # (one event per contribution: they may come from several streams)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream())
            self.events[b].append(ev)
        if self.count_accumulate:
            self.counts[i] += 1
            if self.expected is None:  # learning step: record, issue nothing before finish()
                self.last_seq[i] = sum(self.counts)
                return
            if self.counts[i] < self.expected[i]:
                return
            if self.counts[i] > self.expected[i]:
                # a contribution beyond what the learning step observed: the parameter's bucket
                # may already be in flight, so this add would race its all-reduce
                raise RuntimeError("OverlappedGradSync: parameter %d got %d gradient contributions, the first "
                                   "step observed %d" % (i, self.counts[i], self.expected[i]))
        self.seen.add(i)
        self.order.append(i)
        self.pending[b] -= 1
        while self.next < len(self.buckets) and self.pending[self.next] == 0:
            self._issue(self.next)
            self.next += 1

    def _issue(self, b, after_stream=None):
        off, n = self.spans[b]
        view = self.flat.grad[off:off + n]
        if self.flat.grad.is_cuda:
            with torch.cuda.stream(self.comm):
                for ev in self.events[b]:
                    self.comm.wait_event(ev)
                if after_stream is not None:
                    self.comm.wait_stream(after_stream)
                if self.world > 1:
                    w = dist.all_reduce(view, group=self.group, async_op=True)
                    self.works.append(w)
                    if self.optimizer is not None:
                        w.wait()  # (the communication stream waits for the collective)
                if self.optimizer is not None:
                    self.optimizer(off, n)
        else:
            if self.world > 1:
                self.works.append(dist.all_reduce(view, group=self.group, async_op=True))
            if self.optimizer is not None:
                if self.works:
                    self.works[-1].wait()
                self.optimizer(off, n)

    def finish(self):
        if not self.active:
            return
        tpgan_ops.GRAD_READY_HOOK[0] = None
        self.active = False
        if self.count_accumulate and self.expected is None:
            # the learning step: contributions per parameter, and the completion order by each
            # parameter's last contribution (what the buckets will wait for from now on)
            self.expected = list(self.counts)
            self.order = sorted((i for i in range(len(self.counts)) if self.counts[i] > 0),
                                key=lambda i: self.last_seq[i])
        elif self.count_accumulate:
            bad = [i for i in range(len(self.counts)) if self.counts[i] != self.expected[i]]
            if bad:
                raise RuntimeError("OverlappedGradSync: gradient contribution counts changed since the first step "
                                   "(parameters %s: %s, expected %s)" % (bad[:5], [self.counts[i] for i in bad[:5]],
                                                                          [self.expected[i] for i in bad[:5]]))
        cur = torch.cuda.current_stream() if self.flat.grad.is_cuda else None
        while self.next < len(self.buckets):
            self._issue(self.next, after_stream=cur)
            self.next += 1
        for w in self.works:
            w.wait()
        self.works = []
        if self.optimizer is not None:
            if cur is not None:
                cur.wait_stream(self.comm)
            self.updated = True
        if not self.order_learned:
            self._learn_order()

    def _learn_order(self):
        """Rank 0's completion order (unreported parameters after it, in reverse
        registration order), broadcast and applied to the flat layout on every rank."""
        f = self.flat
        n = len(f.params)
        seen = set(self.order)
        order = list(self.order) + [i for i in reversed(range(n)) if i not in seen]
        t = torch.tensor(order, dtype=torch.int64, device=f.grad.device)
        if self.world > 1:
            dist.broadcast(t, 0, group=self.group)
        # layout: the first-completed parameters at the END of the buffer, so that the
        # reverse-order bucketing of _build() follows the completion order
        f.relayout([int(i) for i in reversed(t.tolist())])
        self.order_learned = True
        self._build()

    def allreduce(self, flat):
        if self.active:  # already being reduced bucket by bucket
            return self.finish()
        return super(OverlappedGradSync, self).allreduce(flat)


def _weak_method(m):
    ref = weakref.WeakMethod(m)

    def call(*args):
        f = ref()
        if f is not None:
            f(*args)
    return call


def _hp_equal(a, b):
    if isinstance(a, (tuple, list)) or isinstance(b, (tuple, list)):
        return len(a) == len(b) and all(_hp_equal(x, y) for x, y in zip(a, b))
    return abs(float(a) - float(b)) <= 1e-12 * max(1.0, abs(float(b)))


# the first train step runs the local pathways ungrouped so that their shapes are autotuned
# (a grouped launch cannot time candidates); False: grouped from the first step (A/B)
TUNE_UNGROUPED = {"enabled": True}

# the G step's pixel / symmetry / total-variation / local terms as the fused HIP ops
# (tpgan_ops.image_losses / l1_means); False: the aten expressions (A/B, tests)
FUSED_LOSSES = {"enabled": True}

# the identity-preserving loss (configs[2] / [4]: a frozen ResNet-50 / MobileNetV2 on the fake
# face) on a side stream, beside D's Adam, the frozen D(fake) and the other G losses; its
# input-gradient backward then runs on that stream too (autograd replays each node on its
# forward's stream), beside D(fake)'s.  Both paths are chains of small-map layers that leave
# most of the chip idle: configs[2] eager 38.19 / 37.95 -> 34.50 / 35.41 ms/step (gpurun r05ak).
# The stream is the real-image features' one (they ran in phase A): a process holding one more
# stream crashed in the first replay of a later whole-step capture (r05aj-r05al; reusing the
# stream, r05aq, it does not).  Not inside capture() ("in_capture"): hipStreamEndCapture
# crashed with the fork in the graph (r05ar).  False: everything on the step's stream.
IDENTITY_STREAM = {"enabled": True, "in_capture": True, "own_stream": False}


def total_variation(x):
    return (x[:, :, 1:, :] - x[:, :, :-1, :]).abs().mean() + (x[:, :, :, 1:] - x[:, :, :, :-1]).abs().mean()


class TPGANTrainer:
    """One process per GPU; call step(batch) with device-resident synthetic or real data.

    batch keys: I128 (B,3,128,128) profile face, left_eye/right_eye (B,3,40,40),
    nose (B,3,32,40), mouth (B,3,32,48), z (B,64), frontal (B,3,128,128) target,
    frontal_left_eye/... local targets, label (B,) int64 identity.
    """

    def __init__(self, G, D, lr=1e-4, betas=(0.5, 0.999), compute_dtype=torch.bfloat16, loss_weights=None,
                 gradient_penalty=False, process_group=None, identity_fn=None, use_dropout=True, overlap=True,
                 bucket_mb=32.0, loss_scale=None, real_ahead=None, overlap_optimizer=None):
        self.G, self.D = G, D
        # fp16 activations / gradients (BASELINE configs[4]): a static loss scale keeps the
        # per-element image gradients (~1/(B*3*H*W)) out of fp16's subnormal range; the scale
        # is divided out in the Adam launch (grad_scale), weight gradients accumulate in fp32
        if loss_scale is None:
            loss_scale = 1024.0 if compute_dtype == torch.float16 else 1.0
        if gradient_penalty and loss_scale != 1.0:
            raise ValueError("WGAN-GP with a loss scale is not supported (fp16: use bf16 for the GP run)")
        self.loss_scale = float(loss_scale)
        self.use_dropout = use_dropout  # FeaturePredict dropout (D_and_G_model.py:331-348)
        dev = next(G.parameters()).device
        self.fG = FlatParams(G, dev)
        self.fD = FlatParams(D, dev)
        self.lr, self.betas = lr, betas
        self.dtype = compute_dtype
        self.w = dict(LOSS_W if loss_weights is None else loss_weights)
        self.gp = gradient_penalty
        self.gp_frozen_first_order = True  # (gradient_penalty: D frozen in the first-order pass; False = A/B)
        self._tuned_ungrouped = False
        self._nsteps = 0
        self.tune_steps = 3  # the tuning window (tpgan_ops.AUTOTUNE["frozen"] after it)
        self.sync = GradSync(process_group)
        self.world = self.sync.world
        # G's 551 MB of gradients are reduced bucket by bucket during the G backward, D's 54 MB
        # during the D-step backward (buckets of bucket_mb / 4: D's backward is ~5x shorter)
        # overlap_optimizer: G's Adam (and the repack of its bf16 weight images) bucket by bucket
        # on the communication stream as each bucket's gradients complete (world > 1: right behind
        # its all-reduce), under the rest of the G backward; never with a loss scale (the fp16
        # step's overflow check must see every gradient before any update).  Off by default:
        # measured 35.14 vs 33.27 ms/step at world 1 (tools/ab_step.py, interleaved rounds,
        # profiles/r04/ab_bucketed_adam.txt) -- the full-chip Adam / pack grids on the second
        # stream slow the backward's kernels more than the ~0.7 ms of update they hide
        if overlap_optimizer is None:
            overlap_optimizer = False
        self.overlap_optimizer = bool(overlap_optimizer) and self.loss_scale == 1.0
        # (a weak reference: a bound method would make trainer <-> gsync a reference cycle, so a
        # dropped trainer's GPU buffers would wait for the cyclic GC -- which may then run in the
        # middle of another trainer's graph capture and free memory there)
        g_opt = _weak_method(self._g_bucket_update) if self.overlap_optimizer else None
        self.gsync = (OverlappedGradSync(self.fG, process_group, bucket_mb, optimizer=g_opt)
                      if (overlap and (self.world > 1 or g_opt is not None)) else None)
        # (with WGAN-GP a D parameter gets a second gradient contribution from the double
        # backward, after its first one: D's buckets then wait for the contribution count the
        # first step observed, OverlappedGradSync(count_accumulate=True))
        self.dsync = (OverlappedGradSync(self.fD, process_group, bucket_mb / 4.0, count_accumulate=gradient_penalty)
                      if (overlap and self.world > 1) else None)
        # the next step's D(real) forward / backward (it depends on the updated D,
        # not on the new G) runs under the G gradients' last buckets and G's Adam; on by default
        # in data-parallel runs, where that tail is the all-reduce's
        self.real_ahead = (self.world > 1) if real_ahead is None else bool(real_ahead)
        self._d_real_next = None
        self.real_ahead_used = 0  # steps whose D(real) came from the previous step's real_ahead pass
        self._capturing = False
        self._segmented = False
        self._graphs = []
        self._graph_setup = False  # (inside capture(), warm-up steps included)
        self.comm_timing = False  # exposed-communication events around each exchange (exposed_comm_ms)
        self.comm_events = []
        self.identity_fn = identity_fn
        self.identity_forks_captured = 0  # identity side-stream forks recorded inside capture()
        self.sync.broadcast(self.fG)
        self.sync.broadcast(self.fD)

    def _g_bucket_update(self, off, n):
        self.fG.adam_bucket(off, n, self.lr, self.betas, grad_scale=self.sync.grad_scale / self.loss_scale)

    def _allreduce(self, flat):
        ov = self.gsync if flat is self.fG else self.dsync
        # comm_timing (bench.py at world > 1): HIP events on the compute stream around the
        # exchange -- the first is reached once the backward's kernels are enqueued ahead of it,
        # the second once that stream has waited for the last bucket's all-reduce, so their
        # distance is the communication time the compute stream was left waiting for
        # (exposed), not the all-reduce time
        t = self.comm_timing and flat.grad.is_cuda and self.world > 1
        if t:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        if ov is not None and ov.active:
            ov.finish()
        else:
            self.sync.allreduce(flat)
        if t:
            e1.record()
            self.comm_events.append(("G" if flat is self.fG else "D", e0, e1))

    def exposed_comm_ms(self):
        """{"G": ms, "D": ms, "steps": n} summed over the steps recorded since the last call
        (comm_timing on); synchronises on the recorded events."""
        out = {"G": 0.0, "D": 0.0}
        for tag, e0, e1 in self.comm_events:
            e1.synchronize()
            out[tag] += e0.elapsed_time(e1)
        n = sum(1 for tag, _, _ in self.comm_events if tag == "G")
        self.comm_events = []
        out["steps"] = n
        return out

    def bucket_stats(self):
        """Gradient buckets of the data-parallel exchange: count and bytes per network."""
        out = {}
        for tag, ov, flat in (("G", self.gsync, self.fG), ("D", self.dsync, self.fD)):
            if ov is None:
                out[tag] = {"buckets": 1 if self.world > 1 else 0, "bytes": flat.grad.numel() * 4, "overlapped": False}
            else:
                sizes = [n * 4 for _, n in ov.spans]
                out[tag] = {"buckets": len(sizes), "bytes": sum(sizes), "min_bucket_bytes": min(sizes),
                            "max_bucket_bytes": max(sizes), "overlapped": True}
        return out

    # The step is three device phases separated by the two data-parallel exchanges:
    #   A: zero grads, G forward, D-step forward/backward           -> all-reduce D grads
    #   B: D Adam, G-step D forward, G losses, G backward            -> all-reduce G grads
    # (world > 1, eager: each exchange is bucketed and overlapped with its backward; the
    # phase boundary only waits for the last buckets)
    #   C: G Adam
    # Eager mode runs them back to back; graph mode (capture()) records each phase as a
    # hipGraph sharing one memory pool and replays them around the RCCL calls.
    def _phase_a(self, b):
        G, D = self.G, self.D
        self.fG.zero_grad()
        # D(real) of this batch already ran at the end of the previous step (_real_ahead): its
        # gradient is in fD.grad and its output is kept for the loss
        d_real_pre, self._d_real_next = self._d_real_next, None
        if d_real_pre is not None and (d_real_pre[0] is not b["frontal"] or
                                       d_real_pre[1] != self._real_key(b["frontal"])):
            # (the caller's next batch was not the one it announced, its images were refilled in
            # place since, or D's weights changed after the pass: a checkpoint load, a relayout)
            d_real_pre = None
        if d_real_pre is None:
            self.fD.zero_grad()
        else:
            self.real_ahead_used += 1
        # the identity loss's real-image features run on a side stream under G's forward
        # (not while phase A is captured as a graph of its own: the fork would stay unjoined
        # at the end of that capture, and phase B's graph would wait on work of another graph)
        pre = getattr(self.identity_fn, "real_features_async", None)
        if self._capturing and self._segmented:
            pre = None
        self._id_pre = pre(b["frontal"]) if pre is not None else None
        with tpgan_ops.compute_dtype(self.dtype):
            with tpgan_ops.roctx_range("G-fwd"):
                outs = G(b["I128"], b["left_eye"], b["right_eye"], b["nose"], b["mouth"], b["z"], self.use_dropout)
            fake = outs[0]
            B = fake.shape[0]
            with tpgan_ops.roctx_range("D-step"):
                real = tpgan_ops.to_cl(b["frontal"], self.dtype)
                if d_real_pre is None:
                    # ---- D-step (critic on real and detached fake as one 2B batch)
                    d_both = D(torch.cat([real, fake.detach()], 0)).float()
                    d_real, d_fake = d_both[:B], d_both[B:]
                else:
                    d_real, d_fake = d_real_pre[2], D(fake.detach()).float()
                loss_D = d_fake.mean() - d_real.mean()
                if self.gp:
                    loss_D = loss_D + self.w["weight_gradient_penalty"] * self.gradient_penalty(real, fake.detach())
                if self.dsync is not None and not self._capturing:
                    self.dsync.begin()
                (loss_D * self.loss_scale if self.loss_scale != 1.0 else loss_D).backward()
        self._st = {"outs": outs, "loss_D": loss_D.detach()}

    def _real_ahead(self, nb):
        """The next step's D(real) forward and backward of -mean D(real) into a fresh fD.grad
        (SURVEY.md §8e): it needs the D this step's Adam produced, not the new G, so it runs
        while G's last gradient buckets are still being reduced and before G's Adam.  Phase A of
        the next step adds D(fake)'s gradient to it (the same sum as the 2B critic batch)."""
        if nb is None or not self.real_ahead or self._capturing:
            return
        with tpgan_ops.roctx_range("D-real-ahead"), tpgan_ops.compute_dtype(self.dtype):
            self.fD.zero_grad()
            d_real = self.D(tpgan_ops.to_cl(nb["frontal"], self.dtype)).float()
            loss = -d_real.mean()
            (loss * self.loss_scale if self.loss_scale != 1.0 else loss).backward()
        self._d_real_next = (nb["frontal"], self._real_key(nb["frontal"]), d_real.detach())

    def _real_key(self, frontal):
        """What a precomputed D(real) pass is valid for: the very tensor (identity, storage
        address, in-place version counter -- a caller refilling one persistent batch buffer
        bumps it) and D's weights (FlatParams.epoch / layout_version: every optimizer update,
        load or relayout changes them)."""
        return (frontal.data_ptr(), frontal._version, self.fD.epoch, self.fD.layout_version)

    def gradient_penalty(self, real, fake, alpha=None):
        """WGAN-GP (config.py:72 weight_gradient_penalty): mean over the batch of
        (||grad_x D(x_hat)||_2 - 1)^2 at x_hat = a*real + (1-a)*fake, a ~ U[0,1) per sample.
        The input gradient is taken with create_graph=True, so loss.backward() runs the
        double backward through D on the HIP conv kernels (tpgan_ops._ConvDgrad/_ConvWgrad/
        _ConvFwdPlain); parameter gradients of this first-order pass are not accumulated
        into the flat buffer (tpgan_ops only fuses when no graph is being built)."""
        B = real.shape[0]
        a = torch.rand(B, 1, 1, 1, device=real.device, dtype=torch.float32) if alpha is None else alpha
        x_hat = (a * real.float() + (1 - a) * fake.float()).requires_grad_(True)
        # D's parameters are frozen for this forward, so the first-order pass (grad w.r.t. x_hat
        # only) skips every weight / bias gradient it would otherwise compute and discard; they
        # require grad again before the graph of gx is built, so gx's own nodes (the input
        # gradients, which read the saved weights) carry the double backward to them
        params = [p for p in self.D.parameters()] if self.gp_frozen_first_order else []
        flags = [p.requires_grad for p in params]
        set_requires_grad(params, False)
        try:
            # (no ActToken links: D's saved outputs of this forward also feed the double backward,
            # so their gradients have more than one contribution)
            with tpgan_ops.act_links(False):
                d_hat = self.D(x_hat).float()
        finally:
            for p, f in zip(params, flags):
                p.requires_grad_(f)
        (gx,) = torch.autograd.grad(d_hat.sum(), x_hat, create_graph=True)
        return ((gx.reshape(B, -1).float().norm(dim=1) - 1.0) ** 2).mean()

    def _phase_b(self, b):
        w = self.w
        D = self.D
        fake, pred, fused_fake, le_f, re_f, no_f, mo_f, _ = self._st.pop("outs")
        front = b["frontal"]
        id_st, l_ip = None, None
        # The identity fork (in eager steps and, since round 6, inside graph captures: the
        # round-5 crashes in hipStreamEndCapture came from an event wait of the features stream
        # on itself, FeatureExtract.IdentityPreservingLoss).  Its fork point is taken here, where
        # `fake` is ready, but its forward is enqueued after D's Adam and D(fake): its autograd
        # nodes are then created later than D(fake)'s, so the backward (latest-created first)
        # enqueues the identity input gradient on its stream before D(fake)'s on the main one,
        # and neither waits for the other (enqueued the other way round, the captured step had
        # the identity backward behind all of D(fake)'s).
        if (self.identity_fn is not None and IDENTITY_STREAM["enabled"] and fake.is_cuda and
                tpgan_ops.MULTISTREAM and
                (not self._graph_setup or IDENTITY_STREAM.get("in_capture", False))):
            main = torch.cuda.current_stream()
            # (the real-image features' stream: they ran in phase A, so the two never overlap)
            id_st = tpgan_ops.side_streams(fake.device, 1, "identity_fork" if IDENTITY_STREAM["own_stream"]
                                           else "identity")[0]
            id_st.wait_stream(main)
            if self._capturing:
                self.identity_forks_captured += 1
        with tpgan_ops.compute_dtype(self.dtype):
            self.fD.adam(self.lr, self.betas, grad_scale=self.sync.grad_scale / self.loss_scale,
                         check_finite=self.loss_scale != 1.0)
            # ---- G-step through the frozen, updated D
            set_requires_grad(D.parameters(), False)
            d_gen = D(fake).float()
            set_requires_grad(D.parameters(), True)
        if id_st is not None:
            with torch.cuda.stream(id_st):
                l_ip = self._identity_loss(fake, front)
        elif self.identity_fn is not None:
            # (the same point of the autograd graph as the side-stream form: the gradients at
            # `fake` are then summed in the same order, and the two forms are bit-identical)
            l_ip = self._identity_loss(fake, front)
        args = (fake, le_f, re_f, no_f, mo_f, d_gen, pred, front, b["frontal_left_eye"], b["frontal_right_eye"],
                b["frontal_nose"], b["frontal_mouth"], b["label"])
        loss_G = self._g_losses(*args)
        if self.identity_fn is not None:
            if id_st is not None:
                main = torch.cuda.current_stream()
                main.wait_stream(id_st)
                l_ip.record_stream(main)
            loss_G = loss_G + w["weight_identity_preserving"] * l_ip
        if self.gsync is not None and not self._capturing:
            if self.gsync.optimizer is not None:
                self.fG.adam_begin(self.betas)  # (the step counter, once, ahead of every bucket's update)
            self.gsync.begin()
        with tpgan_ops.roctx_range("G-bwd"):
            (loss_G * self.loss_scale if self.loss_scale != 1.0 else loss_G).backward()
        self._st["loss_G"] = loss_G.detach()

    def _identity_loss(self, fake, front):
        f32 = fake.float()
        if self._id_pre is not None:
            pre, self._id_pre = self._id_pre, None
            return self.identity_fn(f32, front, pre=pre)
        return self.identity_fn(f32, front)

    def _g_losses(self, fake, le_f, re_f, no_f, mo_f, d_gen, pred, front, fle, fre, fno, fmo, label):
        """The G-step's pixel, local, symmetry, adversarial, total-variation and identity-class
        losses (build-defined, config.py:59-82 weights)."""
        w = self.w
        if not FUSED_LOSSES["enabled"]:  # (the aten form, A/B)
            f32 = fake.float()
            l_pix = w["weight_128"] * (f32 - front).abs().mean()
            l_local = ((le_f.float() - fle).abs().mean() + (re_f.float() - fre).abs().mean() +
                       (no_f.float() - fno).abs().mean() + (mo_f.float() - fmo).abs().mean()) / 4.0
            l_sym = (f32 - f32.flip(3)).abs().mean()
            return (w["weight_pixelwise"] * l_pix + w["weight_pixelwise_local"] * l_local +
                    w["weight_symmetry"] * l_sym + w["weight_adv_G"] * -d_gen.mean() +
                    w["weight_total_varation"] * total_variation(f32) +
                    w["weight_cross_entropy"] * F.cross_entropy(pred.float(), label))
        # w_pixelwise * w_128 * mean|fake - front| + w_symmetry * mean|fake - flip(fake)|
        # + w_tv * total_variation(fake): one fused op (tpg_losses.hip), as the four local
        # w_pixelwise_local * mean|patch - crop| / 4 terms
        l_img = tpgan_ops.image_losses(fake, front, w["weight_pixelwise"] * w["weight_128"], w["weight_symmetry"],
                                       w["weight_total_varation"])
        l_local = tpgan_ops.l1_means([(le_f, fle), (re_f, fre), (no_f, fno), (mo_f, fmo)],
                                     [w["weight_pixelwise_local"] / 4.0] * 4)
        l_adv = -d_gen.mean()
        l_ce = F.cross_entropy(pred.float(), label)
        return l_img + l_local + w["weight_adv_G"] * l_adv + w["weight_cross_entropy"] * l_ce

    def _phase_c(self, b):
        with tpgan_ops.roctx_range("G-adam"):
            if self.gsync is not None and self.gsync.updated:
                self.gsync.updated = False  # (updated bucket by bucket under the G backward)
                self.fG.adam_end()
            else:
                self.fG.adam(self.lr, self.betas, grad_scale=self.sync.grad_scale / self.loss_scale,
                             check_finite=self.loss_scale != 1.0)
        out = {"loss_D": self._st["loss_D"], "loss_G": self._st["loss_G"]}
        if self.loss_scale != 1.0:  # device tensors: reading them is the caller's synchronisation
            out["skipped_D"], out["skipped_G"] = self.fD.skipped, self.fG.skipped
        return out

    # ---- checkpoint / resume.  Files and formats of the reference's
    # UtilityMethods.save_model / save_optimizer (UtilityMethods.py:58-103), one directory per
    # network: <dir>/{G,D}/model_epoch_<e>.pth (state_dict) and optimizer_epoch_<e>.pth
    # ({optimizer: torch.optim.Adam state_dict, model: state_dict, epoch}).  The reference
    # writes these but never reads them back (config.py:56-57); load_checkpoint resumes.
    def _nets(self):
        return (("G", self.G, self.fG), ("D", self.D, self.fD))

    def _rank(self):
        return dist.get_rank(self.sync.group) if self.world > 1 else 0

    def save_checkpoint(self, dir, epoch):
        """Rank 0 writes (every rank holds the same replica); each file goes to a temporary
        name first and is renamed into place (os.replace, atomic on POSIX), so a reader never
        sees a partial file; all ranks leave only after the files exist (barrier)."""
        import os
        torch.cuda.synchronize() if self.fG.data.is_cuda else None
        payload = []
        for tag, net, flat in self._nets():  # collective-free, but every rank walks the same state
            sd = {k: v.detach().cpu().contiguous().clone() for k, v in net.state_dict().items()}
            payload.append((tag, sd, flat.optimizer_state_dict(self.lr, self.betas)))
        if self._rank() == 0:
            for tag, sd, opt in payload:
                d = os.path.join(dir, tag)
                os.makedirs(d, exist_ok=True)
                for name, obj in (("model_epoch_%s.pth" % epoch, sd),
                                  ("optimizer_epoch_%s.pth" % epoch, {"optimizer": opt, "model": sd, "epoch": epoch})):
                    final = os.path.join(d, name)
                    tmp = final + ".tmp%d" % os.getpid()
                    torch.save(obj, tmp)
                    os.replace(tmp, final)
        if self.world > 1:
            dist.barrier(group=self.sync.group)

    def load_checkpoint(self, dir, epoch, adopt_hparams=False):
        """Restore both networks and their Adam states; returns the stored epoch.  Loaded with
        weights_only=True (nothing in the file is executed).  The file's optimizer
        hyperparameters (lr, betas, eps, weight_decay; e.g. the reference's getOptimizer Adam,
        UtilityMethods.py:30-36, betas (0.9, 0.999)) must match this trainer's, since the
        restored moments were built under them: a mismatch raises ValueError, or, with
        adopt_hparams=True, the trainer takes the stored lr and betas (eps 1e-8 and
        weight_decay 0 are fixed here, so those must match either way)."""
        import os
        if self.world > 1:  # the writer's files are complete before anyone reads
            dist.barrier(group=self.sync.group)
        # every file is read and checked before anything is restored: a mismatch (in either
        # network) leaves the trainer exactly as it was
        loaded, adopt = [], {}
        for tag, net, flat in self._nets():
            ck = torch.load(os.path.join(dir, tag, "optimizer_epoch_%s.pth" % epoch), map_location="cpu",
                            weights_only=True)
            _, hp = flat.check_optimizer_state_dict(ck["optimizer"])
            mine = {"lr": self.lr, "betas": tuple(self.betas), "eps": 1e-8, "weight_decay": 0.0}
            bad = {k: (hp[k], mine[k]) for k in hp if k in mine and not _hp_equal(hp[k], mine[k])}
            fixed = {k: v for k, v in bad.items() if k in ("eps", "weight_decay")}
            if bad and (not adopt_hparams or fixed):
                raise ValueError("checkpoint %s/%s optimizer hyperparameters differ from the trainer's "
                                 "(stored, trainer): %s" % (tag, epoch, bad))
            if bad:
                if adopt and any(not _hp_equal(adopt[k], hp[k]) for k in adopt if k in hp):
                    raise ValueError("checkpoint %s: G and D were saved with different hyperparameters" % epoch)
                adopt.update({k: hp[k] for k in ("lr", "betas") if k in hp})
            own = net.state_dict()
            sd = ck["model"]
            if set(sd) != set(own):
                raise ValueError("checkpoint %s/%s: state_dict keys differ (missing %s, unexpected %s)" %
                                 (tag, epoch, sorted(set(own) - set(sd))[:5], sorted(set(sd) - set(own))[:5]))
            for k, v in sd.items():
                if tuple(v.shape) != tuple(own[k].shape):
                    raise ValueError("checkpoint %s/%s: %s has shape %s, model %s" %
                                     (tag, epoch, k, tuple(v.shape), tuple(own[k].shape)))
            loaded.append((net, flat, ck))
        self._d_real_next = None  # (a D(real) pass precomputed with the old weights)
        if adopt:
            self.lr = float(adopt.get("lr", self.lr))
            self.betas = tuple(adopt.get("betas", self.betas))
        out = None
        for net, flat, ck in loaded:
            flat.load_optimizer_state_dict(ck["optimizer"])
            net.load_state_dict(ck["model"])  # copies into the flat-buffer views
            flat.weights_loaded()
            out = ck["epoch"]
        return out  # every rank reads the same files: replicas stay identical without a broadcast

    def step(self, b, next_b=None):
        """One eager G+D train step.  next_b: the batch of the following step, when known --
        its D(real) pass then runs under this step's G-gradient all-reduce tail (real_ahead)."""
        if not self._tuned_ungrouped and TUNE_UNGROUPED["enabled"] and tpgan_ops.AUTOTUNE["enabled"]:
            # the first step runs the local pathways ungrouped (their own streams, same
            # concurrency flag), so the weight-gradient tuner sees their shapes; the grouped
            # launches of later steps take those picks from the tuning cache
            self._tuned_ungrouped = True
            prev = tpgan_ops.GROUP["enabled"]
            tpgan_ops.GROUP["enabled"] = False
            try:
                return self.step(b, next_b)
            finally:
                tpgan_ops.GROUP["enabled"] = prev
        # the autotuners time new shapes during this trainer's first tune_steps steps only; a
        # shape first seen later (a partial last batch) takes the planner's default plan rather
        # than synchronising the device for a tuning sweep mid-training
        frozen = tpgan_ops.AUTOTUNE["frozen"]
        tpgan_ops.AUTOTUNE["frozen"] = frozen or self._nsteps >= self.tune_steps
        self._nsteps += 1
        try:
            self._phase_a(b)
            with tpgan_ops.roctx_range("allreduce-D"):
                self._allreduce(self.fD)
            self._phase_b(b)
            self._real_ahead(next_b)
            with tpgan_ops.roctx_range("allreduce-G"):
                self._allreduce(self.fG)
            return self._phase_c(b)
        finally:
            tpgan_ops.AUTOTUNE["frozen"] = frozen

    def capture(self, b, warmup=3, segmented=None):
        """Record the train step as hipGraphs (torch.cuda.CUDAGraph over HIP streams): one
        graph per phase sharing a memory pool (world > 1: the RCCL all-reduces run between
        replays) or a single graph (world == 1).  `b` becomes the static input batch;
        step_graphed() copies new data into it.  Warm-up steps (which also run the
        weight-gradient autotuner, and train the model) run on a side stream first, as
        capture requires."""
        self._graph_setup = True
        try:
            self._capture(b, warmup, segmented)
        finally:
            self._graph_setup = False

    def _capture(self, b, warmup, segmented):
        self._static = {k: v.clone() for k, v in b.items()}
        self._d_real_next = None  # (graph replays never run the eager real_ahead pass)
        gc.collect()  # (nothing of earlier steps or trainers may be freed while a graph is being captured)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        # the data-parallel bucket layout is re-learned after the first overlapped step
        # (FlatParams.relayout moves every parameter, gradient and packed weight image): that
        # step must run before capture, or the graphs would keep the old buffers' addresses
        pending = any(s is not None and not s.order_learned for s in (self.gsync, self.dsync))
        with torch.cuda.stream(side):
            for _ in range(max(warmup, 1 if pending else 0)):
                self.step(self._static)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        if segmented is None:
            segmented = self.world > 1
        # the captured phase C repacks every weight image with one batched launch, whose job table
        # is built (host -> device copy) on first use: build it now, outside the capture (the eager
        # steps updated G bucket by bucket and never needed it); the images are re-packed unchanged
        tpgan_ops.repack(self.fG)
        tpgan_ops.repack(self.fD)
        torch.cuda.synchronize()
        self._capturing = True  # graph replays reduce G in one call between phases
        self._segmented = bool(segmented)
        phases = (self._phase_a, self._phase_b, self._phase_c)
        self._graphs = []
        # no cyclic garbage collection while a graph is being recorded: a collection run inside
        # the capture window (triggered by any allocation of Python objects) would free the
        # device memory of whatever unreachable cycle it finds -- a dropped trainer, a stale
        # autograd graph -- and a free during capture aborts the process.  The collect() above
        # empties what exists now; this keeps anything that becomes garbage meanwhile alive
        # until the capture has ended.
        gc_was_enabled = gc.isenabled()
        gc.disable()
        try:
            if not segmented:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for ph in phases:
                        out = ph(self._static)
                self._graphs.append(g)
            else:
                pool = None
                for ph in phases:
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, pool=pool):
                        out = ph(self._static)
                    pool = g.pool()
                    self._graphs.append(g)
        finally:
            if gc_was_enabled:
                gc.enable()
        self._graph_out = out
        self._graph_layout = (self.fG.layout_version, self.fD.layout_version)
        torch.cuda.synchronize()

    def reset_capture(self):
        """Drop every graph and the state a (possibly failed) capture() left: the graphs and
        their memory pool, the static batch, the graph outputs; eager step() is then the only
        launch mode, as before capture()."""
        self._capturing = False
        self._segmented = False
        self._graph_setup = False
        self._graphs = []
        self._static = None
        self._graph_out = None
        self._graph_layout = None
        self._st = {}
        self._id_pre = None
        gc.collect()
        torch.cuda.synchronize()

    def step_graphed(self, b=None):
        """One train step by graph replay (capture() first).  Returns the step's losses as
        fresh tensors: the graph's own outputs live in its memory pool and the next replay
        overwrites them, so a caller holding step k's dict would otherwise read step k+1's
        values (round 2's graphed-loss experiment returned such aliased outputs)."""
        if not self._graphs:
            raise RuntimeError("step_graphed() without a captured step: capture() first")
        if (self.fG.layout_version, self.fD.layout_version) != self._graph_layout:
            raise RuntimeError("the parameters were re-laid out after capture(): the graphs hold the old buffers; "
                               "capture() again")
        if b is not None and b is not self._static:
            for k, v in b.items():
                self._static[k].copy_(v, non_blocking=True)
        if len(self._graphs) == 1:
            self._graphs[0].replay()
        else:
            ga, gb, gc = self._graphs
            ga.replay()
            self._allreduce(self.fD)
            gb.replay()
            self._allreduce(self.fG)
            gc.replay()
        return {k: v.clone() for k, v in self._graph_out.items()}


def synthetic_batch(B, device, seed=0, img_size=128):
    """Multi-PIE-shaped synthetic batch, U[-1, 1] images (DataAndDataset.py:220), z, labels.
    img_size 256 (BASELINE configs[4]) doubles the face and the patch sizes (LocalFuser(256))."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    k = img_size // 128

    def u(*s):
        return (torch.rand(*s, generator=g) * 2 - 1).to(device)

    S, E, NH, NW, MH, MW = img_size, 40 * k, 32 * k, 40 * k, 32 * k, 48 * k
    b = {"I128": u(B, 3, S, S), "left_eye": u(B, 3, E, E), "right_eye": u(B, 3, E, E),
         "nose": u(B, 3, NH, NW), "mouth": u(B, 3, MH, MW), "z": u(B, 64), "frontal": u(B, 3, S, S),
         "frontal_left_eye": u(B, 3, E, E), "frontal_right_eye": u(B, 3, E, E), "frontal_nose": u(B, 3, NH, NW),
         "frontal_mouth": u(B, 3, MH, MW),
         "label": torch.randint(0, 347, (B,), generator=g).to(device)}
    return b
