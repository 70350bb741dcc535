"""Device-resident FM / DDPM train step and FM-Euler sampler over the fused HIP engine.

One train step is the body of ``src/pipelines/train/flow_matching_lib.py:150-182``
(FM) or ``src/pipelines/train/diffusion_lib.py:153-185`` (DDPM) for one batch:

    noise ~ N(0,1), t ~ U[0,1) (FM) | timesteps ~ randint (DDPM)
    model input = cat([x_t, ldct]),  pred = UNet(input, timesteps)
    loss = mse(pred, noise - x0) (FM) | mse(pred, noise) (DDPM), backward
    [data-parallel: gradient all-reduce (mean) over RCCL]   <- added: the reference has none
    AdamW + cosine-with-warmup LR

Every stage is a HIP kernel on the current stream, nothing synchronises with
the host, so the whole step can be captured once into a hipGraph
(``torch.cuda.graph``) and replayed.  The LR schedule and Adam step count live
in device memory for that reason.  Parameters, gradients and Adam moments are
single flat fp32 buffers (the model's Parameters become views into them), so
the optimizer is one launch and the gradient all-reduce is over contiguous
buckets.
"""
from __future__ import annotations

import functools
import math
import time
from typing import Optional

import torch

from ...runtime import ops
from ...runtime.dp import bucketed_allreduce, bucketed_allreduce_async, world_size
from ...runtime.engine import get_engine
from ..schedulers import SCHED_NCOEF



def _own_stream(fn):
    """Run a public entry point on the object's private HIP stream when the caller is on the device's default
    (legacy null) stream, handing off with stream waits at entry and exit.

    Measured on MI355X / ROCm 7.x (tests/test_gpu_dp.py, tools/dp_debug.py): with the process on the legacy
    null stream, the 2-rank step's gradient buckets came back corrupted after the second replay (norms of 1e16 /
    inf) -- with the graphs replayed on the null stream, with a host synchronisation between the replay and the
    all-reduce, and also with this hand-off to a private stream; with the whole process on a created stream
    (``torch.cuda.set_stream`` before any work, as bench.py and the trainer loop do) every run was bit-identical
    to the eager reference.  Round 5 ruled out the stream half of that chain: graph replays on the null stream
    handed to a created stream by an event (or ``wait_stream``) are ordered exactly (tests/test_gpu_null_stream.py,
    every copy bit-exact), so the fault lies on the collective side, which no pool box (one GPU) can exercise over
    RCCL.  Until it can be, a multi-rank step from the null stream is refused (RuntimeError) rather than run on
    possibly corrupt gradients; single-process callers keep the hand-off."""
    @functools.wraps(fn)
    def wrapped(self, *a, **kw):
        cur = torch.cuda.current_stream()
        if cur != torch.cuda.default_stream(cur.device):
            return fn(self, *a, **kw)
        if getattr(self, "world", 1) > 1:
            raise RuntimeError("FusedTrainStep with several ranks on the default (null) HIP stream: collectives next "
                               "to graph replays on that stream corrupted gradients on this stack; call "
                               "torch.cuda.set_stream(torch.cuda.Stream()) before building the model (as bench.py "
                               "and fmdiff.pipelines.train.loop do)")
        st = self.__dict__.get("_work_stream")
        if st is None or st.device != cur.device:
            st = self._work_stream = torch.cuda.Stream(device=cur.device)
        st.wait_stream(cur)
        with torch.cuda.stream(st):
            out = fn(self, *a, **kw)
        cur.wait_stream(st)
        if torch.is_tensor(out):
            out.record_stream(cur)   # produced on st, consumed on the caller's stream
        return out
    return wrapped


class FlatParams:
    """Re-point every parameter (and its .grad) into one flat fp32 buffer.  ``first``: parameters laid out
    at the front (``split_at`` elements), e.g. those whose gradients are final early in the backward."""

    def __init__(self, model: torch.nn.Module, first=None):
        params = [p for p in model.parameters()]
        if first:
            ids = {id(p) for p in first}
            params = list(first) + [p for p in params if id(p) not in ids]
        self.split_at = sum(p.numel() for p in first) if first else 0
        self.order = params
        dev = params[0].device
        total = sum(p.numel() for p in params)
        self.data = torch.empty(total, device=dev, dtype=torch.float32)
        self.grad = torch.zeros(total, device=dev, dtype=torch.float32)
        self.slices = []
        self.offsets = {}           # id(param) -> (offset, numel) in the flat buffers
        off = 0
        with torch.no_grad():
            for p in params:
                n = p.numel()
                self.data[off:off + n].copy_(p.detach().reshape(-1))
                p.data = self.data[off:off + n].view_as(p)
                p.grad = self.grad[off:off + n].view_as(p)
                self.slices.append((off, n))
                self.offsets[id(p)] = (off, n)
                off += n
        self.numel = total


def _segment_buckets(sizes, buckets: int):
    """Cut backward segments (element counts, in backward order) into contiguous all-reduce buckets: the
    first segment (head + decoder, final first) alone, the middle segments merged into ``buckets - 2`` runs of
    about equal size, and the last segment (time MLP + grouped emb projections, final only at the very end:
    the one exposed exchange) alone.  Returns [((first_seg, last_seg), (lo, hi) flat range)], backward order."""
    n = len(sizes)
    if n <= 2 or buckets <= 2:
        cuts = [(0, 0), (1, n - 1)] if n > 1 else [(0, 0)]
    else:
        mid = sizes[1:-1]
        k = max(1, min(buckets - 2, len(mid)))
        target = sum(mid) / k
        cuts, first, acc = [(0, 0)], 1, 0
        for j, m in enumerate(mid):
            acc += m
            seg = j + 1
            runs_left = k - (len(cuts) - 1) - 1
            if seg == n - 2 or (acc >= target and runs_left > 0 and (n - 2 - seg) >= runs_left):
                cuts.append((first, seg))
                first, acc = seg + 1, 0
        cuts.append((n - 1, n - 1))
    out, lo = [], 0
    for f, l in cuts:
        hi = lo + sum(sizes[f:l + 1])
        out.append(((f, l), (lo, hi)))
        lo = hi
    return out


class FusedTrainStep:
    def __init__(self, model, *, objective: str = "flow_matching", lr: float = 1e-4, weight_decay: float = 0.0,
                 warmup: int = 500, total_steps: int = 10 ** 9, num_train_timesteps: int = 1000,
                 grad_accum: int = 1, betas=(0.9, 0.999), eps: float = 1e-8, ddpm_scheduler=None,
                 process_group=None, allreduce_buckets: int = 4, overlap_allreduce: Optional[bool] = None):
        self.model = model
        self.eng = get_engine(model)
        world = world_size(process_group)
        # data parallel: the decoder's gradients (final after backward part 1) go first in the flat buffer
        # and are all-reduced while the encoder's backward runs.  With gradient accumulation the exchange overlaps
        # the LAST chunk's backward (the earlier chunks' backward passes run whole, as the reference accumulates
        # .grad over chunks before its optimizer step, flow_matching_lib.py:143-146, 176-182)
        self.overlap = world > 1 if overlap_allreduce is None else bool(overlap_allreduce)
        # overlapped exchange: the flat buffer is laid out in backward-segment order and cut into
        # ``allreduce_buckets`` contiguous buckets of whole segments; bucket b is all-reduced (async) while
        # the segments of the later buckets run, only the last bucket's exchange is exposed
        self.seg_buckets = None
        first = None
        if self.overlap:
            groups = self.eng.backward_param_groups()
            first = [p for g in groups for p in g]
            self.seg_buckets = _segment_buckets([sum(p.numel() for p in g) for g in groups], allreduce_buckets)
        self.flat = FlatParams(model, first)
        dev = self.flat.data.device
        self.m = torch.zeros_like(self.flat.data)
        self.v = torch.zeros_like(self.flat.data)
        self.step_ctr = torch.zeros(1, dtype=torch.int32, device=dev)
        self.loss = torch.zeros(1, dtype=torch.float32, device=dev)
        # sum over chunks of loss * chunk size (flow_matching_lib.py:174), kept on the device so the step never
        # synchronises with the host; read once per epoch (epoch_loss_sum)
        self.loss_sum = torch.zeros(1, dtype=torch.float64, device=dev)
        self.partial = torch.empty(4096, dtype=torch.float32, device=dev)
        self.objective = objective
        self.hp = dict(lr=lr, wd=weight_decay, warmup=warmup, total=total_steps, betas=betas, eps=eps)
        self.N_train = num_train_timesteps
        self.grad_accum = max(1, int(grad_accum))
        self.pg = process_group
        self.world = world_size(process_group)
        self.buckets = allreduce_buckets
        if objective == "ddpm":
            if ddpm_scheduler is None:
                raise ValueError("ddpm objective needs its DDPMScheduler (alphas_cumprod)")
            self.acp = ddpm_scheduler.alphas_cumprod.to(dev, torch.float32)
        self._graph = None
        self._static = None
        self._split = False

    # ---------------------------------------------------------------- body
    def _chunk(self, clean, ldct, noise, t_or_ts, cca=None, last=True):
        N, Cx = clean.shape[:2]
        Cc = ldct.shape[1] if ldct is not None else 0
        Cp = max(8, -(-(Cx + Cc) // 8) * 8)
        if self.objective == "flow_matching":
            inp = ops.noise_prepare(clean, noise, t_or_ts, None, ldct, Cp)        # (1-t) x0 + t eps
            out, ctx = self.eng.forward(inp, t_or_ts, save=True, t_scale=float(self.N_train - 1), t_trunc=True,
                                        context_ca=cca)
            ta, tb, sign = noise, clean, -1.0                                      # target eps - x0
        else:
            sel = self.acp[t_or_ts]
            ca, cb = sel.sqrt(), (1 - sel).sqrt()
            inp = ops.noise_prepare(clean, noise, ca, cb, ldct, Cp)               # add_noise
            out, ctx = self.eng.forward(inp, t_or_ts, save=True, context_ca=cca)
            ta, tb, sign = noise, None, 0.0                                        # target eps
        dpred = torch.empty(out.shape, device=out.device, dtype=torch.bfloat16)
        ops.mse(out, ta, tb, sign, 1.0 / self.grad_accum, self.loss, self.partial, dpred)
        self.loss_sum.add_(self.loss, alpha=float(N))
        if self.overlap and last:
            # bucket 0's segments now; the rest in _bwd_bucket, each after the previous bucket's all-reduce started
            self.eng.backward(ctx, dpred, segs=self.seg_buckets[0][0])
            self._ctx = ctx
        else:
            self.eng.backward(ctx, dpred)
        return self.loss

    def _bwd_bucket(self, b):
        self.eng.backward(self._ctx, None, segs=self.seg_buckets[b][0])
        if b == len(self.seg_buckets) - 1:
            self._ctx = None

    def _bwd_rest(self):
        for b in range(1, len(self.seg_buckets)):
            self._bwd_bucket(b)

    def _allreduce(self):
        bucketed_allreduce(self.flat.grad, self.buckets, self.pg)

    @_own_stream
    def step(self, clean, ldct, noise=None, t=None, context_ca=None):
        """One optimizer step on (clean, ldct) [N,C,H,W] fp32 device tensors; returns the last chunk's loss.
        ``context_ca``: cross-attention conditioning (conditioning "attention", e.g. VAE latents)."""
        loss = self._fwd_bwd(clean, ldct, noise, t, context_ca)
        if self.overlap:
            self._overlapped_tail(self._bwd_bucket)
        else:
            self._allreduce()
        self._adamw()
        return loss

    def _overlapped_tail(self, run_bucket):
        """Bucket b's gradients (final after its backward segments) all-reduced asynchronously while
        ``run_bucket(b + 1)`` runs the next bucket's segments; the last bucket's exchange is the only exposed
        one.  ``run_bucket``: eager segments (_bwd_bucket) or their captured graphs."""
        works = []
        nb = len(self.seg_buckets)
        for b in range(nb):
            lo, hi = self.seg_buckets[b][1]
            if b == nb - 1:
                bucketed_allreduce(self.flat.grad[lo:hi], 1, self.pg)
            else:
                works += bucketed_allreduce_async(self.flat.grad[lo:hi], 1, self.pg)
                run_bucket(b + 1)
        for w in works:
            w.wait()

    def exposed_allreduce_elems(self) -> int:
        """fp32 gradient elements whose all-reduce is not overlapped with backward compute."""
        if not self.overlap:
            return self.flat.numel
        lo, hi = self.seg_buckets[-1][1]
        return hi - lo

    def _adamw(self):
        b1, b2 = self.hp["betas"]
        ops.adamw_sched(self.flat.data, self.flat.grad, self.m, self.v, self.step_ctr, self.hp["lr"], self.hp["warmup"],
                        self.hp["total"], b1, b2, self.hp["eps"], self.hp["wd"], 1.0 / self.world)
        ops.counter_add(self.step_ctr)

    def _fwd_bwd(self, clean, ldct, noise=None, t=None, context_ca=None):
        """Weight refresh, gradient zeroing and forward + backward of every grad-accumulation chunk."""
        self.eng.invalidate_weights()            # bf16 kernel weights re-derived from the updated masters
        self.flat.grad.zero_()
        N = clean.shape[0]
        chunk = -(-N // self.grad_accum)
        loss = None
        for c0 in range(0, N, chunk):
            cl = clean[c0:c0 + chunk]
            ld = ldct[c0:c0 + chunk] if ldct is not None else None
            nz = noise[c0:c0 + chunk] if noise is not None else torch.randn_like(cl)
            if self.objective == "flow_matching":
                tt = t[c0:c0 + chunk] if t is not None else torch.rand(cl.shape[0], device=cl.device)
            else:
                tt = t[c0:c0 + chunk] if t is not None else torch.randint(0, self.N_train, (cl.shape[0],),
                                                                           device=cl.device)
            cc = context_ca[c0:c0 + chunk].contiguous() if context_ca is not None else None
            loss = self._chunk(cl.contiguous(), ld.contiguous() if ld is not None else None, nz.contiguous(), tt, cc,
                               last=c0 + chunk >= N)
        return loss

    # ------------------------------------------------- bookkeeping / state
    def epoch_loss_sum(self, reset: bool = True) -> torch.Tensor:
        """Device fp64 sum of (chunk loss x chunk size) since the last reset (the reference's ``epoch_loss``)."""
        out = self.loss_sum.clone()
        if reset:
            self.loss_sum.zero_()
        return out

    def lr_multiplier(self, s: int) -> float:
        """get_cosine_schedule_with_warmup's multiplier after ``s`` scheduler steps (same formula as
        fmd_adamw_sched)."""
        w, total = self.hp["warmup"], self.hp["total"]
        if s < w:
            return float(s) / float(max(1, w))
        prog = float(s - w) / float(max(1, total - w))
        return max(0.0, 0.5 * (1.0 + math.cos(math.pi * 2.0 * 0.5 * prog)))

    def steps_done(self) -> int:
        return int(self.step_ctr.item())

    def optimizer_state_dict(self) -> dict:
        """The step's AdamW state in ``torch.optim.AdamW.state_dict()`` form (state keyed by the index in
        ``model.parameters()``), so a checkpoint written here resumes the reference's optimizer and back."""
        s = self.steps_done()
        b1, b2 = self.hp["betas"]
        state = {}
        params = list(self.model.parameters())
        if s > 0:
            for i, p in enumerate(params):
                off, n = self.flat.offsets[id(p)]
                state[i] = {"step": torch.tensor(float(s)), "exp_avg": self.m[off:off + n].view_as(p).detach().cpu().clone(),
                            "exp_avg_sq": self.v[off:off + n].view_as(p).detach().cpu().clone()}
        group = {"lr": self.hp["lr"] * self.lr_multiplier(s), "betas": (b1, b2), "eps": self.hp["eps"],
                 "weight_decay": self.hp["wd"], "amsgrad": False, "maximize": False, "foreach": None,
                 "capturable": False, "differentiable": False, "fused": None, "decoupled_weight_decay": True,
                 "initial_lr": self.hp["lr"], "params": list(range(len(params)))}
        return {"state": state, "param_groups": [group]}

    def lr_scheduler_state_dict(self) -> dict:
        """``LambdaLR`` state of get_cosine_schedule_with_warmup after the steps taken."""
        s = self.steps_done()
        return {"base_lrs": [self.hp["lr"]], "last_epoch": s, "_step_count": s + 1, "_is_initial": False,
                "_get_lr_called_within_step": False, "_last_lr": [self.hp["lr"] * self.lr_multiplier(s)],
                "lr_lambdas": [{}]}

    def load_optimizer_state_dict(self, opt_state: dict, sched_state: Optional[dict] = None) -> None:
        """Inverse of optimizer_state_dict (also accepts a torch AdamW checkpoint of the reference).  The step
        count comes from the optimizer state (else the LR scheduler's ``last_epoch``)."""
        params = list(self.model.parameters())
        st = opt_state.get("state", {}) if opt_state else {}
        steps = 0
        with torch.no_grad():
            for i, p in enumerate(params):
                e = st.get(i) if i in st else st.get(str(i))
                if not e:
                    continue
                off, n = self.flat.offsets[id(p)]
                self.m[off:off + n].copy_(torch.as_tensor(e["exp_avg"]).reshape(-1))
                self.v[off:off + n].copy_(torch.as_tensor(e["exp_avg_sq"]).reshape(-1))
                steps = max(steps, int(float(torch.as_tensor(e["step"]))))
        if steps == 0 and sched_state:
            steps = int(sched_state.get("last_epoch", 0))
        self.step_ctr.fill_(steps)

    # ---------------------------------------------------------- hipGraph
    @_own_stream
    def capture(self, clean, ldct, warmup_iters: int = 2, split_collectives: Optional[bool] = None,
                context_ca=None, noise=None, t=None):
        """Capture one step into a hipGraph.  Single process: the whole step (RNG, forward, loss, backward,
        AdamW).  With several ranks (``split_collectives``, default: world > 1) the graph holds RNG +
        forward + backward, and each replay is followed by the bucketed RCCL all-reduce and the AdamW
        launch issued eagerly: no collective is ever recorded into a graph.

        ``noise`` / ``t`` (optional): inject the step's random draws (static buffers, refreshed by
        ``replay(noise=..., t=...)``) instead of drawing them inside the graph.

        The ``warmup_iters`` eager steps that precede the capture (allocator and kernel warm-up) leave no
        trace: parameters, Adam moments and the step counter are restored afterwards, so the first replay
        is optimizer step 1 with the schedule's first LR, as in the reference loop
        (flow_matching_lib.py:148-182)."""
        self._split = self.world > 1 if split_collectives is None else bool(split_collectives)
        self._static = (clean.clone(), ldct.clone() if ldct is not None else None,
                        noise.clone() if noise is not None else None, t.clone() if t is not None else None,
                        context_ca.clone() if context_ca is not None else None)
        snap = (self.flat.data.clone(), self.m.clone(), self.v.clone(), self.step_ctr.clone(), self.loss_sum.clone())
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup_iters):
                self.step(*self._static)
        torch.cuda.current_stream().wait_stream(s)
        for dst, src in zip((self.flat.data, self.m, self.v, self.step_ctr, self.loss_sum), snap):
            dst.copy_(src)
        self.flat.grad.zero_()
        del snap
        # the weight layouts are created lazily by the first forward, after that step's refresh: refresh once
        # more here so the batched job tables exist before capture (a table built while capturing would be a
        # host-to-device copy inside the graph) -- with warmup_iters=1 no eager refresh has seen them yet
        self.eng.invalidate_weights()
        g = torch.cuda.CUDAGraph()
        # multi-rank: thread-local capture, so the process group's watchdog thread may keep querying its
        # (already completed) events while this thread records
        mode = "thread_local" if self._split else "global"
        with torch.cuda.graph(g, stream=ops.capture_stream(), capture_error_mode=mode):
            if self._split:
                self._graph_loss = self._fwd_bwd(*self._static)
            else:
                self._graph_loss = self.step(*self._static)
        self._graph = g
        self._graphs = []
        if self._split and self.overlap:   # each later bucket's backward segments as a graph in the same pool
            for b in range(1, len(self.seg_buckets)):
                gb = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gb, pool=g.pool(), stream=ops.capture_stream(), capture_error_mode=mode):
                    self._bwd_bucket(b)
                self._graphs.append(gb)

    @_own_stream
    def replay(self, clean=None, ldct=None, context_ca=None, noise=None, t=None):
        for i, new in ((0, clean), (1, ldct), (2, noise), (3, t), (4, context_ca)):
            if new is None:
                continue
            if self._static[i] is None:
                raise ValueError("replay: this input was not a static buffer at capture time")
            self._static[i].copy_(new)
        self._graph.replay()
        if self._split:
            if self._graphs:
                self._overlapped_tail(lambda b: self._graphs[b - 1].replay())
            else:
                self._allreduce()
            self._adamw()
        return self._graph_loss


class FusedSampler:
    """The sampling loop of ``src/pipelines/utils.py:163-220`` (``cat([x, cond])`` -> UNet ->
    ``scheduler.step``) with one replayable step for every scheduler that has a HIP step:

    * FlowMatchEuler: ``fmd_flow_euler`` (sigmas on the device);
    * DDPM / DDIM (eta 0): ``fmd_ddpm_step`` with a per-step coefficient table (``scheduler.coefficients``)
      and, for DDPM, the variance noise: an injected [S][N,C,*S] table (the S steps that run), or one
      [N,C,*S] buffer refilled from ``generator`` before every step (outside the graph, so any generator works
      and memory does not grow with the schedule length: 1000 steps of a 512^2 batch would be 8 GB);
    * DPM-Solver(++) / UniPC: ``fmd_sched_step`` over ``scheduler.plan()`` (the host bookkeeping of the
      eager ``step``: order warm-up, lower-order final steps, corrector) and a 4-slot data-prediction ring.

    Every table is indexed by a device step counter, so the step (time embedding row, UNet forward, scheduler
    update, next packed model input) is captured once and replayed S times; a later call with the same shapes
    only re-arms the static buffers.  ``start``: first step index of the schedule (the reference's tail
    selection, ``select_timesteps``); the eager scheduler would begin there from a fresh state, and so does
    the table."""

    def __init__(self, model, scheduler, num_inference_steps: int, start: int = 0):
        from ..schedulers import (DDIMScheduler, DDPMScheduler, DPMSolverMultistepScheduler,
                                  FlowMatchEulerDiscreteScheduler, UniPCMultistepScheduler)
        self.eng = get_engine(model)
        self.sched = scheduler
        self.sched.set_timesteps(num_inference_steps)
        if isinstance(scheduler, FlowMatchEulerDiscreteScheduler):
            self.kind = "fm"
        elif isinstance(scheduler, DDIMScheduler):
            self.kind = "ddim"
        elif isinstance(scheduler, DDPMScheduler):
            self.kind = "ddpm"
        elif isinstance(scheduler, (DPMSolverMultistepScheduler, UniPCMultistepScheduler)):
            self.kind = "ms"
        else:
            raise NotImplementedError(f"no fused step for {type(scheduler).__name__}")
        self.S0 = int(start)
        self.S = len(self.sched.timesteps) - self.S0
        if self.S < 1:
            raise ValueError("No timesteps selected after applying start_step/last_n_steps.")
        self._graph = None
        self._gkey = None
        self.cca = None

    def _key(self, init, cond, context_ca):
        return (tuple(init.shape), init.device, None if cond is None else tuple(cond.shape),
                None if context_ca is None else tuple(context_ca.shape))

    def _tables(self, dev):
        sch = self.sched
        self.ts = sch.timesteps.to(dev).float().contiguous()         # model timestep of every step
        self.sig = self.coef = None
        if self.kind == "fm":
            self.sig = sch.sigmas.to(dev)
        elif self.kind in ("ddpm", "ddim"):
            self.coef = torch.stack([sch.coefficients(int(t)) for t in sch.timesteps]).to(dev).contiguous()
        else:
            self.coef = torch.zeros(len(sch.timesteps), SCHED_NCOEF, dtype=torch.float32)
            self.coef[self.S0:] = sch.plan(self.S0)
            self.coef = self.coef.to(dev)

    def _prepare(self, init, cond):
        dev = init.device
        self._tables(dev)
        self.idx = torch.full((1,), self.S0, dtype=torch.int32, device=dev)
        self.x = init.float().clone()
        self.cond = cond.float().contiguous() if cond is not None else None
        Cx = init.shape[1]
        Cc = cond.shape[1] if cond is not None else 0
        self.inp = ops.noise_prepare(None, self.x, None, None, self.cond, max(8, -(-(Cx + Cc) // 8) * 8))
        self.tbuf = torch.empty(init.shape[0], device=dev, dtype=torch.float32)
        self.noise = None
        self.noise_base = -1
        if self.kind == "ddpm":   # one step's variance noise (NCHW); _arm_noise swaps in an injected table
            self.noise = torch.empty(init.shape, device=dev, dtype=torch.float32)
        self.ring = self.last = None
        if self.kind == "ms":
            self.ring = [torch.zeros_like(self.x) for _ in range(4)]
            self.last = torch.zeros_like(self.x)
        # the schedule is fixed: every step's time embedding is computed once, the step copies its row
        self.eng.set_time_table(self.ts, init.shape[0], self.idx)
        self._tt = self.eng._tt   # the captured step reads these tables: keep them alive with the graph

    def _arm_noise(self, noise, captured: bool):
        """DDPM variance noise for this call: an injected [S, *shape] table (row 0 = step S0) or the per-step
        buffer.  A captured graph keeps the buffer it was recorded with, so a cached graph re-armed with the
        other mode is dropped (returns False)."""
        if self.kind != "ddpm":
            return True
        want_table = noise is not None
        if captured and want_table != (self.noise_base >= 0):
            return False
        if want_table:
            rows = noise.reshape(self.S, *self.x.shape).float()
            if self.noise_base >= 0 and self.noise.shape == rows.shape:
                self.noise.copy_(rows)
            else:
                self.noise = rows.contiguous().clone()
            self.noise_base = self.S0
        elif self.noise_base >= 0 or self.noise is None:
            self.noise = torch.empty(self.x.shape, device=self.x.device, dtype=torch.float32)
            self.noise_base = -1
        return True

    def _pre(self, generator):
        """Before each step: a fresh variance-noise draw into the per-step buffer (DDPM without injection)."""
        if self.kind == "ddpm" and self.noise_base < 0:
            self.noise.normal_(generator=generator)

    def _refresh(self, init, cond, context_ca):
        """Re-arm the cached graph's static buffers for a new call (same shapes): sample, conditioning, the
        packed model input, the step counter, the solver history, and the time-embedding tables (the time
        MLP's weights may have changed since the capture)."""
        self.eng.invalidate_weights()   # bf16 kernel weights re-derived in place from the fp32 masters
        self.x.copy_(init)
        if self.cond is not None:
            self.cond.copy_(cond)
        if self.cca is not None:
            self.cca.copy_(context_ca)
        self.idx.fill_(self.S0)
        if self.ring is not None:
            for r in self.ring:
                r.zero_()
            self.last.zero_()
        Cx = init.shape[1]
        Cc = cond.shape[1] if cond is not None else 0
        ops.noise_prepare(None, self.x, None, None, self.cond, max(8, -(-(Cx + Cc) // 8) * 8), out=self.inp)
        self.eng.set_time_table(self.ts, init.shape[0], self.idx)
        new = self.eng._tt
        self._tt["emb"].copy_(new["emb"])
        if self._tt["eo"] is not None:
            self._tt["eo"].copy_(new["eo"])
        self.eng._tt = self._tt

    def _one(self):
        if self.eng._tt is None:   # no precomputed embedding table: the MLP runs on t = ts[idx]
            ops.fill_from_table(self.ts, self.idx, self.tbuf)
        out, _ = self.eng.forward(self.inp, self.tbuf, save=False, context_ca=self.cca)
        if self.kind == "fm":
            ops.flow_euler(self.x, out, self.sig, self.idx, self.cond, self.inp)
        elif self.kind in ("ddpm", "ddim"):
            ops.ddpm_step(self.x, out, self.coef, self.idx, self.noise, self.cond, self.inp, self.noise_base)
        else:
            ops.sched_step(self.x, out, self.ring, self.last if self._unipc() else None, self.coef, self.idx,
                           self.cond, self.inp)
        ops.counter_add(self.idx)

    def _unipc(self):
        from ..schedulers import UniPCMultistepScheduler
        return isinstance(self.sched, UniPCMultistepScheduler)

    @_own_stream
    @torch.no_grad()
    def sample(self, init: torch.Tensor, cond: Optional[torch.Tensor] = None, use_graph: bool = True,
               context_ca: Optional[torch.Tensor] = None, noise: Optional[torch.Tensor] = None, generator=None,
               timing: Optional[dict] = None):
        """``cond``: concatenated conditioning; ``context_ca``: cross-attention conditioning; ``noise``: DDPM
        variance noise of the S steps ([S, *init.shape]; drawn with ``generator`` when None).  ``timing``: the
        reference's ``model_seconds`` / ``model_calls`` accumulators (pipelines/utils.py:196-200), here the
        S steps of the loop (UNet + scheduler update, which the reference times apart) between two device
        synchronisations; a first call's graph capture is excluded.

        With ``use_graph`` the step is captured once per input shape and the graph is kept: a later call
        with the same shapes only re-arms the static buffers (``_refresh``) and replays it S times.  The
        returned tensor is a copy of the sample buffer."""
        key = self._key(init, cond, context_ca)
        t0 = None
        if use_graph and self._graph is not None and self._gkey == key and self._arm_noise(noise, True):
            self._refresh(init, cond, context_ca)
            if timing is not None:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            for _ in range(self.S):
                self._pre(generator)
                self._graph.replay()
            return self._finish(timing, t0)
        self._graph = None
        self._prepare(init, cond)
        self._arm_noise(noise, False)
        self.cca = context_ca.float().contiguous() if context_ca is not None else None
        if timing is not None:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        if not use_graph:
            for _ in range(self.S):
                self._pre(generator)
                self._one()
            return self._finish(timing, t0)
        self.eng.invalidate_weights()
        self._pre(generator)
        self._one()   # the first step eagerly: re-derives the bf16 weights and warms the allocator
        g = torch.cuda.CUDAGraph()
        mode = "thread_local" if torch.distributed.is_available() and torch.distributed.is_initialized() else "global"
        if timing is not None:   # the capture is set-up, not model time: keep it out of model_seconds
            torch.cuda.synchronize()
            tc = time.perf_counter()
        with torch.cuda.graph(g, stream=ops.capture_stream(), capture_error_mode=mode):   # records, does not execute
            self._one()
        if timing is not None:
            torch.cuda.synchronize()
            t0 += time.perf_counter() - tc
        for _ in range(self.S - 1):
            self._pre(generator)
            g.replay()
        self._graph, self._gkey = g, key
        return self._finish(timing, t0)

    def _finish(self, timing, t0):
        self.eng.set_time_table(None)
        if timing is not None:
            torch.cuda.synchronize()
            timing["model_seconds"] = timing.get("model_seconds", 0.0) + (time.perf_counter() - t0)
            timing["model_calls"] = timing.get("model_calls", 0) + self.S
        return self.x.clone()


class FusedFlowSampler(FusedSampler):
    """FlowMatchEuler sampling loop (``src/pipelines/utils.py:163-220``) with one replayable step."""

    def __init__(self, model, num_inference_steps: int = 50, num_train_timesteps: int = 1000):
        from ..schedulers import FlowMatchEulerDiscreteScheduler
        super().__init__(model, FlowMatchEulerDiscreteScheduler(num_train_timesteps), num_inference_steps)
