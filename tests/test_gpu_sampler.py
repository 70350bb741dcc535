"""Graph-replayed sampling for every scheduler with a HIP step (fmdiff.pipelines.train.fused.FusedSampler) vs the
generic eager loop ``sample_with_scheduler`` (src/pipelines/utils.py:163-220) with the same scheduler class.

Both run the same UNet kernels and the same step arithmetic: the eager loop calls ``scheduler.step`` per step
(fmd_flow_euler / fmd_ddpm_step / fmd_lincomb with host-folded coefficients), the fused sampler replays one
captured step whose scheduler update reads a per-step coefficient table (``coefficients`` / ``plan()``) by a
device counter.  DDPM's variance noise is injected into both.  The two paths differ only in how the time
embedding is produced (one precomputed table vs the MLP per step), so the bound is 2e-3 relative L2 (the
tiny UNet's bf16 forward turns an ulp-level embedding difference into ~1e-4); captured vs eager fused runs
must agree bit for bit.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
BETAS = dict(beta_start=0.00085, beta_end=0.012)   # configs/diffusion/ldct_ddpm.json


def _model(golden):
    from fmdiff.models.generators import DiffusionUNetFactory
    from oracle import spec as S
    from oracle import unet as U
    T, M = golden
    meta = M["ldct_fm_test"]
    tr = meta["training"]
    model = DiffusionUNetFactory().build(meta["unet"], tr["conditioning"], tr["channels"] or 1).to(DEV)
    model.load_state_dict(U.seeded_state_dict(S.derive_spec(meta["unet"], tr["conditioning"], tr["channels"] or 1),
                                              meta["seed"]))
    return model, T["ldct_fm_test/cond"].to(DEV)


def _sched(kind):
    from fmdiff.pipelines import schedulers as SC
    return {
        "flow_match_euler": lambda: SC.FlowMatchEulerDiscreteScheduler(1000),
        "ddpm": lambda: SC.DDPMScheduler(1000, **BETAS),
        "ddim": lambda: SC.DDIMScheduler(1000, **BETAS),
        "dpm++2": lambda: SC.DPMSolverMultistepScheduler(1000, **BETAS),
        "dpm++3": lambda: SC.DPMSolverMultistepScheduler(1000, solver_order=3, **BETAS),
        "dpmsolver2": lambda: SC.DPMSolverMultistepScheduler(1000, algorithm_type="dpmsolver",
                                                             final_sigmas_type="sigma_min", **BETAS),
        "unipc2": lambda: SC.UniPCMultistepScheduler(1000, **BETAS),
        "unipc3_bh1": lambda: SC.UniPCMultistepScheduler(1000, solver_order=3, solver_type="bh1", **BETAS),
    }[kind]()


class _Injected:
    """Feeds the eager DDPM step pre-drawn variance noise (row = step index of the schedule)."""

    def __init__(self, inner, noise, start):
        self.inner, self.noise, self.i = inner, noise, start
        self.config = inner.config

    def set_timesteps(self, n, device=None):
        self.inner.set_timesteps(n, device)

    @property
    def timesteps(self):
        return self.inner.timesteps

    def step(self, pred, t, x, **kw):
        out = self.inner.step(pred, t, x, variance_noise=self.noise[self.i])
        self.i += 1
        return out


@pytest.mark.parametrize("kind,steps,start_step", [
    ("flow_match_euler", 8, None), ("ddpm", 8, None), ("ddim", 8, None), ("ddim", 10, 500),
    ("dpm++2", 10, None), ("dpm++3", 12, None), ("dpmsolver2", 8, None), ("unipc2", 10, None),
    ("unipc3_bh1", 12, None), ("unipc2", 10, 600)])
def test_fused_sampler_matches_generic_loop(golden, kind, steps, start_step):
    from fmdiff.pipelines.train.fused import FusedSampler
    from fmdiff.pipelines.utils import sample_with_scheduler, select_timesteps
    model, cond = _model(golden)
    g = torch.Generator().manual_seed(31)
    init = torch.randn(cond.shape, generator=g).to(DEV)
    noise = torch.randn((steps, *cond.shape), generator=g).to(DEV)
    sch = _sched(kind)
    sch.set_timesteps(steps)
    sel = select_timesteps(sch.timesteps, start_step)
    start = len(sch.timesteps) - len(sel)
    eager_sched = _Injected(_sched(kind), noise, start) if kind == "ddpm" else _sched(kind)
    timing = {}
    with torch.no_grad():
        ref = sample_with_scheduler(model, eager_sched, steps, tuple(init.shape), torch.device(DEV),
                                    conditioning_mode="concatenate", conditioning_batch=cond, init_sample=init,
                                    start_step=start_step)
    outs = []
    for use_graph in (True, False):
        fs = FusedSampler(model, _sched(kind), steps, start=start)
        outs.append(fs.sample(init, cond, use_graph=use_graph, noise=noise[start:] if kind == "ddpm" else None,
                              timing=timing))
    err = ((outs[0] - ref).norm() / ref.norm()).item()
    print(f"{kind} steps {steps} start {start}: fused vs generic rel L2 {err:.3e}; model calls {timing['model_calls']}")
    assert torch.equal(outs[0], outs[1]), "captured and eager fused steps differ"
    assert timing["model_calls"] == 2 * len(sel)
    assert err < 2e-3


def test_fused_ddpm_sampler_graph_reuse_draws_fresh_noise(golden):
    """A cached DDPM graph re-armed for a second call draws new variance noise (generator) and, given the
    same generator state, reproduces a fresh sampler's output bit for bit."""
    from fmdiff.pipelines.train.fused import FusedSampler
    model, cond = _model(golden)
    init = torch.randn(cond.shape, generator=torch.Generator().manual_seed(3)).to(DEV)
    fs = FusedSampler(model, _sched("ddpm"), 6)
    a = fs.sample(init, cond, generator=torch.Generator(DEV).manual_seed(1))
    graph = fs._graph
    b = fs.sample(init, cond, generator=torch.Generator(DEV).manual_seed(2))
    assert fs._graph is graph and not torch.equal(a, b)
    c = FusedSampler(model, _sched("ddpm"), 6).sample(init, cond, generator=torch.Generator(DEV).manual_seed(2))
    assert torch.equal(b, c)


def test_time_table_rows_equal_per_sample_mlp(golden):
    """The sampler's precomputed time-embedding table (engine.set_time_table) evaluates the time MLP and the
    grouped ResBlock projections once per step and repeats each row for the N samples of the batch; every
    (step, sample) row must equal the MLP evaluated on that sample's own t, bit for bit (the kernels are
    row-independent)."""
    from fmdiff.pipelines.train.fused import FusedFlowSampler
    model, _ = _model(golden)
    sampler = FusedFlowSampler(model, 7)
    eng = sampler.eng
    N = 3
    ts = torch.linspace(999.0, 11.0, 7, device=DEV)
    idx = torch.zeros(1, device=DEV, dtype=torch.int32)
    eng.set_time_table(ts, N, idx)
    tt = eng._tt
    eng.set_time_table(None)
    with torch.no_grad():
        ctx = eng.time_mlp(ts.repeat_interleave(N).contiguous(), False, 7 * N)
    assert torch.equal(tt["emb"].view(7 * N, -1), ctx.emb)
    if tt["eo"] is not None:
        assert torch.equal(tt["eo"].view(7 * N, -1), ctx.eo_all)
