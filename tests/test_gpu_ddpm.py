"""Config C's DDPM path on the GPU (diffusion_lib.py:153-185, pipelines/utils.py:163-220) vs the oracle.

* ``DDPMScheduler.add_noise`` (fmd_add_noise): bit-exact with the oracle's eager fp32 expression;
* ``DDPMScheduler.step`` / ``DDIMScheduler.step`` (fmd_ddpm_step) over the 50-step leading schedule of
  ``configs/diffusion/ldct_ddpm.json`` (betas 0.00085 -> 0.012) with injected ``variance_noise``:
  timesteps bit-exact, fp32 step outputs within 1e-6 (FMA contraction / operation-order ulps);
* ``FusedTrainStep(objective="ddpm")``: loss and gradients vs the oracle's ``ddpm_loss`` (UNet tolerances
  of tests/test_gpu_unet.py);
* the generic ``sample_with_scheduler`` on the GPU with FlowMatchEuler, DDIM and DDPM (noise injected)
  vs the oracle's sampling loop (fp32 UNet): relative L2 < 2e-2.

Scheduler parity is pinned by the oracle's closed-form KATs only (diffusers is absent: SURVEY.md 8(c)).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
BETAS = dict(beta_start=0.00085, beta_end=0.012)   # configs/diffusion/ldct_ddpm.json model.scheduler.params


def _rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _tiny(golden, name="ldct_fm_test"):
    from fmdiff.models.generators import DiffusionUNetFactory
    from oracle import spec as S
    from oracle import unet as U
    T, M = golden
    meta = M[name]
    tr = meta["training"]
    model = DiffusionUNetFactory().build(meta["unet"], tr["conditioning"], tr["channels"] or 1).to(DEV)
    spec = S.derive_spec(meta["unet"], tr["conditioning"], tr["channels"] or 1)
    sd = U.seeded_state_dict(spec, meta["seed"])
    model.load_state_dict(sd)
    return model, spec, sd, T, meta


def test_add_noise_bit_exact():
    from fmdiff.pipelines.schedulers import DDPMScheduler
    from oracle import schedulers as OS
    g = torch.Generator().manual_seed(5)
    x0 = torch.rand(4, 1, 64, 64, generator=g)
    eps = torch.randn(4, 1, 64, 64, generator=g)
    ts = torch.tensor([0, 17, 500, 999])
    ref = OS.DDPM(1000, **BETAS).add_noise(x0, eps, ts)
    got = DDPMScheduler(1000, **BETAS).add_noise(x0.to(DEV), eps.to(DEV), ts.to(DEV))
    assert got.dtype == torch.float32
    assert torch.equal(got.cpu(), ref)


@pytest.mark.parametrize("kind", ["ddpm", "ddim"])
def test_ddpm_ddim_step_kernels_vs_oracle(kind):
    """Every step of the 50-step leading schedule, each fed the same (x, eps, z) on both sides."""
    from fmdiff.pipelines.schedulers import DDIMScheduler, DDPMScheduler
    from oracle import schedulers as OS
    cls, ocls = (DDPMScheduler, OS.DDPM) if kind == "ddpm" else (DDIMScheduler, OS.DDIM)
    s, o = cls(1000, **BETAS), ocls(1000, **BETAS)
    s.set_timesteps(50)
    o.set_timesteps(50)
    assert s.timesteps.dtype == torch.int64 and torch.equal(s.timesteps, o.timesteps)
    assert s.timesteps.tolist() == list(range(980, -1, -20))
    g = torch.Generator().manual_seed(9)
    worst = 0.0
    for t in s.timesteps:
        x = torch.randn(2, 1, 32, 32, generator=g)
        eps = torch.randn(2, 1, 32, 32, generator=g)
        z = torch.randn(2, 1, 32, 32, generator=g)
        if kind == "ddpm":
            ref = o.step(eps, t, x, noise=z).prev_sample
            got = s.step(eps.to(DEV), t, x.to(DEV), variance_noise=z.to(DEV)).prev_sample
        else:
            ref = o.step(eps, t, x).prev_sample
            got = s.step(eps.to(DEV), t, x.to(DEV)).prev_sample
        err = (got.cpu() - ref).abs().max().item()
        worst = max(worst, err)
        assert err <= 1e-6, (int(t), err)
    print(f"{kind}: worst |step(gpu) - step(oracle)| over 50 steps {worst:.2e}")


def test_ddpm_fused_train_step_vs_oracle(golden):
    """FusedTrainStep(objective="ddpm") -- add_noise folded into the model-input kernel, target eps --
    vs the oracle's ddpm_loss gradients on the tiny LDCT config (injected eps and integer timesteps)."""
    from fmdiff.pipelines.schedulers import DDPMScheduler
    from fmdiff.pipelines.train.fused import FusedTrainStep
    from oracle import schedulers as OS
    from oracle import train_step as OT
    model, spec, sd, T, meta = _tiny(golden)
    x, cond = T["ldct_fm_test/x"], T["ldct_fm_test/cond"]
    clean = x.clamp(0, 1)
    g = torch.Generator().manual_seed(13)
    noise = torch.randn(clean.shape, generator=g)
    ts = torch.tensor([3, 777])
    sdg = {k: v.clone().requires_grad_() for k, v in sd.items()}
    loss_ref, scaled = OT.ddpm_loss(sdg, spec, OS.DDPM(1000, **BETAS), clean, cond, noise, ts)
    scaled.backward()
    tr = FusedTrainStep(model, objective="ddpm", ddpm_scheduler=DDPMScheduler(1000, **BETAS), lr=1e-4, warmup=10,
                        total_steps=100)
    loss = tr.step(clean.to(DEV), cond.to(DEV), noise=noise.to(DEV), t=ts.to(DEV))
    torch.cuda.synchronize()
    print(f"ddpm loss hip {loss.item():.6f} oracle {loss_ref.item():.6f}")
    assert abs(loss.item() - loss_ref.item()) / loss_ref.item() < 1e-2
    num = den = 0.0
    worst = (1.0, "")
    for k, p in model.named_parameters():
        gk, r = p.grad.double().cpu(), sdg[k].grad.double()
        num += (gk - r).pow(2).sum().item()
        den += r.pow(2).sum().item()
        if r.norm() > 1e-3 * math.sqrt(den + 1e-30):
            cos = ((gk * r).sum() / (gk.norm() * r.norm() + 1e-30)).item()
            worst = min(worst, (cos, k))
    rel = math.sqrt(num / den)
    print(f"ddpm grad rel L2 {rel:.3e}, worst cosine {worst}")
    assert rel < 5e-2 and worst[0] > 0.99


class _InjectedDDPM:
    """Wraps the GPU DDPMScheduler so the generic loop's ``step(pred, t, x)`` uses pre-drawn variance noise."""

    def __init__(self, inner, noises):
        self.inner, self.noises, self.i = inner, noises, 0
        self.config = inner.config

    def set_timesteps(self, n, device=None):
        self.inner.set_timesteps(n, device)

    @property
    def timesteps(self):
        return self.inner.timesteps

    def step(self, pred, t, x, **kw):
        out = self.inner.step(pred, t, x, variance_noise=self.noises[self.i].to(x.device))
        self.i += 1
        return out


@pytest.mark.parametrize("kind", ["flow_match_euler", "ddim", "ddpm"])
def test_sample_with_scheduler_vs_oracle(golden, kind):
    """The generic sampling loop (pipelines/utils.py:163-220: cat([x, cond]) -> UNet -> scheduler.step) on
    the GPU, 6 steps, vs the oracle's loop with the oracle's fp32 UNet and scheduler."""
    from fmdiff.pipelines.schedulers import DDIMScheduler, DDPMScheduler, FlowMatchEulerDiscreteScheduler
    from fmdiff.pipelines.utils import sample_with_scheduler
    from oracle import schedulers as OS
    from oracle import train_step as OT
    model, spec, sd, T, meta = _tiny(golden)
    cond = T["ldct_fm_test/cond"]
    g = torch.Generator().manual_seed(21)
    init = torch.randn(cond.shape, generator=g)
    steps = 6
    noises = [torch.randn(cond.shape, generator=g) for _ in range(steps)]
    if kind == "flow_match_euler":
        sch, osch = FlowMatchEulerDiscreteScheduler(1000), OS.FlowMatchEuler(1000)
    elif kind == "ddim":
        sch, osch = DDIMScheduler(1000, **BETAS), OS.DDIM(1000, **BETAS)
    else:
        sch, osch = _InjectedDDPM(DDPMScheduler(1000, **BETAS), noises), OS.DDPM(1000, **BETAS)
    # DDIM (eta 0) is deterministic from x_T: at t ~ 830 its x0 estimate divides the UNet's bf16 error by
    # sqrt(alpha_bar) ~ 0.09, so the run starts at t <= 500 (start_step; also exercises the tail selection)
    start = 500 if kind == "ddim" else None
    n_calls = 4 if kind == "ddim" else steps
    timing = {}
    with torch.no_grad():
        got = sample_with_scheduler(model, sch, steps, tuple(init.shape), torch.device(DEV),
                                    conditioning_mode="concatenate", conditioning_batch=cond.to(DEV),
                                    timing=timing, init_sample=init, start_step=start)
    ref = OT.sample(sd, spec, osch, steps, init, cond, noises=noises if kind == "ddpm" else None, start_step=start)
    err = _rel(got, ref)
    print(f"{kind}: sample_with_scheduler rel L2 {err:.3e}, model calls {timing.get('model_calls')}")
    assert timing["model_calls"] == n_calls
    assert err < 2e-2


@pytest.mark.parametrize("case", ["c256", "mnist"])
def test_ddpm_fused_train_step_vs_reference_golden(golden_ddpm, case):
    """FusedTrainStep(objective="ddpm"), graph-captured, on the configurations that train with DDPM, vs the
    reference's own step (tests/golden/make_golden_ddpm.py; diffusion_lib.py:153-185):

    * ``c256``: config C's 113 M EfficientUNetND (configs/diffusion/ldct_ddpm.json) at 256x256, batch 2;
    * ``mnist``: config A's UNetDiffusersND (configs/MNIST/mnist_ddpm_diffusers_nd.json) at 32x32, batch 2.

    Injected eps and integer timesteps; the config's betas; AdamW at the config's lr under the cosine
    schedule (warmup 0).  Checks: loss, per-tensor gradient statistics, full small gradients, Rademacher
    projections and strided samples of every large gradient and AdamW delta (test_gpu_unet.py)."""
    from fmdiff.models.generators import DiffusionUNetFactory
    from fmdiff.pipelines.schedulers import DDPMScheduler
    from fmdiff.pipelines.train.fused import FusedTrainStep
    from oracle import spec as S
    from oracle import unet as U
    from test_gpu_unet import _check_step_vs_golden
    T, M = golden_ddpm
    m = M[case]
    tr_cfg = m["training"]
    model = DiffusionUNetFactory().build(m["unet"], tr_cfg["conditioning"], tr_cfg["channels"]).to(DEV)
    spec = S.derive_spec(m["unet"], tr_cfg["conditioning"], tr_cfg["channels"])
    sd = U.seeded_state_dict(spec, m["seed"])
    model.load_state_dict(sd)
    sch = DDPMScheduler(m["num_train_timesteps"], **m["scheduler"].get("params", {}))
    tr = FusedTrainStep(model, objective="ddpm", ddpm_scheduler=sch, lr=m["lr"], weight_decay=m["weight_decay"],
                        warmup=m["warmup"], total_steps=m["total"], num_train_timesteps=m["num_train_timesteps"])
    clean, ldct, noise, ts = (T[f"{case}/{k}"].to(DEV) for k in ("clean", "ldct", "noise", "t"))
    tr.capture(clean, ldct, warmup_iters=2, noise=noise, t=ts)
    loss = tr.replay()
    torch.cuda.synchronize()
    assert int(tr.step_ctr.item()) == 1
    _check_step_vs_golden(model, T, m, case, loss.item(), m["lr"], small=m["small_grads"], sd_before=sd)
