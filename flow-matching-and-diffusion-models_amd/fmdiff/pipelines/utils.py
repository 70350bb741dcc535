"""Scheduler registry and the generic sampling loop.

Mirrors ``src/pipelines/utils.py`` of the reference: ``SCHEDULER_REGISTRY``
(``:22-30``), ``build_scheduler`` (``:40-62``), ``resolve_scheduler_override``
(``:65-90``), ``_forward_model`` (``:93-102``), ``_align_conditioning``
(``:110-119``), ``normalize_latent_conditioning`` (``:122-151``) and
``sample_with_scheduler`` (``:163-220``) keep the same names, arguments and
error messages.  The scheduler classes are the HIP-stepped ones of
``fmdiff.pipelines.schedulers``; the model call goes through the HIP UNet
engine.  For the graph-captured fast path of the flow-matching sampler see
``fmdiff.pipelines.train.fused.FusedFlowSampler``.
"""
from __future__ import annotations

import inspect
import math
import time
from typing import Dict, Tuple

import torch

from .schedulers import (DDIMScheduler, DDPMScheduler, DPMSolverMultistepScheduler,
                         FlowMatchEulerDiscreteScheduler, UniPCMultistepScheduler)


class _NotBuiltScheduler:
    """Registry placeholder for a diffusers scheduler whose HIP step is not built yet."""
    name = "?"

    def __init__(self, num_train_timesteps: int = 1000, **params):
        raise NotImplementedError(f"scheduler '{self.name}' has no HIP step implementation in fmdiff yet")


class DPMSolverSDEScheduler(_NotBuiltScheduler):
    name = "dpm_sde"   # Brownian-tree SDE sampler (torchsde upstream): not on the BASELINE configs


SCHEDULER_REGISTRY: Dict[str, type] = {
    "ddpm": DDPMScheduler,
    "ddim": DDIMScheduler,
    "dpm_multistep": DPMSolverMultistepScheduler,
    "dpm_sde": DPMSolverSDEScheduler,
    "unipc": UniPCMultistepScheduler,
    "flow_match_euler": FlowMatchEulerDiscreteScheduler,
    "flowmatch": FlowMatchEulerDiscreteScheduler,
}

_ALIASES = {
    "ddpm": {"name": "ddpm"},
    "ddim": {"name": "ddim"},
    "dpmsolver1": {"name": "dpm_multistep", "params": {"solver_order": 1, "algorithm_type": "dpmsolver"}},
    "dpmsolver2": {"name": "dpm_multistep", "params": {"solver_order": 2, "algorithm_type": "dpmsolver"}},
    "dpmsolver++": {"name": "dpm_multistep", "params": {"solver_order": 2, "algorithm_type": "dpmsolver++"}},
    "dpmsolversde": {"name": "dpm_sde"},
    "unipc": {"name": "unipc"},
    "flowmatch": {"name": "flow_match_euler"},
    "flow_match_euler": {"name": "flow_match_euler"},
}


def resolve_conditioning_mode(value) -> str | None:
    if value is None:
        return None
    value = str(value).strip().lower()
    return value or None


def build_scheduler(spec: Dict, training_cfg: Dict) -> Tuple[object, int]:
    """(scheduler, num_inference_steps) from the config's ``scheduler`` and ``training`` blocks.

    Name falls back to ``training.scheduler`` then ``"ddpm"``; ctor kwargs in ``params`` are filtered by the
    class signature; ``num_train_timesteps`` / ``num_inference_steps`` fall back scheduler -> training -> 1000 /
    num_train_timesteps (reference ``pipelines/utils.py:40-62``)."""
    sch = dict(spec or {})
    tr = dict(training_cfg or {})
    name = sch.get("name") or tr.get("scheduler") or "ddpm"
    key = str(name).lower()
    if key not in SCHEDULER_REGISTRY:
        raise ValueError(f"Unknown scheduler '{name}'. Available: {', '.join(SCHEDULER_REGISTRY)}")
    cls = SCHEDULER_REGISTRY[key]
    n_train = int(sch.get("num_train_timesteps") or tr.get("num_train_timesteps") or 1000)
    allowed = set(inspect.signature(cls.__init__).parameters) - {"self"}
    params = {k: v for k, v in dict(sch.get("params", {})).items() if k in allowed}
    scheduler = cls(num_train_timesteps=n_train, **params)
    n_inf = int(sch.get("num_inference_steps") or tr.get("num_inference_steps") or n_train)
    return scheduler, n_inf


def resolve_scheduler_override(name: str | None) -> Dict | None:
    """CLI alias -> scheduler config override (``run_model.py --scheduler``)."""
    if not name:
        return None
    key = str(name).strip().lower()
    if not key:
        return None
    if key in _ALIASES:
        return {k: (dict(v) if isinstance(v, dict) else v) for k, v in _ALIASES[key].items()}
    if key in SCHEDULER_REGISTRY:
        return {"name": key}
    raise ValueError(f"Unknown scheduler override '{name}'. Available: {', '.join(sorted(_ALIASES))}")


def _forward_model(model, inputs, timesteps, context_ca=None):
    out = model(inputs, timesteps, context_ca=context_ca) if context_ca is not None else model(inputs, timesteps)
    if isinstance(out, tuple):
        return out[0]
    return out.sample if hasattr(out, "sample") else out


def sync_if_cuda(device: torch.device) -> None:
    if device.type == "cuda" and torch.cuda.is_available():
        torch.cuda.synchronize(device)


def _align_conditioning(condition, target_batch):
    """Repeat/trim the conditioning batch to the sample batch."""
    if condition is None or condition.size(0) == target_batch:
        return condition
    reps = math.ceil(target_batch / condition.size(0))
    if reps > 1:
        condition = condition.repeat(reps, *([1] * (condition.dim() - 1)))
    return condition[:target_batch]


def normalize_latent_conditioning(condition, mode):
    """Per-sample ``standardize`` / ``minmax`` / none normalisation of latent conditioning."""
    if condition is None:
        return None
    m = str(mode or "none").lower()
    if m in {"none", "false", "off"}:
        return condition
    dims = tuple(range(2, condition.dim()))
    if m == "standardize":
        return (condition - condition.mean(dim=dims, keepdim=True)) / (condition.std(dim=dims, keepdim=True) + 1e-6)
    if m == "minmax":
        lo, hi = condition.amin(dim=dims, keepdim=True), condition.amax(dim=dims, keepdim=True)
        return (condition - lo) / (hi - lo + 1e-6)
    raise ValueError(f"Unknown latent_norm mode: {mode}")


def _prepare_attention_context(condition):
    """Cross-attention context as the UNet takes it: (B, C, T) tokens or (B, C, *spatial) maps pass through."""
    if condition is None:
        return None
    if condition.dim() >= 3:
        return condition
    raise ValueError(f"Unsupported conditioning shape for attention: {tuple(condition.shape)}")


def select_timesteps(timesteps: torch.Tensor, start_step=None, last_n_steps=None) -> torch.Tensor:
    """Tail selection of ``sample_with_scheduler`` (reference ``pipelines/utils.py:182-192``)."""
    if start_step is not None:
        start_step = int(start_step)
        if start_step < 0:
            raise ValueError("start_step must be >= 0.")
        timesteps = timesteps[timesteps <= start_step]
    if last_n_steps is not None:
        last_n_steps = int(last_n_steps)
        if last_n_steps <= 0:
            raise ValueError("last_n_steps must be > 0.")
        timesteps = timesteps[-last_n_steps:]
    if timesteps.numel() == 0:
        raise ValueError("No timesteps selected after applying start_step/last_n_steps.")
    return timesteps


def model_throughput(timing: Dict, count: int) -> Dict:
    """The evaluate-side throughput fields of the reference (``src/pipelines/samplers/diffusion_like.py:287-313``):
    from the sampling loop's ``model_seconds`` / ``model_calls`` accumulators and the number of samples produced,
    ``model_samples_per_second = count / model_seconds`` and ``model_seconds_per_sample = model_seconds / count``
    (0 when undefined), formatted as the reference's metrics row formats them."""
    secs = float(timing.get("model_seconds", 0.0))
    sps = count / secs if secs > 0 else 0.0
    spp = secs / count if count else 0.0
    return {"samples": int(count), "model_seconds": f"{secs:.6f}", "model_samples_per_second": f"{sps:.6f}",
            "model_seconds_per_sample": f"{spp:.8f}", "model_calls": int(timing.get("model_calls", 0))}


def sample_with_scheduler(model, scheduler, num_inference_steps: int, sample_shape: Tuple[int, ...],
                          device: torch.device, conditioning_mode: str | None = None,
                          conditioning_batch: torch.Tensor | None = None, latent_norm: str | None = None,
                          timing: dict | None = None, start_step: int | None = None,
                          last_n_steps: int | None = None, init_sample: torch.Tensor | None = None) -> torch.Tensor:
    """Generic sampling loop: per timestep ``cat([x, cond])`` -> UNet -> ``scheduler.step(...).prev_sample``."""
    scheduler.set_timesteps(num_inference_steps)
    timesteps = select_timesteps(scheduler.timesteps, start_step, last_n_steps)
    current = init_sample.to(device) if init_sample is not None else torch.randn(sample_shape, device=device)
    cond = _align_conditioning(conditioning_batch, current.size(0))
    if conditioning_mode == "attention":
        cond = normalize_latent_conditioning(cond, latent_norm)
    ctx = cond if conditioning_mode == "attention" else None
    for t in timesteps:
        inp = current
        if conditioning_mode == "concatenate" and cond is not None:
            inp = torch.cat([inp, cond.to(inp.dtype)], dim=1)
        ts = t.to(current.device) if torch.is_tensor(t) else torch.as_tensor(t, device=current.device)
        if ts.dim() == 0:
            ts = ts.expand(current.size(0))
        if timing is not None:
            sync_if_cuda(current.device)
            t0 = time.perf_counter()
        pred = _forward_model(model, inp, ts, context_ca=ctx)
        if timing is not None:
            sync_if_cuda(current.device)
            timing["model_seconds"] = timing.get("model_seconds", 0.0) + (time.perf_counter() - t0)
            timing["model_calls"] = timing.get("model_calls", 0) + 1
        current = scheduler.step(pred, t, current).prev_sample
    return current
