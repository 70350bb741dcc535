"""Restated diffusers scheduler arithmetic (TEST INFRASTRUCTURE ONLY).

The reference calls third-party ``diffusers`` schedulers
(``src/pipelines/utils.py:13-30``; ``requirements.txt:18`` pins only
``diffusers>=0.24.0``).  diffusers is not installed offline, so this is a
restatement of its published algorithms (FlowMatchEulerDiscreteScheduler,
DDPMScheduler, DDIMScheduler with their default constructor arguments),
pinned only by the closed-form known-answer values in SURVEY.md Appendix B /
8(c): **parity unpinned** beyond those KATs.

Host bookkeeping (timestep tables, step indices) follows the float32 / int64
/ float64 types of the upstream code exactly; the per-step update is plain
fp32 torch on CPU.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch


@dataclass
class StepOut:
    prev_sample: torch.Tensor


class FlowMatchEuler:
    """FlowMatchEulerDiscreteScheduler, shift=1, no dynamic shifting."""

    def __init__(self, num_train_timesteps: int = 1000, shift: float = 1.0):
        self.N = int(num_train_timesteps)
        self.shift = float(shift)
        ts = np.linspace(1, self.N, self.N, dtype=np.float32)[::-1].copy()
        ts = torch.from_numpy(ts).to(torch.float32)
        sig = ts / self.N
        sig = self.shift * sig / (1 + (self.shift - 1) * sig)
        self.timesteps = sig * self.N
        self.sigmas = sig
        self.sigma_min = float(sig[-1].item())
        self.sigma_max = float(sig[0].item())
        self.step_index = None

    def set_timesteps(self, n: int):
        t = np.linspace(self.sigma_max * self.N, self.sigma_min * self.N, n)
        sig = t / self.N
        sig = self.shift * sig / (1 + (self.shift - 1) * sig)
        sig = torch.from_numpy(sig).to(dtype=torch.float32)
        self.timesteps = sig * self.N
        self.sigmas = torch.cat([sig, torch.zeros(1)])
        self.step_index = None

    def index_for_timestep(self, t):
        idx = (self.timesteps == t).nonzero()
        return int(idx[1 if len(idx) > 1 else 0].item())

    def step(self, v, t, x):
        if self.step_index is None:
            self.step_index = self.index_for_timestep(t)
        xs = x.to(torch.float32)
        s = self.sigmas[self.step_index]
        s1 = self.sigmas[self.step_index + 1]
        out = xs + (s1 - s) * v
        self.step_index += 1
        return StepOut(out.to(v.dtype))


def _betas(N, beta_start, beta_end, schedule):
    if schedule == "linear":
        return torch.linspace(beta_start, beta_end, N, dtype=torch.float32)
    if schedule == "scaled_linear":
        return torch.linspace(beta_start ** 0.5, beta_end ** 0.5, N, dtype=torch.float32) ** 2
    if schedule == "squaredcos_cap_v2":
        def ab(t):
            return math.cos((t + 0.008) / 1.008 * math.pi / 2) ** 2
        return torch.tensor([min(1 - ab((i + 1) / N) / ab(i / N), 0.999) for i in range(N)], dtype=torch.float32)
    raise NotImplementedError(schedule)


class DDPM:
    """DDPMScheduler defaults: fixed_small variance, epsilon prediction, clip 1.0, leading spacing."""

    def __init__(self, num_train_timesteps=1000, beta_start=0.0001, beta_end=0.02, beta_schedule="linear",
                 clip_sample=True, clip_sample_range=1.0, timestep_spacing="leading", steps_offset=0,
                 prediction_type="epsilon"):
        self.N = int(num_train_timesteps)
        self.betas = _betas(self.N, beta_start, beta_end, beta_schedule)
        self.alphas = 1.0 - self.betas
        self.alphas_cumprod = torch.cumprod(self.alphas, dim=0)
        self.one = torch.tensor(1.0)
        self.clip = clip_sample
        self.clip_range = clip_sample_range
        self.spacing = timestep_spacing
        self.offset = steps_offset
        self.pred = prediction_type
        self.n = None
        self.timesteps = torch.from_numpy(np.arange(0, self.N)[::-1].copy())

    def set_timesteps(self, n):
        self.n = n
        if self.spacing == "leading":
            r = self.N // n
            ts = (np.arange(0, n) * r).round()[::-1].copy().astype(np.int64) + self.offset
        elif self.spacing == "linspace":
            ts = np.linspace(0, self.N - 1, n).round()[::-1].copy().astype(np.int64)
        elif self.spacing == "trailing":
            r = self.N / n
            ts = np.round(np.arange(self.N, 0, -r)).astype(np.int64) - 1
        else:
            raise ValueError(self.spacing)
        self.timesteps = torch.from_numpy(ts)

    def prev_t(self, t):
        return t - (self.N // self.n if self.n else 1)

    def coefficients(self, t):
        """All fp32 scalars the step uses, in the upstream operation order."""
        t = int(t)
        pt = self.prev_t(t)
        a_t = self.alphas_cumprod[t]
        a_p = self.alphas_cumprod[pt] if pt >= 0 else self.one
        b_t = 1 - a_t
        b_p = 1 - a_p
        cur_a = a_t / a_p
        cur_b = 1 - cur_a
        c_x0 = (a_p ** 0.5 * cur_b) / b_t
        c_xt = cur_a ** 0.5 * b_p / b_t
        var = (1 - a_p) / (1 - a_t) * cur_b
        var = torch.clamp(var, min=1e-20)
        return dict(sqrt_b=b_t ** 0.5, sqrt_a=a_t ** 0.5, c_x0=c_x0, c_xt=c_xt, std=var ** 0.5)

    def step(self, eps, t, x, noise=None):
        c = self.coefficients(t)
        if self.pred == "epsilon":
            x0 = (x - c["sqrt_b"] * eps) / c["sqrt_a"]
        elif self.pred == "sample":
            x0 = eps
        else:
            x0 = c["sqrt_a"] * x - c["sqrt_b"] * eps
        if self.clip:
            x0 = x0.clamp(-self.clip_range, self.clip_range)
        prev = c["c_x0"] * x0 + c["c_xt"] * x
        if int(t) > 0:
            if noise is None:
                noise = torch.randn_like(eps)
            prev = prev + c["std"] * noise
        return StepOut(prev)

    def add_noise(self, x0, noise, timesteps):
        ac = self.alphas_cumprod.to(dtype=x0.dtype)
        sa = ac[timesteps] ** 0.5
        sb = (1 - ac[timesteps]) ** 0.5
        sa = sa.flatten()
        sb = sb.flatten()
        while sa.ndim < x0.ndim:
            sa = sa.unsqueeze(-1)
            sb = sb.unsqueeze(-1)
        return sa * x0 + sb * noise


class DDIM(DDPM):
    """DDIMScheduler defaults: eta 0, set_alpha_to_one, clip 1.0, leading spacing."""

    def __init__(self, num_train_timesteps=1000, beta_start=0.0001, beta_end=0.02, beta_schedule="linear",
                 clip_sample=True, set_alpha_to_one=True, steps_offset=0, clip_sample_range=1.0,
                 timestep_spacing="leading", prediction_type="epsilon"):
        super().__init__(num_train_timesteps, beta_start, beta_end, beta_schedule, clip_sample, clip_sample_range,
                         timestep_spacing, steps_offset, prediction_type)
        self.final = torch.tensor(1.0) if set_alpha_to_one else self.alphas_cumprod[0]

    def step(self, eps, t, x, eta=0.0, noise=None):
        t = int(t)
        pt = t - self.N // self.n
        a_t = self.alphas_cumprod[t]
        a_p = self.alphas_cumprod[pt] if pt >= 0 else self.final
        b_t = 1 - a_t
        x0 = (x - b_t ** 0.5 * eps) / a_t ** 0.5
        if self.clip:
            x0 = x0.clamp(-self.clip_range, self.clip_range)
        b_p = 1 - a_p
        var = (b_p / b_t) * (1 - a_t / a_p)
        std = eta * var ** 0.5
        direction = (1 - a_p - std ** 2) ** 0.5 * eps
        prev = a_p ** 0.5 * x0 + direction
        if eta > 0:
            prev = prev + std * (noise if noise is not None else torch.randn_like(eps))
        return StepOut(prev)


def cosine_with_warmup(step: int, warmup: int, total: int, num_cycles: float = 0.5) -> float:
    """LR multiplier of ``get_cosine_schedule_with_warmup`` (``flow_matching_lib.py:76-79``)."""
    if step < warmup:
        return float(step) / float(max(1, warmup))
    progress = float(step - warmup) / float(max(1, total - warmup))
    return max(0.0, 0.5 * (1.0 + math.cos(math.pi * float(num_cycles) * 2.0 * progress)))
