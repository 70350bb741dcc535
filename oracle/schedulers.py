"""Restated diffusers scheduler arithmetic (TEST INFRASTRUCTURE ONLY).

The reference calls third-party ``diffusers`` schedulers
(``src/pipelines/utils.py:13-30``; ``requirements.txt:18`` pins only
``diffusers>=0.24.0``).  diffusers is not installed offline, so this is a
restatement of its published algorithms (FlowMatchEulerDiscreteScheduler,
DDPMScheduler, DDIMScheduler, DPMSolverMultistepScheduler, UniPCMultistepScheduler with their default
constructor arguments),
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


# --------------------------------------------------------------------------------------------------
# Multistep solvers (diffusers DPMSolverMultistepScheduler / UniPCMultistepScheduler, default constructor
# arguments: linspace spacing, final_sigmas_type "zero", lower_order_final, epsilon prediction; no
# thresholding, karras or lu-lambda sigmas).  Restated from the published algorithms (DPM-Solver++,
# arXiv:2211.01095 multistep update; UniPC, arXiv:2302.04867 B(h) predictor/corrector); parity unpinned.


class _SigmaSchedule:
    def _init_sched(self, N, beta_start, beta_end, beta_schedule, order, final_sigmas_type="zero"):
        self.N = int(N)
        self.final_sigmas_type = final_sigmas_type
        self.betas = _betas(self.N, beta_start, beta_end, beta_schedule)
        self.alphas_cumprod = torch.cumprod(1.0 - self.betas, dim=0)
        self.order = int(order)
        self.timesteps = None
        self.sigmas = None

    def set_timesteps(self, n, spacing="linspace", steps_offset=0):
        N = self.N
        if spacing == "linspace":
            ts = np.linspace(0, N - 1, n + 1).round()[::-1][:-1].copy().astype(np.int64)
        elif spacing == "leading":
            r = N // (n + 1)
            ts = (np.arange(0, n + 1) * r).round()[::-1][:-1].copy().astype(np.int64) + steps_offset
        elif spacing == "trailing":
            r = N / n
            ts = np.arange(N, 0, -r).round().copy().astype(np.int64) - 1
        else:
            raise ValueError(spacing)
        sig = (((1 - self.alphas_cumprod) / self.alphas_cumprod) ** 0.5).numpy()
        last = (((1 - self.alphas_cumprod[0]) / self.alphas_cumprod[0]) ** 0.5).item() \
            if self.final_sigmas_type == "sigma_min" else 0
        sig = np.interp(ts, np.arange(0, len(sig)), sig)
        self.sigmas = torch.from_numpy(np.concatenate([sig, [last]]).astype(np.float32))
        self.timesteps = torch.from_numpy(ts).to(torch.int64)
        self.model_outputs = [None] * self.order
        self.lower_order_nums = 0
        self.step_index = None

    @staticmethod
    def alpha_sigma(sigma):
        alpha_t = 1 / ((sigma ** 2 + 1) ** 0.5)
        return alpha_t, sigma * alpha_t

    def lam(self, i):
        a, s = self.alpha_sigma(self.sigmas[i])
        return torch.log(a) - torch.log(s)

    def init_index(self, t):
        cand = (self.timesteps == int(t)).nonzero()
        if len(cand) == 0:
            self.step_index = len(self.timesteps) - 1
        else:
            self.step_index = int(cand[1 if len(cand) > 1 else 0])

    def to_x0(self, eps, x):
        a, s = self.alpha_sigma(self.sigmas[self.step_index])
        return (x - s * eps) / a


class DPMSolverMultistep(_SigmaSchedule):
    """DPMSolverMultistepScheduler: algorithm dpmsolver++ | dpmsolver, solver_order 1 | 2 | 3, solver_type
    midpoint | heun, lower_order_final."""

    def __init__(self, num_train_timesteps=1000, beta_start=0.0001, beta_end=0.02, beta_schedule="linear",
                 solver_order=2, algorithm_type="dpmsolver++", solver_type="midpoint", lower_order_final=True,
                 final_sigmas_type="zero"):
        if algorithm_type == "dpmsolver" and final_sigmas_type == "zero":
            raise ValueError("final_sigmas_type zero is not supported for algorithm_type dpmsolver")
        self._init_sched(num_train_timesteps, beta_start, beta_end, beta_schedule, solver_order, final_sigmas_type)
        self.algo = algorithm_type
        self.solver_type = solver_type
        self.lower_order_final = lower_order_final

    def first(self, m, x):
        i = self.step_index
        a_t, s_t = self.alpha_sigma(self.sigmas[i + 1])
        a_s, s_s = self.alpha_sigma(self.sigmas[i])
        h = (torch.log(a_t) - torch.log(s_t)) - (torch.log(a_s) - torch.log(s_s))
        if self.algo == "dpmsolver++":
            return (s_t / s_s) * x - (a_t * (torch.exp(-h) - 1.0)) * m
        return (a_t / a_s) * x - (s_t * (torch.exp(h) - 1.0)) * m

    def second(self, x):
        i = self.step_index
        a_t, s_t = self.alpha_sigma(self.sigmas[i + 1])
        a_0, s_0 = self.alpha_sigma(self.sigmas[i])
        l_t, l_0, l_1 = self.lam(i + 1), self.lam(i), self.lam(i - 1)
        m0, m1 = self.model_outputs[-1], self.model_outputs[-2]
        h, h_0 = l_t - l_0, l_0 - l_1
        r0 = h_0 / h
        D0, D1 = m0, (1.0 / r0) * (m0 - m1)
        if self.algo == "dpmsolver++":
            if self.solver_type == "midpoint":
                return ((s_t / s_0) * x - (a_t * (torch.exp(-h) - 1.0)) * D0
                        - 0.5 * (a_t * (torch.exp(-h) - 1.0)) * D1)
            return ((s_t / s_0) * x - (a_t * (torch.exp(-h) - 1.0)) * D0
                    + (a_t * ((torch.exp(-h) - 1.0) / h + 1.0)) * D1)
        if self.solver_type == "midpoint":
            return ((a_t / a_0) * x - (s_t * (torch.exp(h) - 1.0)) * D0
                    - 0.5 * (s_t * (torch.exp(h) - 1.0)) * D1)
        return ((a_t / a_0) * x - (s_t * (torch.exp(h) - 1.0)) * D0
                - (s_t * ((torch.exp(h) - 1.0) / h - 1.0)) * D1)

    def third(self, x):
        i = self.step_index
        a_t, s_t = self.alpha_sigma(self.sigmas[i + 1])
        a_0, s_0 = self.alpha_sigma(self.sigmas[i])
        l_t, l_0, l_1, l_2 = self.lam(i + 1), self.lam(i), self.lam(i - 1), self.lam(i - 2)
        m0, m1, m2 = self.model_outputs[-1], self.model_outputs[-2], self.model_outputs[-3]
        h, h_0, h_1 = l_t - l_0, l_0 - l_1, l_1 - l_2
        r0, r1 = h_0 / h, h_1 / h
        D0 = m0
        D1_0, D1_1 = (1.0 / r0) * (m0 - m1), (1.0 / r1) * (m1 - m2)
        D1 = D1_0 + (r0 / (r0 + r1)) * (D1_0 - D1_1)
        D2 = (1.0 / (r0 + r1)) * (D1_0 - D1_1)
        if self.algo == "dpmsolver++":
            return ((s_t / s_0) * x - (a_t * (torch.exp(-h) - 1.0)) * D0
                    + (a_t * ((torch.exp(-h) - 1.0) / h + 1.0)) * D1
                    - (a_t * ((torch.exp(-h) - 1.0 + h) / h ** 2 - 0.5)) * D2)
        return ((a_t / a_0) * x - (s_t * (torch.exp(h) - 1.0)) * D0
                - (s_t * ((torch.exp(h) - 1.0) / h - 1.0)) * D1
                - (s_t * ((torch.exp(h) - 1.0 - h) / h ** 2 - 0.5)) * D2)

    def step(self, eps, t, x):
        if self.step_index is None:
            self.init_index(t)
        n = len(self.timesteps)
        lof = self.step_index == n - 1 and (self.final_sigmas_type == "zero" or (self.lower_order_final and n < 15))
        los = self.step_index == n - 2 and self.lower_order_final and n < 15
        m = self.to_x0(eps, x) if self.algo == "dpmsolver++" else eps
        self.model_outputs = self.model_outputs[1:] + [m]
        x = x.to(torch.float32)
        if self.order == 1 or self.lower_order_nums < 1 or lof:
            prev = self.first(m, x)
        elif self.order == 2 or self.lower_order_nums < 2 or los:
            prev = self.second(x)
        else:
            prev = self.third(x)
        if self.lower_order_nums < self.order:
            self.lower_order_nums += 1
        self.step_index += 1
        return StepOut(prev.to(eps.dtype))


class UniPCMultistep(_SigmaSchedule):
    """UniPCMultistepScheduler: predict_x0, solver_type bh1 | bh2, solver_order 1..3, corrector on every
    step after the first, lower_order_final."""

    def __init__(self, num_train_timesteps=1000, beta_start=0.0001, beta_end=0.02, beta_schedule="linear",
                 solver_order=2, solver_type="bh2", lower_order_final=True, final_sigmas_type="zero"):
        self._init_sched(num_train_timesteps, beta_start, beta_end, beta_schedule, solver_order, final_sigmas_type)
        self.solver_type = solver_type
        self.lower_order_final = lower_order_final

    def set_timesteps(self, n, spacing="linspace", steps_offset=0):
        super().set_timesteps(n, spacing, steps_offset)
        self.last_sample = None
        self.this_order = None

    def _rb(self, h, rks, order):
        hh = -h
        h_phi_1 = torch.expm1(hh)
        h_phi_k = h_phi_1 / hh - 1
        fact = 1
        B_h = hh if self.solver_type == "bh1" else torch.expm1(hh)
        R, b = [], []
        for i in range(1, order + 1):
            R.append(torch.pow(rks, i - 1))
            b.append(h_phi_k * fact / B_h)
            fact *= i + 1
            h_phi_k = h_phi_k / hh - 1 / fact
        return torch.stack(R), torch.tensor(b), h_phi_1, B_h

    def predictor(self, x, order):
        i = self.step_index
        m0 = self.model_outputs[-1]
        a_t, s_t = self.alpha_sigma(self.sigmas[i + 1])
        a_0, s_0 = self.alpha_sigma(self.sigmas[i])
        l_0 = self.lam(i)
        h = self.lam(i + 1) - l_0
        rks, D1s = [], []
        for k in range(1, order):
            mi = self.model_outputs[-(k + 1)]
            rk = (self.lam(i - k) - l_0) / h
            rks.append(rk)
            D1s.append((mi - m0) / rk)
        rks.append(1.0)
        R, b, h_phi_1, B_h = self._rb(h, torch.tensor(rks), order)
        x_t_ = s_t / s_0 * x - a_t * h_phi_1 * m0
        if D1s:
            rhos = torch.tensor([0.5]) if order == 2 else torch.linalg.solve(R[:-1, :-1], b[:-1])
            pred_res = sum(rhos[k] * D1s[k] for k in range(len(D1s)))
            return x_t_ - a_t * B_h * pred_res
        return x_t_

    def corrector(self, model_t, x, order):
        i = self.step_index
        m0 = self.model_outputs[-1]
        a_t, s_t = self.alpha_sigma(self.sigmas[i])
        a_0, s_0 = self.alpha_sigma(self.sigmas[i - 1])
        l_0 = self.lam(i - 1)
        h = self.lam(i) - l_0
        rks, D1s = [], []
        for k in range(1, order):
            mi = self.model_outputs[-(k + 1)]
            rk = (self.lam(i - (k + 1)) - l_0) / h
            rks.append(rk)
            D1s.append((mi - m0) / rk)
        rks.append(1.0)
        R, b, h_phi_1, B_h = self._rb(h, torch.tensor(rks), order)
        rhos = torch.tensor([0.5]) if order == 1 else torch.linalg.solve(R, b)
        x_t_ = s_t / s_0 * x - a_t * h_phi_1 * m0
        corr = sum(rhos[k] * D1s[k] for k in range(len(D1s))) if D1s else 0
        return x_t_ - a_t * B_h * (corr + rhos[-1] * (model_t - m0))

    def step(self, eps, t, x):
        if self.step_index is None:
            self.init_index(t)
        m = self.to_x0(eps, x)
        if self.step_index > 0 and self.last_sample is not None:
            x = self.corrector(m, self.last_sample, self.this_order)
        self.model_outputs = self.model_outputs[1:] + [m]
        n = len(self.timesteps)
        order = min(self.order, n - self.step_index) if self.lower_order_final else self.order
        self.this_order = min(order, self.lower_order_nums + 1)
        self.last_sample = x
        prev = self.predictor(x, self.this_order)
        if self.lower_order_nums < self.order:
            self.lower_order_nums += 1
        self.step_index += 1
        return StepOut(prev.to(eps.dtype))


def cosine_with_warmup(step: int, warmup: int, total: int, num_cycles: float = 0.5) -> float:
    """LR multiplier of ``get_cosine_schedule_with_warmup`` (``flow_matching_lib.py:76-79``)."""
    if step < warmup:
        return float(step) / float(max(1, warmup))
    progress = float(step - warmup) / float(max(1, total - warmup))
    return max(0.0, 0.5 * (1.0 + math.cos(math.pi * float(num_cycles) * 2.0 * progress)))
