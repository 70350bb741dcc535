"""diffusers-compatible schedulers with HIP step kernels.

The reference instantiates third-party ``diffusers`` schedulers through
``SCHEDULER_REGISTRY`` (``src/pipelines/utils.py:13-30``) and uses
``config.num_train_timesteps``, ``set_timesteps``, ``timesteps``, ``step(...)
.prev_sample`` and ``add_noise``.  These classes keep that protocol; the
timestep / sigma / alpha tables are built on the host with the same dtypes as
the upstream code (float32 / int64 / float64 numpy), so the bookkeeping is
bit-exact, and the per-step update runs in the HIP kernels of
``csrc/misc.hip`` on device tensors.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from types import SimpleNamespace

import numpy as np
import torch

from ..runtime import ops

SCHED_NCOEF = 12   # FMD_SCHED_NCOEF: coefficient row of the table-driven multistep step (fmd_sched_step)


@dataclass
class SchedulerOutput:
    prev_sample: torch.Tensor


def _flat_cfg(**kw):
    return SimpleNamespace(**kw)


def _nhwc_view(t: torch.Tensor):
    """[N, C, H, W] fp32 -> (fp32 NHWC-compatible buffer [N, H, W, C]) for the step kernels."""
    if t.shape[1] == 1:
        return t.contiguous().view(t.shape[0], *t.shape[2:], 1)
    return t.permute(0, 2, 3, 1).contiguous()


class FlowMatchEulerDiscreteScheduler:
    """shift=1, no dynamic shifting (the reference's configs pass ``params: {}``)."""

    def __init__(self, num_train_timesteps: int = 1000, shift: float = 1.0, **_unused):
        self.config = _flat_cfg(num_train_timesteps=int(num_train_timesteps), shift=float(shift))
        N = self.config.num_train_timesteps
        ts = torch.from_numpy(np.linspace(1, N, N, dtype=np.float32)[::-1].copy()).to(torch.float32)
        sig = ts / N
        sig = shift * sig / (1 + (shift - 1) * sig)
        self.timesteps = sig * N
        self.sigmas = sig
        self.sigma_min = float(sig[-1].item())
        self.sigma_max = float(sig[0].item())
        self._step_index = None
        self.num_inference_steps = None
        self._dev = {}

    def set_timesteps(self, num_inference_steps: int, device=None):
        N = self.config.num_train_timesteps
        t = np.linspace(self.sigma_max * N, self.sigma_min * N, num_inference_steps)
        sig = t / N
        s = self.config.shift
        sig = s * sig / (1 + (s - 1) * sig)
        sig = torch.from_numpy(sig).to(dtype=torch.float32)
        self.timesteps = (sig * N).to(device) if device is not None else sig * N
        self.sigmas = torch.cat([sig, torch.zeros(1)])
        self.num_inference_steps = num_inference_steps
        self._step_index = None
        self._dev = {}

    def index_for_timestep(self, timestep):
        ts = self.timesteps.cpu()
        t = timestep.cpu() if torch.is_tensor(timestep) else torch.tensor(timestep)
        idx = (ts == t).nonzero()
        return int(idx[1 if len(idx) > 1 else 0].item())

    @property
    def step_index(self):
        return self._step_index

    def _device_tables(self, device):
        if device not in self._dev:
            self._dev[device] = (self.sigmas.to(device), torch.zeros(1, dtype=torch.int32, device=device))
        return self._dev[device]

    def step(self, model_output: torch.Tensor, timestep, sample: torch.Tensor, return_dict: bool = True, **_kw):
        if self._step_index is None:
            self._step_index = self.index_for_timestep(timestep)
        ops._need_cuda(sample, "FlowMatchEulerDiscreteScheduler.step")
        sig, idx = self._device_tables(sample.device)
        idx.fill_(self._step_index)
        x = sample.float().clone()
        ops.flow_euler(x, _nhwc_view(model_output.float()), sig, idx, None, None)
        self._step_index += 1
        out = x.to(model_output.dtype)
        return SchedulerOutput(out) if return_dict else (out,)


def _betas(N, start, end, schedule):
    if schedule == "linear":
        return torch.linspace(start, end, N, dtype=torch.float32)
    if schedule == "scaled_linear":
        return torch.linspace(start ** 0.5, end ** 0.5, N, dtype=torch.float32) ** 2
    if schedule == "squaredcos_cap_v2":
        def ab(x):
            return math.cos((x + 0.008) / 1.008 * math.pi / 2) ** 2
        return torch.tensor([min(1 - ab((i + 1) / N) / ab(i / N), 0.999) for i in range(N)], dtype=torch.float32)
    raise NotImplementedError(f"beta_schedule {schedule}")


class DDPMScheduler:
    """Defaults: linear betas, fixed_small variance, epsilon prediction, clip 1.0, leading spacing."""

    def __init__(self, num_train_timesteps: int = 1000, beta_start: float = 0.0001, beta_end: float = 0.02,
                 beta_schedule: str = "linear", variance_type: str = "fixed_small", clip_sample: bool = True,
                 prediction_type: str = "epsilon", clip_sample_range: float = 1.0,
                 timestep_spacing: str = "leading", steps_offset: int = 0, **_unused):
        if variance_type != "fixed_small" or prediction_type != "epsilon":
            raise NotImplementedError("fmdiff DDPM step: fixed_small variance + epsilon prediction")
        self.config = _flat_cfg(num_train_timesteps=int(num_train_timesteps), beta_start=beta_start,
                                beta_end=beta_end, beta_schedule=beta_schedule, clip_sample=clip_sample,
                                clip_sample_range=clip_sample_range, timestep_spacing=timestep_spacing,
                                steps_offset=steps_offset, prediction_type=prediction_type)
        N = self.config.num_train_timesteps
        self.betas = _betas(N, beta_start, beta_end, beta_schedule)
        self.alphas = 1.0 - self.betas
        self.alphas_cumprod = torch.cumprod(self.alphas, dim=0)
        self.one = torch.tensor(1.0)
        self.timesteps = torch.from_numpy(np.arange(0, N)[::-1].copy())
        self.num_inference_steps = None
        self._dev = {}
        self._noise_tables = {}

    def set_timesteps(self, num_inference_steps: int, device=None):
        N = self.config.num_train_timesteps
        n = num_inference_steps
        sp = self.config.timestep_spacing
        if sp == "leading":
            ts = (np.arange(0, n) * (N // n)).round()[::-1].copy().astype(np.int64) + self.config.steps_offset
        elif sp == "linspace":
            ts = np.linspace(0, N - 1, n).round()[::-1].copy().astype(np.int64)
        elif sp == "trailing":
            ts = np.round(np.arange(N, 0, -N / n)).astype(np.int64) - 1
        else:
            raise ValueError(sp)
        self.timesteps = torch.from_numpy(ts).to(device) if device is not None else torch.from_numpy(ts)
        self.num_inference_steps = n
        self._dev = {}

    def previous_timestep(self, t: int) -> int:
        return t - (self.config.num_train_timesteps // self.num_inference_steps if self.num_inference_steps else 1)

    def coefficients(self, t: int):
        """fp32 scalars of one step in the upstream operation order:
        [sqrt(1-a_t), sqrt(a_t), c_x0, c_xt, std, clip, c_eps] (csrc/misc.hip ddpm_step_kernel)."""
        pt = self.previous_timestep(t)
        a_t = self.alphas_cumprod[t]
        a_p = self.alphas_cumprod[pt] if pt >= 0 else self.one
        b_t = 1 - a_t
        b_p = 1 - a_p
        cur_a = a_t / a_p
        cur_b = 1 - cur_a
        c_x0 = (a_p ** 0.5 * cur_b) / b_t
        c_xt = cur_a ** 0.5 * b_p / b_t
        var = torch.clamp((1 - a_p) / (1 - a_t) * cur_b, min=1e-20)
        std = var ** 0.5 if t > 0 else torch.tensor(0.0)
        clip = self.config.clip_sample_range if self.config.clip_sample else 0.0
        return torch.stack([b_t ** 0.5, a_t ** 0.5, c_x0, c_xt, std, torch.tensor(float(clip)),
                            torch.tensor(0.0)]).float()

    def step(self, model_output, timestep, sample, generator=None, return_dict: bool = True, variance_noise=None,
             **_kw):
        ops._need_cuda(sample, "DDPMScheduler.step")
        t = int(timestep)
        coef = self.coefficients(t).to(sample.device)
        idx = torch.zeros(1, dtype=torch.int32, device=sample.device)
        noise = None
        if t > 0:
            noise = variance_noise if variance_noise is not None else torch.randn(
                sample.shape, generator=generator, device=sample.device, dtype=torch.float32)
            noise = noise.float().contiguous()
        x = sample.float().clone()
        ops.ddpm_step(x, _nhwc_view(model_output.float()), coef, idx, noise, None, None)
        out = x.to(model_output.dtype)
        return SchedulerOutput(out) if return_dict else (out,)

    def add_noise(self, original_samples, noise, timesteps):
        """sqrt(a_t) x0 + sqrt(1-a_t) eps (diffusers add_noise; training input of diffusion_lib.py:158), fp32,
        bit-exact with the eager torch expression (fmd_add_noise).  The sqrt tables are the host's fp32
        ``alphas_cumprod ** 0.5`` / ``(1 - alphas_cumprod) ** 0.5``, gathered per sample on the device."""
        ops._need_cuda(original_samples, "add_noise")
        dev = original_samples.device
        if dev not in self._noise_tables:
            ac = self.alphas_cumprod.to(torch.float32)
            self._noise_tables[dev] = ((ac ** 0.5).to(dev), ((1 - ac) ** 0.5).to(dev))
        sa, sb = self._noise_tables[dev]
        x0 = original_samples.float().contiguous()
        nz = noise.to(device=dev, dtype=torch.float32).contiguous()
        N = x0.shape[0]
        ts = torch.as_tensor(timesteps).to(device=dev, dtype=torch.int64).reshape(-1)
        if ts.numel() == 1 and N > 1:
            ts = ts.expand(N)
        ts = ts.contiguous()
        if ts.numel() != N or nz.shape != x0.shape:
            raise ValueError("add_noise: one timestep per sample and noise of the samples' shape")
        # the kernel gathers sa[t] / sb[t] unchecked: validate the range here, as torch indexing does in the
        # reference (IndexError); a stream capture cannot read the device tensor, so captures skip the check
        T = int(sa.numel())
        if N and not torch.cuda.is_current_stream_capturing():
            lo, hi = int(ts.min()), int(ts.max())
            if lo < 0 or hi >= T:
                raise IndexError(f"add_noise: timesteps must lie in [0, {T}), got [{lo}, {hi}]")
        out = torch.empty_like(x0)
        from .. import _lib
        _lib.call("fmd_add_noise", x0.data_ptr(), nz.data_ptr(), sa.data_ptr(), sb.data_ptr(), ts.data_ptr(), N,
                  x0[0].numel() if N else 0, out.data_ptr(), ops.stream())
        return out.to(original_samples.dtype)


class DDIMScheduler(DDPMScheduler):
    """Defaults: eta 0, set_alpha_to_one, clip 1.0, leading spacing (deterministic update)."""

    def __init__(self, num_train_timesteps: int = 1000, beta_start: float = 0.0001, beta_end: float = 0.02,
                 beta_schedule: str = "linear", clip_sample: bool = True, set_alpha_to_one: bool = True,
                 steps_offset: int = 0, prediction_type: str = "epsilon", clip_sample_range: float = 1.0,
                 timestep_spacing: str = "leading", **_unused):
        super().__init__(num_train_timesteps, beta_start, beta_end, beta_schedule, "fixed_small", clip_sample,
                         prediction_type, clip_sample_range, timestep_spacing, steps_offset)
        self.final_alpha_cumprod = torch.tensor(1.0) if set_alpha_to_one else self.alphas_cumprod[0]

    def coefficients(self, t: int):
        """eta = 0: prev = sqrt(a_p) * clip(x0_hat) + sqrt(1 - a_p) * eps (DDIMScheduler.step)."""
        pt = t - self.config.num_train_timesteps // self.num_inference_steps
        a_t = self.alphas_cumprod[t]
        a_p = self.alphas_cumprod[pt] if pt >= 0 else self.final_alpha_cumprod
        b_t = 1 - a_t
        clip = self.config.clip_sample_range if self.config.clip_sample else 0.0
        return torch.stack([b_t ** 0.5, a_t ** 0.5, a_p ** 0.5, torch.tensor(0.0), torch.tensor(0.0),
                            torch.tensor(float(clip)), (1 - a_p) ** 0.5]).float()

    def step(self, model_output, timestep, sample, eta: float = 0.0, generator=None, return_dict: bool = True,
             **_kw):
        if eta != 0.0:
            raise NotImplementedError("fmdiff DDIM: eta = 0 (the reference's default)")
        ops._need_cuda(sample, "DDIMScheduler.step")
        coef = self.coefficients(int(timestep)).to(sample.device)
        idx = torch.zeros(1, dtype=torch.int32, device=sample.device)
        x = sample.float().clone()
        ops.ddpm_step(x, _nhwc_view(model_output.float()), coef, idx, None, None, None)
        out = x.to(model_output.dtype)
        return SchedulerOutput(out) if return_dict else (out,)


# --------------------------------------------------------------------------------------------------
# Multistep solvers: diffusers DPMSolverMultistepScheduler / UniPCMultistepScheduler protocol (called by the
# reference at src/pipelines/utils.py:218 through SCHEDULER_REGISTRY "dpm_multistep" / "unipc", and the
# run_model CLI aliases dpmsolver1/2/++).  Host bookkeeping (timesteps, sigmas, step index, warm-up order)
# follows the upstream float32 / int64 / float64 types; every per-step scalar is folded on the host into
# the coefficients of one fused device update ``out = sum_k c_k * t_k`` (fmd_lincomb) over the sample and
# the model-output history, so a step is 2 launches (data-prediction conversion + update).


class _MultistepBase:
    order_max = 3

    def __init__(self, num_train_timesteps, beta_start, beta_end, beta_schedule, solver_order, prediction_type,
                 timestep_spacing, steps_offset, final_sigmas_type, use_karras_sigmas, thresholding):
        if prediction_type != "epsilon":
            raise NotImplementedError("fmdiff multistep solvers: epsilon prediction (the reference's DDPM models)")
        if use_karras_sigmas or thresholding:
            raise NotImplementedError("fmdiff multistep solvers: karras sigmas / thresholding")
        if not 1 <= int(solver_order) <= self.order_max:
            raise ValueError(f"solver_order {solver_order}")
        if final_sigmas_type not in ("zero", "sigma_min"):
            raise ValueError(final_sigmas_type)
        N = int(num_train_timesteps)
        self.betas = _betas(N, beta_start, beta_end, beta_schedule)
        self.alphas_cumprod = torch.cumprod(1.0 - self.betas, dim=0)
        self.init_noise_sigma = 1.0
        self.timesteps = torch.from_numpy(np.linspace(0, N - 1, N, dtype=np.float32)[::-1].copy())
        self.num_inference_steps = None
        self._set_common()

    def _set_common(self):
        self.model_outputs = [None] * self.config.solver_order
        self.lower_order_nums = 0
        self._step_index = None

    @property
    def step_index(self):
        return self._step_index

    def set_timesteps(self, num_inference_steps: int, device=None):
        N = self.config.num_train_timesteps
        n = int(num_inference_steps)
        sp = self.config.timestep_spacing
        if sp == "linspace":
            ts = np.linspace(0, N - 1, n + 1).round()[::-1][:-1].copy().astype(np.int64)
        elif sp == "leading":
            ts = (np.arange(0, n + 1) * (N // (n + 1))).round()[::-1][:-1].copy().astype(np.int64)
            ts += self.config.steps_offset
        elif sp == "trailing":
            ts = np.arange(N, 0, -N / n).round().copy().astype(np.int64) - 1
        else:
            raise ValueError(sp)
        sig = (((1 - self.alphas_cumprod) / self.alphas_cumprod) ** 0.5).numpy()
        sig = np.interp(ts, np.arange(0, len(sig)), sig)
        last = (((1 - self.alphas_cumprod[0]) / self.alphas_cumprod[0]) ** 0.5).item() \
            if self.config.final_sigmas_type == "sigma_min" else 0
        self.sigmas = torch.from_numpy(np.concatenate([sig, [last]]).astype(np.float32))
        self.timesteps = torch.from_numpy(ts).to(device=device, dtype=torch.int64) if device is not None \
            else torch.from_numpy(ts).to(torch.int64)
        self.num_inference_steps = len(ts)
        self._set_common()

    def _init_step_index(self, timestep):
        cand = (self.timesteps.cpu() == int(timestep)).nonzero()
        self._step_index = len(self.timesteps) - 1 if len(cand) == 0 else int(cand[1 if len(cand) > 1 else 0])

    @staticmethod
    def _alpha_sigma(sigma):
        alpha_t = 1 / ((sigma ** 2 + 1) ** 0.5)
        return alpha_t, sigma * alpha_t

    def _lam(self, i):
        a, s = self._alpha_sigma(self.sigmas[i])
        return torch.log(a) - torch.log(s)

    def _to_x0(self, eps, x):
        """x0 = (x - sigma_t * eps) / alpha_t at the current step (fmd_lincomb)."""
        a, s = self._alpha_sigma(self.sigmas[self._step_index])
        return ops.lincomb(torch.empty_like(x), [x, eps], [1.0 / a, -(s / a)])

    @staticmethod
    def _prep(model_output, sample):
        ops._need_cuda(sample, "scheduler.step")
        return model_output.float().contiguous(), sample.float().contiguous()


class DPMSolverMultistepScheduler(_MultistepBase):
    """Defaults as upstream: solver_order 2, dpmsolver++, midpoint, lower_order_final, final_sigmas_type
    zero (rejected for algorithm_type dpmsolver, like upstream), linspace spacing."""

    def __init__(self, num_train_timesteps: int = 1000, beta_start: float = 0.0001, beta_end: float = 0.02,
                 beta_schedule: str = "linear", solver_order: int = 2, prediction_type: str = "epsilon",
                 algorithm_type: str = "dpmsolver++", solver_type: str = "midpoint", lower_order_final: bool = True,
                 euler_at_final: bool = False, use_karras_sigmas: bool = False, final_sigmas_type: str = "zero",
                 timestep_spacing: str = "linspace", steps_offset: int = 0, thresholding: bool = False,
                 **_unused):
        if algorithm_type not in ("dpmsolver++", "dpmsolver"):
            raise NotImplementedError(f"fmdiff DPM-Solver: algorithm_type {algorithm_type}")
        if solver_type not in ("midpoint", "heun"):
            raise ValueError(solver_type)
        if algorithm_type == "dpmsolver" and final_sigmas_type == "zero":
            raise ValueError(f"`final_sigmas_type` {final_sigmas_type} is not supported for `algorithm_type` "
                             f"{algorithm_type}. Please choose `sigma_min` instead.")
        self.config = _flat_cfg(num_train_timesteps=int(num_train_timesteps), beta_start=beta_start,
                                beta_end=beta_end, beta_schedule=beta_schedule, solver_order=int(solver_order),
                                prediction_type=prediction_type, algorithm_type=algorithm_type,
                                solver_type=solver_type, lower_order_final=lower_order_final,
                                euler_at_final=euler_at_final, final_sigmas_type=final_sigmas_type,
                                timestep_spacing=timestep_spacing, steps_offset=steps_offset)
        super().__init__(num_train_timesteps, beta_start, beta_end, beta_schedule, solver_order, prediction_type,
                         timestep_spacing, steps_offset, final_sigmas_type, use_karras_sigmas, thresholding)

    def _coefs(self, order):
        """(coefficient of the sample, [coefficients of model_outputs[-1], [-2], [-3]]) of one update."""
        i = self._step_index
        pp = self.config.algorithm_type == "dpmsolver++"
        heun = self.config.solver_type == "heun"
        a_t, s_t = self._alpha_sigma(self.sigmas[i + 1])
        a_0, s_0 = self._alpha_sigma(self.sigmas[i])
        h = self._lam(i + 1) - self._lam(i)
        cx = s_t / s_0 if pp else a_t / a_0
        c0 = -(a_t * (torch.exp(-h) - 1.0)) if pp else -(s_t * (torch.exp(h) - 1.0))
        if order == 1:
            return cx, [c0]
        if pp:
            cd1 = (a_t * ((torch.exp(-h) - 1.0) / h + 1.0)) if heun else -0.5 * (a_t * (torch.exp(-h) - 1.0))
        else:
            cd1 = -(s_t * ((torch.exp(h) - 1.0) / h - 1.0)) if heun else -0.5 * (s_t * (torch.exp(h) - 1.0))
        h_0 = self._lam(i) - self._lam(i - 1)
        r0 = h_0 / h
        if order == 2:   # D1 = (m0 - m1) / r0
            return cx, [c0 + cd1 / r0, -cd1 / r0]
        # third order: D1 = D1_0 + r0/(r0+r1) (D1_0 - D1_1), D2 = (D1_0 - D1_1)/(r0+r1)
        cd1 = (a_t * ((torch.exp(-h) - 1.0) / h + 1.0)) if pp else -(s_t * ((torch.exp(h) - 1.0) / h - 1.0))
        cd2 = (-(a_t * ((torch.exp(-h) - 1.0 + h) / h ** 2 - 0.5)) if pp
               else -(s_t * ((torch.exp(h) - 1.0 - h) / h ** 2 - 0.5)))
        r1 = (self._lam(i - 1) - self._lam(i - 2)) / h
        k = r0 / (r0 + r1)
        # D1_0 = (m0 - m1)/r0, D1_1 = (m1 - m2)/r1
        d10 = [1.0 / r0, -1.0 / r0, 0.0]
        d11 = [0.0, 1.0 / r1, -1.0 / r1]
        diff = [x - y for x, y in zip(d10, d11)]
        d1 = [x + k * y for x, y in zip(d10, diff)]
        d2 = [y / (r0 + r1) for y in diff]
        return cx, [c0 + cd1 * d1[0] + cd2 * d2[0], cd1 * d1[1] + cd2 * d2[1], cd1 * d1[2] + cd2 * d2[2]]

    def plan(self, start: int = 0) -> torch.Tensor:
        """Coefficient rows of fmd_sched_step for steps ``start`` .. end of the schedule set by set_timesteps, in
        the order ``step`` takes them from a fresh state (the same order decisions and coefficient folding, so
        the table-driven graph step equals this class's eager steps): [n - start][12] fp32."""
        n = len(self.timesteps)
        saved = self._step_index
        pp = self.config.algorithm_type == "dpmsolver++"
        rows, lon = [], 0
        try:
            for i in range(start, n):
                self._step_index = i
                lof = i == n - 1 and (self.config.euler_at_final or (self.config.lower_order_final and n < 15)
                                      or self.config.final_sigmas_type == "zero")
                los = i == n - 2 and self.config.lower_order_final and n < 15
                if self.config.solver_order == 1 or lon < 1 or lof:
                    order = 1
                elif self.config.solver_order == 2 or lon < 2 or los:
                    order = 2
                else:
                    order = 3
                cx, cm = self._coefs(order)
                row = [0.0] * SCHED_NCOEF
                if pp:
                    a, s = self._alpha_sigma(self.sigmas[i])
                    row[0], row[1] = float(1.0 / a), float(-(s / a))
                else:
                    row[1] = 1.0
                row[8] = float(cx)
                for k, c in enumerate(cm):
                    row[9 + k] = float(c)
                rows.append(row)
                if lon < self.config.solver_order:
                    lon += 1
        finally:
            self._step_index = saved
        return torch.tensor(rows, dtype=torch.float32)

    def step(self, model_output, timestep, sample, generator=None, variance_noise=None, return_dict: bool = True,
             **_kw):
        eps, x = self._prep(model_output, sample)
        if self._step_index is None:
            self._init_step_index(timestep)
        n = len(self.timesteps)
        i = self._step_index
        lof = i == n - 1 and (self.config.euler_at_final or (self.config.lower_order_final and n < 15)
                              or self.config.final_sigmas_type == "zero")
        los = i == n - 2 and self.config.lower_order_final and n < 15
        m = self._to_x0(eps, x) if self.config.algorithm_type == "dpmsolver++" else eps.clone()
        self.model_outputs = self.model_outputs[1:] + [m]
        if self.config.solver_order == 1 or self.lower_order_nums < 1 or lof:
            order = 1
        elif self.config.solver_order == 2 or self.lower_order_nums < 2 or los:
            order = 2
        else:
            order = 3
        cx, cm = self._coefs(order)
        hist = [self.model_outputs[-1 - k] for k in range(order)]
        prev = ops.lincomb(torch.empty_like(x), [x] + hist, [cx] + cm)
        if self.lower_order_nums < self.config.solver_order:
            self.lower_order_nums += 1
        self._step_index += 1
        out = prev.to(model_output.dtype)
        return SchedulerOutput(out) if return_dict else (out,)


class UniPCMultistepScheduler(_MultistepBase):
    """Defaults as upstream: solver_order 2, bh2, predict_x0, lower_order_final, corrector on every step after
    the first (disable_corrector = []), final_sigmas_type zero, linspace spacing."""

    def __init__(self, num_train_timesteps: int = 1000, beta_start: float = 0.0001, beta_end: float = 0.02,
                 beta_schedule: str = "linear", solver_order: int = 2, prediction_type: str = "epsilon",
                 predict_x0: bool = True, solver_type: str = "bh2", lower_order_final: bool = True,
                 disable_corrector=(), use_karras_sigmas: bool = False, timestep_spacing: str = "linspace",
                 steps_offset: int = 0, final_sigmas_type: str = "zero", thresholding: bool = False, **_unused):
        if not predict_x0:
            raise NotImplementedError("fmdiff UniPC: predict_x0 (upstream default)")
        if solver_type not in ("bh1", "bh2"):
            raise ValueError(solver_type)
        self.config = _flat_cfg(num_train_timesteps=int(num_train_timesteps), beta_start=beta_start,
                                beta_end=beta_end, beta_schedule=beta_schedule, solver_order=int(solver_order),
                                prediction_type=prediction_type, predict_x0=predict_x0, solver_type=solver_type,
                                lower_order_final=lower_order_final, disable_corrector=list(disable_corrector),
                                timestep_spacing=timestep_spacing, steps_offset=steps_offset,
                                final_sigmas_type=final_sigmas_type)
        super().__init__(num_train_timesteps, beta_start, beta_end, beta_schedule, solver_order, prediction_type,
                         timestep_spacing, steps_offset, final_sigmas_type, use_karras_sigmas, thresholding)

    def _set_common(self):
        super()._set_common()
        self.last_sample = None
        self.this_order = None

    def _rb(self, h, rks, order):
        hh = -h
        h_phi_1 = torch.expm1(hh)
        h_phi_k = h_phi_1 / hh - 1
        fact = 1
        B_h = hh if self.config.solver_type == "bh1" else torch.expm1(hh)
        R, b = [], []
        for i in range(1, order + 1):
            R.append(torch.pow(rks, i - 1))
            b.append(h_phi_k * fact / B_h)
            fact *= i + 1
            h_phi_k = h_phi_k / hh - 1 / fact
        return torch.stack(R), torch.tensor(b), h_phi_1, B_h

    def _update(self, corrector: bool, order: int):
        """Coefficients of x, model_outputs[-1], [-2], ..., (and model_t for the corrector)."""
        i = self._step_index
        it, i0 = (i, i - 1) if corrector else (i + 1, i)
        a_t, s_t = self._alpha_sigma(self.sigmas[it])
        a_0, s_0 = self._alpha_sigma(self.sigmas[i0])
        l_0 = self._lam(i0)
        h = self._lam(it) - l_0
        rks = [(self._lam(i0 - k) - l_0) / h for k in range(1, order)]
        R, b, h_phi_1, B_h = self._rb(h, torch.tensor(rks + [1.0]), order)
        cx = s_t / s_0
        cm = [-(a_t * h_phi_1)] + [0.0] * (order - 1)
        if corrector:
            rhos = torch.tensor([0.5]) if order == 1 else torch.linalg.solve(R, b)
            lin = rhos[:-1]
        else:
            rhos = None
            lin = (torch.tensor([0.5]) if order == 2 else torch.linalg.solve(R[:-1, :-1], b[:-1])) \
                if order > 1 else torch.tensor([])
        # x_t -= a_t B_h * (sum_k lin_k (m_k - m0) / rk  [+ rho_last (model_t - m0)])
        g = a_t * B_h
        for k in range(1, order):
            w = lin[k - 1] / rks[k - 1]
            cm[k] = cm[k] - g * w
            cm[0] = cm[0] + g * w
        cmt = None
        if corrector:
            cmt = -(g * rhos[-1])
            cm[0] = cm[0] + g * rhos[-1]
        return cx, cm, cmt

    def plan(self, start: int = 0) -> torch.Tensor:
        """Coefficient rows of fmd_sched_step (corrector + predictor) for steps ``start`` .. end of the schedule,
        in the order ``step`` takes them from a fresh state: [n - start][12] fp32.  A row holds at most 3 history
        coefficients (corrector and predictor), so solver_order > 3 is the eager ``step``'s only."""
        if int(self.config.solver_order) > 3:
            raise NotImplementedError("UniPC plan(): solver_order > 3 has no table step; use the eager step")
        n = len(self.timesteps)
        saved = (self._step_index, self.this_order)
        rows, lon, this_order = [], 0, None
        try:
            for i in range(start, n):
                self._step_index = i
                row = [0.0] * SCHED_NCOEF
                a, s = self._alpha_sigma(self.sigmas[i])
                row[0], row[1] = float(1.0 / a), float(-(s / a))
                if i > start and (i - 1) not in self.config.disable_corrector:
                    cx, cm, cmt = self._update(True, this_order)
                    row[2], row[3], row[7] = 1.0, float(cx), float(cmt)
                    for k, c in enumerate(cm):
                        row[4 + k] = float(c)
                order = min(self.config.solver_order, n - i) if self.config.lower_order_final \
                    else self.config.solver_order
                this_order = min(order, lon + 1)
                cx, cm, _ = self._update(False, this_order)
                row[8] = float(cx)
                for k, c in enumerate(cm):
                    row[9 + k] = float(c)
                rows.append(row)
                if lon < self.config.solver_order:
                    lon += 1
        finally:
            self._step_index, self.this_order = saved
        return torch.tensor(rows, dtype=torch.float32)

    def step(self, model_output, timestep, sample, return_dict: bool = True, generator=None, **_kw):
        eps, x = self._prep(model_output, sample)
        if self._step_index is None:
            self._init_step_index(timestep)
        m = self._to_x0(eps, x)
        i = self._step_index
        if i > 0 and (i - 1) not in self.config.disable_corrector and self.last_sample is not None:
            cx, cm, cmt = self._update(True, self.this_order)
            hist = [self.model_outputs[-1 - k] for k in range(self.this_order)]
            x = ops.lincomb(torch.empty_like(x), [self.last_sample] + hist + [m], [cx] + cm + [cmt])
        self.model_outputs = self.model_outputs[1:] + [m]
        n = len(self.timesteps)
        order = min(self.config.solver_order, n - i) if self.config.lower_order_final else self.config.solver_order
        self.this_order = min(order, self.lower_order_nums + 1)
        self.last_sample = x
        cx, cm, _ = self._update(False, self.this_order)
        hist = [self.model_outputs[-1 - k] for k in range(self.this_order)]
        prev = ops.lincomb(torch.empty_like(x), [x] + hist, [cx] + cm)
        if self.lower_order_nums < self.config.solver_order:
            self.lower_order_nums += 1
        self._step_index += 1
        out = prev.to(model_output.dtype)
        return SchedulerOutput(out) if return_dict else (out,)

