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
        """sqrt(a_t) x0 + sqrt(1-a_t) eps (diffusers add_noise; training input of diffusion_lib.py:158)."""
        ops._need_cuda(original_samples, "add_noise")
        ac = self.alphas_cumprod.to(device=original_samples.device, dtype=torch.float32)
        sel = ac[timesteps.to(original_samples.device)]
        ca = (sel ** 0.5).contiguous()
        cb = ((1 - sel) ** 0.5).contiguous()
        N, Cx = original_samples.shape[:2]
        buf = ops.noise_prepare(original_samples.float().contiguous(), noise.float().contiguous(), ca, cb, None,
                                max(8, -(-Cx // 8) * 8))
        return ops.nhwc_to_nchw(buf, Cx).to(original_samples.dtype)


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
