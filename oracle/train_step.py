"""FM / DDPM train-step body and the sampler loop on CPU (TEST INFRASTRUCTURE ONLY).

Restates ``src/pipelines/train/flow_matching_lib.py:150-182`` (FM),
``src/pipelines/train/diffusion_lib.py:153-185`` (DDPM) and
``src/pipelines/utils.py:163-220`` (``sample_with_scheduler``).  Random draws
(noise, t, timesteps, DDPM variance noise) are injected so the GPU path can be
compared on identical inputs.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.nn.functional as F

from . import unet as U


def fm_timesteps(t: torch.Tensor, num_train_timesteps: int) -> torch.Tensor:
    """``timesteps = (t * (N - 1)).long()`` (flow_matching_lib.py:153)."""
    return (t * (num_train_timesteps - 1)).long()


def fm_loss(sd, spec, clean, ldct, noise, t, num_train_timesteps=1000, grad_accum=1):
    """Forward + loss of one FM chunk; returns (loss, scaled_loss) (flow_matching_lib.py:151-172)."""
    timesteps = fm_timesteps(t, num_train_timesteps)
    tb = t.view(-1, *([1] * (clean.dim() - 1)))
    x_t = (1.0 - tb) * clean + tb * noise
    inp = torch.cat([x_t, ldct], dim=1) if ldct is not None else x_t
    pred = U.unet_forward(sd, spec, inp, timesteps)
    loss = F.mse_loss(pred, noise - clean)
    return loss, loss / grad_accum


def ddpm_loss(sd, spec, sched, clean, ldct, noise, timesteps, grad_accum=1):
    """Forward + loss of one DDPM chunk (diffusion_lib.py:154-172)."""
    noisy = sched.add_noise(clean, noise, timesteps)
    inp = torch.cat([noisy, ldct], dim=1) if ldct is not None else noisy
    pred = U.unet_forward(sd, spec, inp, timesteps)
    loss = F.mse_loss(pred, noise)
    return loss, loss / grad_accum


def adamw_step(params: Dict[str, torch.Tensor], lr: float, step: int, state: Dict[str, dict],
               betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
    """One ``torch.optim.AdamW`` update (flow_matching_lib.py:73,177-181), written out."""
    b1, b2 = betas
    with torch.no_grad():
        for name, p in params.items():
            g = p.grad
            if g is None:
                continue
            st = state.setdefault(name, dict(m=torch.zeros_like(p), v=torch.zeros_like(p)))
            p.mul_(1 - lr * weight_decay)
            st["m"].lerp_(g, 1 - b1)
            st["v"].mul_(b2).addcmul_(g, g, value=1 - b2)
            bc1 = 1 - b1 ** step
            bc2 = 1 - b2 ** step
            denom = (st["v"].sqrt() / (bc2 ** 0.5)).add_(eps)
            p.addcdiv_(st["m"], denom, value=-lr / bc1)


def sample(sd, spec, sched, num_inference_steps, init, cond=None, noises=None,
           start_step: Optional[int] = None, last_n_steps: Optional[int] = None):
    """``sample_with_scheduler`` for concatenate / unconditional modes (pipelines/utils.py:163-220)."""
    sched.set_timesteps(num_inference_steps)
    ts = sched.timesteps
    if start_step is not None:
        ts = ts[ts <= int(start_step)]
    if last_n_steps is not None:
        ts = ts[-int(last_n_steps):]
    cur = init.clone()
    with torch.no_grad():
        for i, t in enumerate(ts):
            inp = torch.cat([cur, cond], dim=1) if cond is not None else cur
            tt = t.expand(cur.size(0)) if t.dim() == 0 else t
            pred = U.unet_forward(sd, spec, inp, tt)
            if noises is not None and hasattr(sched, "add_noise"):
                cur = sched.step(pred, t, cur, noise=noises[i]).prev_sample
            else:
                cur = sched.step(pred, t, cur).prev_sample
    return cur
