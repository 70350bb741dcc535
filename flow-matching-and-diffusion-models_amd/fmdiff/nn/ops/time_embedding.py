"""Sinusoidal timestep features (reference ``src/nn/ops/time_embedding.py:4-32``), HIP kernel."""
from __future__ import annotations

import torch


def timestep_embedding(timesteps: torch.Tensor, dim: int, max_period: int = 10000, *, flip_sin_to_cos: bool = True,
                       freq_shift: int = 0) -> torch.Tensor:
    from ...runtime import ops
    ops._need_cuda(timesteps, "timestep_embedding")
    return ops.timestep_embedding(timesteps, dim, flip_sin_to_cos, freq_shift, float(max_period))
