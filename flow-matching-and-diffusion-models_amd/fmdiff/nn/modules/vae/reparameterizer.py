"""``DiagonalGaussian`` (reference ``src/nn/modules/vae/reparameterizer.py:13-62``).

``mode()`` is a channel slice of the moments (no arithmetic); ``sample`` / ``kl`` / ``nll`` are the
reference's small latent-sized elementwise formulas (not on the encode -> denoise -> decode hot path)."""
from __future__ import annotations

import math
from typing import Iterable, Optional

import torch


class DiagonalGaussian:
    def __init__(self, parameters: torch.Tensor, deterministic: bool = False):
        mu, logvar = torch.chunk(parameters, 2, dim=1)
        self.mu = mu
        self.logvar = torch.clamp(logvar, -30.0, 20.0)
        self.deter = deterministic
        self.device = parameters.device
        if deterministic:
            self.std = torch.zeros_like(mu)
            self.var = torch.zeros_like(mu)
        else:
            self.std = torch.exp(0.5 * self.logvar)
            self.var = torch.exp(self.logvar)

    def sample(self) -> torch.Tensor:
        if self.deter:
            return self.mu
        return self.mu + self.std * torch.randn_like(self.mu)

    def mode(self) -> torch.Tensor:
        return self.mu

    def kl(self, other: Optional["DiagonalGaussian"] = None, reduce_dims: Iterable[int] = (1, 2, 3)) -> torch.Tensor:
        if self.deter:
            return torch.tensor([0.0], device=self.device)
        if other is None:
            return 0.5 * torch.sum(self.mu.pow(2) + self.var - 1.0 - self.logvar, dim=reduce_dims)
        return 0.5 * torch.sum((self.mu - other.mu).pow(2) / other.var + self.var / other.var - 1.0 - self.logvar
                               + other.logvar, dim=reduce_dims)

    def nll(self, x: torch.Tensor, reduce_dims: Iterable[int] = (1, 2, 3)) -> torch.Tensor:
        return 0.5 * torch.sum(math.log(2.0 * math.pi) + self.logvar + (x - self.mu).pow(2) / self.var,
                               dim=reduce_dims)
