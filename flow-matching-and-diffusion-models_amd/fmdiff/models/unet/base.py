"""``BaseUNetND`` (reference ``src/models/unet/base.py:10-53``).

``forward(x, t, context=None, context_ca=None)`` keeps the reference's call
contract (NCHW fp32 in, NCHW fp32 out, differentiable); underneath it runs the
whole UNet through the fused HIP engine (``fmdiff.runtime.engine``) as one
autograd node whose backward is the hand-scheduled HIP backward pass.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn


class BaseUNetND(nn.Module):
    def _normalize_timesteps(self, t, x: torch.Tensor) -> torch.Tensor:
        if not torch.is_tensor(t):
            t = torch.tensor([t], device=x.device, dtype=torch.long)
        if t.ndim == 0:
            t = t[None].to(x.device)
        return t.expand(x.shape[0]).to(x.device)

    def _prepare_input(self, x, context, context_ca):
        return x

    def forward(self, x: torch.Tensor, t, context: Optional[torch.Tensor] = None,
                context_ca: Optional[torch.Tensor] = None, **kwargs) -> torch.Tensor:
        from ...runtime.engine import unet_apply
        if context_ca is not None:
            self._prepare_input(x, None, context_ca)   # reference validation (unet.py:301)
        t = self._normalize_timesteps(t, x)
        # the channel concat of `context` is fused into the NHWC staging kernel
        return unet_apply(self, x, t, context, context_ca)

    def engine(self):
        """The cached fused engine bound to this module (built on first GPU use)."""
        from ...runtime.engine import get_engine
        return get_engine(self)
