"""``PoolND`` / ``UnPoolND`` (reference ``src/nn/ops/pooling.py:10-30, 87-105``): the patchify down / up
projections of ``EfficientUNetND(pool_factor > 1)`` -- a conv with kernel = stride = pool_factor and its
transposed counterpart; identity for a factor of 1.  Executed by the UNet engine (``runtime/engine.py``)."""
from __future__ import annotations

import torch.nn as nn

from ..params import Identity, SizeArg
from .convolution import ConvND, ConvTransposeND


def _is_one(f) -> bool:
    return f == 1 or (isinstance(f, (tuple, list)) and all(p == 1 for p in f))


class PoolND(nn.Module):
    def __init__(self, spatial_dims: int, in_channels: int, out_channels: int, pool_factor: SizeArg = 2):
        super().__init__()
        self.down = Identity() if _is_one(pool_factor) else ConvND(spatial_dims, in_channels, out_channels,
                                                                    kernel_size=pool_factor, stride=pool_factor,
                                                                    padding=0)

    def forward(self, x):
        return self.down(x)


class UnPoolND(nn.Module):
    def __init__(self, spatial_dims: int, in_channels: int, out_channels: int, pool_factor: SizeArg = 2):
        super().__init__()
        self.up = Identity() if _is_one(pool_factor) else ConvTransposeND(spatial_dims, in_channels, out_channels,
                                                                          kernel_size=pool_factor, stride=pool_factor,
                                                                          padding=0)

    def forward(self, x):
        return self.up(x)
