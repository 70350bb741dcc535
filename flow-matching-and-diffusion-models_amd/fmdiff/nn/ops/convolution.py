"""``ConvND`` envelope (reference ``src/nn/ops/convolution.py:8-54``); the parameter lives under ``.conv``."""
from __future__ import annotations

from typing import Optional

import torch.nn as nn

from ..params import Conv, ConvT, SizeArg


class ConvND(nn.Module):
    def __init__(self, spatial_dims: int, in_channels: int, out_channels: int, kernel_size: SizeArg = 3,
                 stride: SizeArg = 1, padding: Optional[SizeArg] = None, dilation: SizeArg = 1, groups: int = 1,
                 bias: bool = True):
        super().__init__()
        if spatial_dims not in (1, 2, 3):
            raise ValueError("spatial_dims must be 1, 2 or 3")
        if padding is None:
            padding = kernel_size // 2 if isinstance(kernel_size, int) else tuple(k // 2 for k in kernel_size)
        self.conv = Conv(spatial_dims, in_channels, out_channels, kernel_size, stride, padding, dilation, groups, bias)

    def forward(self, x):
        return self.conv(x)


class ConvTransposeND(nn.Module):
    """Reference ``src/nn/ops/convolution.py:56-96``; the parameter lives under ``.convT``."""

    def __init__(self, spatial_dims: int, in_channels: int, out_channels: int, kernel_size: SizeArg = 2,
                 stride: SizeArg = 2, padding: SizeArg = 0, output_padding: Optional[SizeArg] = None, groups: int = 1,
                 bias: bool = True):
        super().__init__()
        if spatial_dims not in (1, 2, 3):
            raise ValueError("spatial_dims must be 1, 2 or 3")
        self.convT = ConvT(spatial_dims, in_channels, out_channels, kernel_size, stride, padding, output_padding or 0,
                           groups, bias)

    def forward(self, x):
        return self.convT(x)
