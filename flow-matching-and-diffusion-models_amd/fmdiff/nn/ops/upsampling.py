"""``UpsampleND`` / ``DownsampleND`` (reference ``src/nn/ops/upsampling.py:8-62``).

Nearest-x2 upsampling is never materialised: the following 3x3 conv gathers
from the low-resolution tensor directly (csrc/conv.hip ``upsample``)."""
from __future__ import annotations

import torch.nn as nn

from .convolution import ConvND


class UpsampleND(nn.Module):
    def __init__(self, spatial_dims: int, channels: int, use_conv: bool = True):
        super().__init__()
        if spatial_dims not in (1, 2, 3):
            raise ValueError("spatial_dims must be 1, 2 or 3")
        self.channels = channels
        self.use_conv = use_conv
        self.spatial_dims = spatial_dims
        if use_conv:
            self.conv = ConvND(spatial_dims, channels, channels, kernel_size=3, padding=1)


class AvgPoolND(nn.Module):
    def __init__(self, spatial_dims: int, kernel_size=2, stride=None, padding=0):
        super().__init__()
        self.spatial_dims = spatial_dims
        self.kernel_size, self.stride, self.padding = kernel_size, stride, padding


class DownsampleND(nn.Module):
    def __init__(self, spatial_dims: int, channels: int, use_conv: bool = True):
        super().__init__()
        if spatial_dims not in (1, 2, 3):
            raise ValueError("spatial_dims must be 1, 2 or 3")
        self.channels = channels
        self.use_conv = use_conv
        self.spatial_dims = spatial_dims
        if use_conv:
            self.op = ConvND(spatial_dims, channels, channels, kernel_size=3, stride=2, padding=1)
        else:
            self.op = AvgPoolND(spatial_dims, kernel_size=2, stride=2)
