"""Parameter-holding leaf modules with the reference's attribute / state_dict names.

``Conv`` stands where the reference has ``nn.Conv{1,2,3}d`` (``weight``
[out, in, *k], ``bias``), ``Linear`` for ``nn.Linear`` and ``GroupNorm`` for
``nn.GroupNorm``; initialisation matches PyTorch's defaults so training from
scratch behaves like the reference.  Their compute runs through the fused
HIP engine (``fmdiff.runtime``); calling one on its own goes through the same
kernels (``fmdiff.runtime.standalone``).
"""
from __future__ import annotations

import math
from typing import Tuple, Union

import torch
import torch.nn as nn

SizeArg = Union[int, Tuple[int, ...]]


def _tuple(v, n):
    return tuple(v) if isinstance(v, (tuple, list)) else (v,) * n


class Conv(nn.Module):
    """Holds ``weight`` / ``bias`` of an N-d convolution (reference ``nn.Conv{1,2,3}d``)."""

    def __init__(self, dims: int, in_channels: int, out_channels: int, kernel_size: SizeArg = 3, stride: SizeArg = 1,
                 padding: SizeArg = 0, dilation: SizeArg = 1, groups: int = 1, bias: bool = True):
        super().__init__()
        if groups != 1 or any(d != 1 for d in _tuple(dilation, dims)):
            raise NotImplementedError("grouped / dilated convolution is not on the fmdiff hot path")
        self.dims = dims
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.kernel_size = _tuple(kernel_size, dims)
        self.stride = _tuple(stride, dims)
        self.padding = _tuple(padding, dims)
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels, *self.kernel_size))
        self.bias = nn.Parameter(torch.empty(out_channels)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):
        # torch.nn.modules.conv._ConvNd.reset_parameters
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            fan_in = self.weight[0].numel()
            bound = 1 / math.sqrt(fan_in) if fan_in > 0 else 0
            nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x):
        from ..runtime.standalone import conv_forward
        return conv_forward(self, x)

    def extra_repr(self):
        return (f"{self.in_channels}, {self.out_channels}, kernel_size={self.kernel_size}, "
                f"stride={self.stride}, padding={self.padding}")


class ConvT(nn.Module):
    """Holds ``weight`` [in, out, *k] / ``bias`` [out] of an N-d transposed convolution (reference
    ``nn.ConvTranspose{1,2,3}d``); executed by the UNet engine (UnPoolND)."""

    def __init__(self, dims: int, in_channels: int, out_channels: int, kernel_size: SizeArg = 2,
                 stride: SizeArg = 2, padding: SizeArg = 0, output_padding: SizeArg = 0, groups: int = 1,
                 bias: bool = True):
        super().__init__()
        if groups != 1:
            raise NotImplementedError("grouped transposed convolution is not on the fmdiff hot path")
        self.dims = dims
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.kernel_size = _tuple(kernel_size, dims)
        self.stride = _tuple(stride, dims)
        self.padding = _tuple(padding, dims)
        self.output_padding = _tuple(output_padding, dims)
        self.weight = nn.Parameter(torch.empty(in_channels, out_channels, *self.kernel_size))
        self.bias = nn.Parameter(torch.empty(out_channels)) if bias else None
        # torch.nn.modules.conv._ConvNd.reset_parameters (fan_in of the [in, out, *k] weight = out * prod(k))
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            fan_in, _ = nn.init._calculate_fan_in_and_fan_out(self.weight)
            bound = 1 / math.sqrt(fan_in) if fan_in > 0 else 0
            nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x):
        raise NotImplementedError("ConvTranspose runs inside the UNet engine (UnPoolND of pool_factor > 1)")


class Linear(nn.Module):
    """Holds ``weight`` [out, in] / ``bias`` (reference ``nn.Linear``)."""

    def __init__(self, in_features: int, out_features: int, bias: bool = True):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.weight = nn.Parameter(torch.empty(out_features, in_features))
        self.bias = nn.Parameter(torch.empty(out_features)) if bias else None
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            bound = 1 / math.sqrt(in_features) if in_features > 0 else 0
            nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x):
        from ..runtime.standalone import linear_forward
        return linear_forward(self, x)


class GroupNorm(nn.Module):
    """Holds GroupNorm affine params (reference ``nn.GroupNorm``)."""

    def __init__(self, num_groups: int, num_channels: int, eps: float = 1e-5, affine: bool = True):
        super().__init__()
        if num_channels % num_groups:
            raise ValueError("num_channels must be divisible by num_groups")
        self.num_groups = num_groups
        self.num_channels = num_channels
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(num_channels))
        self.bias = nn.Parameter(torch.zeros(num_channels))

    def extra_repr(self):
        return f"{self.num_groups}, {self.num_channels}, eps={self.eps}"


class SiLU(nn.Module):
    """Marker for the activation the kernels fuse (reference ``nn.SiLU``)."""


class Identity(nn.Module):
    def forward(self, x):
        return x


def zero_module(module):
    """Zero out the parameters of a module and return it (reference ``nn/blocks/common.py:8-14``)."""
    for p in module.parameters():
        p.detach().zero_()
    return module
