"""Calling a single block outside a UNet.

The fused engine executes whole UNets (``fmdiff.runtime.engine``).  A lone
``Conv`` runs through the same implicit-GEMM kernel (forward only); lone
ResBlock / attention modules are executed by the UNet engine only.
"""
from __future__ import annotations

import torch

from . import ops


def conv_forward(conv, x: torch.Tensor) -> torch.Tensor:
    """NCHW fp32 -> NCHW fp32 through csrc/conv.hip (no autograd)."""
    ops._need_cuda(x, "Conv")
    if conv.dims != 2 and not (conv.dims == 1 and conv.kernel_size == (1,)):
        raise NotImplementedError("standalone Conv: 2-D convs and 1x1 Conv1d only")
    if x.dim() == 3:   # Conv1d k=1 over tokens: treat as [N, C, T, 1]
        x4 = x.unsqueeze(-1)
    else:
        x4 = x
    Cin = x4.shape[1]
    Cp = -(-Cin // 8) * 8
    K = conv.out_channels
    Kp = -(-K // 8) * 8
    xin = ops.nchw_to_nhwc(x4, Cp)
    w = ops.prep_weights(conv.weight.detach(), 0, Kp, Cp)
    ks = conv.kernel_size[0]
    bias = None
    if conv.bias is not None:
        bias = torch.zeros(Kp, device=x.device, dtype=torch.float32)
        bias[:K].copy_(conv.bias.detach())
    out, _ = ops.conv(xin, Kp, w, ks=ks, stride=conv.stride[0], pad=conv.padding[0], bias=bias, out_f32=True)
    y = ops.nhwc_to_nchw(out, K)
    return y.squeeze(-1) if x.dim() == 3 else y


def linear_forward(lin, x: torch.Tensor) -> torch.Tensor:
    ops._need_cuda(x, "Linear")
    if x.dim() != 2 or x.shape[0] > 32:
        raise NotImplementedError("standalone Linear: [B<=32, in] inputs (time-embedding path)")
    return ops.linear(x.float().contiguous(), lin.weight.detach(), lin.bias.detach() if lin.bias is not None else None)


def block_forward(block, x, emb):
    raise NotImplementedError(f"{type(block).__name__} runs inside a UNet through fmdiff.runtime.engine; "
                              "standalone block execution is not provided")
