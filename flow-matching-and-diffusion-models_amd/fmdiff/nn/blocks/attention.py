"""Attention blocks (reference ``src/nn/blocks/attention.py``), same ctors / state_dict keys.

GPU execution: GroupNorm is folded into the qkv 1x1-conv gather, the head
split (incl. SpatialSelfAttention's raw reshape, ``attention.py:111-115``) is
index arithmetic inside the attention kernel, and the output projection adds
the residual in its epilogue (``fmdiff.runtime.engine``)."""
from __future__ import annotations

import math

import torch.nn as nn

from ..params import Conv, GroupNorm, Linear, zero_module


class ContextBlock(nn.Module):
    """Marker for layers that consume an external context tensor."""


class QKVAttention(nn.Module):
    def __init__(self, efficient_attn: bool = True, dropout: float = 0.0):
        super().__init__()
        self.efficient_attn = efficient_attn
        self.dropout = dropout


class LinearQKVAttention(nn.Module):
    def __init__(self, dropout: float = 0.0, eps: float = 1e-6):
        super().__init__()
        self.dropout = dropout
        self.eps = eps


class SpatialSelfAttention(nn.Module):
    def __init__(self, dim: int, heads: int = 4, dim_head: int = 64, use_linear: bool = False,
                 use_efficient_attn: bool = True):
        super().__init__()
        self.dim = dim
        self.heads = heads
        self.dim_head = dim_head
        self.inner_dim = dim_head * heads
        self.use_linear = use_linear
        self.norm = GroupNorm(max(1, math.gcd(dim, 32)), dim)
        self.qkv = Conv(1, dim, self.inner_dim * 3, 1)
        self.attention = LinearQKVAttention() if use_linear else QKVAttention(efficient_attn=use_efficient_attn)
        self.proj_out = zero_module(Conv(1, self.inner_dim, dim, 1))

    def forward(self, x):
        from ...runtime.standalone import block_forward
        return block_forward(self, x, None)


class SpatialCrossAttention(ContextBlock):
    def __init__(self, dim: int, context_dim: int, heads: int = 4, dim_head: int = 64, use_linear: bool = False,
                 use_efficient_attn: bool = True):
        super().__init__()
        self.dim = dim
        self.context_dim = context_dim
        self.heads = heads
        self.dim_head = dim_head
        self.inner_dim = dim_head * heads
        self.use_linear = use_linear
        self.norm = GroupNorm(max(1, math.gcd(dim, 32)), dim)
        self.context_norm = GroupNorm(max(1, math.gcd(context_dim, 32)), context_dim)
        self.q_proj = Conv(1, dim, self.inner_dim, 1)
        self.kv_proj = Conv(1, context_dim, self.inner_dim * 2, 1)
        self.attention = LinearQKVAttention() if use_linear else QKVAttention(efficient_attn=use_efficient_attn)
        self.proj_out = zero_module(Conv(1, self.inner_dim, self.dim, 1))

    def forward(self, x, context):
        from ...runtime.standalone import block_forward
        return block_forward(self, x, None, context)


class DiffusersAttentionND(nn.Module):
    def __init__(self, channels: int, heads: int = 1, context_dim: int | None = None, norm_num_groups: int = 32,
                 eps: float = 1e-5, dropout: float = 0.0, use_efficient_attn: bool = True):
        super().__init__()
        self.channels = channels
        self.heads = max(1, heads)
        self.head_dim = channels // self.heads
        self.context_dim = int(context_dim) if context_dim is not None else None
        self.eps = eps
        self.group_norm = GroupNorm(max(1, math.gcd(channels, norm_num_groups)), channels, eps=eps)
        self.to_q = Linear(channels, channels)
        if self.context_dim is None:
            self.context_norm = None
            self.to_k = Linear(channels, channels)
            self.to_v = Linear(channels, channels)
        else:
            self.context_norm = GroupNorm(max(1, math.gcd(self.context_dim, norm_num_groups)), self.context_dim,
                                          eps=eps)
            self.to_k = Linear(self.context_dim, channels)
            self.to_v = Linear(self.context_dim, channels)
        self.to_out = nn.ModuleList([Linear(channels, channels), nn.Dropout(dropout)])
        self.attention = QKVAttention(efficient_attn=use_efficient_attn, dropout=dropout)

    def forward(self, hidden_states, context=None):
        from ...runtime.standalone import block_forward
        return block_forward(self, hidden_states, None, context if self.context_dim is not None else None)
