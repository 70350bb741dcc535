"""``ResBlockND`` (reference ``src/nn/blocks/residual.py:13-140``).

Same constructor, attributes and state_dict keys.  On the GPU the whole block
runs as two fused implicit-GEMM convolutions: GN1+SiLU feed conv1's gather,
GN2 + time-embedding scale/shift (or add) + SiLU feed conv2's gather, and the
identity / 1x1 skip and residual add live in conv2's epilogue
(``fmdiff.runtime.engine``)."""
from __future__ import annotations

from typing import Optional

import torch.nn as nn

from ..ops.convolution import ConvND
from ..ops.normalization import make_group_norm
from ..params import Identity, Linear, SiLU, zero_module
from .timestep import TimestepBlock


class ResBlockND(TimestepBlock):
    def __init__(self, channels: int, emb_channels: Optional[int], dropout: float, out_channels: int = None,
                 use_conv: bool = False, use_scale_shift_norm: bool = False, spatial_dims: int = 2,
                 norm_type: str = "gn", act: str = "silu", norm_groups: int = 32, norm_eps: float = 1e-5,
                 zero_init_last_conv: bool = True, emb_activation_before_proj: bool = False,
                 add_embedding_to_hidden: bool = False):
        super().__init__()
        if norm_type.lower() != "gn" or act.lower() not in ("silu", "swish"):
            raise NotImplementedError("fmdiff fuses GroupNorm + SiLU; other norm/act pairs are off the hot path")
        self.channels = channels
        self.emb_channels = emb_channels
        self.dropout = dropout
        self.out_channels = out_channels or channels
        self.use_conv = use_conv
        self.use_scale_shift_norm = use_scale_shift_norm and emb_channels is not None
        self.uses_embedding = emb_channels is not None
        self.emb_activation_before_proj = emb_activation_before_proj
        self.add_embedding_to_hidden = add_embedding_to_hidden
        self.spatial_dims = spatial_dims
        if emb_channels is None and use_scale_shift_norm:
            raise ValueError("use_scale_shift_norm requires emb_channels to be provided.")
        self.norm1 = make_group_norm(channels, norm_groups, norm_eps)
        self.act1 = SiLU()
        self.conv1 = ConvND(spatial_dims, channels, self.out_channels, 3, padding=1)
        if self.uses_embedding:
            self.emb_act = SiLU()
            self.emb_layers = Linear(emb_channels, 2 * self.out_channels if self.use_scale_shift_norm
                                     else self.out_channels)
        else:
            self.emb_layers = None
        self.norm2 = make_group_norm(self.out_channels, norm_groups, norm_eps)
        self.act2 = SiLU()
        self.dropout_layer = nn.Dropout(p=dropout)
        self.conv2 = ConvND(spatial_dims, self.out_channels, self.out_channels, 3, padding=1)
        if zero_init_last_conv:
            self.conv2 = zero_module(self.conv2)
        if self.out_channels == channels:
            self.skip_connection = Identity()
        elif use_conv:
            self.skip_connection = ConvND(spatial_dims, channels, self.out_channels, 3, padding=1)
        else:
            self.skip_connection = ConvND(spatial_dims, channels, self.out_channels, 1)

    def forward(self, x, emb=None):
        from ...runtime.standalone import block_forward
        return block_forward(self, x, emb)
