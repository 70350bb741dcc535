"""``UNetDiffusersND`` (reference ``src/models/unet/unet_diffusers_nd.py:19-191``): identical
constructor, module tree and state_dict keys; executed by the fused HIP engine."""
from __future__ import annotations

from typing import Sequence

import torch
import torch.nn as nn

from ...nn.blocks.legacy_unet import DownBlock2DCompat, UNetMidBlock2DCompat, UpBlock2DCompat
from ...nn.ops.convolution import ConvND
from ...nn.ops.normalization import make_group_norm
from ...nn.params import SiLU
from .base import BaseUNetND
from .utils import TimestepEmbedding


class UNetDiffusersND(BaseUNetND):
    def __init__(self, spatial_dims: int = 2, sample_size=None, in_channels: int = 3, out_channels: int = 3,
                 center_input_sample: bool = False, time_embedding_type: str = "positional", freq_shift: int = 0,
                 flip_sin_to_cos: bool = True,
                 down_block_types: Sequence[str] = ("DownBlock2D", "AttnDownBlock2D", "AttnDownBlock2D",
                                                    "AttnDownBlock2D"),
                 mid_block_type: str | None = "UNetMidBlock2D",
                 up_block_types: Sequence[str] = ("AttnUpBlock2D", "AttnUpBlock2D", "AttnUpBlock2D", "UpBlock2D"),
                 block_out_channels: Sequence[int] = (224, 448, 672, 896), layers_per_block: int = 2,
                 downsample_padding: int = 1, dropout: float = 0.0, attention_head_dim: int = 8,
                 norm_num_groups: int = 32, norm_eps: float = 1e-5, resnet_time_scale_shift: str = "default",
                 add_attention: bool = True, cross_attention_dim: int | None = None, **_kwargs):
        super().__init__()
        if time_embedding_type != "positional":
            raise ValueError("UNetDiffusersND currently supports positional time embedding only for strict compat.")
        self.center_input_sample = center_input_sample
        self.sample_size = sample_size
        self.time_embedding_type = time_embedding_type
        self.flip_sin_to_cos = flip_sin_to_cos
        self.freq_shift = freq_shift
        self.block_out_channels = tuple(block_out_channels)
        self.cross_attention_dim = int(cross_attention_dim) if cross_attention_dim is not None else None
        self.norm_num_groups = norm_num_groups
        self.norm_eps = norm_eps
        ted = self.block_out_channels[0] * 4
        self.conv_in = ConvND(spatial_dims, in_channels, self.block_out_channels[0], kernel_size=3, padding=1).conv
        self.time_proj_dim = self.block_out_channels[0]
        self.time_embedding = TimestepEmbedding(self.time_proj_dim, ted)
        self.class_embedding = None
        self.down_blocks = nn.ModuleList()
        self.up_blocks = nn.ModuleList()
        out_c = self.block_out_channels[0]
        for i, t in enumerate(down_block_types):
            in_c = out_c
            out_c = self.block_out_channels[i]
            final = i == len(self.block_out_channels) - 1
            if t not in {"DownBlock2D", "AttnDownBlock2D", "CrossAttnDownBlock2D"}:
                raise ValueError(f"Unsupported down block type in compat model: {t}")
            self.down_blocks.append(DownBlock2DCompat(
                spatial_dims=spatial_dims, num_layers=layers_per_block, in_channels=in_c, out_channels=out_c,
                temb_channels=ted, add_downsample=not final, eps=norm_eps, groups=norm_num_groups, dropout=dropout,
                time_scale_shift=resnet_time_scale_shift, with_attention=t in {"AttnDownBlock2D", "CrossAttnDownBlock2D"},
                attention_head_dim=attention_head_dim,
                cross_attention_dim=self.cross_attention_dim if t == "CrossAttnDownBlock2D" else None))
        self.mid_block = None if mid_block_type is None else UNetMidBlock2DCompat(
            spatial_dims=spatial_dims, in_channels=self.block_out_channels[-1], temb_channels=ted, eps=norm_eps,
            groups=norm_num_groups, dropout=dropout, time_scale_shift=resnet_time_scale_shift,
            add_attention=add_attention, attention_head_dim=attention_head_dim,
            cross_attention_dim=self.cross_attention_dim if mid_block_type == "UNetMidBlock2DCrossAttn" else None)
        rev = list(reversed(self.block_out_channels))
        out_c = rev[0]
        for i, t in enumerate(up_block_types):
            prev = out_c
            out_c = rev[i]
            in_c = rev[min(i + 1, len(self.block_out_channels) - 1)]
            final = i == len(self.block_out_channels) - 1
            if t not in {"UpBlock2D", "AttnUpBlock2D", "CrossAttnUpBlock2D"}:
                raise ValueError(f"Unsupported up block type in compat model: {t}")
            self.up_blocks.append(UpBlock2DCompat(
                spatial_dims=spatial_dims, num_layers=layers_per_block + 1, in_channels=in_c, out_channels=out_c,
                prev_output_channel=prev, temb_channels=ted, add_upsample=not final, eps=norm_eps,
                groups=norm_num_groups, dropout=dropout, time_scale_shift=resnet_time_scale_shift,
                with_attention=t in {"AttnUpBlock2D", "CrossAttnUpBlock2D"}, attention_head_dim=attention_head_dim,
                cross_attention_dim=self.cross_attention_dim if t == "CrossAttnUpBlock2D" else None))
        self.conv_norm_out = make_group_norm(self.block_out_channels[0], groups=norm_num_groups, eps=norm_eps)
        self.conv_act = SiLU()
        self.conv_out = ConvND(spatial_dims, self.block_out_channels[0], out_channels, kernel_size=3, padding=1).conv

    def _prepare_input(self, x, context=None, context_ca=None):
        if context is not None:
            x = torch.cat([x, context], dim=1)
        if self.center_input_sample:
            x = 2 * x - 1.0
        return x


UNetExactND = UNetDiffusersND
