"""``EfficientUNetND`` (reference ``src/models/unet/unet.py:42-326``): identical constructor,
module tree and state_dict keys; executed by the fused HIP engine."""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import torch
import torch.nn as nn

from ...nn.blocks.attention import ContextBlock, SpatialCrossAttention, SpatialSelfAttention
from ...nn.blocks.residual import ResBlockND
from ...nn.blocks.timestep import TimestepBlock
from ...nn.ops.convolution import ConvND
from ...nn.ops.normalization import make_group_norm
from ...nn.ops.pooling import PoolND, UnPoolND
from ...nn.ops.upsampling import DownsampleND, UpsampleND
from ...nn.params import Identity, Linear, SiLU, zero_module
from .base import BaseUNetND


class TimestepEmbedSequential(nn.Sequential, TimestepBlock):
    """Sequential whose children get (x, emb, context) as they need (reference ``unet.py:18-39``)."""


class EfficientUNetND(BaseUNetND):
    def __init__(self, spatial_dims: int, in_channels: int, model_channels: int, out_channels: int,
                 num_res_blocks: int, attention_resolutions: Sequence[int], dropout: float = 0.0,
                 channel_mult: Tuple[int, ...] = (1, 2, 3, 4), conv_resample: bool = True, dim_head: int = 64,
                 num_heads: int = 4, use_linear_attn: bool = True, use_scale_shift_norm: bool = True,
                 pool_factor: int = 1, cross_attention_resolutions: Optional[Sequence[int]] = None,
                 cross_attention_dim: int = 4, cross_attention_in_middle: bool = False,
                 emb_activation_before_proj: bool = False):
        super().__init__()
        if spatial_dims not in (1, 2, 3):
            raise ValueError("spatial_dims must be 1, 2 or 3")
        self.spatial_dims = spatial_dims
        self.in_channels = in_channels
        self.model_channels = model_channels
        self.out_channels = out_channels
        self.num_res_blocks = num_res_blocks
        self.attention_resolutions = tuple(attention_resolutions)
        self.cross_attention_resolutions = tuple(cross_attention_resolutions or ())
        self.dropout = dropout
        self.channel_mult = channel_mult
        self.conv_resample = conv_resample
        self.num_heads = num_heads
        self.pool_factor = pool_factor
        self.cross_attention_dim = cross_attention_dim
        self.cross_attention_in_middle = cross_attention_in_middle
        self.emb_activation_before_proj = emb_activation_before_proj

        ted = model_channels * 4
        self.time_embed = nn.Sequential(Linear(model_channels, ted), SiLU(), Linear(ted, ted))
        # optional input pooling (patchify, reference unet.py:123-129)
        if pool_factor > 1:
            self.pool = PoolND(spatial_dims, in_channels, model_channels, pool_factor)
            start_channels = model_channels
        else:
            self.pool = Identity()
            start_channels = in_channels

        def res(cin, cout=None):
            return ResBlockND(spatial_dims=spatial_dims, channels=cin, emb_channels=ted, out_channels=cout,
                              dropout=dropout, use_scale_shift_norm=use_scale_shift_norm,
                              emb_activation_before_proj=emb_activation_before_proj)

        def attn_layers(ch, ds, linear):
            out = []
            if ds in self.attention_resolutions:
                out.append(SpatialSelfAttention(dim=ch, heads=num_heads, dim_head=dim_head, use_linear=linear,
                                                use_efficient_attn=True))
            if ds in self.cross_attention_resolutions:
                out.append(SpatialCrossAttention(dim=ch, context_dim=cross_attention_dim, heads=num_heads,
                                                 dim_head=dim_head, use_linear=linear, use_efficient_attn=True))
            return out

        self.input_blocks = nn.ModuleList([TimestepEmbedSequential(ConvND(spatial_dims, start_channels,
                                                                          model_channels, 3, padding=1))])
        chans = [model_channels]
        ch = model_channels
        ds = 1
        for level, mult in enumerate(channel_mult):
            for _ in range(num_res_blocks):
                layers = [res(ch, mult * model_channels)]
                ch = mult * model_channels
                layers += attn_layers(ch, ds, use_linear_attn)
                self.input_blocks.append(TimestepEmbedSequential(*layers))
                chans.append(ch)
            if level != len(channel_mult) - 1:
                self.input_blocks.append(TimestepEmbedSequential(DownsampleND(spatial_dims, ch,
                                                                              use_conv=conv_resample)))
                chans.append(ch)
                ds *= 2
        mid = [res(ch), SpatialSelfAttention(ch, heads=num_heads, dim_head=dim_head, use_linear=False,
                                             use_efficient_attn=True)]
        if cross_attention_in_middle or ds in self.cross_attention_resolutions:
            mid.append(SpatialCrossAttention(dim=ch, context_dim=cross_attention_dim, heads=num_heads,
                                             dim_head=dim_head, use_linear=False, use_efficient_attn=True))
        mid.append(res(ch))
        self.middle_block = TimestepEmbedSequential(*mid)
        self.output_blocks = nn.ModuleList([])
        for level, mult in list(enumerate(channel_mult))[::-1]:
            for i in range(num_res_blocks + 1):
                layers = [res(ch + chans.pop(), model_channels * mult)]
                ch = model_channels * mult
                layers += attn_layers(ch, ds, use_linear_attn)
                if level and i == num_res_blocks:
                    layers.append(UpsampleND(spatial_dims, ch, use_conv=conv_resample))
                    ds //= 2
                self.output_blocks.append(TimestepEmbedSequential(*layers))
        if pool_factor > 1:   # reference unet.py:280-287: the head keeps model_channels, UnPoolND projects
            self.out = nn.Sequential(make_group_norm(ch, groups=32), SiLU(),
                                     ConvND(spatial_dims, model_channels, model_channels, 3, padding=1))
            self.unpool = UnPoolND(spatial_dims, model_channels, out_channels, pool_factor)
        else:
            self.out = nn.Sequential(make_group_norm(ch, groups=32), SiLU(),
                                     zero_module(ConvND(spatial_dims, model_channels, out_channels, 3, padding=1)))
            self.unpool = Identity()

    def _prepare_input(self, x, context, context_ca):
        if context_ca is not None and not (self.cross_attention_resolutions or self.cross_attention_in_middle):
            raise ValueError("context_ca provided but cross-attention is disabled.")
        if context is not None:
            x = torch.cat([x, context], dim=1)
        return x
