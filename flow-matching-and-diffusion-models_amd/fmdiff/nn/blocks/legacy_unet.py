"""Diffusers-compat down / up / mid blocks (reference ``src/nn/blocks/legacy_unet.py:11-231``)."""
from __future__ import annotations

import torch.nn as nn

from ..ops.upsampling import DownsampleND, UpsampleND
from .attention import DiffusersAttentionND
from .residual import ResBlockND


def _res(spatial_dims, cin, temb, cout, dropout, time_scale_shift, groups, eps):
    return ResBlockND(spatial_dims=spatial_dims, channels=cin, emb_channels=temb, out_channels=cout, dropout=dropout,
                      use_conv=False, use_scale_shift_norm=(time_scale_shift == "scale_shift"), norm_type="gn",
                      norm_groups=groups, norm_eps=eps, zero_init_last_conv=False, emb_activation_before_proj=True,
                      add_embedding_to_hidden=True)


class DownBlock2DCompat(nn.Module):
    def __init__(self, spatial_dims, num_layers, in_channels, out_channels, temb_channels, add_downsample, eps, groups,
                 dropout, time_scale_shift, with_attention=False, attention_head_dim=8, cross_attention_dim=None):
        super().__init__()
        self.resnets = nn.ModuleList()
        self.attentions = nn.ModuleList() if with_attention else None
        heads = max(1, out_channels // max(attention_head_dim, 1))
        ch = in_channels
        for _ in range(num_layers):
            self.resnets.append(_res(spatial_dims, ch, temb_channels, out_channels, dropout, time_scale_shift, groups,
                                     eps))
            if with_attention:
                self.attentions.append(DiffusersAttentionND(out_channels, heads=heads, context_dim=cross_attention_dim,
                                                            eps=eps, norm_num_groups=groups))
            ch = out_channels
        self.downsamplers = nn.ModuleList([DownsampleND(spatial_dims, out_channels, use_conv=True)]) \
            if add_downsample else None


class UpBlock2DCompat(nn.Module):
    def __init__(self, spatial_dims, num_layers, in_channels, out_channels, prev_output_channel, temb_channels,
                 add_upsample, eps, groups, dropout, time_scale_shift, with_attention=False, attention_head_dim=8,
                 cross_attention_dim=None):
        super().__init__()
        self.resnets = nn.ModuleList()
        self.attentions = nn.ModuleList() if with_attention else None
        heads = max(1, out_channels // max(attention_head_dim, 1))
        for i in range(num_layers):
            skip = in_channels if i == num_layers - 1 else out_channels
            rin = prev_output_channel if i == 0 else out_channels
            self.resnets.append(_res(spatial_dims, rin + skip, temb_channels, out_channels, dropout, time_scale_shift,
                                     groups, eps))
            if with_attention:
                self.attentions.append(DiffusersAttentionND(out_channels, heads=heads, context_dim=cross_attention_dim,
                                                            eps=eps, norm_num_groups=groups))
        self.upsamplers = nn.ModuleList([UpsampleND(spatial_dims, out_channels, use_conv=True)]) \
            if add_upsample else None


class UNetMidBlock2DCompat(nn.Module):
    def __init__(self, spatial_dims, in_channels, temb_channels, eps, groups, dropout, time_scale_shift,
                 add_attention=True, attention_head_dim=8, cross_attention_dim=None):
        super().__init__()
        heads = max(1, in_channels // max(attention_head_dim, 1))
        self.resnets = nn.ModuleList([
            _res(spatial_dims, in_channels, temb_channels, in_channels, dropout, time_scale_shift, groups, eps)
            for _ in range(2)])
        self.attentions = nn.ModuleList([DiffusersAttentionND(in_channels, heads=heads,
                                                              context_dim=cross_attention_dim, eps=eps,
                                                              norm_num_groups=groups)]) if add_attention else None
