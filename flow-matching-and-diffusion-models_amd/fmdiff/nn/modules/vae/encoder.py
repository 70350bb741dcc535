"""``Encoder`` (reference ``src/nn/modules/vae/encoder.py:19-158``): same constructor, attributes and
state_dict keys.  ``forward`` runs the whole encoder through the fused HIP engine
(``fmdiff.runtime.vae_engine``)."""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch.nn as nn

from ...blocks.residual import ResBlockND
from ...ops.convolution import ConvND
from ...ops.upsampling import DownsampleND
from ...params import GroupNorm, Identity
from ._common import attention_layer, out_groups


class Encoder(nn.Module):
    def __init__(self, in_channels: int = 3, base_ch: int = 128, ch_mult: Tuple[int, ...] = (1, 2, 4, 4),
                 down_channels: Optional[Tuple[int, ...]] = None, num_res_blocks: int = 2,
                 attn_resolutions: Tuple[int, ...] = (), resolution: int = 256, z_channels: int = 4,
                 dropout: float = 0.0, use_attention: bool = True, attn_heads: Optional[int] = None,
                 attn_dim_head: Optional[int] = None, double_z: bool = True, spatial_dims: int = 2,
                 emb_channels: Optional[int] = None, use_scale_shift_norm: bool = False,
                 norm_groups: Optional[int] = None, block_factory=None) -> None:
        super().__init__()
        self.resolution = resolution
        self.double_z = double_z
        self.z_channels = z_channels
        self.spatial_dims = spatial_dims
        self.emb_channels = emb_channels
        self.use_attention = use_attention
        self.attn_heads = attn_heads
        self.attn_dim_head = attn_dim_head
        self.use_scale_shift_norm = use_scale_shift_norm and emb_channels is not None
        if emb_channels is None and use_scale_shift_norm:
            raise ValueError("use_scale_shift_norm requires emb_channels to be provided.")
        channels = tuple(down_channels) if down_channels is not None else tuple(base_ch * m for m in ch_mult)
        self.conv_in = ConvND(spatial_dims, in_channels, base_ch, 3, padding=1)
        curr_res, in_ch = resolution, base_ch
        downs: List[nn.Module] = []
        for idx, out_ch in enumerate(channels):
            blocks, attns = [], []
            for _ in range(num_res_blocks):
                factory = block_factory or ResBlockND
                blocks.append(factory(channels=in_ch, emb_channels=emb_channels, dropout=dropout,
                                      out_channels=out_ch, use_conv=False,
                                      use_scale_shift_norm=self.use_scale_shift_norm, spatial_dims=spatial_dims))
                in_ch = out_ch
                if use_attention and curr_res in attn_resolutions:
                    attns.append(attention_layer(in_ch, attn_heads, attn_dim_head))
            stage = nn.Module()
            stage.blocks = nn.ModuleList(blocks)
            stage.attns = nn.ModuleList(attns)
            if idx != len(channels) - 1:
                stage.down = DownsampleND(spatial_dims, in_ch, use_conv=True)
                curr_res //= 2
            downs.append(stage)
        self.downs = nn.ModuleList(downs)
        mk = lambda: ResBlockND(channels=in_ch, emb_channels=emb_channels, dropout=dropout, out_channels=in_ch,
                                use_conv=False, use_scale_shift_norm=self.use_scale_shift_norm,
                                spatial_dims=spatial_dims)
        self.mid_block1 = mk()
        self.mid_attn = attention_layer(in_ch, attn_heads, attn_dim_head) if use_attention else Identity()
        self.mid_block2 = mk()
        self.norm_out = GroupNorm(out_groups(in_ch, norm_groups), in_ch)
        self.conv_out = ConvND(spatial_dims, in_ch, 2 * z_channels if double_z else z_channels, 3, padding=1)

    def forward(self, x):
        from ....runtime.vae_engine import get_vae_engine
        return get_vae_engine(self).encoder_forward(x)
