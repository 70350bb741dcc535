from __future__ import annotations

import math

from ...blocks.attention import SpatialSelfAttention


def attention_layer(channels: int, attn_heads, attn_dim_head) -> SpatialSelfAttention:
    """``_build_attention_layer`` of the reference encoder / decoder (encoder.py:123-137, decoder.py:117-131)."""
    heads = attn_heads if attn_heads is not None else 1
    if attn_dim_head is not None:
        dim_head = attn_dim_head
    elif heads == 1:
        dim_head = channels
    else:
        dim_head = max(1, channels // heads)
    return SpatialSelfAttention(dim=channels, heads=heads, dim_head=dim_head, use_linear=False,
                                use_efficient_attn=True)


def out_groups(channels: int, norm_groups) -> int:
    return norm_groups if norm_groups is not None else max(1, math.gcd(channels, 32))
