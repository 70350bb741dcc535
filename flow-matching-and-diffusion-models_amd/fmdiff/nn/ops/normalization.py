"""Group-norm factory (reference ``src/nn/ops/normalization.py:11-19``)."""
from __future__ import annotations

from ..params import GroupNorm


def group_count(channels: int, groups: int = 32) -> int:
    g = min(groups, channels)
    while channels % g != 0 and g > 1:
        g -= 1
    return g


def make_group_norm(channels: int, groups: int = 32, eps: float = 1e-5) -> GroupNorm:
    """GroupNorm with the largest group count <= ``groups`` that divides ``channels``."""
    return GroupNorm(group_count(channels, groups), channels, eps=eps)
