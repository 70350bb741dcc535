"""Blocks (mirror of reference ``src/nn/blocks``)."""
from .attention import DiffusersAttentionND, SpatialCrossAttention, SpatialSelfAttention, ContextBlock
from .legacy_unet import DownBlock2DCompat, UNetMidBlock2DCompat, UpBlock2DCompat
from .residual import ResBlockND
from .timestep import TimestepBlock
from ..params import zero_module

__all__ = ["DiffusersAttentionND", "SpatialCrossAttention", "SpatialSelfAttention", "ContextBlock",
           "DownBlock2DCompat", "UNetMidBlock2DCompat", "UpBlock2DCompat", "ResBlockND", "TimestepBlock",
           "zero_module"]
