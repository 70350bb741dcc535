"""Dimension-agnostic ops (mirror of reference ``src/nn/ops``)."""
from .convolution import ConvND
from .normalization import make_group_norm
from .time_embedding import timestep_embedding
from .upsampling import UpsampleND, DownsampleND

__all__ = ["ConvND", "make_group_norm", "timestep_embedding", "UpsampleND", "DownsampleND"]
