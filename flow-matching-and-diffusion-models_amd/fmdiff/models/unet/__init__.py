from .base import BaseUNetND
from .unet import EfficientUNetND, TimestepEmbedSequential
from .unet_diffusers_nd import UNetDiffusersND, UNetExactND

__all__ = ["BaseUNetND", "EfficientUNetND", "TimestepEmbedSequential", "UNetDiffusersND", "UNetExactND"]
