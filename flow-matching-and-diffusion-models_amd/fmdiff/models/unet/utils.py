"""Time-embedding MLP module (reference ``src/models/unet/utils.py:9-41``)."""
from __future__ import annotations

import torch.nn as nn

from ...nn.ops.time_embedding import timestep_embedding
from ...nn.params import Linear, SiLU


class TimestepEmbedding(nn.Module):
    def __init__(self, in_channels: int, out_channels: int):
        super().__init__()
        self.linear_1 = Linear(in_channels, out_channels)
        self.act = SiLU()
        self.linear_2 = Linear(out_channels, out_channels)


def build_timestep_features(timesteps, channels, *, max_period=10000, flip_sin_to_cos=True, freq_shift=0):
    return timestep_embedding(timesteps, channels, max_period=max_period, flip_sin_to_cos=flip_sin_to_cos,
                              freq_shift=freq_shift)
