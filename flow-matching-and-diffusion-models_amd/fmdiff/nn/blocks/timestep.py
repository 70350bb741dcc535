"""Marker base for blocks that take the timestep embedding (reference ``src/nn/blocks/timestep.py:13-23``)."""
import torch.nn as nn


class TimestepBlock(nn.Module):
    pass
