"""Building blocks with the reference ``src/nn`` module / state_dict API."""
from .params import Conv, GroupNorm, Linear, zero_module
