"""Order-independent seeded parameter fill shared by golden generators and the GPU tests (test infrastructure).

Large fixtures (config D's 84 M-parameter VAE, config E's 308 M-parameter 3-D UNet) cannot store their weights,
so both sides regenerate them: every parameter is drawn from a CPU ``torch.Generator`` seeded by
(seed, crc32(name)), so the values depend only on the parameter's name and shape, never on module order.

Rule (every path non-degenerate, activations O(1) through deep stacks):
* GroupNorm / norm weights: 1 + 0.1 N(0,1);  other 1-D tensors (biases, norm shifts): 0.05 N(0,1);
* >= 2-D weights: N(0,1) / sqrt(fan_in) with fan_in = numel / shape[0] (zero-initialised layers of the
  reference -- conv2 of each ResBlock, proj_out, the head -- are filled too, so their paths are exercised).
"""
from __future__ import annotations

import math
import zlib
from typing import Dict, Iterable, Tuple

import torch


def _is_norm_weight(name: str) -> bool:
    leaf = name.rsplit(".", 1)[0].rsplit(".", 1)[-1]
    return name.endswith(".weight") and ("norm" in leaf or leaf.startswith("gn"))


def seeded_tensor(name: str, shape: Tuple[int, ...], seed: int) -> torch.Tensor:
    g = torch.Generator().manual_seed((int(seed) * 1000003 + zlib.crc32(name.encode())) & 0x7FFFFFFF)
    r = torch.randn(tuple(shape), generator=g)
    if len(shape) <= 1:
        return 1.0 + 0.1 * r if _is_norm_weight(name) else 0.05 * r
    fan = math.prod(shape[1:])
    return r / math.sqrt(max(fan, 1))


def seeded_params(named_shapes: Iterable[Tuple[str, Tuple[int, ...]]], seed: int) -> Dict[str, torch.Tensor]:
    return {k: seeded_tensor(k, tuple(s), seed) for k, s in named_shapes}


def fill_module(module: torch.nn.Module, seed: int) -> Dict[str, torch.Tensor]:
    """Fill every parameter of ``module`` in place by the rule above; returns the values (CPU)."""
    vals = seeded_params(((k, tuple(p.shape)) for k, p in module.named_parameters()), seed)
    with torch.no_grad():
        for k, p in module.named_parameters():
            p.copy_(vals[k].to(p.device))
    return vals
