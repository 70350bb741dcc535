"""Order-sensitive fingerprints of large per-parameter tensors (gradients, AdamW deltas) for the golden fixtures.

Sums and norms are permutation-invariant: a tap- or channel-permuted weight gradient passes both.  These
fingerprints are not:

* ``projections``: for each tensor i and k < NPROJ, <t_i, r_k[seg_i]> with r_k a seeded Rademacher (+-1)
  vector over the concatenation of all tensors (torch.Generator on the CPU, so the GPU tests regenerate the
  same signs).  By Johnson-Lindenstrauss the cosine of two tensors' 8-vectors tracks their full cosine;
  a permuted tensor gives ~0.
* ``strided_sample``: every STRIDE-th element of the same concatenation (element-wise comparison of a
  fixed 1/STRIDE subset).

Shared by tests/golden/make_golden_steps.py / make_golden_b256.py (generation) and tests/test_gpu_unet.py /
tests/test_gpu_ddpm.py (checks).  Test infrastructure only.
"""
from __future__ import annotations

from typing import List, Sequence

import torch

NPROJ = 8
STRIDE = 397


def _flat(tensors: Sequence[torch.Tensor]) -> torch.Tensor:
    return torch.cat([t.detach().reshape(-1).double().cpu() for t in tensors])


def projections(tensors: Sequence[torch.Tensor], seed: int) -> torch.Tensor:
    """[len(tensors)][NPROJ] float64 Rademacher projections of each tensor."""
    numels = [t.numel() for t in tensors]
    flat = _flat(tensors)
    out = torch.empty(len(tensors), NPROJ, dtype=torch.float64)
    for k in range(NPROJ):
        g = torch.Generator().manual_seed(seed * 100 + k)
        r = torch.randint(0, 2, (flat.numel(),), generator=g, dtype=torch.int8)
        prod = torch.where(r.bool(), flat, -flat)
        out[:, k] = torch.stack([s.sum() for s in prod.split(numels)])
        del r, prod
    return out


def strided_sample(tensors: Sequence[torch.Tensor]) -> torch.Tensor:
    """float64 elements 0, STRIDE, 2*STRIDE, ... of the concatenation."""
    return _flat(tensors)[::STRIDE].clone()


def sample_segments(numels: Sequence[int]) -> List[slice]:
    """Slice of strided_sample's output that belongs to each tensor."""
    out, off = [], 0
    for n in numels:
        lo = -(-off // STRIDE)
        hi = -(-(off + n) // STRIDE)
        out.append(slice(lo, hi))
        off += n
    return out


def cosine(a: torch.Tensor, b: torch.Tensor) -> float:
    a, b = a.double().flatten(), b.double().flatten()
    return float((a @ b) / (a.norm() * b.norm() + 1e-300))
