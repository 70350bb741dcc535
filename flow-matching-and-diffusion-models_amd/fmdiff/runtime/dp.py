"""Data-parallel gradient exchange.

The reference shards ``LDCTDataset`` with ``DistributedSampler``
(``flow_matching_lib.py:81``) but never synchronises gradients (only the
epoch loss is all-reduced, ``:187-192``), so its ranks drift apart.  Here the
N-rank step is defined to equal a single-process step on the concatenated
global batch: the flat fp32 gradient buffer is summed over ranks in a few
large contiguous buckets (RCCL over xGMI; ring all-reduce is per-link bound,
so few big buckets beat many small ones) and the 1/world mean is folded into
the AdamW launch (``grad_scale``), not a separate pass.
"""
from __future__ import annotations

from typing import List, Tuple

import torch
import torch.distributed as dist


def world_size(group=None) -> int:
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def bucket_bounds(n: int, buckets: int) -> List[Tuple[int, int]]:
    """Contiguous [lo, hi) ranges covering n elements in at most ``buckets`` equal pieces."""
    buckets = max(1, int(buckets))
    per = -(-n // buckets) if n else 0
    return [(lo, min(n, lo + per)) for lo in range(0, n, per)] if per else []


def bucketed_allreduce(flat: torch.Tensor, buckets: int = 4, group=None) -> None:
    """In-place SUM all-reduce of a flat buffer, bucket by bucket (no-op at world 1)."""
    if world_size(group) <= 1:
        return
    for lo, hi in bucket_bounds(flat.numel(), buckets):
        dist.all_reduce(flat[lo:hi], op=dist.ReduceOp.SUM, group=group)


def bucketed_allreduce_async(flat: torch.Tensor, buckets: int = 2, group=None) -> list:
    """Start in-place SUM all-reduces of ``flat`` (bucket by bucket) without making the current stream wait:
    compute issued afterwards overlaps them; call ``.wait()`` on every returned work before reading ``flat``."""
    if world_size(group) <= 1:
        return []
    return [dist.all_reduce(flat[lo:hi], op=dist.ReduceOp.SUM, group=group, async_op=True)
            for lo, hi in bucket_bounds(flat.numel(), buckets)]

