"""Host -> device batch pipeline: pinned staging buffers and a side HIP stream.

The reference copies each batch with ``.to(device, non_blocking=True)`` at the top of the step
(``flow_matching_lib.py:139-141``); with DataLoader ``pin_memory`` that copy still runs on the compute
stream, in front of the step's kernels.  ``DevicePrefetcher`` instead keeps a ring of pinned host
buffers and device buffers per field: batch i+1 is staged into pinned memory and copied on a separate
stream while step i computes, and the compute stream waits only on that batch's copy event.  Device
buffers are reused (a ring of ``depth``), so a captured train step can read a batch without new
allocations; a slot's copy is ordered after the compute work already queued when it is staged, which
includes the step that last read that slot.
"""
from __future__ import annotations

from typing import Dict, Iterable, Iterator, Optional

import torch

FIELDS = ("target", "image")


class DevicePrefetcher:
    """Iterate ``loader`` (yielding dicts with tensor ``target`` / ``image`` entries, ``image`` may be None) and
    yield the same dicts with those tensors on ``device``, one batch ahead, copied on a side stream."""

    def __init__(self, loader: Iterable, device, depth: int = 2, fields=FIELDS):
        self.loader = loader
        self.device = torch.device(device)
        self.depth = max(2, int(depth))
        self.fields = tuple(fields)
        self._stream = torch.cuda.Stream(device=self.device)
        self._host: Dict[tuple, torch.Tensor] = {}
        self._dev: Dict[tuple, torch.Tensor] = {}
        self._copied = [None] * self.depth     # side-stream event after slot i's last host -> device copy

    def _buf(self, pool, key, like: torch.Tensor, pinned: bool):
        b = pool.get(key)
        if b is None or b.shape != like.shape or b.dtype != like.dtype:
            if pinned:
                b = torch.empty(like.shape, dtype=like.dtype, pin_memory=True)
            else:
                b = torch.empty(like.shape, dtype=like.dtype, device=self.device)
            pool[key] = b
        return b

    def _stage(self, batch: dict, slot: int):
        out = dict(batch)
        if self._copied[slot] is not None:   # the pinned buffers of this slot are free once their copy landed
            self._copied[slot].synchronize()
        pairs = []
        for f in self.fields:   # buffers come from the compute stream's pool: a replaced one is freed in its order
            t = batch.get(f)
            if torch.is_tensor(t):
                h = self._buf(self._host, (f, slot), t, pinned=True)
                h.copy_(t)
                d = self._buf(self._dev, (f, slot), t, pinned=False)
                pairs.append((d, h))
                out[f] = d
        # the copy is ordered after every kernel already queued on the compute stream: that covers the step
        # that last read this slot (batch i-1, staged while batch i is still to be issued) and any earlier user
        # of freshly allocated memory, and still overlaps step i
        self._stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self._stream):
            for d, h in pairs:
                d.copy_(h, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self._stream)
        self._copied[slot] = ev
        return out, ev

    def __iter__(self) -> Iterator[dict]:
        it = iter(self.loader)
        slot = 0
        try:
            nxt = self._stage(next(it), slot)
        except StopIteration:
            return
        while nxt is not None:
            batch, ev = nxt
            slot = (slot + 1) % self.depth
            try:
                nxt = self._stage(next(it), slot)   # overlaps the consumer's step on `batch`
            except StopIteration:
                nxt = None
            torch.cuda.current_stream(self.device).wait_event(ev)
            yield batch

    def __len__(self):
        return len(self.loader)
