"""LDCT tensor-cache datasets (reference ``src/datasets/base.py:202-280``,
``src/datasets/ldct.py:25-113, 286-293``, ``src/utils/dataset_utils.py:398-472``).

The reference's ``LDCTDataset`` reads DICOM / npy slices, converts HU and windows them to [0, 1]
(skimage, pydicom), and caches each preprocessed slice as an fp32 ``(1, H, W)`` tensor at
``<root>/<cache_subdir>/<rel_parent>/<stem>[_split_<i>].pt``; once cached, a training epoch only
reads those files.  This module serves that cached form -- the part of the input path a training
run actually spends its time in -- with the same split-file contract (tab-separated
``Case / SDCT / LDCT`` columns in ``train.txt`` / ``test.txt``), the same cache-path rule and the
same sample dict (``{"image", "target", "img_id", "img_path", "img_size"}``, ``image`` falling back
to ``target`` without conditioning).  DICOM decoding / HU windowing stay out of scope:
an entry whose cache file is missing raises instead of silently reading something else.
Cache files are read with ``torch.load(weights_only=True)``.
"""
from __future__ import annotations

import csv
import os
from pathlib import Path
from typing import List, Optional, Sequence, Tuple

import torch
from torch.utils.data import Dataset


def cache_path_for_entry(base_path, cache_root, entry, split_index: Optional[int] = None,
                         split_count: int = 1) -> Optional[Path]:
    """``cache_root/<parent of entry relative to base_path>/<stem>[_split_<i>].pt`` (None if unresolvable).

    ``entry`` may be a path, a list of paths (first one names the file) or a dict with ``path`` / ``paths``."""
    if cache_root is None:
        return None
    if isinstance(entry, (list, tuple)):
        first = entry[0] if entry else None
    elif isinstance(entry, dict):
        first = entry.get("path")
        if first is None and isinstance(entry.get("paths"), (list, tuple)) and entry["paths"]:
            first = entry["paths"][0]
    else:
        first = entry
    if first is None:
        return None
    p = Path(str(first))
    if p.is_absolute():
        try:
            p = p.relative_to(base_path)
        except ValueError:
            p = Path(p.name)
    name = f"{p.stem}_split_{split_index}.pt" if (split_count > 1 and split_index is not None) else f"{p.stem}.pt"
    return Path(cache_root) / p.parent / name


def save_tensor_cache(tensor: torch.Tensor, cache_path) -> None:
    """Write a cache file atomically: temporary file, fsync, rename over the destination."""
    if cache_path is None:
        return
    cache_path = Path(cache_path)
    cache_path.parent.mkdir(parents=True, exist_ok=True)
    tmp = cache_path.with_suffix(cache_path.suffix + ".tmp")
    torch.save(tensor, tmp)
    try:
        with open(tmp, "rb+") as fh:
            os.fsync(fh.fileno())
    except OSError:
        pass
    os.replace(tmp, cache_path)


def _read_split(path: Path, names: Optional[Sequence[str]]) -> List[dict]:
    with open(path, newline="") as fh:
        rows = list(csv.reader(fh, delimiter="\t"))
    if not rows:
        return []
    if names is None:
        header, body = rows[0], rows[1:]
    else:
        header, body = list(names), rows
        if body and [c.strip() for c in body[0]] == list(names):   # a header line that repeats the names
            body = body[1:]
    out = []
    for r in body:
        if len(r) < len(header) or any(not c.strip() for c in r[:len(header)]):
            continue   # pandas dropna()
        out.append({h: c.strip() for h, c in zip(header, r)})
    return out


class LDCTCacheDataset(Dataset):
    """LDCT (SDCT target, LDCT conditioning) slices served from the reference's tensor cache.

    Arguments follow ``LDCTDataset`` (``src/datasets/ldct.py:29-45``): ``file_path`` = dataset root holding
    ``train.txt`` / ``test.txt``; ``load_ldct`` = conditioning on; ``names`` = split-file columns; ``cache_subdir``.
    Each split-file row is one sample (window_size 1, per-slice files)."""

    def __init__(self, file_path, train: bool = True, img_size=None, load_ldct: bool = False,
                 names: Tuple[str, ...] = ("Case", "SDCT", "LDCT"), split_file=None, cache_subdir: str = "cache",
                 **_unused):
        self.base_path = Path(file_path)
        self.train = bool(train)
        self.names = tuple(names)
        self.conditioning = bool(load_ldct)
        self.cache_root = self.base_path / cache_subdir
        self.img_size = (img_size, img_size) if isinstance(img_size, int) else (tuple(img_size) if img_size else None)
        split = Path(split_file) if split_file is not None else Path("train.txt" if self.train else "test.txt")
        if not split.is_absolute():
            split = self.base_path / split
        if not split.exists():
            raise FileNotFoundError(f"Annotations file not found: {split}")
        self.data = _read_split(split, self.names)
        self.size = len(self.data)
        if self.size == 0:
            raise ValueError("Empty Dataset")

    def __len__(self):
        return self.size

    def _load(self, entry) -> torch.Tensor:
        path = cache_path_for_entry(self.base_path, self.cache_root, entry)
        if path is None or not path.exists():
            raise FileNotFoundError(f"tensor cache entry missing for {entry!r} (expected {path}); build the cache "
                                    "with the reference's LDCTDataset(save_tensor_cache=True) first")
        return torch.as_tensor(torch.load(path, map_location="cpu", weights_only=True)).float().contiguous()

    def _load_conditioning(self, row) -> torch.Tensor:
        return self._load(row[self.names[2]])

    def __getitem__(self, idx):
        row = self.data[idx]
        tgt = self._load(row[self.names[1]])
        img = self._load_conditioning(row) if self.conditioning else None
        return {"image": img if img is not None else tgt, "target": tgt, "img_id": row.get(self.names[0]),
                "img_path": row[self.names[1]], "img_size": self.img_size}


class LDCTAttentionCacheDataset(LDCTCacheDataset):
    """``LDCTAttentionDataset`` (``ldct.py:286-293``): the conditioning column holds pre-computed latents (e.g.
    VAE encodings) that are loaded as stored, without image preprocessing -- here, straight from the cache."""


class TensorPairDataset(Dataset):
    """In-memory ``{"target", "image"}`` samples from two stacked tensors (synthetic LDCT-shaped data)."""

    def __init__(self, target: torch.Tensor, image: Optional[torch.Tensor] = None):
        self.target = target
        self.image = image

    def __len__(self):
        return self.target.shape[0]

    def __getitem__(self, i):
        t = self.target[i]
        return {"target": t, "image": self.image[i] if self.image is not None else t, "img_id": i}
