"""Keep masks of fmd_dropout_apply (TEST INFRASTRUCTURE ONLY).

numpy restatement of csrc/groupnorm.hip's counter-based mask: keep = mix32(key ^ index) >= p * 2^32 with
key = mix32(seed * 0x9e3779b9 + salt) and ``index`` the flat NHWC element index.  The reference draws its
ResBlockND dropout mask (src/nn/blocks/residual.py:117, nn.Dropout) from torch's generator, which no
other implementation reproduces; parity is therefore checked with the SAME mask on both sides (the engine's
mask regenerated here, applied in oracle.unet.resblock(drop=...)) plus the mask's keep rate.
"""
from __future__ import annotations

import numpy as np

M32 = np.uint64(0xFFFFFFFF)


def mix32(x):
    x = np.asarray(x, dtype=np.uint64) & M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & M32
    x ^= x >> np.uint64(16)
    return x


def keep_mask_nhwc(seed: int, salt: int, shape_nhwc, p: float) -> np.ndarray:
    key = mix32((np.uint64(seed) * np.uint64(0x9E3779B9) + np.uint64(salt)) & M32)
    idx = np.arange(int(np.prod(shape_nhwc)), dtype=np.uint64)
    thr = min(int(float(np.float32(p)) * 4294967296.0), 4294967295)   # the kernel takes p as fp32
    return (mix32(key ^ idx) >= np.uint64(thr)).reshape(shape_nhwc)
