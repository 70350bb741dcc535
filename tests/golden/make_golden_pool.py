"""Reference fixture for EfficientUNetND(pool_factor=2) -- the patchify PoolND / UnPoolND path
(/root/reference/src/models/unet/unet.py:123-129, 280-287, nn/ops/pooling.py).  Build container only:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_pool.py

Parameters from oracle.unet.seeded_state_dict (only seeds, inputs and outputs are stored); writes
tests/golden/golden_pool.pt (tensors only, weights_only=True) + golden_pool.json."""
from __future__ import annotations

import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, "/root/reference/src")

from models.unet.unet import EfficientUNetND  # noqa: E402  (reference)

from oracle import spec as S  # noqa: E402
from oracle import unet as U  # noqa: E402

CASES = [("pool2_2d", dict(spatial_dims=2, in_channels=2, out_channels=1, layers_per_block=1,
                           block_out_channels=[32, 64], attention_resolutions=[], pool_factor=2), (2, 2, 32, 32), 800),
         ("pool2_3d", dict(spatial_dims=3, in_channels=2, out_channels=1, layers_per_block=1,
                           block_out_channels=[32, 64], attention_resolutions=[], pool_factor=2), (1, 2, 16, 16, 16),
          810)]


def main():
    out, meta = {}, {}
    for name, cfg, shape, seed in CASES:
        spec = S.derive_spec(cfg, None, 1)
        m = EfficientUNetND(spatial_dims=cfg["spatial_dims"], in_channels=2, model_channels=32, out_channels=1,
                            num_res_blocks=1, attention_resolutions=[], channel_mult=(1, 2), pool_factor=2)
        m.load_state_dict(U.seeded_state_dict(spec, seed))
        g = torch.Generator().manual_seed(seed + 1)
        x = torch.randn(*shape, generator=g)
        t = torch.tensor([3, 700][:shape[0]])
        with torch.no_grad():
            out[f"{name}/y"] = m(x, t)
        out[f"{name}/x"] = x
        out[f"{name}/t"] = t
        meta[name] = dict(cfg=cfg, seed=seed)
    torch.save(out, os.path.join(HERE, "golden_pool.pt"))
    with open(os.path.join(HERE, "golden_pool.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote golden_pool.pt")


if __name__ == "__main__":
    main()
