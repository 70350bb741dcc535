"""Generate the AutoencoderKL golden fixture from the reference itself (config D).

Run in the build container only (the reference never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_vae_golden.py

Builds the reference ``models.vae.AutoencoderKL`` from ``/root/reference/src`` (pure PyTorch, CPU, fp32)
at a reduced width of the ``configs/LDCT/LDCT_autoencoder_kl.json`` layout (1 channel, 3 levels, mid
attention with 4 heads x 16), fills every parameter from a seeded normal (the reference zero-inits
conv2 / proj_out, which would hide those paths), and records encode moments / ``posterior.mode()`` and
``decode`` outputs.  Writes ``tests/golden/vae_golden.pt`` (tensors + the config as JSON text; load with
``weights_only=True``).
"""
from __future__ import annotations

import json
import math
import os
import sys
import warnings

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join("/root/reference", "src"))

from models.vae import AutoencoderKL  # noqa: E402  (reference)

CFG = dict(in_channels=1, out_channels=1, resolution=32, base_ch=32, down_channels=[32, 64, 64], num_res_blocks=1,
           attn_resolutions=[], z_channels=4, embed_dim=4, dropout=0.0, use_attention=True, spatial_dims=2,
           emb_channels=None, use_scale_shift_norm=False, double_z=True, attn_heads=4, attn_dim_head=16)


def main():
    torch.manual_seed(0)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        vae = AutoencoderKL(**CFG).eval()
    g = torch.Generator().manual_seed(1234)
    with torch.no_grad():
        for name, p in vae.named_parameters():
            fan = p[0].numel() if p.dim() > 1 else 1
            if name.endswith("norm1.weight") or name.endswith("norm2.weight") or ".norm" in name and name.endswith("weight"):
                p.copy_(1.0 + 0.1 * torch.randn(p.shape, generator=g))
            elif p.dim() == 1:
                p.copy_(0.05 * torch.randn(p.shape, generator=g))
            else:
                p.copy_(torch.randn(p.shape, generator=g) / math.sqrt(fan))
    x = torch.rand(2, 1, 32, 32, generator=g)
    with torch.no_grad():
        post = vae.encode(vae.image_to_model_range(x), normalize=False)
        moments = torch.cat([post.mu, post.logvar], 1)   # logvar clamped as the reference stores it
        z = torch.randn(2, 4, 8, 8, generator=g)
        rec = vae.decode(z, denorm=False)
    out = {"state": {k: v.clone() for k, v in vae.state_dict().items()}, "x": x, "moments": moments,
           "mode": post.mode().clone(), "z": z, "rec": rec, "cfg_json": torch.tensor(list(json.dumps(CFG).encode()),
                                                                                  dtype=torch.uint8)}
    torch.save(out, os.path.join(HERE, "vae_golden.pt"))
    print("wrote vae_golden.pt", {k: tuple(v.shape) for k, v in out.items() if torch.is_tensor(v)})


if __name__ == "__main__":
    main()
