"""Config D probe (BASELINE.json configs[3]): AutoencoderKL (configs/LDCT/LDCT_autoencoder_kl.json
layout, random init) + latent flow-matching UNet (the ldct_flow_matching.json UNet with 4 latent channels,
concatenate conditioning -> 8 input channels, 32x32), encode -> 50-step FM-Euler sampler -> decode on one
MI355X.  Prints one JSON line with images/s of the whole path and each stage's ms.

    python tools/bench_latent.py --batch 8 --steps 50
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import warnings

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "flow-matching-and-diffusion-models_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

from bench import LDCT_FM_UNET  # noqa: E402

VAE_CFG = dict(in_channels=1, out_channels=1, resolution=256, base_ch=128, down_channels=[128, 256, 512, 512],
               num_res_blocks=2, attn_resolutions=[], z_channels=4, embed_dim=4, dropout=0.0, use_attention=True,
               spatial_dims=2, emb_channels=None, use_scale_shift_norm=False, double_z=True, attn_heads=4,
               attn_dim_head=64)
ENC_GF, DEC_GF, UNET_STEP_GF = 269.2, 618.7, 7.748   # SURVEY.md 8(d) D, per image [probe]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_stream(torch.cuda.Stream(dev))   # as bench.py: all work on a created stream
    from fmdiff.models.generators import DiffusionUNetFactory
    from fmdiff.models.vae import AutoencoderKL
    from fmdiff.pipelines.latent import decode_vae_batch, encode_vae_batch
    from fmdiff.pipelines.train.fused import FusedFlowSampler
    torch.manual_seed(0)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        vae = AutoencoderKL(**VAE_CFG).to(dev).eval()
    ucfg = dict(LDCT_FM_UNET, in_channels=4, out_channels=4, sample_size=32)
    unet = DiffusionUNetFactory().build(ucfg, "concatenate", 4).to(dev)
    sampler = FusedFlowSampler(unet, args.steps)
    B = args.batch
    g = torch.Generator(device=dev).manual_seed(3)
    img = torch.rand(B, 1, 256, 256, device=dev, generator=g)
    times = {"encode": [], "sample": [], "decode": []}
    for r in range(args.reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cond = encode_vae_batch(vae, img).contiguous()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        lat = sampler.sample(torch.randn_like(cond), cond, use_graph=True)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out = decode_vae_batch(vae, lat)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        if r:
            times["encode"].append(t1 - t0)
            times["sample"].append(t2 - t1)
            times["decode"].append(t3 - t2)
    med = {k: sorted(v)[len(v) // 2] for k, v in times.items()}
    tot = sum(med.values())
    gf = B * (ENC_GF + DEC_GF + args.steps * UNET_STEP_GF)
    print(json.dumps({"workload": f"config D: AutoencoderKL encode -> {args.steps}-step latent FM-Euler -> decode, "
                                  f"batch {B}, 256x256 -> 4x32x32", "images_per_sec": B / tot,
                      "ms": {k: v * 1e3 for k, v in med.items()}, "tflops": gf / tot / 1e3,
                      "out_range": [float(out.min()), float(out.max())]}), flush=True)


if __name__ == "__main__":
    main()
