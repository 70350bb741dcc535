"""Config E probe (BASELINE.json configs[4]): EfficientUNetND with spatial_dims=3 built from the
reference's ldct_flow_matching.json model block, one FM train step per iteration on a (B,1,S,S,S) synthetic volume,
on one MI355X.  Prints one JSON line: train samples/s, ms/step and the fraction of dense bf16 MFMA peak at the
algorithmic 3 x fwd FLOPs.  Not the headline bench (config B, bench.py); the 8-GPU DDP leg of config E is the same
FusedTrainStep with the all-reduce path bench.py exercises.

    python tools/bench3d.py --size 128 --batch 1 --steps 3 --warmup 2
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "flow-matching-and-diffusion-models_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

from bench import LDCT_FM_UNET, PEAK_BF16_TFLOPS  # noqa: E402

FWD_GFLOP_128 = 32854.2   # fwd GFLOP per 128^3 sample [probe]; conv FLOPs scale with voxels


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--graph", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_stream(torch.cuda.Stream(dev))   # as bench.py: all work on a created stream
    from fmdiff.models.generators import DiffusionUNetFactory
    from fmdiff.pipelines.train.fused import FusedTrainStep
    torch.manual_seed(0)
    cfg = dict(LDCT_FM_UNET, spatial_dims=3, sample_size=args.size)
    model = DiffusionUNetFactory().build(cfg, "concatenate", 1).to(dev)
    nparam = sum(p.numel() for p in model.parameters())
    S, B = args.size, args.batch
    g = torch.Generator(device=dev).manual_seed(7)
    clean = torch.rand(B, 1, S, S, S, device=dev, generator=g)
    ldct = (clean + 0.05 * torch.randn(B, 1, S, S, S, device=dev, generator=g)).clamp(0, 1)
    tr = FusedTrainStep(model, lr=1e-4, warmup=500, total_steps=100000, num_train_timesteps=1000)
    if args.graph:
        tr.capture(clean, ldct, warmup_iters=2)
        run = tr.replay
    else:
        def run():
            return tr.step(clean, ldct)
    for i in range(args.warmup):
        t0 = time.perf_counter()
        loss = run()
        torch.cuda.synchronize()
        print(f"[bench3d] warmup {i}: {time.perf_counter() - t0:.3f} s loss {float(loss):.4f}", flush=True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    gflop = 3 * FWD_GFLOP_128 * (S / 128) ** 3 * B
    print(json.dumps({"workload": f"config E: EfficientUNetND 3-D {S}^3, batch {B}, FM train step", "params": nparam,
                      "ms_per_step": dt * 1e3, "samples_per_sec": B / dt, "tflops": gflop / dt / 1e3,
                      "mfma_frac": gflop / dt / 1e3 / PEAK_BF16_TFLOPS, "loss": float(loss),
                      "peak_mem_gb": torch.cuda.max_memory_allocated() / 2**30, "hipgraph": args.graph}), flush=True)


if __name__ == "__main__":
    main()
