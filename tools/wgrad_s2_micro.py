"""Time the stride-2 3x3 weight gradients (generic wgrad kernel) of config B (2-D, 256^2 -> 128^2 etc.) and config E
(3-D, 128^3 -> 64^3 etc.) with HIP events, to price a halo (space-to-depth) form.  usage: python tools/wgrad_s2_micro.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "flow-matching-and-diffusion-models_amd")]

import torch  # noqa: E402

from fmdiff.runtime import ops  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    probs = [("2d 8x256^2 128->128", (8, 256, 256), 128, 128), ("2d 8x128^2 128->128", (8, 128, 128), 128, 128),
             ("2d 8x64^2 256->256", (8, 64, 64), 256, 256), ("3d 1x128^3 128->128", (1, 128, 128, 128), 128, 128),
             ("3d 1x64^3 128->128", (1, 64, 64, 64), 128, 128), ("3d 1x32^3 256->256", (1, 32, 32, 32), 256, 256)]
    s = torch.cuda.current_stream()
    for name, shp, C, K in probs:
        N, sp = shp[0], shp[1:]
        x = torch.randn(N, *sp, C, device=dev, generator=g).to(torch.bfloat16)
        dy = torch.randn(N, *[v // 2 for v in sp], K, device=dev, generator=g).to(torch.bfloat16)
        dw = torch.zeros(K, C, *([3] * len(sp)), device=dev)
        db = torch.zeros(K, device=dev)
        for _ in range(3):
            ops.wgrad(x, dy, dw, ks=3, stride=2, pad=1, db=db)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        it = 10
        e0.record(s)
        for _ in range(it):
            ops.wgrad(x, dy, dw, ks=3, stride=2, pad=1, db=db)
        e1.record(s)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / it
        fl = 2.0 * dy[..., 0].numel() * K * C * 3 ** len(sp)
        print(f"{name:24s} {us:8.1f} us  {fl / us / 1e6:7.1f} TF/s  ({fl / us / 1e6 / 2500:.3f} of peak)", flush=True)


if __name__ == "__main__":
    main()
