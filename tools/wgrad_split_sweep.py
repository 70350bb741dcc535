"""Split-count sweep of the halo weight gradient (kernel + split-K combine) on config B's levels (GPU box).

usage: python tools/wgrad_split_sweep.py [--iters 20]
Prints, per (H, C, K) problem, the automatic split count and the time of each tried split count.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "flow-matching-and-diffusion-models_amd")]

import torch  # noqa: E402

from fmdiff.runtime import ops  # noqa: E402


def auto_splits(N, H, W, C, K):
    tiles = N * (H // 8) * (W // 16)
    base = (K // 128) * (C // 64)
    return max(1, min(tiles, -(-ops.WGRAD_HALO_WG // base), (ops.WGRAD_SLAB_MB << 20) // (K * C * 36)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    g = torch.Generator(device=dev).manual_seed(0)
    N = 8
    for H, C, K in ((256, 128, 128), (128, 128, 128), (64, 256, 256), (32, 256, 256), (32, 512, 256),
                    (16, 512, 512), (16, 1024, 512)):
        x = torch.randn(N, H, H, C, device=dev, generator=g).to(torch.bfloat16)
        dy = torch.randn(N, H, H, K, device=dev, generator=g).to(torch.bfloat16)
        pa, pb = torch.rand(N, C, device=dev) + 0.5, torch.randn(N, C, device=dev) * 0.1
        dw = torch.zeros(K, C, 3, 3, device=dev)
        db = torch.zeros(K, device=dev)
        s0 = auto_splits(N, H, H, C, K)
        tiles = N * (H // 8) * (H // 16)
        cands = sorted({max(1, s0 // 4), max(1, s0 // 2), s0, min(tiles, s0 * 2)})
        res = []
        for s in cands:
            f = lambda: ops.wgrad(x, dy, dw, pro=(pa, pb, True), db=db, splits=s)  # noqa: E731
            for _ in range(3):
                f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.iters):
                f()
            e1.record()
            torch.cuda.synchronize()
            res.append((s, e0.elapsed_time(e1) / a.iters * 1e3))
        print(f"H={H} C={C} K={K} auto={s0} " + " ".join(f"s{s}:{t:.1f}us" for s, t in res), flush=True)


if __name__ == "__main__":
    main()
