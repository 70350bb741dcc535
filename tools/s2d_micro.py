"""Stride-2 conv micro-benchmark (GPU box): the implicit GEMM vs the space-to-depth halo kernel (fmd_conv_s2d) on
config B's DownsampleND forwards and UpsampleND data gradients.

usage: python tools/s2d_micro.py [--iters 50]
"""
import argparse
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "flow-matching-and-diffusion-models_amd")]

import torch  # noqa: E402

from fmdiff.runtime import ops as O  # noqa: E402


def timeit(fn, iters):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    g = torch.Generator(device=dev).manual_seed(0)
    # (kind, N, full-resolution H, C in, K out)
    for kind, N, H, C, K in (("down", 8, 256, 128, 128), ("down", 8, 128, 256, 256), ("down", 8, 64, 256, 256),
                             ("updgrad", 8, 256, 256, 256), ("updgrad", 8, 128, 256, 256), ("updgrad", 8, 64, 512, 512),
                             ("s2dgrad", 8, 256, 128, 128), ("s2dgrad", 8, 128, 256, 256), ("s2dgrad", 8, 64, 256, 256)):
        h = H // 2
        if kind == "down":
            x = torch.randn(N, H, H, C, device=dev, generator=g).to(torch.bfloat16)
            w = torch.randn(K, C, 3, 3, device=dev, generator=g) / math.sqrt(9 * C)
            wg, ws = O.prep_weights(w, 0), O.s2d_tile_weights(w, 0)
            flops = 2 * N * h * h * K * C * 9
            gen = lambda: O.conv(x, K, wg, ks=3, stride=2, pad=1)
            s2d = (lambda: O.conv(x, K, None, ks=3, stride=2, pad=1, s2d_tiled=ws)) \
                if O.s2d_eligible(N, H, H, h, h, K, C, 3) else None
        elif kind == "s2dgrad":   # data gradient of the stride-2 conv x [N, H, H, C] -> y [N, h, h, K]
            dy = torch.randn(N, h, h, K, device=dev, generator=g).to(torch.bfloat16)
            w = torch.randn(K, C, 3, 3, device=dev, generator=g) / math.sqrt(9 * C)
            wg, ws = O.prep_weights(w, 1), O.s2d_tile_weights(w, 2)
            flops = 2 * N * h * h * K * C * 9
            gen = lambda: O.conv(dy, C, wg, ks=3, stride=2, pad=1, transposed=True, out_hw_=(H, H))
            s2d = (lambda: O.conv(dy, C, None, ks=3, stride=2, pad=1, transposed=True, out_hw_=(H, H), s2d_tiled=ws)) \
                if O.d2s_eligible(N, h, h, H, H, C, K) else None
        else:   # data gradient of conv3x3(nearest_x2(x)): x [N, h, h, C] -> conv output K channels at H
            dy = torch.randn(N, H, H, K, device=dev, generator=g).to(torch.bfloat16)
            w = torch.randn(K, C, 3, 3, device=dev, generator=g) / math.sqrt(9 * C)
            wg, ws = O.prep_weights(w, 2), O.s2d_tile_weights(w, 1)
            flops = 2 * N * H * H * K * C * 9
            gen = lambda: O.conv(dy, C, wg, ks=4, stride=2, pad=1, out_hw_=(h, h))
            s2d = (lambda: O.conv(dy, C, None, ks=4, stride=2, pad=1, out_hw_=(h, h), s2d_tiled=ws)) \
                if O.s2d_eligible(N, H, H, h, h, C, K, 4) else None
        tg = timeit(gen, a.iters)
        line = f"{kind:8s} N={N} {H}^2 {C}->{K}: generic {tg * 1e3:7.1f} us ({flops / tg / 1e9:6.1f} TF/s)"
        if s2d is not None:
            ts = timeit(s2d, a.iters)
            line += f"  s2d {ts * 1e3:7.1f} us ({flops / ts / 1e9:6.1f} TF/s)"
        print(line, flush=True)


if __name__ == "__main__":
    main()
