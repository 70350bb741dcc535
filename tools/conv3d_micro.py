"""Micro-benchmark of config E's dominant 3-D conv problems (GPU box; also run under rocprofv3 for PMC passes).

usage: python tools/conv3d_micro.py [--size 128] [--c 128] [--iters 10] [--only fwd,dgrad,wgrad,dgrad_s2]
Problems (config E, EfficientUNetND spatial_dims=3, batch 1, the 128^3 level):
  fwd      : GN+SiLU -> 3x3x3 conv C->C (depth-tap halo kernel), fused stats
  dgrad    : 3x3x3 data gradient C->C with the SiLU'/GN-stats epilogue (halo kernel, flipped taps)
  wgrad    : 3x3x3 weight gradient C->C with the GN+SiLU prologue (halo weight-gradient kernel)
  dgrad_s2 : data gradient of the stride-2 3x3x3 DownsampleND conv (transposed gather, parity classes)
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "flow-matching-and-diffusion-models_amd")]

import torch  # noqa: E402

from fmdiff.runtime import ops  # noqa: E402
from fmdiff.runtime.engine import WeightCache  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="")
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--c", type=int, default=128)
    ap.add_argument("--warm", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    N, S, C = 1, a.size, a.c
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(N, S, S, S, C, device=dev, generator=g).to(torch.bfloat16)
    x2 = torch.randn(N, S, S, S, C, device=dev, generator=g).to(torch.bfloat16)
    dyh = torch.randn(N, S // 2, S // 2, S // 2, C, device=dev, generator=g).to(torch.bfloat16)
    wf = torch.randn(C, C, 3, 3, 3, device=dev, generator=g) * 0.02
    wc = WeightCache()
    wt, wdt = wc.dtiled(wf, 0), wc.dtiled(wf, 3)
    w0, w1 = wc.get(wf, 0), wc.get(wf, 1)
    pa = torch.rand(N, C, device=dev) + 0.5
    pb = torch.randn(N, C, device=dev) * 0.1
    bias = torch.zeros(C, device=dev)
    out = torch.empty(N, S, S, S, C, device=dev, dtype=torch.bfloat16)
    dw = torch.zeros(C, C, 3, 3, 3, device=dev)
    db = torch.zeros(C, device=dev)
    sp = (S, S, S)

    def fwd():
        ops.conv(x, C, w0, pro=(pa, pb, True), bias=bias, out=out, want_stats=True, wgt_tiled=wt, out_hw_=sp)

    def dgrad():
        ops.conv(x, C, wc.get(wf, 3), out=out, want_stats=True, ep=(x2, None, pa, pb), wgt_tiled=wdt, out_hw_=sp)

    def wgrad():
        ops.wgrad(x, x2, dw, pro=(pa, pb, True), db=db)

    def dgrad_s2():
        ops.conv(dyh, C, w1, stride=2, transposed=True, out_hw_=sp, out=out)

    fl = 2 * N * S ** 3 * C * C * 27
    probs = dict(fwd=(fwd, fl), dgrad=(dgrad, fl), wgrad=(wgrad, fl), dgrad_s2=(dgrad_s2, fl // 8))
    for name, (fn, flops) in probs.items():
        if a.only and name not in a.only.split(","):
            continue
        for _ in range(a.warm):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        print(f"{name:8s} {ms * 1e3:9.1f} us/call  {flops / ms / 1e9:7.1f} TFLOP/s (useful)", flush=True)


if __name__ == "__main__":
    main()
