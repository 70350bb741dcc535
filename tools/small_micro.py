"""Split-factor sweep for the small-level (8x8 / 16x16) convs of config B (GPU box helper).

usage: python tools/small_micro.py
Times fmd_conv (3x3, GN+SiLU prologue, fused stats, incl. the split-K combine) and fmd_wgrad
(incl. its reduction) at N=8 for several split factors.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "flow-matching-and-diffusion-models_amd")]

import torch  # noqa: E402

from fmdiff.runtime import ops  # noqa: E402


def timeit(fn, iters=20):
    """Device time per call: `iters` calls captured into one hipGraph (no host launch overhead)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(iters):
            fn()
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        gr.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (3 * iters) * 1e3


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    N = 8
    for hw, C in ((8, 512), (16, 512), (32, 256)):
        K = C
        x = torch.randn(N, hw, hw, C, device=dev, generator=g).to(torch.bfloat16)
        dy = torch.randn(N, hw, hw, K, device=dev, generator=g).to(torch.bfloat16)
        wf = torch.randn(K, C, 3, 3, device=dev, generator=g) * 0.03
        w = ops.prep_weights(wf, 0)
        pa = torch.rand(N, C, device=dev) + 0.5
        pb = torch.randn(N, C, device=dev) * 0.1
        flops = 2 * N * hw * hw * K * C * 9
        for sp in (1, 2, 4, 6, 9, 12, 18, 24, 36):
            try:
                us = timeit(lambda: ops.conv(x, K, w, pro=(pa, pb, True), want_stats=True, splits=sp,
                                             force_generic=True))
                print(f"fwd   {hw:3d}^2 C={C} splits={sp:3d} {us:8.1f} us {flops / us / 1e6:7.1f} TF/s", flush=True)
            except Exception as e:  # noqa: BLE001
                print(f"fwd   {hw}^2 splits={sp}: {e}", flush=True)
        if ops.halo_eligible(N, hw, hw, hw, K, Cin=C, pro=True):
            us = timeit(lambda: ops.conv(x, K, None, pro=(pa, pb, True), want_stats=True,
                                         wgt_tiled=ops.tile_weights(w)))
            print(f"halo  {hw:3d}^2 C={C} auto        {us:8.1f} us {flops / us / 1e6:7.1f} TF/s", flush=True)
        dw = torch.zeros(K, C, 3, 3, device=dev)
        for sp in (1, 2, 4, 8, 16, 32):
            us = timeit(lambda: ops.wgrad(x, dy, dw, pro=(pa, pb, True), splits=sp, force_generic=True))
            print(f"wgrad {hw:3d}^2 C={C} splits={sp:3d} {us:8.1f} us {flops / us / 1e6:7.1f} TF/s", flush=True)
        us = timeit(lambda: ops.wgrad(x, dy, dw, pro=(pa, pb, True)))
        print(f"wgrad {hw:3d}^2 C={C} auto        {us:8.1f} us {flops / us / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
