"""Small-level conv probe (GPU box helper): one 3x3 conv at a tiny spatial size, every split factor, each
captured 20x in a hipGraph; run under rocprofv3 --kernel-trace to split main kernel vs combine.

usage: python tools/small_conv_probe.py [H] [C] [K]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "flow-matching-and-diffusion-models_amd")]

import torch  # noqa: E402

from fmdiff.runtime import ops  # noqa: E402


def timeit(fn, iters=20):
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
    for _ in range(5):
        gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        gr.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (5 * iters) * 1e3


def main():
    H = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    C = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 512
    N = 8
    dev = torch.device("cuda", 0)
    x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
    w = torch.randn(K, C, 3, 3, device=dev) * 0.05
    wk = ops.prep_weights(w, 0)
    nk = -(-C // 64) * 9
    for sp in (1, 2, 4, 9, 18, 36, 72):
        if sp > nk:
            break
        us = timeit(lambda: ops.conv(x, K, wk, splits=sp, force_generic=True))
        print(f"H={H} C={C} K={K} M={N * H * H} splits={sp:3d}: {us:7.1f} us per conv (main + combine)", flush=True)


if __name__ == "__main__":
    main()
