"""Weight-gradient ablation timings (GPU box): the halo weight gradient on config B's bench problem (8x256^2,
128 -> 128, GN+SiLU prologue) and config E's 128^3 level (128 -> 128, materialised prologue), with the FMD_HALO_DBG
ablation flags of csrc/wgrad_halo.hip (needs FMD_LIB pointing at a -DFMD_HALO_DBG build for nonzero flags).

usage: python tools/wgrad_abl.py [--dbg 1,2,4,8,16,32] [--iters 20] [--only b,e]
Times ops.wgrad (kernel + split-K reduce) per call.
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "flow-matching-and-diffusion-models_amd")]

import torch  # noqa: E402

from fmdiff import _lib  # noqa: E402
from fmdiff.runtime import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dbg", default="")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="b,e")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    g = torch.Generator(device=dev).manual_seed(0)
    probs = {}
    if "b" in a.only.split(","):
        x = torch.randn(8, 256, 256, 128, device=dev, generator=g).to(torch.bfloat16)
        dy = torch.randn(8, 256, 256, 128, device=dev, generator=g).to(torch.bfloat16)
        pa, pb = torch.rand(8, 128, device=dev) + 0.5, torch.randn(8, 128, device=dev) * 0.1
        dw = torch.zeros(128, 128, 3, 3, device=dev)
        probs["wgrad_b"] = (lambda: ops.wgrad(x, dy, dw, pro=(pa, pb, True)), 2 * 8 * 256 * 256 * 128 * 128 * 9)
    if "e" in a.only.split(","):
        S = 128
        x3 = torch.randn(1, S, S, S, 128, device=dev, generator=g).to(torch.bfloat16)
        dy3 = torch.randn(1, S, S, S, 128, device=dev, generator=g).to(torch.bfloat16)
        dw3 = torch.zeros(128, 128, 3, 3, 3, device=dev)
        probs["wgrad_e"] = (lambda: ops.wgrad(x3, dy3, dw3), 2 * S ** 3 * 128 * 128 * 27)
    flags = [0] + [int(f) for f in a.dbg.split(",") if f]
    for name, (fn, flops) in probs.items():
        for fl in flags:
            if a.dbg:
                _lib.lib().fmd_debug_halo_flags(ctypes.c_int(fl))
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            print(f"{name:8s} dbg={fl:3d} {ms * 1e3:9.1f} us/call  {flops / ms / 1e9:7.1f} TFLOP/s", flush=True)
        if a.dbg:
            _lib.lib().fmd_debug_halo_flags(ctypes.c_int(0))


if __name__ == "__main__":
    main()
