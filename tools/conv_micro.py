"""Micro-benchmark of the UNet's dominant conv problems (GPU box; used under rocprofv3 for PMC passes).

usage: python tools/conv_micro.py [--iters 20] [--only fwd|dgrad|wgrad]
Problems (batch 8, 256x256 level):
  fwd   : GN+SiLU -> 3x3 conv 128->128 (halo kernel), fused stats
  cat   : GN+SiLU -> 3x3 conv (128|128)->128 (decoder concat)
  dgrad : 3x3 data gradient 128->128 with the SiLU'/GN-stats epilogue (halo kernel, flipped taps)
  wgrad : weight gradient 128->128 3x3 with the GN+SiLU prologue
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "flow-matching-and-diffusion-models_amd")]

import torch  # noqa: E402

from fmdiff.runtime import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--hw", type=int, default=256)
    ap.add_argument("--c", type=int, default=128)
    ap.add_argument("--dbg", default="", help="comma list of halo ablation flag values to time as well")
    ap.add_argument("--variants", default="1", help="(kept for the output format)")
    ap.add_argument("--staggers", default="", help="comma list of v2 stagger values to time (default: library's)")
    ap.add_argument("--warm", type=int, default=300, help="back-to-back launches before the first timing (clock ramp)")
    ap.add_argument("--cold", action="store_true", help="evict L2 / Infinity Cache (512 MiB write) before every call")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    N, H, W, C, K = 8, a.hw, a.hw, a.c, a.c
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(N, H, W, C, device=dev, generator=g).to(torch.bfloat16)
    x2 = torch.randn(N, H, W, C, device=dev, generator=g).to(torch.bfloat16)
    wf = torch.randn(K, C, 3, 3, device=dev, generator=g) * 0.03
    w = ops.prep_weights(wf, 0)
    wt = ops.tile_weights(w)
    wf2 = torch.randn(K, 2 * C, 3, 3, device=dev, generator=g) * 0.03
    w2 = ops.prep_weights(wf2, 0)
    wt2 = ops.tile_weights(w2)
    wd = ops.prep_weights(wf, 3)
    wdt = ops.tile_weights(wd)
    pa = torch.rand(N, 2 * C, device=dev) + 0.5
    pb = torch.randn(N, 2 * C, device=dev) * 0.1
    bias = torch.zeros(K, device=dev)
    out = torch.empty(N, H, W, K, device=dev, dtype=torch.bfloat16)
    dw = torch.zeros(K, C, 3, 3, device=dev)
    db = torch.zeros(K, device=dev)

    def fwd():
        ops.conv(x, K, w, pro=(pa[:, :C].contiguous(), pb[:, :C].contiguous(), True), bias=bias, out=out,
                 want_stats=True, wgt_tiled=wt)

    pac, pbc = pa[:, :C].contiguous(), pb[:, :C].contiguous()

    def cat():
        ops.conv(x, K, w2, src1=x2, pro=(pa, pb, True), bias=bias, out=out, want_stats=True, wgt_tiled=wt2)

    def dgrad():
        ops.conv(x, C, wd, out=out, want_stats=True, ep=(x2, None, pac, pbc), wgt_tiled=wdt)

    def wgrad():
        ops.wgrad(x, x2, dw, pro=(pac, pbc, True), db=db)

    def fwd0():
        ops.conv(x, K, w, bias=bias, out=out, want_stats=True, wgt_tiled=wt)

    def wgrad0():
        ops.wgrad(x, x2, dw, db=db)

    def gnapply():
        ops.gn_apply_fwd(x, None, pac, pbc)

    def gnapply_cat():
        ops.gn_apply_fwd(x, x2, pa, pb)

    probs = dict(fwd=(fwd, 2 * N * H * W * K * C * 9), cat=(cat, 2 * N * H * W * K * 2 * C * 9),
                 fwd0=(fwd0, 2 * N * H * W * K * C * 9), wgrad0=(wgrad0, 2 * N * H * W * K * C * 9),
                 gnapply=(gnapply, 4 * N * H * W * C), gnapply_cat=(gnapply_cat, 8 * N * H * W * C),
                 dgrad=(dgrad, 2 * N * H * W * K * C * 9), wgrad=(wgrad, 2 * N * H * W * K * C * 9))
    import ctypes
    from fmdiff import _lib
    L = _lib.lib()
    flush = torch.zeros(128 << 20, device=dev) if a.cold else None   # 512 MiB
    flagsets = [0] + [int(f) for f in a.dbg.split(",") if f]
    stg = [int(x) for x in a.staggers.split(",") if x] or [None]
    todo = [(name, fl, v, sg) for name in probs for fl in flagsets for v in [int(x) for x in a.variants.split(",")]
            for sg in stg]
    warmed = False
    for name, fl, var, sg in todo:
        fn, flops = probs[name]
        if a.only and name not in a.only.split(","):
            continue
        L.fmd_debug_halo_flags(ctypes.c_int(fl))
        for _ in range(3 if warmed else a.warm):   # the chip ramps its clock over the first few hundred ms
            fn()
        warmed = True
        torch.cuda.synchronize()
        if a.cold:
            ms = 0.0
            for _ in range(a.iters):
                flush.add_(1.0)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                ms += e0.elapsed_time(e1) / a.iters
        else:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
        print(f"{name:6s} v{var} stagger={sg} dbg={fl:2d} {'cold' if a.cold else 'hot '} {ms * 1e3:8.1f} us/call  {flops / ms / 1e9:7.1f} TFLOP/s",
              flush=True)
    L.fmd_debug_halo_flags(ctypes.c_int(0))


if __name__ == "__main__":
    main()
