"""A/B of the halo conv v10 (producer / consumer, csrc/conv_halo10.hip) against v9b on the UNet's halo problems
(GPU box).  For every problem: output and statistics of v10 vs v9b (max |diff| / max |ref|), then interleaved warm
timings of both (fmd_debug_halo10 0 / 1 in one process).

usage: python tools/h10_micro.py [--iters 20] [--reps 3] [--only fwd,dgrad,...] [--hw 256]
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
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--warm", type=int, default=200)
    ap.add_argument("--only", default="")
    ap.add_argument("--hw", default="256")
    ap.add_argument("--check-only", action="store_true")
    ap.add_argument("--dbg", default="", help="comma list of v10 ablation flags (needs FMD_LIB = a -DFMD_HALO_DBG build)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    L = _lib.lib()
    g = torch.Generator(device=dev).manual_seed(0)

    def rn(*s):
        return torch.randn(*s, device=dev, generator=g).to(torch.bfloat16)

    probs = {}
    for hw in [int(v) for v in a.hw.split(",")]:
        N = 8
        for C, K in ((128, 128), (256, 256)):
            x, x2, side = rn(N, hw, hw, C), rn(N, hw, hw, C), rn(N, hw, hw, K)
            wf = torch.randn(K, C, 3, 3, device=dev, generator=g) * 0.03
            w, wd = ops.prep_weights(wf, 0), ops.prep_weights(wf, 3)   # dgrad: flipped taps of the same weight
            wt, wdt = ops.tile_weights(w), ops.tile_weights(wd)
            wf2 = torch.randn(K, 2 * C, 3, 3, device=dev, generator=g) * 0.03
            w2 = ops.prep_weights(wf2, 0)
            wt2 = ops.tile_weights(w2)
            pa, pb = torch.rand(N, 2 * C, device=dev) + 0.5, torch.randn(N, 2 * C, device=dev) * 0.1
            pac, pbc = pa[:, :C].contiguous(), pb[:, :C].contiguous()
            ea, eb = torch.rand(N, K, device=dev) + 0.5, torch.randn(N, K, device=dev) * 0.1
            bias = torch.randn(K, device=dev) * 0.1
            bnc = torch.randn(N, K, device=dev) * 0.1
            ws = torch.randn(K, 2 * C, device=dev) * 0.05
            wsk = ops.prep_weights(ws.reshape(K, 2 * C, 1, 1), 0)
            wskt = ops.tile_weights(wsk)
            f = 2 * N * hw * hw * K * C * 9
            tag = f"{hw}_{C}"
            probs[f"fwd_{tag}"] = (lambda x=x, K=K, w=w, pac=pac, pbc=pbc, wt=wt, bias=bias, bnc=bnc: ops.conv(
                x, K, w, pro=(pac, pbc, True), bias=bias, bias_nc=bnc, want_stats=True, wgt_tiled=wt), f)
            probs[f"resid_{tag}"] = (lambda x=x, K=K, w=w, pac=pac, pbc=pbc, wt=wt, bias=bias, side=side: ops.conv(
                x, K, w, pro=(pac, pbc, True), bias=bias, resid=side, want_stats=True, wgt_tiled=wt), f)
            probs[f"cat_{tag}"] = (lambda x=x, x2=x2, K=K, w2=w2, pa=pa, pb=pb, wt2=wt2, bias=bias: ops.conv(
                x, K, w2, src1=x2, pro=(pa, pb, True), bias=bias, want_stats=True, wgt_tiled=wt2), 2 * f)
            probs[f"skip_{tag}"] = (lambda x=x, x2=x2, K=K, w=w, pac=pac, pbc=pbc, wt=wt, wsk=wsk, wskt=wskt: ops.conv(
                x, K, w, pro=(pac, pbc, True), src2=x, src3=x2, wgt2=wsk, want_stats=True, wgt_tiled=wt,
                wgt2_tiled=wskt),
                f + 2 * N * hw * hw * K * 2 * C)
            probs[f"dgrad_{tag}"] = (lambda side=side, C=C, wd=wd, wdt=wdt, x=x, ea=ea, eb=eb: ops.conv(
                side, C, wd, want_stats=True, ep=(x, None, ea[:, :C].contiguous(), eb[:, :C].contiguous()),
                wgt_tiled=wdt), f)
    todo = [k for k in probs if not a.only or any(k.startswith(p) for p in a.only.split(","))]
    for name in todo:
        fn, flops = probs[name]
        outs = []
        for v in (0, 1):
            L.fmd_debug_halo10(ctypes.c_int(v))
            o, st = fn()
            torch.cuda.synchronize()
            outs.append((o.float(), None if st is None else st.slab.clone()))
        (o0, s0), (o1, s1) = outs
        err = ((o1 - o0).abs().max() / o0.abs().max().clamp_min(1e-30)).item()
        serr = float("nan") if s0 is None else ((s1 - s0).abs().max() / s0.abs().max().clamp_min(1e-30)).item()
        print(f"{name:14s} v10 vs v9b: out max rel {err:.2e}, stats max rel {serr:.2e}", flush=True)
        if a.check_only:
            continue
        res = {0: [], 1: []}
        for v in (0, 1):
            L.fmd_debug_halo10(ctypes.c_int(v))
            for _ in range(a.warm if v == 0 else 20):
                fn()
        for _ in range(a.reps):
            for v in (0, 1):
                L.fmd_debug_halo10(ctypes.c_int(v))
                fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res[v].append(e0.elapsed_time(e1) / a.iters)
        m0, m1 = min(res[0]), min(res[1])
        print(f"{name:14s} v9b {m0 * 1e3:8.1f} us ({flops / m0 / 1e9:6.0f} TF/s)   v10 {m1 * 1e3:8.1f} us "
              f"({flops / m1 / 1e9:6.0f} TF/s)   x{m0 / m1:.3f}", flush=True)
        for fl in [int(v) for v in a.dbg.split(",") if v]:
            L.fmd_debug_halo10(ctypes.c_int(1))
            L.fmd_debug_halo_flags(ctypes.c_int(fl))
            for _ in range(20):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            L.fmd_debug_halo_flags(ctypes.c_int(0))
            print(f"{name:14s}   v10 dbg={fl:3d} {ms * 1e3:8.1f} us", flush=True)
    L.fmd_debug_halo10(ctypes.c_int(1))


if __name__ == "__main__":
    main()
