"""v11 (ping-pong halo conv, csrc/conv_halo11.hip) against v9b on the GPU box: bit-equality of outputs and
statistics, then interleaved HIP-event timings, on config B's 256^2 problems.

usage: python tools/h11_check.py [--iters 30]   (needs the library built at commit 0a067f5, where v11 lives)
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
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    L = _lib.lib()
    L.fmd_debug_halo11.argtypes = [ctypes.c_int]
    g = torch.Generator(device=dev).manual_seed(0)
    N, H = 8, 256
    probs = {}
    for name, C, K, resid, pro in (("fwd_128", 128, 128, False, 2), ("resid_128", 128, 128, True, 2),
                                   ("cat_256", 256, 128, False, 2), ("fwd_256", 256, 256, False, 2),
                                   ("raw_128", 128, 128, False, 0)):
        x = torch.randn(N, H, H, C, device=dev, generator=g).to(torch.bfloat16)
        wf = torch.randn(K, C, 3, 3, device=dev, generator=g) * 0.03
        w = ops.prep_weights(wf, 0)
        wt = ops.tile_weights(w)
        pa = torch.rand(N, C, device=dev, generator=g) + 0.5
        pb = torch.randn(N, C, device=dev, generator=g) * 0.1
        bias = torch.randn(K, device=dev, generator=g) * 0.1
        rs = torch.randn(N, H, H, K, device=dev, generator=g).to(torch.bfloat16) if resid else None
        out = torch.empty(N, H, H, K, device=dev, dtype=torch.bfloat16)
        kw = dict(bias=bias, out=out, want_stats=True, wgt_tiled=wt)
        if pro:
            kw["pro"] = (pa, pb, pro == 2)
        if resid:
            kw["resid"] = rs

        def run(x=x, K=K, w=w, kw=kw):
            return ops.conv(x, K, w, **kw)
        probs[name] = (run, out, 2.0 * N * H * H * C * K * 9)
    for name, (run, out, fl) in probs.items():
        res = []
        for v in (0, 1):
            L.fmd_debug_halo11(v)
            o, st = run()
            torch.cuda.synchronize()
            res.append((o.clone(), st.slab.clone() if st is not None else None))
        eq = torch.equal(res[0][0], res[1][0])
        se = (res[0][1] is None and res[1][1] is None) or torch.equal(res[0][1], res[1][1])
        print(f"{name:10s} v11 vs v9b: out equal {eq}, stats equal {se}", flush=True)
        if not (eq and se):
            d = (res[0][0].float() - res[1][0].float()).abs().max().item()
            print(f"   max |diff| {d:.3e}", flush=True)
    s = torch.cuda.current_stream()
    for name, (run, out, fl) in probs.items():
        t = {0: [], 1: []}
        for rep in range(2):
            for v in (0, 1):
                L.fmd_debug_halo11(v)
                for _ in range(50):
                    run()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(a.iters):
                    run()
                e1.record(s)
                torch.cuda.synchronize()
                t[v].append(e0.elapsed_time(e1) * 1e3 / a.iters)
        print(f"{name:10s} v9b {t[0][0]:7.1f} / {t[0][1]:7.1f} us   v11 {t[1][0]:7.1f} / {t[1][1]:7.1f} us   "
              f"({fl / min(t[1]) / 1e6:.0f} vs {fl / min(t[0]) / 1e6:.0f} TF/s)", flush=True)
    L.fmd_debug_halo11(0)


if __name__ == "__main__":
    main()
