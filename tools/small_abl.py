"""Ablation timings of fmd_conv_small (csrc/conv_small.hip) on the latent UNet's shapes (GPU box).

Needs the debug build (tools/build_variant.sh small -DFMD_SMALL_DBG) loaded with FMD_LIB=.../libfmdiff_small.so; flags
(fmd_debug_small_flags): 1 no staging DMA, 2 no GroupNorm fold, 4 no main loop, 8 no epilogue stores, 16 no stats.

usage: FMD_LIB=flow-matching-and-diffusion-models_amd/fmdiff/lib/variants/libfmdiff_small.so python tools/small_abl.py
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "flow-matching-and-diffusion-models_amd"), os.path.join(REPO, "tests")]

import torch  # noqa: E402

import test_gpu_conv_small as T  # noqa: E402
from fmdiff import _lib  # noqa: E402


def prepared(p):
    """(closure running ONLY fmd_conv_small, as tests/test_gpu_conv_small.py._run_small sets it up)."""
    ops = p["ops"]
    x0 = p["x0"].to("cuda")
    x1 = p["x1"].to("cuda") if p["x1"] is not None else None
    wk = ops.prep_weights(p["w"].to("cuda"), 0)
    gn = None
    if p["gn"]:
        gn = dict(st0=ops.channel_stats(x0), st1=ops.channel_stats(x1) if x1 is not None else None, groups=p["G"],
                  eps=1e-6, gamma=p["gamma"].to("cuda"), beta=p["beta"].to("cuda"))
        if "emb" in p:
            gn["emb"] = p["emb"].to("cuda")
    kw = dict(bias=p["bias"].to("cuda"))
    if "skip_w" in p:
        kw.update(skip_wgt=ops.prep_weights(p["skip_w"].to("cuda"), 0), bias2=p["bias2"].to("cuda"),
                  src2=p["xs0"].to("cuda"), src3=p["xs1"].to("cuda") if p["xs1"] is not None else None)
    if "bias_nc_full" in p:
        kw["bias_nc"] = p["bias_nc_full"].to("cuda")[:, :p["K"]]
    if "resid" in p:
        kw["resid"] = p["resid"].to("cuda")
    out = torch.empty((p["N"], p["Ho"], p["Ho"], p["K"]), device="cuda", dtype=torch.bfloat16)
    return lambda: ops.conv_small(x0, p["K"], wk, src1=x1, mode=p["mode"], gn=gn, out=out, **kw)


def phase_times(L, fn, name, flags=0):
    """One eager launch with phase timestamps (wave 0 of each workgroup, 100 MHz wall clock): per phase the median
    and max over workgroups of its duration, and the spread of workgroup start times."""
    import numpy as np
    ts = L.fmd_debug_small_ts
    ts.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    nb = 4096
    buf = np.zeros(nb * 12, dtype=np.uint64)
    ts(buf.ctypes.data, nb, 1)
    torch.cuda.synchronize()
    fn()
    torch.cuda.synchronize()
    ts(buf.ctypes.data, nb, 0)
    t = buf.reshape(nb, 12).astype(np.int64)
    t = t[t[:, 0] > 0]
    if not len(t):
        return
    names = ["issue", "dma_wait", "gn", "main", "sync", "ticket", "epilogue"]
    parts = []
    t0 = t[:, 0].min()
    for k in range(1, 8):
        ok = (t[:, k] > 0) & (t[:, k - 1] > 0)
        if ok.any():
            d = (t[ok, k] - t[ok, k - 1]) * 0.01
            parts.append(f"{names[k - 1]} {np.median(d):5.2f}/{d.max():5.2f}")
    if len(t) > 256:   # workgroups that started after the first wave of 256 (their CU ran one before them)
        order = np.argsort(t[:, 0])
        late = t[order[256:]]
        early = t[order[:256]]
        for lab, tt in (("first 256", early), ("later", late)):
            d = [(np.median(tt[:, k] - tt[:, k - 1]) * 0.01) for k in range(1, 5)]
            parts.append(f"{lab}: " + " ".join(f"{x:5.2f}" for x in d))
    end = np.where(t[:, 7] > 0, t[:, 7], np.where(t[:, 6] > 0, t[:, 6], t[:, 5]))
    parts.append(f"start spread {(t[:, 0].max() - t0) * 0.01:5.2f} end {(end.max() - t0) * 0.01:5.2f} wgs {len(t)}")
    if (t[:, 10] > 0).any() and (t[:, 11] > 0).any():
        w = np.median(t[:, 10] - t[:, 0]) * 0.01
        f = np.median(t[:, 11] - t[:, 2]) * 0.01
        parts.append(f"(weights issue {w:5.2f}, GN fold {f:5.2f})")
    if (t[:, 9] > 0).any():
        ok = t[:, 9] > 0
        d = (t[ok, 9] - t[ok, 8]) * 0.01
        parts.append(f"main 2nd pass {np.median(d):5.2f}/{d.max():5.2f}")
    print(f"  {name:22s} phases us (median/max): " + " | ".join(parts), flush=True)


def main():
    torch.cuda.set_stream(torch.cuda.Stream())
    L = _lib.lib()
    dbg = getattr(L, "fmd_debug_small_flags", None)
    names = sys.argv[1:] or ["s1_32_cat_skip", "s1_16_cat_skip_embadd", "s1_8_cat_skip", "s1_2_cat", "s1_2_conv2_skip",
                             "point_1_cat_skip", "s2_32", "up_16"]
    flagsets = [0, 1, 2, 4, 8 | 16, 1 | 2 | 4 | 8 | 16, 127, 32] if dbg else [0]
    for name in names:
        p = T._make(name)
        fn = prepared(p)
        row = []
        for fl in flagsets:
            if dbg:
                dbg.argtypes = [ctypes.c_int]
                dbg(fl)
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            # GPU time only: 20 calls captured in a graph, replayed (no host launch overhead in the timing)
            n = 20
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(n):
                    fn()
            for _ in range(10):
                g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            row.append(f"{fl:3d}:{e0.elapsed_time(e1) / (5 * n) * 1e3:6.1f}")
        print(f"{name:24s} " + "  ".join(row) + "   (us per call, graph-replayed)", flush=True)
        if hasattr(L, "fmd_debug_small_ts"):
            if dbg:
                dbg(0)
            phase_times(L, fn, name)
            if dbg:
                dbg(128)
                phase_times(L, fn, name + " x2")
                dbg(0)
    if dbg:
        dbg(0)


if __name__ == "__main__":
    main()
