"""Phase timeline of the v10 halo conv (GPU box; needs the -DFMD_HALO_TIME variant library built by
tools/build_variant.sh time -DFMD_HALO_TIME).

usage: FMD_LIB=flow-matching-and-diffusion-models_amd/fmdiff/lib/variants/libfmdiff_time.so \
       python tools/h10_timeline.py [--prob fwd|resid|dgrad] [--hw 256] [--c 128]
One armed launch after a warm-up; per chunk interval g (medians over workgroups, shader-clock ticks):
  consumer: MFMA stream (stamp 1 - 0), barrier wait (next 0 - 1), epilogue (3 - 2 at a tile's last chunk)
  producer: commit (1 - 0), issue (2 - 1), jobs (3 - 2), barrier wait (next 0 - 3)
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "flow-matching-and-diffusion-models_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from fmdiff import _lib  # noqa: E402
from fmdiff.runtime import ops  # noqa: E402

NS = 512


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prob", default="fwd")
    ap.add_argument("--hw", type=int, default=256)
    ap.add_argument("--c", type=int, default=128)
    a = ap.parse_args()
    assert "time" in _lib.LIB_PATH, "set FMD_LIB to the -DFMD_HALO_TIME variant"
    dev = torch.device("cuda", 0)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    N, H, C, K = 8, a.hw, a.c, a.c
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(N, H, H, C, device=dev, generator=g).to(torch.bfloat16)
    x2 = torch.randn(N, H, H, C, device=dev, generator=g).to(torch.bfloat16)
    wf = torch.randn(K, C, 3, 3, device=dev, generator=g) * 0.03
    w, wd = ops.prep_weights(wf, 0), ops.prep_weights(wf, 3)
    wt, wdt = ops.tile_weights(w), ops.tile_weights(wd)
    pa, pb = torch.rand(N, C, device=dev) + 0.5, torch.randn(N, C, device=dev) * 0.1
    bias = torch.zeros(K, device=dev)
    fns = dict(fwd=lambda: ops.conv(x, K, w, pro=(pa, pb, True), bias=bias, want_stats=True, wgt_tiled=wt),
               resid=lambda: ops.conv(x, K, w, pro=(pa, pb, True), bias=bias, resid=x2, want_stats=True, wgt_tiled=wt),
               dgrad=lambda: ops.conv(x, C, wd, want_stats=True, ep=(x2, None, pa, pb), wgt_tiled=wdt))
    fn = fns[a.prob]
    L = _lib.lib()
    buf = torch.zeros(256 * 2 * NS + 1024, dtype=torch.int64, device=dev)
    L.fmd_debug_halo_timebuf(ctypes.c_void_p(buf.data_ptr()))
    for _ in range(200):
        fn()
    torch.cuda.synchronize()
    buf.zero_()
    fn()
    torch.cuda.synchronize()
    t = buf[:256 * 2 * NS].view(256, 2, NS).cpu().numpy().astype(np.int64)
    ntiles = N * (H // 16) ** 2 * ((K + 127) // 128)
    nch = -(-C // 32)
    G = min(256, ntiles)
    nt = -(-ntiles // G)
    total = nt * nch
    cons, prod = t[:G, 0], t[:G, 1]
    base = np.minimum(cons[:, 0], prod[:, 0])[:, None]
    print(f"{a.prob} {N}x{H}^2 {C}->{K}: {G} workgroups x {nt} tiles x {nch} chunks; ticks relative to each "
          f"workgroup's first stamp (medians over workgroups)")
    print(" g | cons mma  wait  epi | prod commit (ldwait) issue  jobs  wait | cons start  prod start")
    sums = np.zeros(9)
    for gi in range(total):
        c0, c1 = cons[:, 4 * gi], cons[:, 4 * gi + 1]
        cn = cons[:, 4 * (gi + 1)] if gi + 1 < total else None
        p0, p1, p2, p3 = (prod[:, 4 * gi + k] for k in range(4))
        pn = prod[:, 4 * (gi + 1)] if gi + 1 < total else None
        last = (gi + 1) % nch == 0
        mma = np.median(c1 - c0)
        epi = np.median(cons[:, 4 * gi + 3] - cons[:, 4 * gi + 2]) if last else 0
        cw = np.median(cn - c1) - epi if cn is not None else 0
        cm, iss, jb = np.median(p1 - p0), np.median(p2 - p1), np.median(p3 - p2)
        lw = np.median(prod[:, 256 + gi] - p0) if 256 + gi < NS and prod[:, 256 + gi].any() else 0
        pw = np.median(pn - p3) if pn is not None else 0
        sums += [mma, cw, epi, cm, iss, jb, pw, 0, 0]
        print(f"{gi:2d} | {mma:8.0f} {cw:5.0f} {epi:4.0f} | {cm:11.0f} ({lw:6.0f}) {iss:5.0f} {jb:5.0f} {pw:5.0f} | "
              f"{np.median(c0 - base[:, 0]):10.0f} {np.median(p0 - base[:, 0]):10.0f}")
    print(f"sum | {sums[0]:8.0f} {sums[1]:5.0f} {sums[2]:4.0f} | {sums[3]:11.0f} {sums[4]:5.0f} {sums[5]:5.0f} "
          f"{sums[6]:5.0f}")
    life = np.median(cons[:, 4 * (total - 1) + 3] - cons[:, 0])
    print(f"consumer stamped lifetime (first chunk start -> last epilogue end): {life:.0f} ticks; MFMA floor "
          f"{total * 144 * 32} ticks")


if __name__ == "__main__":
    main()
