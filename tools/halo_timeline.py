"""Phase timeline of the halo conv (GPU box; needs the -DFMD_HALO_TIME variant library).

usage: FMD_LIB=flow-matching-and-diffusion-models_amd/fmdiff/lib/variants/libfmdiff_time.so \
       python tools/halo_timeline.py [--prob fwd|fwd0|dgrad] [--out gpurun_out/halo_time.npy]
Runs the conv_micro problem warm, then one launch with the timestamp buffer armed, and saves the raw
[workgroups][2 waves][32] u64 buffer (HW_ID, XCC_ID, s_memtime per phase) for tools/halo_timeline_report.py.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prob", default="fwd")
    ap.add_argument("--hw", type=int, default=256)
    ap.add_argument("--c", type=int, default=128)
    ap.add_argument("--out", default="gpurun_out/halo_time.npy")
    a = ap.parse_args()
    assert "time" in _lib.LIB_PATH, "set FMD_LIB to the -DFMD_HALO_TIME variant"
    dev = torch.device("cuda", 0)
    N, H, W, C, K = 8, a.hw, a.hw, a.c, a.c
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(N, H, W, C, device=dev, generator=g).to(torch.bfloat16)
    x2 = torch.randn(N, H, W, C, device=dev, generator=g).to(torch.bfloat16)
    wf = torch.randn(K, C, 3, 3, device=dev, generator=g) * 0.03
    w = ops.prep_weights(wf, 0)
    wt = ops.tile_weights(w)
    wd = ops.prep_weights(wf, 3)
    wdt = ops.tile_weights(wd)
    pa = torch.rand(N, C, device=dev) + 0.5
    pb = torch.randn(N, C, device=dev) * 0.1
    bias = torch.zeros(K, device=dev)
    out = torch.empty(N, H, W, K, device=dev, dtype=torch.bfloat16)
    fns = dict(fwd=lambda: ops.conv(x, K, w, pro=(pa, pb, True), bias=bias, out=out, want_stats=True, wgt_tiled=wt),
               fwd0=lambda: ops.conv(x, K, w, bias=bias, out=out, want_stats=True, wgt_tiled=wt),
               dgrad=lambda: ops.conv(x, C, wd, out=out, want_stats=True, ep=(x2, None, pa, pb), wgt_tiled=wdt))
    fn = fns[a.prob]
    L = _lib.lib()
    nwg = N * (H // 16) * (W // 16) * ((K + 127) // 128)
    buf = torch.zeros(nwg * 2 * 32 + 1024, dtype=torch.int64, device=dev)
    # the instrumented kernel stores unconditionally: the buffer is armed before the first launch
    L.fmd_debug_halo_timebuf(ctypes.c_void_p(buf.data_ptr()))
    for _ in range(300):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"{a.prob}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us/launch (instrumented build)")
    buf.zero_()
    fn()
    torch.cuda.synchronize()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    np.save(a.out, buf[:nwg * 64].view(nwg, 2, 32).cpu().numpy())
    print("saved", a.out)


if __name__ == "__main__":
    main()
