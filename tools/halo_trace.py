"""Per-phase timing of the halo conv (GPU box): s_memtime stamps from the first 16 workgroups.

usage: python tools/halo_trace.py [--case fwd|dgrad|cat]
Prints, per tap-step, the median cycles spent in: load issue -> compute issue, compute -> store done,
store -> barrier released; plus prologue / epilogue lengths.
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

TRACE_WG, STEPS, PH = 16, 40, 4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="fwd")
    ap.add_argument("--hw", type=int, default=256)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    N, H, W, C, K = 8, a.hw, a.hw, 128, 128
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(N, H, W, C, device=dev, generator=g).to(torch.bfloat16)
    x2 = torch.randn(N, H, W, C, device=dev, generator=g).to(torch.bfloat16)
    Cin = 2 * C if a.case == "cat" else C
    w = ops.prep_weights(torch.randn(K, Cin, 3, 3, device=dev, generator=g) * 0.03, 0)
    wt = ops.tile_weights(w)
    pa = torch.rand(N, Cin, device=dev) + 0.5
    pb = torch.randn(N, Cin, device=dev) * 0.1
    out = torch.empty(N, H, W, K, device=dev, dtype=torch.bfloat16)

    def run():
        if a.case == "dgrad":
            ops.conv(x, K, w, out=out, want_stats=True, ep=(x2, None, pa, pb), wgt_tiled=wt)
        else:
            ops.conv(x, K, w, src1=x2 if a.case == "cat" else None, pro=(pa, pb, True), out=out,
                     want_stats=True, wgt_tiled=wt)

    for _ in range(3):
        run()
    buf = torch.zeros(TRACE_WG * 8 * STEPS * PH, dtype=torch.int64, device=dev)
    L = _lib.lib()
    L.fmd_debug_halo_trace.argtypes = [ctypes.c_void_p]
    L.fmd_debug_halo_trace(ctypes.c_void_p(buf.data_ptr()))
    run()
    torch.cuda.synchronize()
    L.fmd_debug_halo_trace(ctypes.c_void_p(0))
    t = buf.view(TRACE_WG, 8, STEPS, PH).cpu().double()
    nsteps = int((t[0, 0, 1:, 0] > 0).sum())
    t0 = t[:, :, 0, 0]
    print(f"case {a.case}: {nsteps} steps traced, {TRACE_WG} WGs x 8 waves")
    pro = (t[:, :, 1, 0] - t0).median().item()
    print(f"prologue (start -> step1 load issued): {pro:.0f} cycles")
    rows = []
    for s in range(1, nsteps + 1):
        ld = (t[:, :, s, 0] - (t[:, :, s - 1, 3] if s > 1 else t[:, :, 1, 0])).median().item()
        cmp_ = (t[:, :, s, 1] - t[:, :, s, 0]).median().item()
        st = (t[:, :, s, 2] - t[:, :, s, 1]).median().item()
        bar = (t[:, :, s, 3] - t[:, :, s, 2]).median().item()
        tot = (t[:, :, s, 3] - (t[:, :, s - 1, 3] if s > 1 else t[:, :, 1, 0])).median().item()
        rows.append((s, ld, cmp_, st, bar, tot))
        print(f"step {s:2d}: issue-loads {ld:6.0f}  compute {cmp_:6.0f}  store {st:6.0f}  barrier {bar:6.0f}  total {tot:6.0f}")
    main_end = t[:, :, 0, 1]
    epi = (t[:, :, 0, 2] - main_end).median().item()
    total = (t[:, :, 0, 2] - t0).median().item()
    print(f"epilogue (to stats): {epi:.0f} cycles; whole WG: {total:.0f} cycles")
    # per-wave spread of the store phase (who waits for whom)
    for wv in range(8):
        st = (t[:, wv, 2:nsteps, 2] - t[:, wv, 2:nsteps, 1]).median().item()
        cp = (t[:, wv, 2:nsteps, 1] - t[:, wv, 2:nsteps, 0]).median().item()
        print(f"  wave {wv}: compute {cp:6.0f} store {st:6.0f}")


if __name__ == "__main__":
    main()
