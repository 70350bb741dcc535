"""Tensor-level launchers over the C ABI (device memory from PyTorch's allocator).

Every function launches on the current HIP stream and returns new device
tensors; none of them synchronises, so the whole train / sample step can be
captured into a hipGraph.  Activations are NHWC bf16 ``[N, H, W, C]``.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional, Tuple

import torch

from .. import _lib
from . import tuning
from .._lib import ConvDesc, GnApplyDesc, GnOutDesc, WgradDesc

BF16 = torch.bfloat16
F32 = torch.float32
NUM_CU = 256


def _p(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _need_cuda(t: torch.Tensor, what: str):
    if t.device.type != "cuda":
        raise RuntimeError(f"{what}: fmdiff HIP kernels need ROCm device tensors (got {t.device}); "
                           "there is no CPU path")


@dataclass
class Stats:
    """Per-channel partial sums of an activation: slab [N*HW/rows][C][2] (sum, sum of squares)."""
    slab: torch.Tensor
    rows: int


def channel_stats(x: torch.Tensor, rows: Optional[int] = None, y: Tuple = None) -> Stats:
    """(sum x, sum x^2) per (n, channel, row-block), or (sum x, sum x*y) when ``y=(y0, y1, C0)`` is given."""
    N, Cc = x.shape[0], x.shape[-1]
    HW = x[0, ..., 0].numel()   # pixels per image (H*W, or D*H*W for NDHWC)
    if rows is None:
        # 64-pixel slab rows (like the conv epilogues): enough blocks to cover the chip even at 32x32
        rows = 64 if HW % 64 == 0 else HW
    slab = torch.empty((N * HW // rows, Cc, 2), device=x.device, dtype=F32)
    y0, y1, C0 = (None, None, Cc) if y is None else y
    _lib.call("fmd_channel_stats", _p(x), _p(y0), _p(y1), C0, N, HW, Cc, rows, _p(slab), stream())
    return Stats(slab, rows)


# slabs with at least STATS_FOLD_MIN rows per image are folded STATS_FOLD rows at a time before the GroupNorm
# (n, group) reductions (fmd_stats_fold): config E's 128^3 levels (32768 rows of 64 pixels)
STATS_FOLD_MIN = tuning.get("STATS_FOLD_MIN")
STATS_FOLD = 128


def fold_stats(st: Optional[Stats], HW: int) -> Optional[Stats]:
    """``st`` with STATS_FOLD consecutive slab rows summed (same per-image sums), or ``st`` itself when small."""
    if st is None or not STATS_FOLD_MIN:
        return st
    E = HW // st.rows
    C = st.slab.shape[1]
    if E < STATS_FOLD_MIN or E % STATS_FOLD or C % 2 or not st.slab.is_contiguous():
        return st
    rows_total = st.slab.shape[0]
    out = torch.empty((rows_total // STATS_FOLD, C, 2), device=st.slab.device, dtype=F32)
    _lib.call("fmd_stats_fold", _p(st.slab), rows_total, C, STATS_FOLD, _p(out), stream())
    return Stats(out, st.rows * STATS_FOLD)


def gn_prep(st0: Stats, st1: Optional[Stats], N: int, HW: int, C0: int, C1: int, groups: int, eps: float,
            gamma, beta, emb=None, emb_stride=0, emb_mode=0):
    """Fold GroupNorm (+ scale/shift) into a[n][c], b[n][c]; returns (a, b, mean_rstd)."""
    st0, st1 = fold_stats(st0, HW), fold_stats(st1, HW)
    dev = st0.slab.device
    Ct = C0 + C1
    a = torch.empty((N, Ct), device=dev, dtype=F32)
    b = torch.empty((N, Ct), device=dev, dtype=F32)
    mr = torch.empty((N, groups, 2), device=dev, dtype=F32)
    _lib.call("fmd_gn_prep", _p(st0.slab), st0.rows, _p(st1.slab) if st1 else None, st1.rows if st1 else 1,
              N, HW, C0, C1, groups, float(eps), _p(gamma), _p(beta), _p(emb), emb_stride, emb_mode,
              _p(a), _p(b), _p(mr), stream())
    return a, b, mr


# deferred gamma/beta gradient folds (gb_defer / gb_flush): (ws, N, C, dgamma, dbeta) per GroupNorm backward
_gb_pending: Optional[list] = None


def gb_defer():
    """Start collecting gn_bwd_prep's gamma/beta folds; gb_flush() applies them in batched launches."""
    global _gb_pending
    _gb_pending = []


def gb_flush():
    """Fold every deferred (dgamma, dbeta) contribution (fmd_gn_gb_fold, <= GB_MAX jobs per launch) and stop
    deferring.  Same sums in the same order as the per-call fold."""
    global _gb_pending
    jobs, _gb_pending = _gb_pending or [], None
    for i in range(0, len(jobs), _lib.GB_MAX):
        part = jobs[i:i + _lib.GB_MAX]
        arr = (_lib.GbJob * len(part))()
        for k, (ws, N, Cc, dg, dbt) in enumerate(part):
            arr[k].ws, arr[k].dgamma, arr[k].dbeta, arr[k].N, arr[k].C = _p(ws), _p(dg), _p(dbt), N, Cc
        _lib.call("fmd_gn_gb_fold", arr, len(part), stream())


def gn_bwd_prep(s12: Stats, N: int, HW: int, Ct: int, groups: int, mr, gamma, beta, dgamma, dbeta,
                emb=None, emb_stride=0, emb_mode=0, demb=None, demb_stride=0, fwd: Optional[Stats] = None):
    s12, fwd = fold_stats(s12, HW), fold_stats(fwd, HW)
    dev = s12.slab.device
    P = torch.empty((N, Ct), device=dev, dtype=F32)
    Q = torch.empty((N, Ct), device=dev, dtype=F32)
    R = torch.empty((N, Ct), device=dev, dtype=F32)
    ws = torch.empty((N, Ct, 2), device=dev, dtype=F32)
    if _gb_pending is not None and (dgamma is not None or dbeta is not None):
        _gb_pending.append((ws, N, Ct, dgamma, dbeta))   # ws stays referenced until the fold is issued
        dgamma = dbeta = None
    _lib.call("fmd_gn_bwd_prep", _p(s12.slab), s12.rows, N, HW, Ct, groups, _p(mr), _p(gamma), _p(beta), _p(emb),
              emb_stride, emb_mode, _p(P), _p(Q), _p(R), _p(dgamma), _p(dbeta), _p(demb), demb_stride,
              _p(fwd.slab) if fwd else None, fwd.rows if fwd else 1, _p(ws), stream())
    return P, Q, R


def gn_apply_fwd(x0, x1, a, b, silu=True):
    """t = SiLU(a*x + b) over the channel concat of x0|x1 (NHWC bf16): the materialised GN prologue."""
    N, C0 = x0.shape[0], x0.shape[-1]
    HW = x0[0, ..., 0].numel()                    # any spatial rank (N, *sp, C)
    C1 = x1.shape[-1] if x1 is not None else 0
    t = torch.empty((*x0.shape[:-1], C0 + C1), device=x0.device, dtype=BF16)
    _lib.call("fmd_gn_apply_fwd", _p(x0), _p(x1), C0, C1, N * HW, HW, _p(a), _p(b), int(silu), _p(t), stream())
    return t


GN_FUSED_MAX = 16384   # elements per (n, group) that fmd_gn_fused_apply holds in one workgroup's registers
GN_FUSED = bool(tuning.get("GN_FUSED"))   # A/B switch (0: slab statistics + gn_prep + apply)


def gn_fused_eligible(HW: int, C: int, C0: int, groups: int) -> bool:
    """Mirror of fmd_gn_fused_apply's applicability test (csrc/groupnorm.hip)."""
    Cg = C // groups if C % groups == 0 else 0
    return GN_FUSED and Cg > 0 and Cg % 4 == 0 and C0 % 4 == 0 and 256 % (Cg // 4) == 0 and HW * Cg <= GN_FUSED_MAX


# the GroupNorm forward of a split-K conv's output inside its combine (fmd_conv_gn); CONV_GN=0 (runtime/tuning.py): the separate
# fmd_gn_fused_apply launch (A/B runs)
CONV_GN = bool(tuning.get("CONV_GN"))
# fewest combine blocks (images x channel blocks) for which the fused form beats the two launches it replaces
# (latent step profile: 64 blocks 13.1 us vs 5-7 + 5.2 us; 128 blocks 8.0 us, 256 blocks 7.2 us)
CONV_GN_MIN_BLOCKS = tuning.get("CONV_GN_MIN_BLOCKS")
CONV_GN_CB = tuning.get("CONV_GN_CB")   # fewest channels per combine block (fmd_conv_gn; _lib sets the library's)
if CONV_GN_CB not in (4, 8, 16, 32, 64):
    raise ValueError(f"CONV_GN_CB must be 4, 8, 16, 32 or 64, not {CONV_GN_CB}")


def conv_gn_eligible(K: int, groups: int, N: int = 1 << 30) -> bool:
    """Mirror of fmd_conv_gn's channel test (whole groups per block of max(CONV_GN_CB, K/groups) <= 64 channels,
    CONV_GN_CB from runtime/tuning.py, default 4) plus the block-count floor."""
    if K % 64 or K % groups or 64 % (K // groups):
        return False
    return N * (K // max(CONV_GN_CB, K // groups)) >= CONV_GN_MIN_BLOCKS


def gn_fused_apply(x0, x1, groups: int, eps: float, gamma, beta, emb=None, emb_stride=0, emb_mode=0, silu=True):
    """GroupNorm of x0|x1 from the activations themselves (no statistics slab): returns (a, b, mean_rstd, t)
    with t = SiLU(a*x + b) materialised -- channel_stats + gn_prep + gn_apply_fwd in one launch."""
    N, C0 = x0.shape[0], x0.shape[-1]
    HW = x0[0, ..., 0].numel()
    C1 = x1.shape[-1] if x1 is not None else 0
    Ct = C0 + C1
    dev = x0.device
    a = torch.empty((N, Ct), device=dev, dtype=F32)
    b = torch.empty((N, Ct), device=dev, dtype=F32)
    mr = torch.empty((N, groups, 2), device=dev, dtype=F32)
    t = torch.empty((*x0.shape[:-1], Ct), device=dev, dtype=BF16)
    _lib.call("fmd_gn_fused_apply", _p(x0), _p(x1), C0, C1, N, HW, groups, float(eps), _p(gamma), _p(beta), _p(emb),
              emb_stride, emb_mode, int(silu), _p(a), _p(b), _p(mr), _p(t), stream())
    return a, b, mr, t


def dropout_apply(x, p: float, seed: torch.Tensor, salt: int, ep=None, out=None):
    """y = x * keep / (1 - p) over NHWC bf16 ``x``, keep regenerated from (seed[0], salt, element index)
    (fmd_dropout_apply); ``ep=(h, a, b)``: the backward through the dropout and the GN+SiLU prologue,
    y = x * keep / (1 - p) * silu'(a * h + b).  ``out`` may be ``x`` (in place)."""
    _need_cuda(x, "dropout")
    N, Cc = x.shape[0], x.shape[-1]
    HW = x[0, ..., 0].numel()
    y = torch.empty_like(x) if out is None else out
    h, a, b = ep if ep is not None else (None, None, None)
    _lib.call("fmd_dropout_apply", _p(x), Cc, N * HW, HW, float(p), _p(seed), int(salt) & 0xffffffff, _p(h), _p(a),
              _p(b), _p(y), stream())
    return y


def gn_bwd_apply(dz, x0, x1, P, Q, R, extra, dx0, acc0, dx1=None, acc1=0):
    N = dz.shape[0]
    HW = dz[0, ..., 0].numel()                    # any spatial rank (N, *sp, C)
    C0 = x0.shape[-1]
    C1 = x1.shape[-1] if x1 is not None else 0
    _lib.call("fmd_gn_bwd_apply", _p(dz), _p(x0), _p(x1), C0, C1, N * HW, HW, _p(P), _p(Q), _p(R),
              _p(extra), _p(dx0), int(acc0), _p(dx1), int(acc1), stream())


def conv1x1_gn_apply(dy, wgt_t, dz, x0, x1, P, Q, R, dx0, acc0, dx1=None, acc1=0):
    """dx = dy @ W^T (1x1 data gradient, ``wgt_t`` = mode-1 weights [C][1][K]) + P*dz + Q*x + R (+ dx):
    the ResBlock skip-conv data gradient fused into the block input's GroupNorm backward
    (fmd_conv_gn_apply; == conv(..., transposed=True) followed by gn_bwd_apply(extra=...))."""
    _need_cuda(dy, "conv1x1_gn_apply")
    N, Kd = dy.shape[0], dy.shape[-1]
    W = dy.shape[-2]
    H = dy[0, ..., 0, 0].numel()                  # pointwise: a (D, H, W) volume runs as a (D*H, W) plane
    Ct = dz.shape[-1]
    d = ConvDesc()
    d.N, d.Hs, d.Ws, d.C0, d.C1, d.Ho, d.Wo, d.K = N, H, W, Kd, 0, H, W, Ct
    d.ks, d.stride, d.pad, d.upsample, d.transposed = 1, 1, 0, 0, 1
    d.src0, d.wgt, d.splits = _p(dy), _p(wgt_t), 1
    g = GnApplyDesc()
    g.dz, g.x0, g.x1, g.C0 = _p(dz), _p(x0), _p(x1), x0.shape[-1]
    g.P, g.Q, g.R = _p(P), _p(Q), _p(R)
    g.dx0, g.acc0, g.dx1, g.acc1 = _p(dx0), int(acc0), _p(dx1), int(acc1)
    _lib.call("fmd_conv_gn_apply", C.byref(d), C.byref(g), stream())


def out_hw(Hs, ks, stride, pad, upsample):
    Hin = Hs * (2 if upsample else 1)
    return (Hin + 2 * pad - ks) // stride + 1


# split-K of the generic implicit GEMM on small grids: >= SPLIT_MIN_STEPS k-steps per split, about
# SPLIT_CU_MULT workgroups per CU, at most SPLIT_CAP splits (env overrides for A/B measurements)
SPLIT_MIN_STEPS = tuning.get("SPLIT_MIN_STEPS")
SPLIT_CU_MULT = tuning.get("SPLIT_CU_MULT")
SPLIT_CAP = tuning.get("SPLIT_CAP")
# outputs of at most BPX64_M pixels (K > 64, split-K) run on 64-pixel tiles (csrc/conv.hip small_m)
# (train step 24.94 / 25.03 -> 24.83 / 24.87 ms, config D batch 8 77 -> 82.6 images/s); at most BPX32_M: 32-pixel
# tiles (the latent UNet's 4x4 .. 1x1 levels: 82.3 -> 83.1 images/s)
BPX64_M = 2048
BPX32_M = 128


def _choose_splits(M, K, nk, bpx=128, bco=128):
    tiles = -(-M // bpx) * -(-K // bco)
    if tiles >= NUM_CU or nk < 8:
        return 1
    return max(1, min(nk // SPLIT_MIN_STEPS, -(-SPLIT_CU_MULT * NUM_CU // tiles), SPLIT_CAP))


HALO_CMAX = 512   # widest GN-prologue input of the halo kernel's affine table (csrc/conv_halo.hip CMAX)
HALO_BK = 32      # input channels per halo chunk (FMD_HALO_BK)
SPLIT_STATS_ROWS = 16   # pixels per statistics row of a split-K conv (FMD_SPLIT_STATS_ROWS)


# halo split-K on the small levels: ~HALO_SPLIT_WG workgroups, >= HALO_MIN_CHUNKS 32-channel chunks per split,
# <= HALO_SPLIT_CAP splits (env overrides for A/B runs)
HALO_SPLIT_WG = tuning.get("HALO_SPLIT_WG")
# forward-only GroupNorm folded in the halo conv's prologue from the statistics slabs (fmd_conv_desc.fold_*) where
# the slab has at most HALO_FOLD_MAX_ROWS rows per image (runtime/tuning.py)
HALO_FOLD = bool(tuning.get("HALO_FOLD"))
HALO_FOLD_MAX_ROWS = tuning.get("HALO_FOLD_MAX_ROWS")
# split-K halo convs (2-D) combine their parts inside the launch (fmd_conv_desc.tickets; statistics from the conv
# epilogue with 64-pixel rows) instead of the splitk_reduce_rows launch
HALO_TICKET = bool(tuning.get("HALO_TICKET"))
SPLIT_TICKET = bool(tuning.get("SPLIT_TICKET"))   # the implicit GEMM's split-K likewise (whole tiles)
HALO_MIN_CHUNKS = tuning.get("HALO_MIN_CHUNKS")
HALO_SPLIT_CAP = tuning.get("HALO_SPLIT_CAP")
# fewest halo workgroups (tiles x splits); mirrors fmd_halo_set_min_workgroups (tuning HALO_MIN_WG, applied at _lib load)
HALO_MIN_WG = tuning.get("HALO_MIN_WG")


def halo_splits(N, Ho, Wo, K, Cin, ztaps=1) -> int:
    """Split-K factor the halo kernel uses: 1 when the 16x16 tiles x cout tiles already give >= 128
    workgroups, else enough chunk-range splits (>= 2 chunks each) to reach ~256; 0 = not eligible
    (fewer than HALO_MIN_WG workgroups)."""
    nwg = N * (Ho // 16) * (Wo // 16) * -(-K // 128)
    if nwg >= max(128, HALO_MIN_WG):   # the kernel's own threshold (fmd_halo_set_min_workgroups) may be higher
        return 1
    nch = -(-max(Cin, 1) // HALO_BK) * ztaps
    sp = min(-(-HALO_SPLIT_WG // max(nwg, 1)), nch // HALO_MIN_CHUNKS, HALO_SPLIT_CAP)
    if sp < 2 and nwg >= HALO_MIN_WG:
        return 1
    if sp < 2 or nwg * sp < HALO_MIN_WG:
        return 0
    cps = -(-nch // sp)
    while sp > 1 and (sp - 1) * cps >= nch:   # every split owns at least one chunk (mirrors the kernel)
        sp -= 1
    return sp if nwg * sp >= HALO_MIN_WG else 0


def halo_eligible(N, Hs, Ho, Wo, K, ks=3, stride=1, pad=1, upsample=False, transposed=False, Cin=0,
                  pro=False, ztaps=1) -> bool:
    """Mirror of fmd_conv_halo's applicability test (csrc/conv_halo.hip): 3x3 s1 p1 forward gather,
    16x16 output tiles, K > 16, at least HALO_MIN_WG (default 32) workgroups (with split-K over channel chunks
    when the level is small), GN-prologue inputs of at most HALO_CMAX channels."""
    Ws = Wo // 2 if upsample else Wo
    return (K > 16 and ks == 3 and stride == 1 and pad == 1 and not transposed and not (pro and Cin > HALO_CMAX)
            and Ho % 16 == 0 and Wo % 16 == 0 and (Ho == 2 * Hs if upsample else Ho == Hs)
            and N * Hs * Ws * max(Cin, 1) < (1 << 31)   # the kernel's 32-bit element offsets (conv_halo.hip)
            and halo_splits(N, Ho, Wo, K, Cin, ztaps) > 0)


def s2d_eligible(N, Hs, Ws, Ho, Wo, K, C, ks, Ds=0, Do=0) -> bool:
    """Mirror of fmd_conv_s2d's applicability test (csrc/conv_halo9.hip): a stride-2 pad-1 3x3 / 4x4 forward
    gather onto 16x16 output tiles, C % 32 == 0, K % 128 == 0, >= 128 workgroups.  3-D: ``Ds`` = 2 ``Do`` input /
    output depths (stride 2 in depth too; the depth taps run as chunks)."""
    d3 = Ds > 0 or Do > 0
    if d3 and Ds != 2 * Do:
        return False
    Ni, No = N * (Ds if d3 else 1), N * (Do if d3 else 1)
    return (ks in (3, 4) and Hs == 2 * Ho and Ws == 2 * Wo and Ho % 16 == 0 and Wo % 16 == 0 and C % 32 == 0
            and K % 128 == 0 and No * (Ho // 16) * (Wo // 16) * (K // 128) >= 128
            and Ni * Hs * Ws * C < (1 << 31) and No * Ho * Wo * K < (1 << 31))


def d2s_eligible(N, Hs, Ws, Ho, Wo, K, C, Ds=0, Do=0) -> bool:
    """Mirror of fmd_conv_d2s's applicability test: the transposed gather of a stride-2 pad-1 3x3 conv from an
    Hs x Ws gradient (multiples of 16) onto Ho = 2 Hs, Wo = 2 Ws, C % 32 == 0, K % 128 == 0, >= 128 workgroups.
    3-D: ``Do`` = 2 ``Ds`` (8 output classes per tile)."""
    d3 = Ds > 0 or Do > 0
    if d3 and Do != 2 * Ds:
        return False
    Ni, No = N * (Ds if d3 else 1), N * (Do if d3 else 1)
    return (Ho == 2 * Hs and Wo == 2 * Ws and Hs % 16 == 0 and Ws % 16 == 0 and C % 32 == 0 and K % 128 == 0
            and Ni * (Hs // 16) * (Ws // 16) * (8 if d3 else 4) * (K // 128) >= 128
            and Ni * Hs * Ws * C < (1 << 31) and No * Ho * Wo * K < (1 << 31))


def s2d_tile_weights(w: torch.Tensor, mode: int, out=None) -> torch.Tensor:
    """fp32 [K][C][ks][ks] (3-D: [K][C][3][3][3]) -> fmd_conv_s2d / fmd_conv_d2s tiles (mode 0 stride-2 forward,
    1 data gradient of a 3x3 conv on a nearest-x2 input, 2 stride-2 3x3 data gradient)."""
    K, Cc, ks = w.shape[0], w.shape[1], w.shape[2]
    dims = w.dim() - 2
    n = int(_lib.lib().fmd_s2d_tiled_size_nd(K, Cc, mode, ks, dims))
    if out is None:
        out = torch.empty((n,), device=w.device, dtype=BF16)
    _lib.call("fmd_s2d_tile_weights_nd", _p(w.contiguous()), K, Cc, ks, mode, dims, _p(out), stream())
    return out


def conv(src0, K, wgt, *, src1=None, ks=3, stride=1, pad=1, upsample=False, transposed=False, out_hw_=None,
         pro=None, src2=None, src3=None, wgt2=None, bias=None, bias2=None, bias_nc=None, resid=None, out=None,
         out_f32=False,
         accumulate=False, want_stats=False, ep=None, splits=None, force_generic=False, wgt_tiled=None,
         wgt2_tiled=None, gout=None, s2d_tiled=None, gn=None,
         pro_fold=None) -> Tuple[torch.Tensor, Optional[Stats]]:
    """Implicit-GEMM conv (see csrc/conv.hip, csrc/conv_halo.hip).  ``pro=(a, b, silu)``, ``ep=(x0, x1, a, b)``.
    ``want_stats``: True = per-channel statistics of the output (a separate fmd_channel_stats pass when the
    kernel cannot emit them); "free" = only when the kernel emits them (else None: Act statistics are then
    derived on demand, and a small-level consumer that computes its own GroupNorm never pays for them).
    ``gout``: bf16 tensor shaped like the (concatenated) input; the halo path writes the prologue's output
    G = SiLU(a*x+b) into it (the weight gradient's operand).  Requires ``pro``, (C0+C1) % 32 == 0 and a
    halo-eligible problem (:func:`halo_eligible`); raises otherwise.
    ``pro_fold``: dict(st0=Stats, st1=Stats or None, groups, eps, gamma, beta[, emb, emb_stride], silu) -- a
    forward-only GroupNorm prologue in place of ``pro``: on the halo path each workgroup folds its sample's affine
    from the statistics slabs (fmd_conv_desc.fold_*, no gn_prep launch); elsewhere it is folded by :func:`gn_prep`
    first and passed as ``pro``.
    ``gn``: dict(groups, eps, gamma, beta[, emb, emb_stride, emb_mode]) -- when the conv runs split-K and
    :func:`conv_gn_eligible` holds, its combine also computes the GroupNorm + SiLU of the output (fmd_conv_gn)
    and stores ``gn["res"] = (a, b, mean_rstd, t)`` as :func:`gn_fused_apply` returns them; otherwise ``gn`` is
    left without "res" and the caller runs the GroupNorm itself.
    ``s2d_tiled``: :func:`s2d_tile_weights` of the stride-2 conv's weight -- the problem runs on the space-to-depth
    halo kernel (fmd_conv_s2d; the caller checks :func:`s2d_eligible`), ``wgt`` unused."""
    _need_cuda(src0, "conv")
    # 3-D (spatial_dims = 3): NDHWC tensors, cubic kernels; ``out_hw_`` is then (Do, Ho, Wo)
    d3 = src0.dim() == 5
    if d3:
        N, Ds, Hs, Ws, C0 = src0.shape
    else:
        N, Hs, Ws, C0 = src0.shape
        Ds = 0
    C1 = src1.shape[-1] if src1 is not None else 0
    if out_hw_ is not None:
        Do, Ho, Wo = out_hw_ if d3 else (0, *out_hw_)
    else:
        Ho, Wo = out_hw(Hs, ks, stride, pad, upsample), out_hw(Ws, ks, stride, pad, upsample)
        Do = out_hw(Ds, ks, stride, pad, upsample) if d3 else 0
    M = N * max(Do, 1) * Ho * Wo
    dev = src0.device
    if out is None:
        shape = (N, Do, Ho, Wo, K) if d3 else (N, Ho, Wo, K)
        out = torch.empty(shape, device=dev, dtype=F32 if out_f32 else BF16)
    d = ConvDesc()
    d.N, d.Hs, d.Ws, d.C0, d.C1, d.Ho, d.Wo, d.K = N, Hs, Ws, C0, C1, Ho, Wo, K
    d.Ds, d.Do = Ds, Do
    d.ks, d.stride, d.pad, d.upsample, d.transposed = ks, stride, pad, int(upsample), int(transposed)
    d.src0, d.src1 = _p(src0), _p(src1)
    if pro is not None:
        d.pro_a, d.pro_b, d.pro_silu = _p(pro[0]), _p(pro[1]), int(pro[2])
    d.wgt = _p(wgt)
    if src2 is not None:
        d.src2, d.src3, d.C2, d.C3, d.wgt2 = _p(src2), _p(src3), src2.shape[-1], (src3.shape[-1] if src3 is not None else 0), _p(wgt2)
    d.bias, d.bias2, d.bias_nc, d.resid, d.out = _p(bias), _p(bias2), _p(bias_nc), _p(resid), _p(out)
    d.out_f32, d.accumulate = int(out_f32), int(accumulate)
    if ep is not None:
        x0, x1, ea, eb = ep
        d.ep_x0, d.ep_x1, d.ep_C0, d.ep_a, d.ep_b = _p(x0), _p(x1), x0.shape[-1], _p(ea), _p(eb)
        if x1 is None and x0.shape[-1] != K:
            raise ValueError("epilogue tensor channels must match the conv output channels")
    T = ks * ks * (ks if d3 else 1)
    # host-side operand checks: the kernels index weights as [>=K rows][T][exactly C0+C1] (main) and
    # [>=K][1][C2+C3] (1x1 segment); halo tiles as [K/128][C/32][9][32][128] blocks
    if wgt is not None and (wgt.dim() != 3 or wgt.shape[0] < K or wgt.shape[1] != T or wgt.shape[2] != C0 + C1):
        raise ValueError(f"conv weights {tuple(wgt.shape)} do not match K={K}, taps={T}, C={C0 + C1}")
    if src2 is not None and wgt2 is not None and (wgt2.shape[0] < K or wgt2.shape[-1] != d.C2 + d.C3):
        raise ValueError(f"1x1 segment weights {tuple(wgt2.shape)} do not match K={K}, C={d.C2 + d.C3}")
    for tw, cc, taps in ((wgt_tiled, C0 + C1, 27 if d3 else 9), (wgt2_tiled if src2 is not None else None,
                                                               d.C2 + d.C3, 1)):
        if tw is not None and tw.numel() < -(-K // 128) * 128 * -(-cc // HALO_BK) * HALO_BK * taps:
            raise ValueError(f"halo-tiled weights ({tw.numel()} elements) too small for K={K}, C={cc}")
    nk = -(-(C0 + C1) // 64) * T + (-(-(d.C2 + d.C3) // 64) if src2 is not None else 0)
    bco = 16 if K <= 16 else (64 if K <= 64 else 128)
    # pixel tile the generic kernel will use IF it runs split-K (csrc/conv.hip fmd_conv: the 64 / 32-pixel tiles
    # exist only for splits > 1); re-decided below once the split count is known
    bpx_split = 256 if K <= 16 else (128 if K <= 64 or M > BPX64_M else (32 if M <= BPX32_M else 64))
    bpx = bpx_split
    if d3:   # depth-tap chunks on the halo kernel: pre-tiled (kz, channel block) weights are required
        halo = (not force_generic and wgt_tiled is not None and Do == (2 * Ds if upsample else Ds) and
                halo_eligible(N * Do, Hs, Ho, Wo, K, ks, stride, pad, upsample, transposed, C0 + C1,
                              pro is not None, ztaps=3))
    else:
        halo = not force_generic and halo_eligible(N, Hs, Ho, Wo, K, ks, stride, pad, upsample, transposed,
                                                   C0 + C1, pro is not None or pro_fold is not None)
    d.force_generic = int(force_generic)
    fold = None
    if pro_fold is not None:
        if pro is not None:
            raise ValueError("conv: pro and pro_fold are exclusive")
        rows_ok = all(st is None or (Hs * Ws) % st.rows == 0 and (Hs * Ws) // st.rows <= HALO_FOLD_MAX_ROWS
                      for st in (pro_fold["st0"], pro_fold.get("st1")))
        if halo and not d3 and gout is None and s2d_tiled is None and HALO_FOLD and rows_ok:
            fold = pro_fold
            _set_fold(d, fold)
        else:
            pro = _fold_now(pro_fold, N, Hs * Ws, C0, C1)
            d.pro_a, d.pro_b, d.pro_silu = _p(pro[0]), _p(pro[1]), int(pro[2])
    if s2d_tiled is not None:   # stride-2 on the halo kernel: one launch, statistics in its epilogue
        ok = (s2d_eligible(N, Hs, Ws, Ho, Wo, K, C0 + C1, ks, Ds, Do) if not transposed else
              (ks == 3 and pro is None and d2s_eligible(N, Hs, Ws, Ho, Wo, K, C0 + C1, Ds, Do)))
        if not ok or stride != 2 or pad != 1 or upsample or src2 is not None or out_f32 or gout is not None:
            raise ValueError("conv: s2d_tiled given for a problem fmd_conv_s2d / fmd_conv_d2s does not take")
        d.wgt_tiled, d.splits = _p(s2d_tiled), 1
        st = None
        if want_stats and (max(Do, 1) * Ho * Wo) % 64 == 0:
            slab = torch.empty((M // 64, K, 2), device=dev, dtype=F32)
            d.stats = _p(slab)
            st = Stats(slab, 64)
        _lib.call("fmd_conv_d2s" if transposed else "fmd_conv_s2d", C.byref(d), stream())
        if want_stats is True and st is None:
            st = channel_stats(out)
        return out, st
    if gout is not None:
        want = (N, Ds, Hs, Ws, C0 + C1) if d3 else (N, Hs, Ws, C0 + C1)
        if pro is None or not halo or (C0 + C1) % HALO_BK or tuple(gout.shape) != want or gout.dtype != BF16:
            raise ValueError(f"gout {tuple(gout.shape)} needs a GN prologue, the halo path and shape {want} bf16")
        d.gout = _p(gout)
    if halo:
        splits = halo_splits(N * max(Do, 1), Ho, Wo, K, C0 + C1, 3 if d3 else 1)
        bpx = 256
        if wgt_tiled is None:
            wgt_tiled = tile_weights(wgt)
        if src2 is not None and wgt2_tiled is None:
            wgt2_tiled = tile_weights(wgt2)
        d.wgt_tiled, d.wgt2_tiled = _p(wgt_tiled), _p(wgt2_tiled)
    if splits is None:
        splits = _choose_splits(M, K, nk, bpx, bco)
    if not halo and splits <= 1 and K > 64:
        bpx = 128   # the kernel's rule: small-pixel tiles only with split-K
    ws = None
    if splits > 1:
        ws = torch.empty((splits, M, K), device=dev, dtype=F32)
        d.ws, d.splits = _p(ws), splits
    else:
        d.splits = 1
    ticket, trows = split_ticket(halo, splits, K, M, bpx, bco, d3=d3, transposed=transposed, stride=stride, ks=ks,
                                 pad=pad, Ho=Ho, Wo=Wo, out_f32=out_f32, accumulate=accumulate,
                                 resid_and_ep=resid is not None and ep is not None, gout=gout is not None)
    st = None
    # statistics from the conv epilogue (no split, or the in-launch combine) or from the split-K combine launch
    # (csrc/conv.hip splitk_reduce_rows)
    fused_stats = want_stats and (max(Do, 1) * Ho * Wo) % 64 == 0 and (
        (splits == 1 and M % bpx == 0) or (splits > 1 and K % 4 == 0 and not out_f32 and not accumulate))
    if fused_stats:
        rows = 64 if splits == 1 else trows if ticket else SPLIT_STATS_ROWS
        slab = torch.empty((M // rows, K, 2), device=dev, dtype=F32)
        d.stats = _p(slab)
        st = Stats(slab, rows)
    if (gn is not None and CONV_GN and splits > 1 and not want_stats and d.stats is None and not out_f32
            and not accumulate and ep is None and conv_gn_eligible(K, gn["groups"], N)):
        a = torch.empty((N, K), device=dev, dtype=F32)
        b = torch.empty((N, K), device=dev, dtype=F32)
        mr = torch.empty((N, gn["groups"], 2), device=dev, dtype=F32)
        t = torch.empty_like(out)
        g = GnOutDesc()
        g.G, g.eps, g.gamma, g.beta = gn["groups"], float(gn["eps"]), _p(gn["gamma"]), _p(gn["beta"])
        emb = gn.get("emb")
        g.emb, g.emb_stride, g.emb_mode = _p(emb), gn.get("emb_stride", 0), gn.get("emb_mode", 0) if emb is not None else 0
        g.silu, g.a, g.b, g.mean_rstd, g.t = int(gn.get("silu", True)), _p(a), _p(b), _p(mr), _p(t)
        _lib.call("fmd_conv_gn", C.byref(d), C.byref(g), stream())
        gn["res"] = (a, b, mr, t)
        return out, None
    if ticket:
        d.tickets, d.n_tickets, d.tickets_rows = _p(_small_workspace(dev)[1]), SMALL_TICKETS, trows
    rc = int(_lib.lib().fmd_conv(C.byref(d), stream()))
    if rc == -14:   # the halo kernel did not take the in-launch combine: the combine launch (16-pixel statistics rows)
        d.tickets, d.n_tickets, d.tickets_rows = None, 0, 0
        if st is not None:
            slab = torch.empty((M // SPLIT_STATS_ROWS, K, 2), device=dev, dtype=F32)
            d.stats = _p(slab)
            st = Stats(slab, SPLIT_STATS_ROWS)
        rc = int(_lib.lib().fmd_conv(C.byref(d), stream()))
    if rc == -13 and fold is not None:   # the halo kernel did not take it: the fold as its own launch
        pro = _fold_now(fold, N, Hs * Ws, C0, C1)
        _clear_fold(d)
        d.pro_a, d.pro_b, d.pro_silu = _p(pro[0]), _p(pro[1]), int(pro[2])
        rc = int(_lib.lib().fmd_conv(C.byref(d), stream()))
    _lib.check(rc, "fmd_conv")
    if want_stats == "free":   # only statistics the kernel emits for free; the consumer derives others lazily
        return out, st
    if want_stats and not fused_stats:
        if ep is not None:
            st = channel_stats(out, y=(ep[0], ep[1], ep[0].shape[-1]))
        else:
            st = channel_stats(out)
    return out, st


def split_ticket(halo, splits, K, M, bpx, bco, *, d3=False, transposed=False, stride=1, ks=3, pad=1, Ho=0, Wo=0,
                 out_f32=False, accumulate=False, resid_and_ep=False, gout=False):
    """(ticket, rows): whether a split-K conv combines its parts inside the launch (fmd_conv_desc.tickets), and the
    pixels per statistics row its epilogue then writes -- mirroring the kernels' conditions.  The halo kernel
    (csrc/conv_halo9.hip halo9_launch): 2-D, whole 128-cout tiles, the unsplit epilogue's forms, no G side output,
    rows of 64 pixels.  The implicit GEMM (csrc/conv.hip launch): 2-D, whole pixel and cout tiles, no parity classes
    (transposed stride-2 3x3), one row per wave's pixels (bpx / 2; 64 for K <= 16, whose tile has 4 waves across)."""
    if splits <= 1 or d3 or out_f32 or accumulate:
        return False, 0
    if halo:
        return bool(HALO_TICKET and K % 128 == 0 and not resid_and_ep and not gout), 64
    par = transposed and stride == 2 and ks == 3 and pad == 1 and Ho % 2 == 0 and Wo % 2 == 0
    ok = SPLIT_TICKET and not par and M % bpx == 0 and K % bco == 0
    return bool(ok), (64 if K <= 16 else bpx // 2)


def _set_fold(d, f):
    d.fold_st0, d.fold_rows0 = _p(f["st0"].slab), f["st0"].rows
    if f.get("st1") is not None:
        d.fold_st1, d.fold_rows1 = _p(f["st1"].slab), f["st1"].rows
    d.fold_G, d.fold_eps = f["groups"], float(f["eps"])
    d.fold_gamma, d.fold_beta = _p(f.get("gamma")), _p(f.get("beta"))
    emb = f.get("emb")
    d.fold_emb = _p(emb)
    d.fold_emb_stride = (f.get("emb_stride") or emb.shape[-1]) if emb is not None else 0
    d.pro_silu = int(f.get("silu", True))


def _clear_fold(d):
    d.fold_st0 = d.fold_st1 = d.fold_gamma = d.fold_beta = d.fold_emb = None
    d.fold_rows0 = d.fold_rows1 = d.fold_G = d.fold_emb_stride = 0


def _fold_now(f, N, HW, C0, C1):
    """(a, b, silu) of a pro_fold dict by fmd_gn_prep (the fold as its own launch)."""
    emb = f.get("emb")
    a, b, _ = gn_prep(f["st0"], f.get("st1"), N, HW, C0, C1, f["groups"], f["eps"], f.get("gamma"), f.get("beta"),
                      emb=emb, emb_stride=(f.get("emb_stride") or emb.shape[-1]) if emb is not None else 0,
                      emb_mode=1 if emb is not None else 0)
    return a, b, bool(f.get("silu", True))


CONV_SMALL_MODES = {"s1": 0, "s2": 1, "up": 2, "point": 3}
# forward-only small levels in one launch per conv (fmd_conv_small, runtime/tuning.py SMALL_CONV / SMALL_CONV_MAX_HW)
SMALL_CONV = bool(tuning.get("SMALL_CONV"))
SMALL_CONV_MAX_HW = tuning.get("SMALL_CONV_MAX_HW")
SMALL_CONV_MAX_WORK = tuning.get("SMALL_CONV_MAX_WORK")
SMALL_CONV_SPLIT = tuning.get("SMALL_CONV_SPLIT")
# the in-launch combine of a split reduction: fp32 partial tiles + arrival tickets, one set per (device, stream) --
# launches on one stream serialise, so they can share it; the tickets start at zero and every launch leaves them so
SMALL_PART_BYTES = 8 << 20
SMALL_TICKETS = 4096
_small_ws = {}


_cap_streams = {}
CAPTURE_STREAM = bool(tuning.get("CAPTURE_STREAM"))


def capture_stream():
    """The stream graph captures run on: a side stream whose in-launch-combine workspace (tickets zeroed) is created
    before the first capture, so a capture records no fill of it (a fresh per-stream workspace allocated inside the
    capture would replay its zero-fill every step)."""
    if not CAPTURE_STREAM:
        return None   # torch's own capture stream
    idx = torch.cuda.current_device()
    s = _cap_streams.get(idx)
    if s is None:
        s = torch.cuda.Stream(idx)
        with torch.cuda.stream(s):
            _small_workspace(torch.device("cuda", idx))
        _cap_streams[idx] = s
    return s


def _small_workspace(dev):
    key = (dev.index, torch.cuda.current_stream(dev).cuda_stream)
    ws = _small_ws.get(key)
    if ws is None:
        ws = (torch.empty(SMALL_PART_BYTES // 4, device=dev, dtype=F32),
              torch.zeros(SMALL_TICKETS, device=dev, dtype=torch.int32))
        _small_ws[key] = ws
    return ws


def _conv_small_desc(shape0, C1, K, mode, gn, skip, ptrs, split=None):
    """fmd_conv_small_desc for input shape ``shape0`` = (N, Hs, Ws, C0) (+ C1 concat channels).  ``ptrs``: dict of
    device pointers (a host-only plan query passes placeholders)."""
    from .._lib import ConvSmallDesc
    N, Hs, Ws, C0 = shape0
    m = CONV_SMALL_MODES[mode]
    Ho, Wo = (Hs // 2, Ws // 2) if m == 1 else (2 * Hs, 2 * Ws) if m == 2 else (Hs, Ws)
    d = ConvSmallDesc()
    d.N, d.Hs, d.Ws, d.C0, d.C1, d.Ho, d.Wo, d.K, d.mode = N, Hs, Ws, C0, C1, Ho, Wo, K, m
    d.src0, d.src1, d.wgt, d.out = ptrs["src0"], ptrs.get("src1"), ptrs["wgt"], ptrs["out"]
    if gn is not None:
        d.st0, d.rows0 = ptrs["st0"], gn["st0"].rows
        if gn.get("st1") is not None:
            d.st1, d.rows1 = ptrs["st1"], gn["st1"].rows
        d.G, d.eps = gn["groups"], float(gn["eps"])
        d.gamma, d.beta, d.emb = ptrs.get("gamma"), ptrs.get("beta"), ptrs.get("emb")
        emb = gn.get("emb")
        d.emb_stride = (gn.get("emb_stride") or emb.shape[-1]) if emb is not None else 0
        d.silu = int(gn.get("silu", True))
    if skip:   # (C2, C3): channels of the raw 1x1-segment sources at the output pixels
        d.C2, d.C3 = skip
        d.src2, d.src3, d.wgt2 = ptrs["src2"], ptrs.get("src3"), ptrs["wgt2"]
    d.split = SMALL_CONV_SPLIT if split is None else split
    if d.split != 1:
        d.part, d.part_bytes, d.tickets, d.n_tickets = ptrs["part"], SMALL_PART_BYTES, ptrs["tickets"], SMALL_TICKETS
    return d, (N, Ho, Wo)


def _conv_small_query(fn, shape0, K, C1, mode, gn, skip, split):
    fake = dict(src0=16, src1=16 if C1 else None, wgt=16, out=16, st0=16, st1=16, wgt2=16, src2=16,
                src3=16 if skip and skip[1] else None, part=16, tickets=16)
    d, _ = _conv_small_desc(tuple(shape0), C1, K, mode, gn, skip, fake, split)
    return int(getattr(_lib.lib(), fn)(C.byref(d)))


def conv_small_ok(shape0, K, *, C1=0, mode="s1", gn=None, skip=None, split=None) -> bool:
    """Whether fmd_conv_small takes the problem on input shape ``shape0`` = (N, Hs, Ws, C0) (fmd_conv_small_plan:
    geometry, channel counts, one CU's LDS; a host-side query, nothing is launched), within the SMALL_CONV switches.
    ``skip``: (C2, C3) channels of a 1x1 segment's sources, or None.  ``split``: parts of the reduction (None:
    SMALL_CONV_SPLIT; 0 the plan's choice, 1 none)."""
    if not SMALL_CONV or len(shape0) != 4 or K % 16:
        return False
    m = CONV_SMALL_MODES[mode]
    HWo = shape0[1] * shape0[2] * (4 if m == 2 else 1) // (4 if m == 1 else 1)
    if HWo > SMALL_CONV_MAX_HW or HWo * (shape0[3] + C1) > SMALL_CONV_MAX_WORK:
        return False
    return _conv_small_query("fmd_conv_small_plan", shape0, K, C1, mode, gn, skip, split) > 0


def conv_small_split(shape0, K, *, C1=0, mode="s1", gn=None, skip=None, split=None) -> int:
    """The parts fmd_conv_small splits the reduction of this problem into (fmd_conv_small_split; host-side)."""
    return _conv_small_query("fmd_conv_small_split", shape0, K, C1, mode, gn, skip, split)


def conv_small(src0, K, wgt, *, src1=None, mode="s1", gn=None, src2=None, src3=None, skip_wgt=None, bias=None,
               bias2=None, bias_nc=None, resid=None, out=None, want_stats=True,
               split=None) -> Tuple[torch.Tensor, Optional[Stats]]:
    """One-launch small-level conv (fmd_conv_small, csrc/conv_small.hip; forward only).

    ``mode``: "s1" 3x3 stride 1, "s2" 3x3 stride 2 (DownsampleND), "up" nearest-x2 + 3x3 (UpsampleND), "point" 1x1
    (the centre tap of a 3x3 on 1x1 images).  ``wgt``: fmd_prep_weights mode-0 layout [K][T][C0 + C1].
    ``gn``: GroupNorm(+scale/shift)+SiLU prologue folded from the inputs' statistics:
    dict(st0=Stats, st1=Stats or None, groups, eps, gamma, beta[, emb, emb_stride, silu]).  ``src2`` | ``src3``,
    ``skip_wgt`` (bf16 [K][1][C2 + C3]): a 1x1 conv over raw tensors at the output resolution (the ResBlock skip
    connection over the block input).  ``bias_nc``: [N][>=K] per-sample bias
    (row stride taken from the tensor).  Returns (out, Stats of the bf16 output: 64-pixel rows, or one row per
    image when Ho*Wo < 64).  ``split``: parts of the reduction, combined inside the launch (None: SMALL_CONV_SPLIT;
    0 the plan's choice -- enough workgroups for the chip --, 1 none, 2..16 forced)."""
    _need_cuda(src0, "conv_small")
    C1 = src1.shape[-1] if src1 is not None else 0
    ptrs = dict(src0=_p(src0), src1=_p(src1), wgt=_p(wgt), out=_p(out), wgt2=_p(skip_wgt), src2=_p(src2),
                src3=_p(src3))
    if gn is not None:
        ptrs.update(st0=_p(gn["st0"].slab), st1=_p(gn["st1"].slab) if gn.get("st1") is not None else None,
                    gamma=_p(gn.get("gamma")), beta=_p(gn.get("beta")), emb=_p(gn.get("emb")))
    skip = (src2.shape[-1], src3.shape[-1] if src3 is not None else 0) if skip_wgt is not None else None
    part, tickets = _small_workspace(src0.device)
    ptrs.update(part=_p(part), tickets=_p(tickets))
    d, (N, Ho, Wo) = _conv_small_desc(tuple(src0.shape), C1, K, mode, gn, skip, ptrs, split)
    d.bias, d.bias2, d.resid = _p(bias), _p(bias2), _p(resid)
    if bias_nc is not None:
        d.bias_nc, d.bias_nc_stride = _p(bias_nc), bias_nc.stride(0)
    if out is None:
        out = torch.empty((N, Ho, Wo, K), device=src0.device, dtype=BF16)
        d.out = _p(out)
    st = None
    if want_stats:
        rows = 64 if (Ho * Wo) % 64 == 0 else Ho * Wo
        slab = torch.empty((N * Ho * Wo // rows, K, 2), device=src0.device, dtype=F32)
        d.stats = _p(slab)
        st = Stats(slab, rows)
    _lib.call("fmd_conv_small", C.byref(d), stream())
    return out, st


def conv_combine(ws, K, out_shape, *, bias=None, bias2=None, bias_nc=None, resid=None, ep=None, out=None,
                 accumulate=False, want_stats=False):
    """out (bf16, N-D ``out_shape`` = (N, *sp)) = sum of the fp32 slabs ws [S][M][K] + conv epilogue
    (fmd_conv_combine); returns (out, Stats)."""
    N, sp = out_shape[0], tuple(out_shape[1:])
    Do, Ho, Wo = (0, *sp) if len(sp) == 2 else sp
    if out is None:
        out = torch.empty((N, *sp, K), device=ws.device, dtype=BF16)
    d = ConvDesc()
    d.N, d.Ho, d.Wo, d.Do, d.Hs, d.Ws, d.Ds, d.K = N, Ho, Wo, Do, Ho, Wo, Do, K
    d.ks, d.stride, d.pad = 3, 1, 1
    d.ws, d.splits = _p(ws), ws.shape[0]
    d.bias, d.bias2, d.bias_nc, d.resid, d.out = _p(bias), _p(bias2), _p(bias_nc), _p(resid), _p(out)
    d.accumulate = int(accumulate)
    if ep is not None:
        x0, x1, ea, eb = ep
        d.ep_x0, d.ep_x1, d.ep_C0, d.ep_a, d.ep_b = _p(x0), _p(x1), x0.shape[-1], _p(ea), _p(eb)
    HWo = max(Do, 1) * Ho * Wo
    M = N * HWo
    st = None
    fused = want_stats and not accumulate and K % 4 == 0 and HWo % SPLIT_STATS_ROWS == 0
    if fused:
        slab = torch.empty((M // SPLIT_STATS_ROWS, K, 2), device=ws.device, dtype=F32)
        d.stats = _p(slab)
        st = Stats(slab, SPLIT_STATS_ROWS)
    _lib.call("fmd_conv_combine", C.byref(d), stream())
    if want_stats and not fused:
        st = channel_stats(out, y=(ep[0], ep[1], ep[0].shape[-1])) if ep is not None else channel_stats(out)
    return out, st


def head_eligible(H, W, C, K, D=0) -> bool:
    """Mirror of the head kernels' shape test (csrc/head.hip); D > 0: 3-D data of depth D."""
    return H % 16 == 0 and W % 16 == 0 and C % 32 == 0 and 1 <= K <= (2 if D else 8)


def _head_dims(h):
    """(N, D, H, W, C) of a 2-D NHWC (D = 0) or 3-D NDHWC head input."""
    if h.dim() == 4:
        N, H, W, Cc = h.shape
        return N, 0, H, W, Cc
    return tuple(h.shape)


def head_fwd(h, pro, w, bias, K, Kp=8):
    """out fp32 channels-last [..., Kp] = conv3x3(x3)(SiLU(a*h+b)) for the first K channels (csrc/head.hip)."""
    _need_cuda(h, "head_fwd")
    N, D, H, W, Cc = _head_dims(h)
    out = torch.empty((*h.shape[:-1], Kp), device=h.device, dtype=F32)
    _lib.call("fmd_head_fwd", _p(h), N, D, H, W, Cc, _p(pro[0]), _p(pro[1]), _p(w.contiguous()), _p(bias), K,
              _p(out), stream())
    return out


def head_dgrad(dpred, w, K, h, pro):
    """(dz bf16 channels-last, Stats(sum dz, sum dz*h)) of the head conv (csrc/head.hip)."""
    N, D, H, W, Cc = _head_dims(h)
    dz = torch.empty_like(h)
    slab = torch.empty((h.numel() // Cc // 64, Cc, 2), device=h.device, dtype=F32)
    _lib.call("fmd_head_dgrad", _p(dpred), _p(w.contiguous()), K, _p(h), _p(pro[0]), _p(pro[1]), N, D, H, W, Cc,
              _p(dz), _p(slab), stream())
    return dz, Stats(slab, 64)


def head_wgrad(dpred, K, h, pro, dw, db):
    N, D, H, W, Cc = _head_dims(h)
    n = int(_lib.lib().fmd_head_wgrad_workspace(N, D, H, W, Cc, K))
    ws = torch.empty((n,), device=h.device, dtype=F32)
    _lib.call("fmd_head_wgrad", _p(dpred), K, _p(h), _p(pro[0]), _p(pro[1]), N, D, H, W, Cc, _p(dw), _p(db), _p(ws),
              stream())


# generic weight-gradient split-K: >= WGRAD_MIN_STEPS 32-pixel steps per split, ~WGRAD_CU_MULT workgroups per CU
WGRAD_MIN_STEPS = tuning.get("WGRAD_MIN_STEPS")
WGRAD_CU_MULT = tuning.get("WGRAD_CU_MULT")
# workgroups the halo weight gradient aims for (one per CU); fewer means fewer pixel splits, i.e. smaller
# split-K slabs (their write + reduce read) at the small levels (tuning WGRAD_HALO_WG: A/B override)
WGRAD_HALO_WG = tuning.get("WGRAD_HALO_WG") or NUM_CU
# split-K slab caps (MB): the partial slabs' write + reduce read bound the small levels (A/B: tuning WGRAD_SLAB_MB,
# WGRAD_GEN_SLAB_MB)
WGRAD_SLAB_MB = tuning.get("WGRAD_SLAB_MB")
WGRAD_GEN_SLAB_MB = tuning.get("WGRAD_GEN_SLAB_MB")
WGRAD_S2D = bool(tuning.get("WGRAD_S2D"))


def wgrad_halo_eligible(Hs, Ws, Ho, Wo, K, C, C0, ks=3, stride=1, pad=1, upsample=False, ldy=None) -> bool:
    """Mirror of fmd_wgrad_halo's applicability test (csrc/wgrad_halo.hip): 3x3 pad 1, stride 1 (optionally on a
    nearest-x2 input) or 2-D stride 2 (the space-to-depth planes as chunks; 3-D stride 2 stays generic)."""
    if stride == 2:
        geo = WGRAD_S2D and not upsample and Hs == 2 * Ho and Ws == 2 * Wo
    else:
        geo = stride == 1 and (Ho == 2 * Hs and Wo == 2 * Ws if upsample else Ho == Hs and Wo == Ws)
    return (ks == 3 and pad == 1 and geo and Ho % 8 == 0
            and Wo % 16 == 0 and K % 128 == 0 and C % 64 == 0 and C0 % 8 == 0 and (ldy or K) % 8 == 0)


def wgrad(src0, dy, dw, *, src1=None, ks=3, stride=1, pad=1, upsample=False, pro=None, db=None, accumulate=True,
          splits=None, dy_offset=0, force_generic=False):
    """dW (+)= conv weight gradient in the reference [K][C][kh][kw] fp32 layout (and db).

    ``dy_offset``: use channels [dy_offset, dy_offset + dw.shape[0]) of a wider dY (fused q/k/v).
    A 1-D k-tap weight ([K][C][k], k > 1) on (L, 1)-image activations: the k x k gradient of its embedding
    is computed and its centre column (the only one that meets data) is added in."""
    if dw.dim() == 3 and dw.shape[2] > 1 and src0.dim() == 4:
        full = torch.zeros((*dw.shape[:2], ks, ks), device=dw.device, dtype=F32)
        wgrad(src0, dy, full, src1=src1, ks=ks, stride=stride, pad=pad, upsample=upsample, pro=pro, db=db,
              accumulate=accumulate, splits=splits, dy_offset=dy_offset, force_generic=force_generic)
        col = full[..., (ks - 1) // 2]
        if accumulate:
            dw.add_(col)
        else:
            dw.copy_(col)
        return
    d3 = src0.dim() == 5
    if d3:
        N, Ds, Hs, Ws, C0 = src0.shape
        _, Do, Ho, Wo, ldy = dy.shape
    else:
        N, Hs, Ws, C0 = src0.shape
        _, Ho, Wo, ldy = dy.shape
        Ds = Do = 0
    C1 = src1.shape[-1] if src1 is not None else 0
    K = dw.shape[0]
    M = N * max(Do, 1) * Ho * Wo
    Ct = C0 + C1
    d = WgradDesc()
    d.N, d.Hs, d.Ws, d.C0, d.C1, d.Ho, d.Wo, d.K = N, Hs, Ws, C0, C1, Ho, Wo, K
    d.Ds, d.Do = Ds, Do
    d.ks, d.stride, d.pad, d.upsample = ks, stride, pad, int(upsample)
    d.src0, d.src1 = _p(src0), _p(src1)
    if pro is not None:
        d.pro_a, d.pro_b, d.pro_silu = _p(pro[0]), _p(pro[1]), int(pro[2])
    d.dy, d.ldy, d.dw, d.db, d.accumulate = dy.data_ptr() + 2 * dy_offset, ldy, _p(dw), _p(db), int(accumulate)
    d.force_generic = int(force_generic)
    if splits is None:
        if (not force_generic and (not d3 or (stride == 1 and Do == (2 * Ds if upsample else Ds))) and
                wgrad_halo_eligible(Hs, Ws, Ho, Wo, K, Ct, C0, ks, stride, pad, upsample, ldy)):
            # halo kernel: one workgroup per CU over (cout tile, 64-cin chunk [x depth tap | x stride-2 plane],
            # pixel-tile split); partial slabs capped at ~96 MB (their write + reduce read)
            zt = 3 if d3 else 1
            tiles = N * max(Do, 1) * (Ho // 8) * (Wo // 16)
            base = (K // 128) * (Ct // 64) * zt * (4 if stride == 2 else 1)
            splits = max(1, min(tiles, -(-WGRAD_HALO_WG // base), (WGRAD_SLAB_MB << 20) // (K * Ct * 36 * zt)))
        else:
            # narrow inputs (Ct < 128, T > 1) tile the flattened (tap, cin) pairs (csrc/wgrad.hip make_args
            # ``merged``): ceil(T * Ct / 128) column tiles -- the 3-D stem's 27 x 8 is 2 tiles, not 27
            T = ks * ks * (ks if d3 else 1)
            tiles = -(-K // 128) * (-(-(T * Ct) // 128) if T > 1 and Ct < 128 else -(-Ct // 128) * T)
            steps = -(-M // 32)
            # up to WGRAD_CU_MULT workgroups per CU (the kernel is latency-bound at one), >= WGRAD_MIN_STEPS
            # 32-pixel steps per split, partial slabs <= 48 MB
            cap = max(256, min(1024, (WGRAD_GEN_SLAB_MB << 20) // (K * Ct * T * 4)))
            splits = max(1, min(steps // WGRAD_MIN_STEPS, -(-WGRAD_CU_MULT * NUM_CU // tiles), cap))
    d.splits = splits
    ws = torch.empty((int(_lib.lib().fmd_wgrad_workspace(C.byref(d))),), device=dy.device, dtype=F32)
    d.ws = _p(ws)
    _lib.call("fmd_wgrad", C.byref(d), stream())


def prep_weights(w: torch.Tensor, mode: int, Kpad: Optional[int] = None, Cpad: Optional[int] = None, out=None):
    """fp32 [K][C][kh][kw] -> bf16 kernel layout (mode 0 fwd [Kpad][T][Cpad]; 1 dgrad [Cpad][T][Kpad]; 2 up-dgrad)."""
    K, Cc = w.shape[0], w.shape[1]
    ks = w.shape[2] if w.dim() >= 4 else 1
    Kpad = Kpad or K
    Cpad = Cpad or Cc
    if w.dim() == 5:   # 3-D: ks^3 taps (modes 0, 1, 3)
        T = ks ** 3
        shape = (Kpad, T, Cpad) if mode == 0 else (Cpad, T, Kpad)
        if out is None:
            out = torch.empty(shape, device=w.device, dtype=BF16)
        _lib.call("fmd_prep_weights_t", _p(w.contiguous()), K, Cc, T, mode, Kpad, Cpad, _p(out), stream())
        return out
    T = 16 if mode == 2 else ks * ks
    shape = (Kpad, T, Cpad) if mode == 0 else (Cpad, T, Kpad)
    if out is None:
        out = torch.empty(shape, device=w.device, dtype=BF16)
    _lib.call("fmd_prep_weights", _p(w.contiguous()), K, Cc, ks, mode, Kpad, Cpad, _p(out), stream())
    return out


def tile_weights(wk: torch.Tensor, out=None):
    """bf16 kernel-layout weights [rows][T][cols] -> halo-kernel tiles (csrc/conv_halo.hip)."""
    R, T, Cc = wk.shape
    n = int(_lib.lib().fmd_halo_tiled_size(R, T, Cc))
    if out is None:
        out = torch.empty((n,), device=wk.device, dtype=BF16)
    _lib.call("fmd_tile_weights_halo", _p(wk), R, T, Cc, _p(out), stream())
    return out


def nchw_to_nhwc(x: torch.Tensor, Cpad: Optional[int] = None) -> torch.Tensor:
    _need_cuda(x, "nchw_to_nhwc")
    x = x.contiguous().float()
    N, Cc = x.shape[:2]
    HW = x[0, 0].numel()
    Cpad = Cpad or Cc
    y = torch.empty((N, *x.shape[2:], Cpad), device=x.device, dtype=BF16)
    _lib.call("fmd_nchw_to_nhwc", _p(x), N, Cc, HW, Cpad, _p(y), stream())
    return y


def nhwc_to_nchw(y: torch.Tensor, Cc: int) -> torch.Tensor:
    N = y.shape[0]
    sp = y.shape[1:-1]
    Cs = y.shape[-1]
    x = torch.empty((N, Cc, *sp), device=y.device, dtype=F32)
    _lib.call("fmd_nhwc_to_nchw", _p(y), int(y.dtype == F32), N, Cc, x[0, 0].numel(), Cs, _p(x), stream())
    return x


def timestep_embedding(t: torch.Tensor, dim: int, flip: bool, shift: int = 0, max_period: float = 10000.0,
                       t_scale: float = 1.0, t_trunc: bool = False):
    if t.dtype != F32:
        t = t.float()
    t = t.contiguous()
    out = torch.empty((t.shape[0], dim), device=t.device, dtype=F32)
    _lib.call("fmd_timestep_embedding", _p(t), t.shape[0], dim, int(flip), shift, float(max_period), float(t_scale),
              int(t_trunc), _p(out), stream())
    return out


def linear(x, w, b, in_silu=False, out=None, out_stride=None):
    B, I = x.shape
    O = w.shape[0]
    if out is None:
        out = torch.empty((B, O), device=x.device, dtype=F32)
    _lib.call("fmd_linear", _p(x), B, I, _p(w), _p(b), O, int(in_silu), _p(out), out_stride or O, stream())
    return out


def linear_bwd(x, w, dy, dw, db, dx=None, dx_acc=False, in_silu=False, dy_stride=None):
    B, I = x.shape
    O = w.shape[0]
    _lib.call("fmd_linear_bwd", _p(x), B, I, _p(w), O, int(in_silu), _p(dy), dy_stride or dy.shape[-1], _p(dx),
              int(dx_acc), _p(dw), _p(db), stream())


class GroupedLinear:
    """Every ResBlock ``emb_layers`` projection (residual.py:63-68) of a UNet as one launch each way
    (csrc/misc.hip glinear_*): outputs are concatenated [B][sum O]; group g owns columns
    [off_g, off_g + O_g).  The device descriptor table is rebuilt only when a parameter or gradient
    storage moves (never during hipGraph capture once warmed up)."""

    ROWS = 64

    def __init__(self, linears, in_silu: bool):
        self.linears = list(linears)
        self.in_silu = bool(in_silu)
        self.O = [int(l.weight.shape[0]) for l in self.linears]
        self.I = int(self.linears[0].weight.shape[1])
        self.off = []
        o = 0
        for n in self.O:
            self.off.append(o)
            o += n
        self.total = o
        self.blocks_host = [(g, r0) for g, n in enumerate(self.O) for r0 in range(0, n, self.ROWS)]
        self._key = None
        self._groups = None
        self._blocks = None

    def _table(self, dev):
        key = tuple((l.weight.data_ptr(), l.bias.data_ptr() if l.bias is not None else 0,
                     l.weight.grad.data_ptr() if l.weight.grad is not None else 0,
                     l.bias.grad.data_ptr() if (l.bias is not None and l.bias.grad is not None) else 0)
                    for l in self.linears)
        if key != self._key:
            rows = [[w, b, gw, gb, n, off] for (w, b, gw, gb), n, off in zip(key, self.O, self.off)]
            self._groups = torch.tensor(rows, dtype=torch.int64).to(dev)
            self._blocks = torch.tensor(self.blocks_host, dtype=torch.int32).to(dev)
            self._key = key
        return self._groups, self._blocks

    def forward(self, x):
        _need_cuda(x, "GroupedLinear")
        B = x.shape[0]
        x = x.contiguous()
        g, blk = self._table(x.device)
        y = torch.empty((B, self.total), device=x.device, dtype=F32)
        _lib.call("fmd_grouped_linear", _p(x), B, self.I, _p(g), _p(blk), blk.shape[0], int(self.in_silu), _p(y),
                  self.total, stream())
        return y

    def backward(self, x, dy, dx=None, dx_acc=False):
        for l in self.linears:
            if l.weight.grad is None:
                l.weight.grad = torch.zeros_like(l.weight)
            if l.bias is not None and l.bias.grad is None:
                l.bias.grad = torch.zeros_like(l.bias)
        B = x.shape[0]
        g, blk = self._table(x.device)
        nws = int(_lib.lib().fmd_grouped_linear_bwd_workspace(B, self.I, blk.shape[0]))
        ws = torch.empty((nws,), device=x.device, dtype=F32)
        _lib.call("fmd_grouped_linear_bwd", _p(x.contiguous()), B, self.I, _p(g), _p(blk), blk.shape[0],
                  int(self.in_silu), _p(dy), self.total, _p(dx), int(dx_acc), _p(ws), stream())


def silu_bwd(x, dy):
    dx = torch.empty_like(x)
    _lib.call("fmd_silu_bwd_f32", _p(x), _p(dy), _p(dx), x.numel(), stream())
    return dx


# softmax attention: MFMA kernels over canonical [B*heads][rows][head_pad] planes (csrc/attention_mfma.hip)


def _attn_planes(B, heads, rows, dh, dev):
    D = int(_lib.lib().fmd_attn_head_pad(dh))
    if D < 0:
        raise ValueError(f"attention head dim {dh} > 64 is not supported")
    return torch.empty((B * heads, rows, D), device=dev, dtype=BF16)


def _attn_pack(src_q, src_kv, B, Tq, Tk, heads, dh, raw, cross, which0, which1, cq, ck=None, cv=None):
    _lib.call("fmd_attn_pack", _p(src_q), _p(src_kv), B, Tq, Tk, heads, dh, int(raw), int(cross), which0, which1,
              _p(cq), _p(ck), _p(cv), stream())


class AttnSaved:
    """What the MFMA softmax attention forward keeps for its backward: lse [B][heads][Tq] and the canonical
    q, k, v, o planes (so the backward packs only dout)."""
    __slots__ = ("lse", "cq", "ck", "cv", "co")

    def __init__(self, lse, cq, ck, cv, co):
        self.lse, self.cq, self.ck, self.cv, self.co = lse, cq, ck, cv, co


def _attn_softmax_fwd(src_q, src_kv, B, Tq, Tk, heads, dh, raw, cross):
    dev = src_q.device
    cq, ck, cv = _attn_planes(B, heads, Tq, dh, dev), _attn_planes(B, heads, Tk, dh, dev), _attn_planes(B, heads, Tk, dh, dev)
    _attn_pack(src_q, src_kv, B, Tq, Tk, heads, dh, raw, cross, 0, 2, cq, ck, cv)
    co = torch.empty_like(cq)
    lse = torch.empty((B, heads, Tq), device=dev, dtype=F32)
    _lib.call("fmd_attn_mfma_fwd", _p(cq), _p(ck), _p(cv), B * heads, Tq, Tk, dh, _p(co), _p(lse), stream())
    o = torch.empty((B, Tq, heads * dh), device=dev, dtype=BF16)
    _lib.call("fmd_attn_unpack", _p(co), None, None, B, Tq, Tk, heads, dh, int(raw), int(cross), 3, 3, _p(o), None,
              stream())
    return o, AttnSaved(lse, cq, ck, cv, co)


def _attn_softmax_bwd(src_q, src_kv, o, dout, saved, B, Tq, Tk, heads, dh, raw, cross, dst_q, dst_kv):
    """``saved``: the forward's AttnSaved, or a bare lse tensor (q, k, v, o are then packed again)."""
    dev = src_q.device
    if isinstance(saved, AttnSaved):
        lse, cq, ck, cv, co = saved.lse, saved.cq, saved.ck, saved.cv, saved.co
    else:
        lse = saved
        cq, ck = _attn_planes(B, heads, Tq, dh, dev), _attn_planes(B, heads, Tk, dh, dev)
        cv = _attn_planes(B, heads, Tk, dh, dev)
        _attn_pack(src_q, src_kv, B, Tq, Tk, heads, dh, raw, cross, 0, 2, cq, ck, cv)
        co = torch.empty_like(cq)
        _attn_pack(o, o, B, Tq, Tk, heads, dh, raw, cross, 3, 3, co)
    cdo = torch.empty_like(cq)
    _attn_pack(dout.contiguous(), dout, B, Tq, Tk, heads, dh, raw, cross, 3, 3, cdo)
    cdq, cdk, cdv = torch.empty_like(cq), torch.empty_like(ck), torch.empty_like(cv)
    delta = torch.empty_like(lse)
    _lib.call("fmd_attn_mfma_bwd", _p(cq), _p(ck), _p(cv), _p(co), _p(cdo), _p(lse), _p(delta), B * heads, Tq, Tk,
              dh, _p(cdq), _p(cdk), _p(cdv), stream())
    _lib.call("fmd_attn_unpack", _p(cdq), _p(cdk), _p(cdv), B, Tq, Tk, heads, dh, int(raw), int(cross), 0, 2,
              _p(dst_q), _p(dst_kv), stream())


def attention_fwd(qkv, T, heads, dh, raw):
    """Softmax self-attention over the fused qkv projection [B][T][3*inner] -> (o [B][T][inner], lse)."""
    return _attn_softmax_fwd(qkv, qkv, qkv.shape[0], T, T, heads, dh, raw, 0)


def _la_workspace(B, heads, dev):
    return torch.empty((int(_lib.lib().fmd_linear_attention_workspace(B, heads)),), device=dev, dtype=F32)


def linear_attention_fwd(qkv, T, heads, dh, raw, eps=1e-6):
    """LinearQKVAttention over the fused qkv projection (csrc/attention.hip); returns (o, state)."""
    B = qkv.shape[0]
    o = torch.empty((B, T, heads * dh), device=qkv.device, dtype=BF16)
    state = torch.empty((int(_lib.lib().fmd_linear_attention_state(B, heads)),), device=qkv.device, dtype=F32)
    _lib.call("fmd_linear_attention_fwd", _p(qkv), B, T, heads, dh, int(raw), float(eps), _p(o), _p(state),
              _p(_la_workspace(B, heads, qkv.device)), stream())
    return o, state


def linear_attention_bwd(qkv, dout, state, T, heads, dh, raw, eps=1e-6):
    B = qkv.shape[0]
    dqkv = torch.empty_like(qkv)
    _lib.call("fmd_linear_attention_bwd", _p(qkv), _p(dout), _p(state), _p(_la_workspace(B, heads, qkv.device)), B, T,
              heads, dh, int(raw), float(eps), _p(dqkv), stream())
    return dqkv


def cross_attention_fwd(q, kv, Tq, Tk, heads, dh, linear_eps=None, raw=1):
    """SpatialCrossAttention core (csrc/attention.hip): q [B][Tq][inner], kv [B][Tk][2*inner] -> (o, saved),
    softmax (saved = lse) or LinearQKVAttention when ``linear_eps`` is given (saved = state)."""
    B = q.shape[0]
    if linear_eps is None:
        return _attn_softmax_fwd(q, kv, B, Tq, Tk, heads, dh, raw, 1)
    o = torch.empty((B, Tq, heads * dh), device=q.device, dtype=BF16)
    saved = torch.empty((int(_lib.lib().fmd_linear_attention_state(B, heads)),), device=q.device, dtype=F32)
    ws = _la_workspace(B, heads, q.device)
    _lib.call("fmd_cross_attention_fwd", _p(q), _p(kv), B, Tq, Tk, heads, dh, int(raw), 1, float(linear_eps),
              _p(o), _p(saved), _p(ws), stream())
    return o, saved


def cross_attention_bwd(q, kv, o, dout, saved, Tq, Tk, heads, dh, linear_eps=None, raw=1):
    B = q.shape[0]
    dq, dkv = torch.empty_like(q), torch.empty_like(kv)
    if linear_eps is None:
        _attn_softmax_bwd(q, kv, o, dout, saved, B, Tq, Tk, heads, dh, raw, 1, dq, dkv)
        return dq, dkv
    _lib.call("fmd_cross_attention_bwd", _p(q), _p(kv), _p(o), _p(dout), _p(saved), _p(_la_workspace(B, heads, q.device)),
              B, Tq, Tk, heads, dh, int(raw), 1, float(linear_eps), _p(dq), _p(dkv), stream())
    return dq, dkv


def context_norm_fwd(ctx, tok_major, groups, eps, gamma, beta, Cpad):
    """GroupNorm of a cross-attention context (fp32 [N][C][T] or token-major [N][T][C]) -> bf16 [N][T][1][Cpad]
    (a 1-wide NHWC plane for the kv 1x1 conv) and the (mean, rstd) table."""
    _need_cuda(ctx, "context_norm_fwd")
    N = ctx.shape[0]
    C, T = (ctx.shape[2], ctx.shape[1]) if tok_major else (ctx.shape[1], ctx.shape[2])
    out = torch.empty((N, T, 1, Cpad), device=ctx.device, dtype=BF16)
    mr = torch.empty((N, groups, 2), device=ctx.device, dtype=F32)
    _lib.call("fmd_context_norm_fwd", _p(ctx), N, C, T, int(tok_major), groups, float(eps), _p(gamma), _p(beta), Cpad,
              _p(out), _p(mr), stream())
    return out, mr


def context_norm_bwd(ctx, tok_major, groups, mr, dout, dgamma, dbeta):
    N = ctx.shape[0]
    C, T = (ctx.shape[2], ctx.shape[1]) if tok_major else (ctx.shape[1], ctx.shape[2])
    _lib.call("fmd_context_norm_bwd", _p(ctx), N, C, T, int(tok_major), groups, _p(mr), _p(dout), dout.shape[-1],
              _p(dgamma), _p(dbeta), stream())


def attention_bwd(qkv, o, dout, lse, T, heads, dh, raw):
    dqkv = torch.empty_like(qkv)
    _attn_softmax_bwd(qkv, qkv, o, dout, lse, qkv.shape[0], T, T, heads, dh, raw, 0, dqkv, dqkv)
    return dqkv


def _dhw(t):
    """(N, D, H, W, C) view extents of an N(D)(H)WC tensor (missing leading spatial dims = 1)."""
    N, C = t.shape[0], t.shape[-1]
    sp = list(t.shape[1:-1])
    sp = [1] * (3 - len(sp)) + sp
    return N, sp, C


def resample2(src, dst, up: bool, scale: float, acc: bool = False, factors=None):
    """dst (+)= avg/sum-pool-by-2 (up=False) or nearest-x2 (up=True) of src; ``factors`` (per spatial dim, 1 or
    2; default every dim 2) -- a 1-D signal as an (L, 1) image resamples its first dim only."""
    _need_cuda(src, "resample2")
    N, s_sp, C = _dhw(src)
    _, d_sp, _ = _dhw(dst)
    lo, hi = (s_sp, d_sp) if up else (d_sp, s_sp)
    nd = src.dim() - 2
    f = [1] * (3 - nd) + (list(factors) if factors is not None else [2] * nd)
    _lib.call("fmd_resample2", _p(src), N, lo[0], lo[1], lo[2], hi[0], hi[1], hi[2], C, f[0], f[1], f[2], int(up),
              float(scale), _p(dst), int(acc), stream())


def sum_pool2(src, dst, acc):
    N, H, W, Cc = dst.shape
    _lib.call("fmd_sum_pool2", _p(src), N, H, W, Cc, _p(dst), int(acc), stream())


def sum_pool2_3d(src, dst, acc=False):
    """dst (+)= 2x2x2 block sums of src (bf16 NDHWC): the data gradient of a nearest-x2 3-D upsample."""
    N, D, H, W, Cc = dst.shape
    _lib.call("fmd_sum_pool2_3d", _p(src), N, D, H, W, Cc, _p(dst), int(acc), stream())


def add_(dst, a):
    _lib.call("fmd_add_bf16", _p(a), _p(dst), dst.numel(), stream())


def noise_prepare(x0, noise, ca, cb, cond, Cpad, out=None):
    N, Cx = noise.shape[:2]
    HW = noise[0, 0].numel()
    Cc = cond.shape[1] if cond is not None else 0
    if out is None:
        out = torch.empty((N, *noise.shape[2:], Cpad), device=noise.device, dtype=BF16)
    _lib.call("fmd_noise_prepare", _p(x0), _p(noise), _p(ca), _p(cb), _p(cond), N, HW, Cx, Cc, Cpad, _p(out),
              stream())
    return out


def mse(pred_nhwc, ta, tb, tb_sign, grad_scale, loss, partial, dpred=None):
    N = pred_nhwc.shape[0]
    Kpad = pred_nhwc.shape[-1]
    Cx = ta.shape[1]
    HW = ta[0, 0].numel()
    _lib.call("fmd_mse", _p(pred_nhwc), Kpad, _p(ta), _p(tb), float(tb_sign), N, Cx, HW, float(grad_scale),
              _p(partial), partial.numel(), _p(loss), _p(dpred), stream())


def adamw_sched(p, g, m, v, step_ctr, base_lr, warmup, total, beta1=0.9, beta2=0.999, eps=1e-8, wd=0.0,
                grad_scale=1.0):
    _lib.call("fmd_adamw_sched", _p(p), _p(g), _p(m), _p(v), p.numel(), _p(step_ctr), float(base_lr), int(warmup),
              int(total), float(beta1), float(beta2), float(eps), float(wd), float(grad_scale), stream())


def counter_add(ctr, v=1):
    _lib.call("fmd_counter_add", _p(ctr), int(v), stream())


def fill_from_table(table, index, out):
    _lib.call("fmd_fill_from_table", _p(table), _p(index), _p(out), out.numel(), stream())


def lincomb(out, inputs, coefs):
    """out = sum_k coefs[k] * inputs[k] (fp32 device tensors of out's size; out may be one of the inputs)."""
    _need_cuda(out, "lincomb")
    if not 1 <= len(inputs) <= _lib.LINCOMB_MAX or len(inputs) != len(coefs):
        raise ValueError("lincomb: 1..6 inputs, one coefficient each")
    d = _lib.LincombDesc()
    d.out, d.nin, d.n = _p(out), len(inputs), out.numel()
    for k, (t, c) in enumerate(zip(inputs, coefs)):
        if t.dtype != F32 or not t.is_contiguous() or t.numel() != out.numel():
            raise ValueError("lincomb: contiguous fp32 inputs of the output's size")
        d.in_[k] = _p(t)
        d.c[k] = float(c)
    _lib.call("fmd_lincomb", C.byref(d), stream())
    return out


def gather_row(table, index, out):
    """out = table[index[0]] (row of ``out.numel()`` fp32 elements; ``index`` is a device int32 counter)."""
    _lib.call("fmd_gather_row", _p(table), _p(index), out.numel(), _p(out), stream())


def flow_euler(x, v_nhwc, sigmas, index, cond, next_inp):
    N, Cx = x.shape[:2]
    HW = x[0, 0].numel()
    Cc = cond.shape[1] if cond is not None else 0
    _lib.call("fmd_flow_euler", _p(x), _p(v_nhwc), v_nhwc.shape[-1], _p(sigmas), _p(index), N, Cx, HW, _p(cond), Cc,
              next_inp.shape[-1] if next_inp is not None else 0, _p(next_inp), stream())


def affine_channels(x, C: int, scale: float, shift: float):
    """y = x (channels-last bf16) with channels [0, C) mapped to scale * x + shift (fmd_affine_channels)."""
    _need_cuda(x, "affine_channels")
    y = torch.empty_like(x)
    _lib.call("fmd_affine_channels", _p(x), int(C), x.shape[-1], x.numel() // x.shape[-1], float(scale), float(shift),
              _p(y), stream())
    return y


def ddpm_step(x, eps_nhwc, coef, index, noise, cond, next_inp, noise_base=-1):
    """``noise``: one [N,Cx,*S] buffer (``noise_base`` < 0) or a per-step table [rows][N,Cx,*S] whose row 0 is step
    ``noise_base`` (fmd_ddpm_step)."""
    N, Cx = x.shape[:2]
    HW = x[0, 0].numel()
    Cc = cond.shape[1] if cond is not None else 0
    _lib.call("fmd_ddpm_step", _p(x), _p(eps_nhwc), eps_nhwc.shape[-1], _p(coef), _p(index), _p(noise),
              int(noise_base), N, Cx, HW,
              _p(cond), Cc, next_inp.shape[-1] if next_inp is not None else 0, _p(next_inp), stream())


def sched_step(x, eps_nhwc, ring, last, coef, index, cond, next_inp):
    """One table-driven DPM-Solver / UniPC step (fmd_sched_step): x [N,Cx,*S] fp32 updated in place, ring = 4
    fp32 history buffers of x's shape, last (UniPC corrector state) or None, coef [steps][12] fp32."""
    N, Cx = x.shape[:2]
    d = _lib.SchedStepDesc()
    d.x, d.eps, d.last, d.coef, d.index = _p(x), _p(eps_nhwc), _p(last), _p(coef), _p(index)
    for k in range(4):
        d.ring[k] = _p(ring[k])
    d.N, d.Cx, d.HW, d.Kpad = N, Cx, x[0, 0].numel(), eps_nhwc.shape[-1]
    d.cond, d.Cc = _p(cond), cond.shape[1] if cond is not None else 0
    d.Cpad, d.next = (next_inp.shape[-1], _p(next_inp)) if next_inp is not None else (0, None)
    _lib.call("fmd_sched_step", C.byref(d), stream())


def adamw(p, g, m, v, lr, beta1, beta2, eps, wd, step):
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    _lib.call("fmd_adamw", _p(p), _p(g), _p(m), _p(v), p.numel(), float(lr), float(beta1), float(beta2), float(eps),
              float(wd), float(bc1), float(bc2), stream())
