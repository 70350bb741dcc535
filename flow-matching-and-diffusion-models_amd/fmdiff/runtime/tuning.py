"""Dispatch constants of the runtime (kernel-path choices and split heuristics), in one table.

Every value is the measured default (DESIGN.md section 8 and the round logs cite the A/B runs behind each).  The
only runtime override is ONE environment variable for A/B runs on the GPU box::

    FMD_TUNE="HALO_MIN_WG=64,SPLIT_CAP=8" python bench.py

Unknown names raise, so a typo cannot silently measure the default.  (``FMD_LIB`` -- which library file to load --
is the other variable the package reads; tools/build_variant.sh builds instrumented libraries for it.)
"""
from __future__ import annotations

import os

# name: (default, meaning)
TABLE = {
    # ---- kernel-path switches (1 = on; 0 = the older path, kept for A/B and parity bisection)
    "MAT3D": (1, "3-D: materialise the GN+SiLU operand of depth-tap halo convs once (0: fused prologue + G side "
                 "output)"),
    "DEPTH_HALO": (1, "3x3x3 stride-1 convs on the halo kernel with (depth tap, channel block) chunks"),
    "S2D_HALO": (1, "stride-2 3x3 forwards / nearest-x2 data gradients on the space-to-depth halo kernel"),
    "S2D_3D": (1, "3-D: the same stride-2 modes with the depth taps as chunks (0: generic implicit GEMM, and the "
                  "nearest-x2 data gradient at full resolution + 2x2x2 box sum)"),
    "WGRAD_S2D": (1, "2-D stride-2 3x3 weight gradients on the halo weight-gradient kernel (space-to-depth planes as "
                     "chunks; 0: the generic weight-gradient kernel).  2-D only: 3-D stride-2 weight gradients always "
                     "run on the generic kernel (fmd_wgrad_halo rejects them)"),
    "POINT_1X1": (1, "ResBlock 3x3 convs on 1x1 images as their centre tap"),
    "GN_FUSED": (1, "small levels: GroupNorm statistics + affine + SiLU operand in one launch"),
    "CONV_GN": (1, "split-K conv1 -> GroupNorm-2 in the split combine (fmd_conv_gn)"),
    "HALO_FOLD": (1, "forward only: the GroupNorm affine folded in the halo conv's prologue (no gn_prep launch)"),
    "HALO_FOLD_MAX_ROWS": (64, "... where the statistics slab has at most this many rows per image"),
    "HALO_TICKET": (1, "split-K halo convs combined inside the launch (arrival tickets) instead of a combine launch"),
    "SPLIT_TICKET": (0, "... and split-K implicit-GEMM convs on whole tiles likewise (off: their 8-16 parts make one "
                        "workgroup's serial combine slower than the combine launch -- train 369.6 -> 363.5 img/s)"),
    "CAPTURE_STREAM": (1, "graph captures on a side stream whose in-launch-combine workspace exists beforehand"),
    "SMALL_ATTN": (1, "forward-only small levels: attention's qkv (GroupNorm folded) and output projections on fmd_conv_small"),
    "SMALL_CONV": (1, "forward-only small levels: one launch per conv with the GroupNorm folded in (fmd_conv_small)"),
    "SMALL_CONV_MAX_HW": (256, "fmd_conv_small only on outputs of at most this many pixels per image"),
    "SMALL_CONV_MAX_WORK": (65536, "... and output pixels per image x input channels at most this (16^2 x 256: config D's "
                                   "16^2 level, not config B's 512-channel one; DESIGN.md round 6)"),
    "SMALL_CONV_SPLIT": (0, "fmd_conv_small reduction parts combined in-launch: 0 plan's choice, 1 none, 2..16 forced"),
    # ---- split heuristics
    "CONV_GN_MIN_BLOCKS": (128, "fmd_conv_gn only from this many combine blocks up"),
    "CONV_GN_CB": (4, "fmd_conv_gn combine block channels (4, 8, 16, 32, 64; at least one group)"),
    "STATS_FOLD_MIN": (4096, "statistics slabs with at least this many rows per image are folded first"),
    "SPLIT_MIN_STEPS": (2, "generic conv split-K: at least this many K-steps per split"),
    "SPLIT_CU_MULT": (2, "generic conv split-K: target workgroups per CU"),
    "SPLIT_CAP": (64, "generic conv split-K: most splits"),
    "HALO_SPLIT_WG": (256, "halo conv split-K: target workgroups"),
    "HALO_MIN_CHUNKS": (2, "halo conv split-K: at least this many 32-channel chunks per split"),
    "HALO_SPLIT_CAP": (16, "halo conv split-K: most splits"),
    "HALO_MIN_WG": (32, "halo conv only from this many workgroups (tiles x cout tiles x splits) up"),
    "HALO_TH8_MAX_WG": (1024, "halo conv: 8-row tiles for grids of fewer 16-row workgroups than this (0: never)"),
    "HALO_TH4_MAX_WG": (512, "halo conv: 4-row tiles for 8-row grids of fewer workgroups than this (0: never)"),
    "WGRAD_MIN_STEPS": (8, "generic weight gradient: at least this many 32-pixel steps per split"),
    "WGRAD_CU_MULT": (4, "generic weight gradient: target workgroups per CU"),
    "WGRAD_HALO_WG": (0, "halo weight gradient: target workgroups (0 = one per CU)"),
    "WGRAD_SLAB_MB": (96, "halo weight gradient: split-K slab cap (MB)"),
    "WGRAD_GEN_SLAB_MB": (48, "generic weight gradient: split-K slab cap (MB)"),
}

# the per-switch environment variables this table replaced in round 5 (and earlier retired switches): setting one
# would silently measure the default, so it raises instead
RETIRED = sorted({f"FMD_{k}" for k in TABLE} | {
    "FMD_HALO9", "FMD_HALO10", "FMD_WGRAD9", "FMD_WGRAD_REDUCE", "FMD_WGRAD_REDUCE1", "FMD_WGRAD_PIPE", "FMD_WGRAD_KS",
    "FMD_SPLITK_FUSE", "FMD_WRED_BATCH", "FMD_SIDE_WGRAD", "FMD_MAT_PRO", "FMD_GOUT", "FMD_CONV_LOG", "FMD_X"})


def check_environment(env=None) -> None:
    """Raise if a retired per-switch FMD_* variable is set (use FMD_TUNE=NAME=value instead)."""
    env = os.environ if env is None else env
    stale = [k for k in RETIRED if k in env]
    if stale:
        raise ValueError(f"retired environment switch(es) {', '.join(stale)}: the runtime no longer reads them; use "
                         f"FMD_TUNE=\"NAME=value,...\" with the names of fmdiff/runtime/tuning.py TABLE")


check_environment()
_over = {}
for _item in filter(None, (s.strip() for s in os.environ.get("FMD_TUNE", "").split(","))):
    _k, _, _v = _item.partition("=")
    if _k not in TABLE or not _v:
        raise ValueError(f"FMD_TUNE: unknown or empty setting {_item!r} (known: {', '.join(TABLE)})")
    _over[_k] = int(_v)


def get(name: str) -> int:
    """The value of one constant: its FMD_TUNE override, else the table default."""
    return _over.get(name, TABLE[name][0])


def overridden(name: str) -> bool:
    return name in _over
