"""ctypes binding of the C ABI in ``include/fmdiff.h`` (libfmdiff_hip.so).

There is deliberately no fallback: if the library is missing the import of
any GPU op raises, so a GPU run can never silently use another path.
"""
from __future__ import annotations

import ctypes as C
import os

LIB_PATH = os.environ.get("FMD_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib",
                                                     "libfmdiff_hip.so")

p = C.c_void_p
i32 = C.c_int32
i64 = C.c_int64
f32 = C.c_float
u32 = C.c_uint32


class ConvDesc(C.Structure):
    """Mirror of ``fmd_conv_desc``."""
    _fields_ = [
        ("N", i32), ("Hs", i32), ("Ws", i32), ("C0", i32), ("C1", i32), ("Ho", i32), ("Wo", i32), ("K", i32),
        ("ks", i32), ("stride", i32), ("pad", i32), ("upsample", i32), ("transposed", i32),
        ("src0", p), ("src1", p), ("pro_a", p), ("pro_b", p), ("pro_silu", i32), ("wgt", p),
        ("src2", p), ("src3", p), ("C2", i32), ("C3", i32), ("wgt2", p),
        ("bias", p), ("bias2", p), ("bias_nc", p), ("resid", p), ("out", p), ("out_f32", i32), ("accumulate", i32),
        ("stats", p), ("ep_x0", p), ("ep_x1", p), ("ep_C0", i32), ("ep_a", p), ("ep_b", p),
        ("ws", p), ("splits", i32), ("force_generic", i32), ("wgt_tiled", p), ("wgt2_tiled", p),
        ("Ds", i32), ("Do", i32), ("gout", p),
        ("fold_st0", p), ("fold_rows0", i32), ("fold_st1", p), ("fold_rows1", i32), ("fold_G", i32),
        ("fold_eps", f32), ("fold_gamma", p), ("fold_beta", p), ("fold_emb", p), ("fold_emb_stride", i32),
        ("tickets", p), ("n_tickets", i32), ("tickets_rows", i32),
    ]


class WgradDesc(C.Structure):
    """Mirror of ``fmd_wgrad_desc``."""
    _fields_ = [
        ("N", i32), ("Hs", i32), ("Ws", i32), ("C0", i32), ("C1", i32), ("Ho", i32), ("Wo", i32), ("K", i32),
        ("ks", i32), ("stride", i32), ("pad", i32), ("upsample", i32),
        ("src0", p), ("src1", p), ("pro_a", p), ("pro_b", p), ("pro_silu", i32), ("dy", p), ("ldy", i32), ("dw", p), ("db", p),
        ("accumulate", i32), ("ws", p), ("splits", i32), ("force_generic", i32), ("Ds", i32), ("Do", i32),
    ]


class GnApplyDesc(C.Structure):
    """Mirror of ``fmd_gn_apply_desc``."""
    _fields_ = [
        ("dz", p), ("x0", p), ("x1", p), ("C0", i32), ("P", p), ("Q", p), ("R", p),
        ("dx0", p), ("acc0", i32), ("dx1", p), ("acc1", i32),
    ]


class GnOutDesc(C.Structure):
    """Mirror of ``fmd_gn_out_desc``."""
    _fields_ = [("G", i32), ("eps", f32), ("gamma", p), ("beta", p), ("emb", p), ("emb_stride", i32),
                ("emb_mode", i32), ("silu", i32), ("a", p), ("b", p), ("mean_rstd", p), ("t", p)]


class ConvSmallDesc(C.Structure):
    """Mirror of ``fmd_conv_small_desc``."""
    _fields_ = [
        ("N", i32), ("Hs", i32), ("Ws", i32), ("C0", i32), ("C1", i32), ("Ho", i32), ("Wo", i32), ("K", i32),
        ("mode", i32), ("src0", p), ("src1", p), ("wgt", p), ("st0", p), ("rows0", i32), ("st1", p), ("rows1", i32),
        ("G", i32), ("eps", f32), ("gamma", p), ("beta", p), ("emb", p), ("emb_stride", i32), ("silu", i32),
        ("src2", p), ("src3", p), ("C2", i32), ("C3", i32), ("wgt2", p), ("bias", p), ("bias2", p), ("bias_nc", p),
        ("bias_nc_stride", i32), ("resid", p),
        ("out", p), ("stats", p), ("part", p), ("part_bytes", i64), ("tickets", p), ("n_tickets", i32), ("split", i32),
    ]


LINCOMB_MAX = 6   # FMD_LINCOMB_MAX


class LincombDesc(C.Structure):
    """Mirror of ``fmd_lincomb_desc``."""
    _fields_ = [("out", p), ("in_", p * LINCOMB_MAX), ("c", C.c_float * LINCOMB_MAX), ("nin", i32), ("n", i64)]


SCHED_NCOEF = 12  # FMD_SCHED_NCOEF


class SchedStepDesc(C.Structure):
    """Mirror of ``fmd_sched_step_desc``."""
    _fields_ = [("x", p), ("eps", p), ("ring", p * 4), ("last", p), ("coef", p), ("index", p), ("N", i32), ("Cx", i32),
                ("HW", i32), ("Kpad", i32), ("cond", p), ("Cc", i32), ("Cpad", i32), ("next", p)]


class GbJob(C.Structure):
    """Mirror of ``fmd_gb_job``."""
    _fields_ = [("ws", p), ("dgamma", p), ("dbeta", p), ("N", i32), ("C", i32)]


GB_MAX = 64   # FMD_GB_MAX


# name -> argtypes (restype is int32 unless listed in _RESTYPE)
SIGNATURES = {
    "fmd_conv": [C.POINTER(ConvDesc), p],
    "fmd_conv_halo": [C.POINTER(ConvDesc), p],
    "fmd_conv_gn_apply": [C.POINTER(ConvDesc), C.POINTER(GnApplyDesc), p],
    "fmd_conv_gn": [C.POINTER(ConvDesc), C.POINTER(GnOutDesc), p],
    "fmd_wgrad": [C.POINTER(WgradDesc), p],
    "fmd_wgrad_workspace": [C.POINTER(WgradDesc)],
    "fmd_wgrad_halo": [C.POINTER(WgradDesc), p],
    "fmd_halo_tiled_size": [i32, i32, i32],
    "fmd_tile_weights_halo": [p, i32, i32, i32, p, p],
    "fmd_conv_s2d": [C.POINTER(ConvDesc), p],
    "fmd_conv_d2s": [C.POINTER(ConvDesc), p],
    "fmd_conv_small_plan": [C.POINTER(ConvSmallDesc)],
    "fmd_conv_small_split": [C.POINTER(ConvSmallDesc)],
    "fmd_conv_small": [C.POINTER(ConvSmallDesc), p],
    "fmd_s2d_tiled_size": [i32, i32, i32],
    "fmd_s2d_tile_weights": [p, i32, i32, i32, i32, p, p],
    "fmd_s2d_tiled_size_nd": [i32, i32, i32, i32, i32],
    "fmd_s2d_tile_weights_nd": [p, i32, i32, i32, i32, i32, p, p],
    "fmd_channel_stats": [p, p, p, i32, i32, i32, i32, i32, p, p],
    "fmd_stats_fold": [p, i64, i32, i32, p, p],
    "fmd_gn_prep": [p, i32, p, i32, i32, i32, i32, i32, i32, f32, p, p, p, i32, i32, p, p, p, p],
    "fmd_gn_bwd_prep": [p, i32, i32, i32, i32, i32, p, p, p, p, i32, i32, p, p, p, p, p, p, i32, p, i32, p, p],
    "fmd_gn_apply_fwd": [p, p, i32, i32, i64, i32, p, p, i32, p, p],
    "fmd_gn_fused_apply": [p, p, i32, i32, i32, i32, i32, f32, p, p, p, i32, i32, i32, p, p, p, p, p],
    "fmd_dropout_apply": [p, i32, i64, i32, f32, p, u32, p, p, p, p, p],
    "fmd_gn_gb_fold": [p, i32, p],
    "fmd_lincomb": [C.POINTER(LincombDesc), p],
    "fmd_sched_step": [C.POINTER(SchedStepDesc), p],
    "fmd_halo_set_min_workgroups": [i32],
    "fmd_halo_set_th8_max_workgroups": [i32],
    "fmd_halo_set_th4_max_workgroups": [i32],
    "fmd_conv_gn_set_block_channels": [i32],
    "fmd_gn_bwd_apply": [p, p, p, i32, i32, i64, i32, p, p, p, p, p, i32, p, i32, p],
    "fmd_prep_weights": [p, i32, i32, i32, i32, i32, i32, p, p],
    "fmd_prep_weights_t": [p, i32, i32, i32, i32, i32, i32, p, p],
    "fmd_prep_weights_batch": [p, i32, i32, p],
    "fmd_prep_weights_batch_cubic": [p, i32, i32, p],
    "fmd_nchw_to_nhwc": [p, i32, i32, i32, i32, p, p],
    "fmd_nhwc_to_nchw": [p, i32, i32, i32, i32, i32, p, p],
    "fmd_sum_pool2": [p, i32, i32, i32, i32, p, i32, p],
    "fmd_resample2": [p, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32, f32, p, i32, p],
    "fmd_sum_pool2_3d": [p, i32, i32, i32, i32, i32, p, i32, p],
    "fmd_add_bf16": [p, p, i64, p],
    "fmd_timestep_embedding": [p, i32, i32, i32, i32, f32, f32, i32, p, p],
    "fmd_adamw_sched": [p, p, p, p, i64, p, f32, i32, i32, f32, f32, f32, f32, f32, p],
    "fmd_linear": [p, i32, i32, p, p, i32, i32, p, i32, p],
    "fmd_linear_bwd": [p, i32, i32, p, i32, i32, p, i32, p, i32, p, p, p],
    "fmd_silu_bwd_f32": [p, p, p, i64, p],
    "fmd_grouped_linear": [p, i32, i32, p, p, i32, i32, p, i32, p],
    "fmd_grouped_linear_bwd_workspace": [i32, i32, i32],
    "fmd_grouped_linear_bwd": [p, i32, i32, p, p, i32, i32, p, i32, p, i32, p, p],
    "fmd_conv_combine": [C.POINTER(ConvDesc), p],
    "fmd_attn_head_pad": [i32],
    "fmd_attn_pack": [p, p, i32, i32, i32, i32, i32, i32, i32, i32, i32, p, p, p, p],
    "fmd_attn_unpack": [p, p, p, i32, i32, i32, i32, i32, i32, i32, i32, i32, p, p, p],
    "fmd_attn_mfma_fwd": [p, p, p, i32, i32, i32, i32, p, p, p],
    "fmd_attn_mfma_bwd": [p, p, p, p, p, p, p, i32, i32, i32, i32, p, p, p, p],
    "fmd_cross_attention_fwd": [p, p, i32, i32, i32, i32, i32, i32, i32, f32, p, p, p, p],
    "fmd_cross_attention_bwd": [p, p, p, p, p, p, i32, i32, i32, i32, i32, i32, i32, f32, p, p, p],
    "fmd_context_norm_fwd": [p, i32, i32, i32, i32, i32, f32, p, p, i32, p, p, p],
    "fmd_context_norm_bwd": [p, i32, i32, i32, i32, i32, p, p, i32, p, p, p],
    "fmd_linear_attention_workspace": [i32, i32],
    "fmd_linear_attention_state": [i32, i32],
    "fmd_linear_attention_fwd": [p, i32, i32, i32, i32, i32, f32, p, p, p, p],
    "fmd_linear_attention_bwd": [p, p, p, p, i32, i32, i32, i32, i32, f32, p, p],
    "fmd_noise_prepare": [p, p, p, p, p, i32, i32, i32, i32, i32, p, p],
    "fmd_add_noise": [p, p, p, p, p, i32, i64, p, p],
    "fmd_mse": [p, i32, p, p, f32, i32, i32, i32, f32, p, i32, p, p, p],
    "fmd_adamw": [p, p, p, p, i64, f32, f32, f32, f32, f32, f32, f32, p],
    "fmd_flow_euler": [p, p, i32, p, p, i32, i32, i32, p, i32, i32, p, p],
    "fmd_affine_channels": [p, i32, i32, i64, f32, f32, p, p],
    "fmd_ddpm_step": [p, p, i32, p, p, p, i32, i32, i32, i32, p, i32, i32, p, p],
    "fmd_fill_from_table": [p, p, p, i32, p],
    "fmd_gather_row": [p, p, i64, p, p],
    "fmd_counter_add": [p, i32, p],
    "fmd_head_fwd": [p, i32, i32, i32, i32, i32, p, p, p, p, i32, p, p],
    "fmd_head_dgrad": [p, p, i32, p, p, p, i32, i32, i32, i32, i32, p, p, p],
    "fmd_head_wgrad_workspace": [i32, i32, i32, i32, i32, i32],
    "fmd_head_wgrad": [p, i32, p, p, p, i32, i32, i32, i32, i32, p, p, p, p],
}
_RESTYPE = {"fmd_linear_attention_workspace": i64, "fmd_linear_attention_state": i64, "fmd_wgrad_workspace": i64, "fmd_head_wgrad_workspace": i64, "fmd_halo_tiled_size": i64, "fmd_s2d_tiled_size": i64, "fmd_s2d_tiled_size_nd": i64, "fmd_grouped_linear_bwd_workspace": i64}

_lib = None


def lib():
    """Load (once) and return the library; raises if it was not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"fmdiff HIP library not found at {LIB_PATH}; run __graft_entry__.build() "
                "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
        L = C.CDLL(LIB_PATH)
        for name, args in SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = _RESTYPE.get(name, i32)
        from .runtime import tuning   # FMD_TUNE overrides the library mirrors too
        if tuning.overridden("HALO_MIN_WG"):
            check(L.fmd_halo_set_min_workgroups(tuning.get("HALO_MIN_WG")), "fmd_halo_set_min_workgroups")
        if tuning.overridden("HALO_TH8_MAX_WG"):
            check(L.fmd_halo_set_th8_max_workgroups(tuning.get("HALO_TH8_MAX_WG")), "fmd_halo_set_th8_max_workgroups")
        if tuning.overridden("HALO_TH4_MAX_WG"):
            check(L.fmd_halo_set_th4_max_workgroups(tuning.get("HALO_TH4_MAX_WG")), "fmd_halo_set_th4_max_workgroups")
        if tuning.overridden("CONV_GN_CB"):
            check(L.fmd_conv_gn_set_block_channels(tuning.get("CONV_GN_CB")), "fmd_conv_gn_set_block_channels")
        _lib = L
    return _lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with code {rc}")


def call(name: str, *args) -> None:
    check(getattr(lib(), name)(*args), name)
