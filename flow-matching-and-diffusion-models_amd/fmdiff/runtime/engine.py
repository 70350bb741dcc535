"""Fused HIP execution of EfficientUNetND / UNetDiffusersND (forward + hand-scheduled backward).

The engine walks the model's module tree (same order as the reference's
``_run_network``: ``src/models/unet/unet.py:310-326`` and
``src/models/unet/unet_diffusers_nd.py:172-191``) and issues the fused kernels
of ``csrc/``:

* a ResBlockND (``src/nn/blocks/residual.py:84-120``) is two implicit-GEMM
  convs: GN1+SiLU live in conv1's gather, the time-embedding add lives in
  conv1's epilogue, GN2 (+scale/shift)+SiLU in conv2's gather, the identity /
  1x1 skip and residual add in conv2's epilogue; both convs emit the channel
  statistics the next GroupNorm needs;
* the decoder ``torch.cat([h, skip])`` is a two-source gather, never copied;
* UpsampleND's nearest-x2 is a gather mode of the following conv;
* attention blocks: GN folded into the qkv 1x1-conv gather, head split
  (incl. the raw reshape) inside the attention kernel, residual in the
  projection epilogue.

The backward pass is written out (no autograd tape of primitive ops): each
layer pushes one closure that issues weight-gradient GEMMs (activations
recomputed in their gather prologue), data-gradient convs (with the SiLU'
multiply and the GroupNorm-backward sums in the epilogue) and the exact
GroupNorm backward ``dx = P*dz + Q*x + R``.  Parameter gradients are
accumulated straight into ``param.grad`` (fp32, reference layout).
"""
from __future__ import annotations

import math
import weakref
from typing import List, Optional, Tuple

import torch

from . import ops, tuning
from ..nn.blocks.attention import DiffusersAttentionND, SpatialCrossAttention, SpatialSelfAttention
from ..nn.blocks.residual import ResBlockND
from ..nn.ops.convolution import ConvND
from ..nn.ops.upsampling import DownsampleND, UpsampleND
from ..nn.params import Conv, Identity

BF16 = torch.bfloat16
F32 = torch.float32
CPAD = 8      # NHWC channel padding of the model input / output (16-byte rows)
HALO_BK = 32  # input channels per halo-kernel chunk (FMD_HALO_BK, include/fmdiff.h)
# 3-D: materialise the GN+SiLU operand of depth-tap halo convs (MAT3D=0: fused prologue + G side output)
MAT3D = bool(tuning.get("MAT3D"))
# 3x3x3 stride-1 convs on the halo kernel with (depth tap, channel block) chunks (csrc/conv_halo.hip)
DEPTH_HALO = bool(tuning.get("DEPTH_HALO"))
# stride-2 3x3 forwards and nearest-x2 data gradients on the space-to-depth halo kernel (fmd_conv_s2d); 0: the
# implicit GEMM (A/B runs, runtime/tuning.py)
S2D_HALO = bool(tuning.get("S2D_HALO"))
S2D_3D = S2D_HALO and bool(tuning.get("S2D_3D"))
# ResBlock 3x3 convs on 1x1 images run as their centre tap (WeightCache.center); POINT_1X1=0 for A/B runs
POINT_1X1 = bool(tuning.get("POINT_1X1"))
# forward-only self-attention at the fmd_conv_small levels: both projections on it (runtime/tuning.py SMALL_ATTN)
SMALL_ATTN = bool(tuning.get("SMALL_ATTN"))
# training, 3-D fused-prologue halo convs (MAT3D=0): the conv writes G = SiLU(GN(x)) for the weight gradient
# (fmd_conv_desc.gout), which would otherwise recompute G once per depth tap.  Not on 2-D: there the extra
# 2 B/element of HBM writes cost the forward more than the weight gradient saves.


class Act:
    """One NHWC bf16 activation, its per-channel statistics and its gradient."""
    __slots__ = ("t", "stats", "grad", "need_grad")

    def __init__(self, t: torch.Tensor, stats: Optional[ops.Stats] = None, need_grad: bool = True):
        self.t = t
        self.stats = stats
        self.grad = None
        self.need_grad = need_grad

    @property
    def C(self):
        return self.t.shape[-1]


def _stats(a: Optional[Act]):
    if a is None:
        return None
    if a.stats is None:
        a.stats = ops.channel_stats(a.t)
    return a.stats


def _gdest(a: Optional[Act]):
    """(buffer, accumulate) for writing a's gradient."""
    if a is None:
        return None, 0
    if a.grad is None:
        a.grad = torch.empty_like(a.t)
        return a.grad, 0
    return a.grad, 1


def _materialise(halo: bool, x1, Cin: int, HW: int, d3: bool = False) -> bool:
    """Materialise the GN+SiLU prologue (fmd_gn_apply_fwd) instead of fusing it into the conv: always on
    the generic implicit-GEMM path (small levels), whose gather would redo the transform once per tap
    (9x, VALU-bound at the low occupancy of those levels); on the 3-D depth-tap halo path when MAT3D (its
    chunks stage every input slice for 3 depth taps, so the fused transform runs ~3.8x per element, and the
    weight gradient reads the same materialised operand); never on the 2-D halo path (a 41 us streaming pass
    per 256^2 conv against ~23 us of in-kernel transform saved: measured net-negative)."""
    if not halo:
        return True
    return bool(d3 and MAT3D)


class WeightCache:
    """bf16 kernel-layout copies of the fp32 master weights.

    Entries are created lazily by the layers; after an optimizer step ``invalidate`` re-derives ALL of
    them -- base layouts and halo tiles, directly from the fp32 masters -- in one batched launch
    (fmd_prep_weights_batch), after refreshing the few fp32 derived buffers (padded biases, fused
    q/k/v).  The device job table is rebuilt only when the set of entries or their storage changes."""

    def __init__(self):
        self._c = {}
        self._force = set()
        self._tables = {}   # cubic (3x3x3 masters) or not -> (key, device job table, njobs, nblocks)
        # job tables replaced by a rebuild: a captured graph (train step, sampler) holds the raw pointer of
        # the table it recorded and replays fmd_prep_weights_batch on it, so a table lives as long as the cache
        self._retired: List[torch.Tensor] = []

    @staticmethod
    def _ver(t):
        return (t._version, t.data_ptr())

    def invalidate(self):
        for key, e in self._c.items():          # fp32 derived buffers first: they feed the bf16 layouts
            if e["kind"] == "pad":
                e["buf"][: e["src"].numel()].copy_(e["src"].detach().reshape(-1))
            elif e["kind"] == "e1d":
                self._embed1d(e["src"], e["buf"])
            elif e["kind"] == "ctr":
                e["buf"].copy_(e["src"].detach()[:, :, 1:2, 1:2])
            elif e["kind"] == "fused":
                o = 0
                for w in e["src"]:
                    e["buf"][o:o + w.shape[0]].copy_(w.detach())
                    o += w.shape[0]
            elif e["kind"] == "s2d":
                ops.s2d_tile_weights(e["src"].detach(), e["mode"], out=e["buf"])
        for cubic in (False, True):   # square (<= 9 taps) and cubic (27 taps) masters: one launch each
            jobs = [(key, e) for key, e in self._c.items()
                    if e["kind"] in ("prep", "tiled") and (e["job"][7] == 27) == cubic]
            if jobs:
                self._launch_batch(jobs, cubic)
        for key, e in self._c.items():
            e["ver"] = self._ver(e["src"]) if e["kind"] != "fused" else tuple(self._ver(w) for w in e["src"])
        self._force.clear()

    def _launch_batch(self, jobs, cubic=False):
        """One fmd_prep_weights_batch job per fp32 master: every layout of it from one read of each tile
        (``cubic``: 3x3x3 masters, fmd_prep_weights_batch_cubic, 16-row k tiles)."""
        key = tuple((e["src"].data_ptr(), e["buf"].data_ptr(), e["job"]) for _, e in jobs)
        ptk = 16 if cubic else 32
        tab = self._tables.get(cubic)
        if tab is None or key != tab[0]:
            per_src = {}
            for src_ptr, buf_ptr, job in key:
                per_src.setdefault(src_ptr, []).append((buf_ptr, job))
            rows, blk = [], 0
            for src_ptr, outs in per_src.items():
                for i in range(0, len(outs), 6):
                    part = outs[i:i + 6]
                    K, C, ks = part[0][1][:3]
                    kp = cp = 0
                    descs = []
                    for buf_ptr, (_, _, _, mode, R, Cc, kind, _T, _n) in part:
                        r_ext = -(-R // 128) * 128 if kind else R
                        c_ext = -(-Cc // HALO_BK) * HALO_BK if kind else Cc
                        k_ext, c_ext2 = (r_ext, c_ext) if mode == 0 else (c_ext, r_ext)
                        kp, cp = max(kp, k_ext), max(cp, c_ext2)
                        descs += [buf_ptr, mode | (kind << 8) | (R << 16) | (Cc << 40)]
                    kt, ct = -(-kp // ptk), -(-cp // 32)
                    row = [src_ptr, K | (C << 32), ks | (len(part) << 32), blk | (kt << 32)] + descs
                    rows.append(row + [0] * (16 - len(row)))
                    blk += kt * ct
            dev = jobs[0][1]["buf"].device
            if tab is not None:
                self._retired.append(tab[1])
            tab = (key, torch.tensor(rows, dtype=torch.int64).to(dev), len(rows), blk)
            self._tables[cubic] = tab
        from .. import _lib as L
        L.call("fmd_prep_weights_batch_cubic" if cubic else "fmd_prep_weights_batch", tab[1].data_ptr(), tab[2], tab[3],
               ops.stream())

    def _fresh(self, key, src_ver):
        e = self._c.get(key)
        return e is not None and e["ver"] == src_ver and key not in self._force

    @staticmethod
    def _embed1d(w, buf):
        """fp32 [K][C][k] weight of a 1-D conv -> [K][C][k][k] with the taps in column (k-1)/2: a 1-D signal runs
        as an (L, 1) image, where that column is the only one that meets data (the others read zero padding)."""
        buf.zero_()
        buf[..., (w.shape[2] - 1) // 2].copy_(w.detach())

    def embed1d(self, w: torch.Tensor) -> torch.Tensor:
        key = (id(w), "e1d")
        if not self._fresh(key, self._ver(w)):
            e = self._c.get(key)
            k = w.shape[2]
            buf = e["buf"] if e is not None else torch.empty((*w.shape[:2], k, k), device=w.device, dtype=F32)
            self._embed1d(w, buf)
            self._c[key] = dict(kind="e1d", src=w, buf=buf, ver=self._ver(w))
            self._force.discard(key)
        return self._c[key]["buf"]

    def center(self, w: torch.Tensor) -> torch.Tensor:
        """fp32 [K][C][1][1] centre tap of a 3x3 weight: on a 1x1 image (zero padding all round) the 3x3 conv is
        exactly the 1x1 conv with this weight, a ninth of the weight bytes and K-steps."""
        key = (id(w), "ctr")
        if not self._fresh(key, self._ver(w)):
            e = self._c.get(key)
            buf = e["buf"] if e is not None else torch.empty((*w.shape[:2], 1, 1), device=w.device, dtype=F32)
            buf.copy_(w.detach()[:, :, 1:2, 1:2])
            self._c[key] = dict(kind="ctr", src=w, buf=buf, ver=self._ver(w))
            self._force.discard(key)
        return self._c[key]["buf"]

    def get(self, w: torch.Tensor, mode: int, Kpad=None, Cpad=None):
        if w.dim() == 3 and w.shape[2] > 1:   # 1-D k-tap conv: its (L, 1)-image embedding
            w = self.embed1d(w)
        key = (id(w), mode, Kpad, Cpad)
        if not self._fresh(key, self._ver(w)):
            e = self._c.get(key)
            buf = ops.prep_weights(w.detach(), mode, Kpad, Cpad, out=None if e is None else e["buf"])
            K, C = w.shape[0], w.shape[1]
            ks = w.shape[2] if w.dim() >= 4 else 1
            R, T, Cc = buf.shape
            self._c[key] = dict(kind="prep", src=w, buf=buf, ver=self._ver(w),
                                job=(K, C, ks, mode, R, Cc, 0, T, buf.numel()))
            self._force.discard(key)
        return self._c[key]["buf"]

    def tiled(self, w: torch.Tensor, mode: int, Kpad=None, Cpad=None):
        """Halo-kernel tiling of ``get(w, mode, ...)`` (csrc/conv_halo.hip)."""
        key = (id(w), "tiled", mode, Kpad, Cpad)
        if not self._fresh(key, self._ver(w)):
            base = self.get(w, mode, Kpad, Cpad)
            e = self._c.get(key)
            buf = ops.tile_weights(base, out=None if e is None else e["buf"])
            K, C = w.shape[0], w.shape[1]
            ks = w.shape[2] if w.dim() == 4 else 1
            R, T, Cc = base.shape
            self._c[key] = dict(kind="tiled", src=w, buf=buf, ver=self._ver(w),
                                job=(K, C, ks, mode, R, Cc, 1, T, buf.numel()))
            self._force.discard(key)
        return self._c[key]["buf"]

    @staticmethod
    def _dpack(w, mode, buf):
        """fp32 [R][3 * Cr][3][3] 2-D view of a 3x3x3 weight for the depth-tap halo conv: channel block
        kz*Cr + c holds tap kz of input channel c (Cr = C rounded up to 32, zero padded).  mode 0: the
        forward weight; mode 3: the data-gradient weight W'[c][k][kz][ky][kx] = W[k][c][2-kz][2-ky][2-kx]."""
        src = w.detach() if mode == 0 else w.detach().flip(2, 3, 4).transpose(0, 1)
        R, Cs = src.shape[:2]
        Cr = buf.shape[1] // 3
        v = buf.view(R, 3, Cr, 3, 3)
        if Cr != Cs:
            v[:, :, Cs:].zero_()
        v[:, :, :Cs].copy_(src.permute(0, 2, 1, 3, 4))

    def dtiled(self, w: torch.Tensor, mode: int):
        """Halo-tiled depth-tap layout of a 3x3x3 weight (mode 0 forward, 3 data gradient): the 2-D tiles of the
        ``_dpack`` view, re-derived by the cubic batched prep (kind 2) after each optimizer step; the first
        fill goes through the fp32 view + fmd_tile_weights_halo (the same single bf16 rounding)."""
        key = (id(w), "dtiled", mode)
        if not self._fresh(key, self._ver(w)):
            e = self._c.get(key)
            K, C = w.shape[0], w.shape[1]
            R, Cs = (K, C) if mode == 0 else (C, K)
            view = torch.empty((R, 3 * (-(-Cs // HALO_BK) * HALO_BK), 3, 3), device=w.device, dtype=F32)
            self._dpack(w, mode, view)
            buf = ops.tile_weights(ops.prep_weights(view, 0), out=None if e is None else e["buf"])
            self._c[key] = dict(kind="tiled", src=w, buf=buf, ver=self._ver(w),
                                job=(K, C, 3, mode, R, Cs, 2, 27, buf.numel()))
            self._force.discard(key)
        return self._c[key]["buf"]

    def s2d(self, w: torch.Tensor, mode: int):
        """Stride-2 halo tiles of a 3x3 (3x3x3) weight (fmd_s2d_tile_weights_nd): mode 0 the stride-2 forward, 1 the data
        gradient of the conv on a nearest-x2 input, 2 the stride-2 data gradient; re-derived by one launch per
        optimizer step."""
        key = (id(w), "s2d", mode)
        if not self._fresh(key, self._ver(w)):
            e = self._c.get(key)
            buf = ops.s2d_tile_weights(w.detach(), mode, out=None if e is None else e["buf"])
            self._c[key] = dict(kind="s2d", src=w, buf=buf, ver=self._ver(w), mode=mode)
            self._force.discard(key)
        return self._c[key]["buf"]

    def padded(self, v: torch.Tensor, n: int):
        key = (id(v), "pad", n)
        if not self._fresh(key, self._ver(v)):
            e = self._c.get(key)
            buf = e["buf"] if e is not None else torch.zeros(n, device=v.device, dtype=F32)
            buf[: v.numel()].copy_(v.detach().reshape(-1))
            self._c[key] = dict(kind="pad", src=v, buf=buf, ver=self._ver(v))
            self._force.discard(key)
        return self._c[key]["buf"]

    def fused(self, ws, key_name):
        """Concatenate several fp32 tensors along dim 0 (fused q/k/v projection)."""
        key = (tuple(id(w) for w in ws), key_name)
        ver = tuple(self._ver(w) for w in ws)
        if not self._fresh(key, ver):
            e = self._c.get(key)
            buf = e["buf"] if e is not None else torch.empty((sum(w.shape[0] for w in ws), *ws[0].shape[1:]),
                                                             device=ws[0].device, dtype=F32)
            o = 0
            for w in ws:
                buf[o:o + w.shape[0]].copy_(w.detach())
                o += w.shape[0]
            self._c[key] = dict(kind="fused", src=list(ws), buf=buf, ver=ver)
            self._force.discard(key)
        return self._c[key]["buf"]


class Ctx:
    __slots__ = ("emb", "demb", "tape", "N", "eo_all", "demb_all", "mark", "cca", "marks", "drop_seeded")

    def __init__(self, emb, save, N):
        self.emb = emb
        self.demb = torch.zeros_like(emb) if save else None
        self.tape: Optional[List] = [] if save else None
        self.N = N
        self.eo_all = None      # [N][sum O] grouped emb projections of all ResBlocks
        self.demb_all = None
        self.mark = 0           # tape length when the decoder started (backward part 1 = tape[mark:])
        self.marks: List[int] = []   # tape length before each encoder stage (backward segments, see seg_ranges)
        self.cca = None         # cross-attention context (context_ca), fp32 as passed to the model
        self.drop_seeded = False   # this forward has advanced the dropout seed counter


def _check_conv(c: Conv, ks, stride, pad):
    if c.dims not in (1, 2, 3):
        raise NotImplementedError(f"spatial_dims={c.dims}")
    n = c.dims
    if c.kernel_size != (ks,) * n or c.stride != (stride,) * n or c.padding != (pad,) * n:
        raise NotImplementedError(f"unexpected conv geometry {c.kernel_size}/{c.stride}/{c.padding}")


class UNetEngine:
    def __init__(self, model):
        from ..models.unet.unet import EfficientUNetND
        from ..models.unet.unet_diffusers_nd import UNetDiffusersND
        self._model = weakref.ref(model)
        if isinstance(model, EfficientUNetND):
            self.kind = "efficient"
        elif isinstance(model, UNetDiffusersND):
            self.kind = "diffusers"
        else:
            raise TypeError(type(model))
        self.wc = WeightCache()
        self._tt = None   # precomputed per-step time embeddings (set_time_table)
        self.gl, self.gl_slot = self._group_emb_layers(model)
        # spatial_dims = 1: signals run as (L, 1) images -- 1-D k-tap weights embedded as k x k
        # (WeightCache.embed1d), resampling along the first dim only
        self.dims1 = next(c for c in model.modules() if isinstance(c, Conv)).dims == 1

    @staticmethod
    def _group_emb_layers(model):
        """ResBlocks whose emb projection feeds the block (scale-shift or added embedding) share one
        grouped launch; a mixed emb_activation_before_proj keeps the per-block path."""
        blocks = [mod for mod in model.modules() if isinstance(mod, ResBlockND)
                  and (mod.use_scale_shift_norm or mod.add_embedding_to_hidden)]
        if not blocks or len({bool(b.emb_activation_before_proj) for b in blocks}) != 1:
            return None, {}
        gl = ops.GroupedLinear([b.emb_layers for b in blocks], blocks[0].emb_activation_before_proj)
        return gl, {id(b): (gl.off[i], gl.O[i]) for i, b in enumerate(blocks)}

    @property
    def m(self):
        return self._model()

    def invalidate_weights(self):
        self.wc.invalidate()

    # ------------------------------------------------------------- layers
    def conv_layer(self, conv: Conv, x: Act, ctx: Ctx, *, stride=1, upsample=False, cpad=None):
        """Plain 3x3 conv (input conv, DownsampleND, UpsampleND)."""
        _check_conv(conv, 3, stride, 1)
        Cin = x.C
        N_, sp = x.t.shape[0], tuple(x.t.shape[1:-1])
        if (ctx.tape is None and len(sp) == 2 and not self.dims1 and conv.weight.dim() == 4 and
                conv.weight.shape[1] == Cin):
            # forward only, small level: one launch with the output statistics (fmd_conv_small)
            mode = "s2" if stride == 2 else "up" if upsample else "s1"
            if ops.conv_small_ok(tuple(x.t.shape), conv.out_channels, mode=mode):
                out, st = ops.conv_small(x.t, conv.out_channels, self.wc.get(conv.weight, 0), mode=mode,
                                         bias=conv.bias)
                return Act(out, st)
        Ho_ = ops.out_hw(sp[0], 3, stride, 1, upsample)
        if len(sp) == 2:
            halo = stride == 1 and ops.halo_eligible(N_, sp[0], Ho_, ops.out_hw(sp[1], 3, stride, 1, upsample),
                                                     conv.out_channels, upsample=upsample, Cin=Cin)
        else:   # depth-tap halo, nearest-x2 included (output depth 2D)
            Do_ = 2 * sp[0] if upsample else sp[0]
            halo = DEPTH_HALO and stride == 1 and ops.halo_eligible(
                N_ * Do_, sp[1], ops.out_hw(sp[1], 3, 1, 1, upsample), ops.out_hw(sp[2], 3, 1, 1, upsample),
                conv.out_channels, upsample=upsample, Cin=Cin, ztaps=3)
        s2d = S2D_HALO and stride == 2 and conv.weight.shape[1] == Cin and (
            ops.s2d_eligible(N_, sp[0], sp[1], sp[0] // 2, sp[1] // 2, conv.out_channels, Cin, 3) if len(sp) == 2
            else S2D_3D and ops.s2d_eligible(N_, sp[1], sp[2], sp[1] // 2, sp[2] // 2, conv.out_channels, Cin, 3,
                                             sp[0], sp[0] // 2))
        if s2d:   # DownsampleND's conv on the space-to-depth halo kernel (3-D: depth taps as chunks)
            out, st = ops.conv(x.t, conv.out_channels, None, ks=3, stride=2, pad=1, bias=conv.bias, want_stats="free",
                               s2d_tiled=self.wc.s2d(conv.weight, 0))
        else:
            w, wt = self._wts(conv.weight, 0, halo, None, Cin)
            out, st = ops.conv(x.t, conv.out_channels, w, ks=3, stride=stride, pad=1, upsample=upsample,
                               bias=conv.bias, want_stats="free", wgt_tiled=wt)
        o = Act(out, st)
        if ctx.tape is not None:
            def bwd():
                dy = o.grad

                def wg():
                    tgt = self._wgrad_target(conv, Cin)
                    ops.wgrad(x.t, dy, tgt, ks=3, stride=stride, pad=1, upsample=upsample,
                              db=conv.bias.grad if conv.bias is not None else None)
                    self._wgrad_finish(conv, Cin, tgt)
                self._wg(wg, dy.numel() // dy.shape[-1])
                if not x.need_grad:
                    return
                g, acc = _gdest(x)
                # the tiled mode-1 weight covers exactly conv.weight.shape[0] gradient channels: a channel-padded dy
                # would read past it, so such a dy takes the generic path
                if upsample and len(sp) == 2 and S2D_HALO and conv.weight.shape[1] == Cin and \
                        dy.shape[-1] == conv.weight.shape[0] and ops.s2d_eligible(
                        N_, 2 * sp[0], 2 * sp[1], sp[0], sp[1], Cin, dy.shape[-1], 4):
                    # nearest-x2 folded into a 4x4 stride-2 gather, on the space-to-depth halo kernel
                    ops.conv(dy, Cin, None, ks=4, stride=2, pad=1, out_hw_=sp, out=g, accumulate=bool(acc),
                             s2d_tiled=self.wc.s2d(conv.weight, 1))
                elif upsample and len(sp) == 3 and S2D_3D and conv.weight.shape[1] == Cin and \
                        dy.shape[-1] == conv.weight.shape[0] and ops.s2d_eligible(
                        N_, 2 * sp[1], 2 * sp[2], sp[1], sp[2], Cin, dy.shape[-1], 4, 2 * sp[0], sp[0]):
                    # 3-D: the nearest-x2 copy folded into a 4x4x4 stride-2 gather (the depth taps as chunks)
                    ops.conv(dy, Cin, None, ks=4, stride=2, pad=1, out_hw_=sp, out=g, accumulate=bool(acc),
                             s2d_tiled=self.wc.s2d(conv.weight, 1))
                elif upsample and len(sp) == 2:
                    # nearest-x2 folded into the weights: a 4x4 stride-2 transposed gather (mode 2)
                    wd = self.wc.get(conv.weight, 2)
                    ops.conv(dy, Cin, wd, ks=4, stride=2, pad=1, out_hw_=sp, out=g, accumulate=bool(acc))
                elif upsample:
                    # 3-D: data gradient at the upsampled resolution, then the 2x2x2 box sum the
                    # nearest-x2 copy implies
                    hi = self.dgrad3x3(conv.weight, dy, Cin, tuple(2 * v for v in sp))[0]
                    ops.sum_pool2_3d(hi, g, acc=bool(acc))
                else:
                    self.dgrad3x3(conv.weight, dy, Cin, sp, stride=stride, out=g, accumulate=bool(acc))
            ctx.tape.append(bwd)
        return o

    def pool_layer(self, conv: Conv, x: Act, ctx: Ctx):
        """PoolND (reference nn/ops/pooling.py:10-30, unet.py:124-126): conv with kernel = stride = pool_factor,
        no padding, on the (channel-padded) model input; weight gradient only (the input is data)."""
        pf = conv.stride[0]
        if self.dims1:
            raise NotImplementedError("pool_factor > 1 with spatial_dims=1")
        if conv.kernel_size != (pf,) * conv.dims or conv.padding != (0,) * conv.dims:
            raise NotImplementedError(f"PoolND geometry {conv.kernel_size}/{conv.stride}/{conv.padding}")
        Cin = x.C
        out, _ = ops.conv(x.t, conv.out_channels, self.wc.get(conv.weight, 0, None, Cin), ks=pf, stride=pf, pad=0,
                          bias=conv.bias)
        o = Act(out)
        if ctx.tape is not None:
            def bwd():
                def wg():
                    tgt = self._wgrad_target(conv, Cin)
                    ops.wgrad(x.t, o.grad, tgt, ks=pf, stride=pf, pad=0,
                              db=conv.bias.grad if conv.bias is not None else None)
                    self._wgrad_finish(conv, Cin, tgt)
                self._wg(wg)
            ctx.tape.append(bwd)
        return o

    def unpool_layer(self, ct, hb: torch.Tensor, ctx: Ctx):
        """UnPoolND (reference pooling.py:87-105, unet.py:280-287): ConvTranspose with kernel = stride =
        pool_factor = the transposed gather of the conv F (hi -> lo) whose weight is ct.weight [in, out, *k],
        to the fp32 NHWC model output with CPAD-padded channels.  Backward: dx = F(dy), dW = F's weight
        gradient with dy in F's input role, db = channel sums of dy."""
        pf = ct.stride[0]
        if ct.kernel_size != (pf,) * ct.dims or ct.padding != (0,) * ct.dims or any(ct.output_padding):
            raise NotImplementedError(f"UnPoolND geometry {ct.kernel_size}/{ct.stride}/{ct.padding}")
        K, mc = ct.out_channels, ct.in_channels
        Kp = max(CPAD, -(-K // 8) * 8)
        sp_hi = tuple(pf * v for v in hb.shape[1:-1])
        bias = self.wc.padded(ct.bias, Kp) if ct.bias is not None else None
        out, _ = ops.conv(hb, Kp, self.wc.get(ct.weight, 1, None, Kp), ks=pf, stride=pf, pad=0, transposed=True,
                          out_hw_=sp_hi, bias=bias, out_f32=True)
        if ctx.tape is not None:
            head_bwd = self._head_bwd

            def bwd(dpred):
                def wg():
                    tmp = torch.zeros((mc, Kp, *ct.kernel_size), device=hb.device, dtype=F32)
                    ops.wgrad(dpred, hb, tmp, ks=pf, stride=pf, pad=0, accumulate=False)
                    ct.weight.grad.add_(tmp[:, :K])
                    if ct.bias is not None:
                        ct.bias.grad.add_(ops.channel_stats(dpred).slab[..., 0].sum(0)[:K])
                self._wg(wg)
                dh, _ = ops.conv(dpred, mc, self.wc.get(ct.weight, 0, None, Kp), ks=pf, stride=pf, pad=0)
                head_bwd(dh)
            self._head_bwd = bwd
        return out

    def resample_layer(self, x: Act, ctx: Ctx, up: bool):
        """Parameter-free resampling (fmd_resample2): AvgPoolND(kernel=stride=2) of DownsampleND(use_conv=False)
        (src/nn/ops/upsampling.py:52-58, pooling.py:33-53) or the nearest-x2 F.interpolate of
        UpsampleND(use_conv=False) (upsampling.py:24-29).  Output statistics are computed where a GroupNorm
        consumes them."""
        N, sp, C = x.t.shape[0], tuple(x.t.shape[1:-1]), x.C
        fac = (2, 1) if self.dims1 else (2,) * len(sp)
        osp = tuple(v * f for v, f in zip(sp, fac)) if up else tuple(v // f for v, f in zip(sp, fac))
        scale = 1.0 if up else 1.0 / math.prod(fac)
        out = torch.empty((N, *osp, C), device=x.t.device, dtype=torch.bfloat16)
        ops.resample2(x.t, out, up, scale, factors=fac)
        o = Act(out)
        if ctx.tape is not None and x.need_grad:
            def bwd():
                if o.grad is None:
                    return
                g, acc = _gdest(x)
                ops.resample2(o.grad, g, not up, 1.0 if up else scale, acc=bool(acc), factors=fac)
            ctx.tape.append(bwd)
        return o

    def _wg(self, fn, px=None):
        """Weight-gradient work, issued in line on the current stream.  (A side-stream variant beside the
        data-gradient chain measured no gain on MI355X -- the halo wgrad / dgrad kernels contend for LDS and
        the issue port -- and was retired in round 4.)"""
        fn()

    def _join(self):
        pass

    def _wts(self, w, mode, halo: bool, Kpad=None, Cpad=None):
        """(base, tiled) kernel layouts of ``w``: only the one the chosen conv path reads is derived
        (and refreshed by every optimizer step), the other is None."""
        if halo:
            if w.dim() == 5 and w.shape[2] == 3:
                return None, self.wc.dtiled(w, mode)
            return None, self.wc.tiled(w, mode, Kpad, Cpad)
        return self.wc.get(w, mode, Kpad, Cpad), None

    def dgrad3x3(self, w, dy, Cin, sp, *, stride=1, Kpad=None, **kw):
        """Data gradient of a 3x3 (3x3x3) pad-1 conv onto the input grid ``sp`` ((H, W) or (D, H, W)).
        Stride 1 = forward gather with flipped taps (so a 2-D one runs on the halo-tiled kernel);
        stride 2 = transposed gather."""
        sp = tuple(sp)
        if stride == 1:
            halo = self._halo_ok(dy.shape[0], sp, Cin, dy.shape[-1])
            base, tiled = self._wts(w, 3, halo, Kpad, None)
            return ops.conv(dy, Cin, base, ks=3, stride=1, pad=1, out_hw_=sp, wgt_tiled=tiled, **kw)
        if S2D_HALO and Kpad is None and w.shape[1] == Cin and not kw.get("pro") and (
                ops.d2s_eligible(dy.shape[0], dy.shape[1], dy.shape[2], sp[0], sp[1], Cin, dy.shape[-1])
                if len(sp) == 2 and w.dim() == 4 else
                S2D_3D and len(sp) == 3 and w.dim() == 5 and ops.d2s_eligible(dy.shape[0], dy.shape[2], dy.shape[3], sp[1], sp[2],
                                                                    Cin, dy.shape[-1], dy.shape[1], sp[0])):
            # transposed stride-2 gather onto the depth-to-space view, on the halo kernel (3-D: 8 classes)
            return ops.conv(dy, Cin, None, ks=3, stride=2, pad=1, transposed=True, out_hw_=sp,
                            s2d_tiled=self.wc.s2d(w, 2), **kw)
        return ops.conv(dy, Cin, self.wc.get(w, 1, Kpad, None), ks=3, stride=stride, pad=1, transposed=True,
                        out_hw_=sp, **kw)

    @staticmethod
    def _halo_ok(N, sp, K, Cin, pro=False) -> bool:
        """3x3 (3x3x3) stride-1 conv onto the grid ``sp`` on the halo kernel (3-D: depth-tap chunks)."""
        if len(sp) == 2:
            return ops.halo_eligible(N, sp[0], sp[0], sp[1], K, Cin=Cin, pro=pro)
        D, H, W = sp
        return DEPTH_HALO and ops.halo_eligible(N * D, H, H, W, K, Cin=Cin, pro=pro, ztaps=3)

    def _wgrad_target(self, conv: Conv, Cin: int):
        """fp32 buffer the wgrad kernel writes: param.grad itself unless channels were padded."""
        if conv.weight.shape[1] == Cin and conv.weight.shape[0] % 8 == 0:
            return conv.weight.grad
        return torch.zeros((max(8, -(-conv.weight.shape[0] // 8) * 8), Cin, *conv.weight.shape[2:]),
                           device=conv.weight.device, dtype=F32)

    def _wgrad_finish(self, conv: Conv, Cin: int, tgt):
        if tgt is conv.weight.grad:
            return
        K, C = conv.weight.shape[:2]
        conv.weight.grad.add_(tgt[:K, :C])

    def res_block(self, m: ResBlockND, xs: List[Act], ctx: Ctx):
        x0 = xs[0]
        x1 = xs[1] if len(xs) > 1 else None
        N, C0, sp = x0.t.shape[0], x0.t.shape[-1], tuple(x0.t.shape[1:-1])
        C1 = x1.C if x1 is not None else 0
        Cin, Cout, HW = C0 + C1, m.out_channels, math.prod(sp)
        H, W = sp[-2], sp[-1]
        if Cin != m.channels:
            raise ValueError(f"ResBlockND expects {m.channels} channels, got {Cin}")
        drop = float(m.dropout) if (m.dropout and m.training) else 0.0
        if drop:
            seed, salt = self._dropout_seed(m, ctx, x0.t.device)
        c1, c2 = m.conv1.conv, m.conv2.conv
        _check_conv(c1, 3, 1, 1)
        _check_conv(c2, 3, 1, 1)
        g1, g2 = m.norm1, m.norm2
        el = m.emb_layers
        ss = m.use_scale_shift_norm
        add = (not ss) and m.add_embedding_to_hidden and el is not None
        slot = self.gl_slot.get(id(m)) if ctx.eo_all is not None else None
        if slot is not None:   # view into the grouped projection (row stride = gl.total)
            eo = ctx.eo_all[:, slot[0]:slot[0] + slot[1]]
            es = self.gl.total
        elif ss or add:
            eo = ops.linear(ctx.emb, el.weight, el.bias, in_silu=m.emb_activation_before_proj)
            es = eo.shape[1]
        else:   # the embedding projection feeds nothing (or the block has none: VAE ResBlocks)
            eo, es = None, 0
        if ctx.tape is None and not drop and len(sp) == 2 and not self.dims1:
            o = self._res_block_small(m, x0, x1, eo, es, ss, add)
            if o is not None:
                return o
        halo1 = self._halo_ok(N, sp, Cout, Cin, pro=True)
        mat1 = _materialise(halo1, x1, Cin, HW, len(sp) == 3)
        if mat1 and not halo1:   # without the fused prologue the halo kernel's affine-table limit is moot
            halo1 = self._halo_ok(N, sp, Cout, Cin)
        # a 1x1 level (the bottom of a small latent UNet): the 3x3 convs are their centre taps (exact)
        point = POINT_1X1 and sp == (1, 1) and c1.weight.dim() == 4 and not halo1
        pk = dict(ks=1, pad=0) if point else {}
        w1, w1t = (self.wc.get(self.wc.center(c1.weight), 0), None) if point else self._wts(c1.weight, 0, halo1)
        if mat1 and ops.gn_fused_eligible(HW, Cin, C0, g1.num_groups):
            # small level: statistics, affine and the materialised prologue in one launch from x0|x1
            a1, b1, mr1, t1 = ops.gn_fused_apply(x0.t, x1.t if x1 else None, g1.num_groups, g1.eps, g1.weight,
                                                 g1.bias)
        elif ctx.tape is None and not mat1 and halo1 and len(sp) == 2 and ops.HALO_FOLD:
            # forward only, halo conv1: the GroupNorm-1 affine folded inside the conv from the statistics slabs
            a1 = b1 = mr1 = t1 = None
        else:
            a1, b1, mr1 = ops.gn_prep(_stats(x0), _stats(x1), N, HW, C0, C1, g1.num_groups, g1.eps, g1.weight,
                                      g1.bias)
            t1 = ops.gn_apply_fwd(x0.t, x1.t if x1 else None, a1, b1) if mat1 else None
        pf1 = (dict(st0=_stats(x0), st1=_stats(x1), groups=g1.num_groups, eps=g1.eps, gamma=g1.weight, beta=g1.bias)
               if a1 is None and t1 is None else None)
        halo2 = self._halo_ok(N, sp, Cout, Cout, pro=True)
        mat2 = _materialise(halo2, None, Cout, HW, len(sp) == 3) or bool(drop)   # dropout acts on the materialised operand
        fuse2 = mat2 and ops.gn_fused_eligible(HW, Cout, Cout, g2.num_groups)
        src1 = x1.t if (x1 is not None and t1 is None) else None
        keep_g = ctx.tape is not None and len(sp) == 3
        gg1 = (torch.empty((N, *sp, Cin), device=x0.t.device, dtype=torch.bfloat16)
               if keep_g and t1 is None and halo1 and not point and Cin % HALO_BK == 0 else None)
        # small level, split-K conv1: GroupNorm-2 (+ scale/shift) + SiLU inside conv1's combine (fmd_conv_gn);
        # not with the additive embedding under a tape (its backward needs conv1's statistics slab)
        gnreq = (dict(groups=g2.num_groups, eps=g2.eps, gamma=g2.weight, beta=g2.bias, emb=eo if ss else None,
                      emb_stride=es if ss else 0, emb_mode=1 if ss else 0)
                 if fuse2 and not (add and ctx.tape is not None) else None)
        h, hst = ops.conv(t1 if t1 is not None else x0.t, Cout, w1, src1=src1,
                          pro=None if (t1 is not None or pf1 is not None) else (a1, b1, True), pro_fold=pf1,
                          bias=c1.bias, bias_nc=eo.contiguous() if add else None,
                          want_stats=(add and ctx.tape is not None) or not fuse2,
                          wgt_tiled=w1t, gout=gg1, gn=gnreq, **pk)
        t2 = None
        if fuse2 and gnreq is not None and "res" in gnreq:
            a2, b2, mr2, t2 = gnreq["res"]
        elif fuse2:
            a2, b2, mr2, t2 = ops.gn_fused_apply(h, None, g2.num_groups, g2.eps, g2.weight, g2.bias,
                                                 emb=eo if ss else None, emb_stride=es if ss else 0,
                                                 emb_mode=1 if ss else 0)
        elif ctx.tape is None and not mat2 and halo2 and len(sp) == 2 and hst is not None and ops.HALO_FOLD:
            a2 = b2 = mr2 = None   # forward only, halo conv2: GroupNorm-2 folded inside the conv (as conv1)
        elif ss:
            a2, b2, mr2 = ops.gn_prep(hst, None, N, HW, Cout, 0, g2.num_groups, g2.eps, g2.weight, g2.bias, emb=eo,
                                      emb_stride=es, emb_mode=1)
        else:
            a2, b2, mr2 = ops.gn_prep(hst, None, N, HW, Cout, 0, g2.num_groups, g2.eps, g2.weight, g2.bias)
        pf2 = (dict(st0=hst, groups=g2.num_groups, eps=g2.eps, gamma=g2.weight, beta=g2.bias, emb=eo if ss else None,
                    emb_stride=es if ss else 0) if a2 is None and t2 is None else None)
        sk = m.skip_connection
        kw = {}
        if isinstance(sk, Identity):
            if x1 is not None:
                raise ValueError("identity skip with concatenated input")
            kw["resid"] = x0.t
        else:
            _check_conv(sk.conv, 1, 1, 0)
        if mat2 and not halo2:
            halo2 = self._halo_ok(N, sp, Cout, Cout)
        if not isinstance(sk, Identity):
            s2, s2t = self._wts(sk.conv.weight, 0, halo2)
            kw.update(src2=x0.t, src3=x1.t if x1 else None, wgt2=s2, wgt2_tiled=s2t, bias2=sk.conv.bias)
        point2 = POINT_1X1 and sp == (1, 1) and c2.weight.dim() == 4 and not halo2
        w2, w2t = (self.wc.get(self.wc.center(c2.weight), 0), None) if point2 else self._wts(c2.weight, 0, halo2)
        if point2:
            kw.update(ks=1, pad=0)
        if mat2 and t2 is None:
            t2 = ops.gn_apply_fwd(h, None, a2, b2)
        if drop:
            ops.dropout_apply(t2, drop, seed, salt, out=t2)
        gg2 = (torch.empty_like(h) if keep_g and t2 is None and halo2 and not point2 and Cout % HALO_BK == 0
               else None)
        out, ost = ops.conv(t2 if t2 is not None else h, Cout, w2,
                            pro=None if (t2 is not None or pf2 is not None) else (a2, b2, True), pro_fold=pf2,
                            bias=c2.bias, want_stats="free", wgt_tiled=w2t, gout=gg2, **kw)
        o = Act(out, ost)
        if ctx.tape is None:
            return o

        def bwd():
            dy = o.grad

            def wg2():
                if t2 is not None or gg2 is not None:   # materialised operand / the forward's G side output
                    ops.wgrad(t2 if t2 is not None else gg2, dy, c2.weight.grad, db=c2.bias.grad)
                else:
                    ops.wgrad(h, dy, c2.weight.grad, pro=(a2, b2, True), db=c2.bias.grad)
                if not isinstance(sk, Identity):
                    ops.wgrad(x0.t, dy, sk.conv.weight.grad, src1=x1.t if x1 else None, ks=1, pad=0,
                              db=sk.conv.bias.grad)
            self._wg(wg2, N * HW)
            # the skip data gradient (non-identity) is fused into the GroupNorm-1 backward below
            extra = dy if isinstance(sk, Identity) else None
            if drop:   # d(conv2 input) -> through the regenerated mask and SiLU'(GN) -> GN backward statistics
                dd, _ = self.dgrad3x3(c2.weight, dy, Cout, sp)
                dz2 = ops.dropout_apply(dd, drop, seed, salt, ep=(h, a2, b2), out=dd)
                s2 = ops.channel_stats(dz2, y=(h, None, Cout))
            else:
                dz2, s2 = self.dgrad3x3(c2.weight, dy, Cout, sp, ep=(h, None, a2, b2), want_stats=True)
            if slot is not None:
                demb, ds_ = ctx.demb_all[:, slot[0]:slot[0] + slot[1]], self.gl.total
            elif eo is not None:
                demb = torch.empty_like(eo)
                ds_ = demb.shape[1]
            else:
                demb, ds_ = None, 0
            if ss:
                P2, Q2, R2 = ops.gn_bwd_prep(s2, N, HW, Cout, g2.num_groups, mr2, g2.weight, g2.bias, g2.weight.grad,
                                             g2.bias.grad, emb=eo, emb_stride=es, emb_mode=1, demb=demb,
                                             demb_stride=ds_)
            elif add:
                P2, Q2, R2 = ops.gn_bwd_prep(s2, N, HW, Cout, g2.num_groups, mr2, g2.weight, g2.bias, g2.weight.grad,
                                             g2.bias.grad, emb_mode=2, demb=demb, demb_stride=ds_, fwd=hst)
            else:
                P2, Q2, R2 = ops.gn_bwd_prep(s2, N, HW, Cout, g2.num_groups, mr2, g2.weight, g2.bias, g2.weight.grad,
                                             g2.bias.grad)
            dh = torch.empty_like(h)
            ops.gn_bwd_apply(dz2, h, None, P2, Q2, R2, None, dh, 0)
            del dz2
            if t1 is not None or gg1 is not None:
                self._wg(lambda: ops.wgrad(t1 if t1 is not None else gg1, dh, c1.weight.grad, db=c1.bias.grad),
                         N * HW)
            else:
                self._wg(lambda: ops.wgrad(x0.t, dh, c1.weight.grad, src1=x1.t if x1 else None, pro=(a1, b1, True),
                                           db=c1.bias.grad), N * HW)
            dz1, s1 = self.dgrad3x3(c1.weight, dh, Cin, sp, ep=(x0.t, x1.t if x1 else None, a1, b1),
                                    want_stats=True)
            P1, Q1, R1 = ops.gn_bwd_prep(s1, N, HW, Cin, g1.num_groups, mr1, g1.weight, g1.bias, g1.weight.grad,
                                         g1.bias.grad)
            d0, acc0 = _gdest(x0)
            d1, acc1 = _gdest(x1)
            if isinstance(sk, Identity):
                ops.gn_bwd_apply(dz1, x0.t, x1.t if x1 else None, P1, Q1, R1, extra, d0, acc0, d1, acc1)
            else:
                ops.conv1x1_gn_apply(dy, self.wc.get(sk.conv.weight, 1), dz1, x0.t, x1.t if x1 else None,
                                     P1, Q1, R1, d0, acc0, d1, acc1)
            if (ss or add) and slot is None:
                ops.linear_bwd(ctx.emb, el.weight, demb, el.weight.grad, el.bias.grad, dx=ctx.demb, dx_acc=True,
                               in_silu=m.emb_activation_before_proj)
        ctx.tape.append(bwd)
        return o

    def _res_block_small(self, m: ResBlockND, x0: Act, x1: Optional[Act], eo, es, ss: bool, add: bool):
        """Forward-only ResBlockND on a small level in TWO launches (fmd_conv_small, csrc/conv_small.hip): conv1 folds
        GroupNorm-1 from the inputs' statistics slabs, applies it + SiLU while staging, adds the conv bias and the
        time-embedding (add form); conv2 folds GroupNorm-2 (+ the scale-shift embedding) from conv1's statistics and
        adds its bias and the identity residual or the 1x1 skip conv over the block input.  Both emit the statistics
        of their outputs for the next GroupNorm.  Reference: residual.py:84-120.  Returns None (caller takes the
        general path) when either conv does not qualify."""
        N, H, W, C0 = x0.t.shape
        C1 = x1.C if x1 is not None else 0
        Cout = m.out_channels
        c1, c2 = m.conv1.conv, m.conv2.conv
        if c1.weight.dim() != 4 or c2.weight.dim() != 4:
            return None
        _check_conv(c1, 3, 1, 1)
        _check_conv(c2, 3, 1, 1)
        point = POINT_1X1 and (H, W) == (1, 1)
        mode = "point" if point else "s1"
        g1, g2 = m.norm1, m.norm2
        sk = m.skip_connection
        ident = isinstance(sk, Identity)
        if ident and x1 is not None:
            raise ValueError("identity skip with concatenated input")
        if not ident:
            _check_conv(sk.conv, 1, 1, 0)
        rows = 64 if (H * W) % 64 == 0 else H * W   # the slab rows fmd_channel_stats / fmd_conv_small write

        def probe(a):
            return a.stats if a.stats is not None else ops.Stats(None, rows)
        gn1 = dict(st0=probe(x0), st1=probe(x1) if x1 is not None else None, groups=g1.num_groups, eps=g1.eps)
        gn2 = dict(st0=ops.Stats(None, rows), groups=g2.num_groups, eps=g2.eps, emb=eo if ss else None,
                   emb_stride=es if ss else 0)
        if not (ops.conv_small_ok((N, H, W, C0), Cout, C1=C1, mode=mode, gn=gn1) and
                ops.conv_small_ok((N, H, W, Cout), Cout, mode=mode, gn=gn2, skip=None if ident else (C0, C1))):
            return None
        gn1.update(st0=_stats(x0), st1=_stats(x1), gamma=g1.weight, beta=g1.bias)
        w1 = self.wc.get(self.wc.center(c1.weight), 0) if point else self.wc.get(c1.weight, 0)
        h, hst = ops.conv_small(x0.t, Cout, w1, src1=x1.t if x1 is not None else None, mode=mode, gn=gn1,
                                bias=c1.bias, bias_nc=eo if add else None)
        gn2.update(st0=hst, gamma=g2.weight, beta=g2.bias)
        w2 = self.wc.get(self.wc.center(c2.weight), 0) if point else self.wc.get(c2.weight, 0)
        kw = {}
        if ident:
            kw["resid"] = x0.t
        else:
            kw.update(src2=x0.t, src3=x1.t if x1 is not None else None, skip_wgt=self.wc.get(sk.conv.weight, 0),
                      bias2=sk.conv.bias)
        out, ost = ops.conv_small(h, Cout, w2, mode=mode, gn=gn2, bias=c2.bias, **kw)
        return Act(out, ost)

    def _dropout_seed(self, m, ctx: Ctx, dev):
        """(device seed counter, per-block salt) for ResBlockND dropout; the counter advances once per forward
        (a device-side add, so every replay of a captured step draws fresh masks) and the backward reuses the
        forward's value to regenerate its masks."""
        st = getattr(self, "_drop_state", None)
        if st is None:
            # the counter starts from torch's (host) generator, so training.seed / set_seed selects the mask
            # sequence, and is offset by the data-parallel rank so ranks draw different masks for the same local
            # sample position (the reference draws every mask from torch's RNG). Not saved in checkpoints: a
            # resumed run restarts the sequence from the seeded generator.
            import torch.distributed as dist
            rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
            base = int(torch.randint(0, 1 << 30, (1,)).item())
            start = (base + rank * 1000003) % (1 << 31)
            st = self._drop_state = (torch.full((1,), start, device=dev, dtype=torch.int32), {})
        seed, salts = st
        if not ctx.drop_seeded:
            ops.counter_add(seed, 1)
            ctx.drop_seeded = True
        return seed, salts.setdefault(id(m), len(salts) + 1)

    def attention(self, m, x: Act, ctx: Ctx):
        """SpatialSelfAttention (raw reshape) or DiffusersAttentionND (self-attention only)."""
        N, Cc, sp = x.t.shape[0], x.t.shape[-1], tuple(x.t.shape[1:-1])
        T = math.prod(sp)
        H, W = T // sp[-1], sp[-1]        # 1x1 convs only: a 3-D volume runs as a (D*H, W) plane
        x4 = x.t.view(N, H, W, Cc)
        if isinstance(m, SpatialSelfAttention):
            norm, heads, dh, inner, raw = m.norm, m.heads, m.dim_head, m.inner_dim, 1
            lin = m.attention.eps if m.use_linear else None      # LinearQKVAttention (attention.py:53-70)
            wq = m.qkv.weight
            bq = m.qkv.bias
            wo, bo = m.proj_out.weight, m.proj_out.bias
            qparts = None
        elif isinstance(m, DiffusersAttentionND):
            if m.context_dim is not None:
                return self.cross_attention(m, x, ctx)
            norm, heads, dh, inner, raw = m.group_norm, m.heads, m.head_dim, m.channels, 0
            qparts = (m.to_q, m.to_k, m.to_v)
            wq = self.wc.fused([l.weight for l in qparts], "w")
            bq = self.wc.fused([l.bias for l in qparts], "b")
            wo, bo = m.to_out[0].weight, m.to_out[0].bias
            lin = None
        else:
            raise NotImplementedError(type(m).__name__)
        if ctx.tape is None and len(sp) == 2 and SMALL_ATTN:
            # forward only, small level: the GroupNorm folded into the qkv projection and the output projection with
            # its residual and statistics, one fmd_conv_small launch each (no gn_prep, split-K combine or
            # channel_stats launches)
            rows = 64 if T % 64 == 0 else T
            gnq = dict(st0=x.stats if x.stats is not None else ops.Stats(None, rows), groups=norm.num_groups,
                       eps=norm.eps, silu=False)
            if (ops.conv_small_ok((N, H, W, Cc), 3 * inner, mode="point", gn=gnq) and
                    ops.conv_small_ok((N, H, W, inner), Cc, mode="point")):
                gnq.update(st0=_stats(x), gamma=norm.weight, beta=norm.bias)
                qkv, _ = ops.conv_small(x4, 3 * inner, self.wc.get(wq, 0), mode="point", gn=gnq, bias=bq,
                                        want_stats=False)
                if lin is not None:
                    o, _ = ops.linear_attention_fwd(qkv, T, heads, dh, raw, lin)
                else:
                    o, _ = ops.attention_fwd(qkv, T, heads, dh, raw)
                out, st = ops.conv_small(o.view(N, H, W, inner), Cc, self.wc.get(wo, 0), mode="point", bias=bo,
                                         resid=x4)
                return Act(out.view(x.t.shape), st)
        a, b, mr = ops.gn_prep(_stats(x), None, N, T, Cc, 0, norm.num_groups, norm.eps, norm.weight, norm.bias)
        qkv, _ = ops.conv(x4, 3 * inner, self.wc.get(wq, 0), ks=1, pad=0, pro=(a, b, False), bias=bq)
        if lin is not None:
            o, lse = ops.linear_attention_fwd(qkv, T, heads, dh, raw, lin)
        else:
            o, lse = ops.attention_fwd(qkv, T, heads, dh, raw)
        o4 = o.view(N, H, W, inner)
        out, st = ops.conv(o4, Cc, self.wc.get(wo, 0), ks=1, pad=0, bias=bo, resid=x4, want_stats="free")
        y = Act(out.view(x.t.shape), st)
        if ctx.tape is None:
            return y

        def bwd():
            dy = y.grad.view(N, H, W, Cc)
            self._wg(lambda: ops.wgrad(o4, dy, wo.grad, ks=1, pad=0, db=bo.grad))
            do, _ = ops.conv(dy, inner, self.wc.get(wo, 1), ks=1, pad=0, transposed=True, out_hw_=(H, W))
            if lin is not None:
                dqkv = ops.linear_attention_bwd(qkv, do, lse, T, heads, dh, raw, lin)
            else:
                dqkv = ops.attention_bwd(qkv, o, do, lse, T, heads, dh, raw)
            def wgq():
                if qparts is None:
                    ops.wgrad(x4, dqkv, wq.grad, ks=1, pad=0, pro=(a, b, False), db=bq.grad)
                else:
                    for i, l in enumerate(qparts):
                        ops.wgrad(x4, dqkv, l.weight.grad, ks=1, pad=0, pro=(a, b, False), db=l.bias.grad,
                                  dy_offset=i * inner)
            self._wg(wgq)
            dz, s12 = ops.conv(dqkv, Cc, self.wc.get(wq, 1), ks=1, pad=0, transposed=True, out_hw_=(H, W),
                               ep=(x4, None, None, None), want_stats=True)
            P, Q, R = ops.gn_bwd_prep(s12, N, T, Cc, norm.num_groups, mr, norm.weight, norm.bias, norm.weight.grad,
                                      norm.bias.grad)
            g, acc = _gdest(x)
            ops.gn_bwd_apply(dz, x4, None, P, Q, R, dy, g, acc)
        ctx.tape.append(bwd)
        return y

    @staticmethod
    def _context_flat(context: torch.Tensor, cdim: int):
        """(fp32 contiguous context, token_major) with SpatialCrossAttention's shape rules
        (attention.py:163-177): (b, c_ctx, tokens) / (b, tokens, c_ctx) / (b, c_ctx, *spatial)."""
        if context.dim() == 3:
            if context.shape[1] == cdim:
                return context.float().contiguous(), False
            if context.shape[-1] == cdim:
                return context.float().contiguous(), True
            raise ValueError(f"Context channels mismatch: expected {cdim}, got {context.shape}.")
        if context.shape[1] != cdim:
            raise ValueError(f"Context channels mismatch: expected {cdim}, got {context.shape}.")
        return context.float().reshape(context.shape[0], cdim, -1).contiguous(), False

    def cross_attention(self, m, x: Act, ctx: Ctx):
        """SpatialCrossAttention (attention.py:157-189) or DiffusersAttentionND with a context (:236-274):
        GN(x) folded into the q projection's gather; context_norm of the context into the k|v projection
        operand (fmd_context_norm_fwd); raw (Spatial) or view/transpose (Diffusers) head split; softmax or
        linear attention over the context tokens; output projection + residual in one epilogue.  No gradient
        flows into the context."""
        if ctx.cca is None:
            raise ValueError(f"{type(m).__name__} cross-attention requires a non-empty context tensor.")
        if isinstance(m, SpatialCrossAttention):
            norm, cnm, heads, dh, inner, raw = m.norm, m.context_norm, m.heads, m.dim_head, m.inner_dim, 1
            lin = m.attention.eps if m.use_linear else None
            wq, bq = m.q_proj.weight, m.q_proj.bias
            kvp = [(m.kv_proj.weight, m.kv_proj.bias)]          # one projection: k | v
            wo, bo = m.proj_out.weight, m.proj_out.bias
        else:
            norm, cnm, heads, dh, inner, raw = m.group_norm, m.context_norm, m.heads, m.head_dim, m.channels, 0
            lin = None
            wq, bq = m.to_q.weight, m.to_q.bias
            kvp = [(m.to_k.weight, m.to_k.bias), (m.to_v.weight, m.to_v.bias)]
            wo, bo = m.to_out[0].weight, m.to_out[0].bias
        if any(w.shape[0] % 8 for w, _ in kvp) or inner % 8:
            raise NotImplementedError(f"{type(m).__name__}: the fused k|v projection needs projection widths that "
                                      f"are multiples of 8 (got {[w.shape[0] for w, _ in kvp]})")
        if len(kvp) == 1:
            wkv, bkv = kvp[0]
        else:   # to_k / to_v as one fused projection
            wkv, bkv = self.wc.fused([w for w, _ in kvp], "w"), self.wc.fused([b for _, b in kvp], "b")
        cf, tok = self._context_flat(ctx.cca, m.context_dim)
        Tk = cf.shape[1] if tok else cf.shape[2]
        N, Cc, sp = x.t.shape[0], x.t.shape[-1], tuple(x.t.shape[1:-1])
        T = math.prod(sp)
        H, W = T // sp[-1], sp[-1]
        x4 = x.t.view(N, H, W, Cc)
        Cp = max(8, -(-m.context_dim // 8) * 8)
        a, b, mr = ops.gn_prep(_stats(x), None, N, T, Cc, 0, norm.num_groups, norm.eps, norm.weight, norm.bias)
        q, _ = ops.conv(x4, inner, self.wc.get(wq, 0), ks=1, pad=0, pro=(a, b, False), bias=bq)
        cn, cmr = ops.context_norm_fwd(cf, tok, cnm.num_groups, cnm.eps, cnm.weight, cnm.bias, Cp)
        kv, _ = ops.conv(cn, 2 * inner, self.wc.get(wkv, 0, None, Cp), ks=1, pad=0, bias=bkv)
        o, saved = ops.cross_attention_fwd(q, kv, T, Tk, heads, dh, lin, raw)
        o4 = o.view(N, H, W, inner)
        out, st = ops.conv(o4, Cc, self.wc.get(wo, 0), ks=1, pad=0, bias=bo, resid=x4, want_stats="free")
        y = Act(out.view(x.t.shape), st)
        if ctx.tape is None:
            return y

        def bwd():
            dy = y.grad.view(N, H, W, Cc)
            self._wg(lambda: ops.wgrad(o4, dy, wo.grad, ks=1, pad=0, db=bo.grad))
            do, _ = ops.conv(dy, inner, self.wc.get(wo, 1), ks=1, pad=0, transposed=True, out_hw_=(H, W))
            dq, dkv = ops.cross_attention_bwd(q, kv, o, do, saved, T, Tk, heads, dh, lin, raw)

            def wg():
                ops.wgrad(x4, dq, wq.grad, ks=1, pad=0, pro=(a, b, False), db=bq.grad)
                off = 0
                for w_, b_ in kvp:   # context channels padded to Cp: through a temporary unless they match
                    Ki = w_.shape[0]
                    tgt = w_.grad if w_.shape[1] == Cp else torch.zeros((Ki, Cp, *w_.shape[2:]), device=w_.device,
                                                                       dtype=F32)
                    ops.wgrad(cn, dkv, tgt, ks=1, pad=0, db=b_.grad, dy_offset=off)
                    if tgt is not w_.grad:
                        w_.grad.add_(tgt[:, :m.context_dim])
                    off += Ki
            self._wg(wg)
            dcn, _ = ops.conv(dkv, Cp, self.wc.get(wkv, 1, None, Cp), ks=1, pad=0, transposed=True, out_hw_=(Tk, 1))
            ops.context_norm_bwd(cf, tok, cnm.num_groups, cmr, dcn, cnm.weight.grad, cnm.bias.grad)
            dz, s12 = ops.conv(dq, Cc, self.wc.get(wq, 1), ks=1, pad=0, transposed=True, out_hw_=(H, W),
                               ep=(x4, None, None, None), want_stats=True)
            P, Q, R = ops.gn_bwd_prep(s12, N, T, Cc, norm.num_groups, mr, norm.weight, norm.bias, norm.weight.grad,
                                      norm.bias.grad)
            g, acc = _gdest(x)
            ops.gn_bwd_apply(dz, x4, None, P, Q, R, dy, g, acc)
        ctx.tape.append(bwd)
        return y

    def head(self, norm, conv: Conv, h: Act, ctx: Ctx, bf16_out: bool = False):
        """GroupNorm -> SiLU -> 3x3 conv to an fp32 NHWC output with CPAD channels (``bf16_out``: a bf16
        intermediate with K channels, the input of UnPoolND when pool_factor > 1)."""
        _check_conv(conv, 3, 1, 1)
        N, Cc, sp = h.t.shape[0], h.t.shape[-1], tuple(h.t.shape[1:-1])
        HW = math.prod(sp)
        K = conv.out_channels
        Kp = max(CPAD, -(-K // 8) * 8)
        a, b, mr = ops.gn_prep(_stats(h), None, N, HW, Cc, 0, norm.num_groups, norm.eps, norm.weight, norm.bias)
        if (not bf16_out and Kp == CPAD and len(sp) in (2, 3)
                and ops.head_eligible(*sp[-2:], Cc, K, sp[0] if len(sp) == 3 else 0)):
            # VALU head kernels (csrc/head.hip): the GN/SiLU transform once per element, no MFMA padding
            out = ops.head_fwd(h.t, (a, b), conv.weight, conv.bias, K, Kp)
            if ctx.tape is not None:
                def bwd(dpred):
                    self._wg(lambda: ops.head_wgrad(dpred, K, h.t, (a, b), conv.weight.grad,
                                                    conv.bias.grad if conv.bias is not None else None))
                    dz, s12 = ops.head_dgrad(dpred, conv.weight, K, h.t, (a, b))
                    P, Q, R = ops.gn_bwd_prep(s12, N, HW, Cc, norm.num_groups, mr, norm.weight, norm.bias,
                                              norm.weight.grad, norm.bias.grad)
                    g, acc = _gdest(h)
                    ops.gn_bwd_apply(dz, h.t, None, P, Q, R, None, g, acc)
                self._head_bwd = bwd
            return out
        w = self.wc.get(conv.weight, 0, Kp, None)
        bias = self.wc.padded(conv.bias, Kp)
        out, _ = ops.conv(h.t, Kp, w, pro=(a, b, True), bias=bias, out_f32=not bf16_out)
        if ctx.tape is not None:
            def bwd(dpred):
                def wgh():
                    tmpw = torch.zeros((Kp, Cc, *conv.weight.shape[2:]), device=out.device, dtype=F32)
                    tmpb = torch.zeros((Kp,), device=out.device, dtype=F32)
                    ops.wgrad(h.t, dpred, tmpw, pro=(a, b, True), db=tmpb, accumulate=False)
                    conv.weight.grad.add_(tmpw[:K])
                    conv.bias.grad.add_(tmpb[:K])
                self._wg(wgh)
                dz, s12 = self.dgrad3x3(conv.weight, dpred, Cc, sp, Kpad=Kp, ep=(h.t, None, a, b),
                                        want_stats=True)
                P, Q, R = ops.gn_bwd_prep(s12, N, HW, Cc, norm.num_groups, mr, norm.weight, norm.bias,
                                          norm.weight.grad, norm.bias.grad)
                g, acc = _gdest(h)
                ops.gn_bwd_apply(dz, h.t, None, P, Q, R, None, g, acc)
            self._head_bwd = bwd
        return out

    def set_time_table(self, t_steps: Optional[torch.Tensor], N: int = 0, index: Optional[torch.Tensor] = None):
        """Precompute the time embedding (+ grouped ResBlock projections) of every step of a fixed sampling
        schedule ``t_steps`` [S] (each for a batch of N); forward(save=False) then copies row ``index[0]``
        (device step counter) instead of running the time MLP -- one launch per step instead of four.
        ``None`` clears the table."""
        self._tt = None
        if t_steps is None:
            return
        S = t_steps.shape[0]
        # every sample of a step shares its t: the MLP runs once per step (its kernels are row-independent, so
        # each row is bit-identical to a per-sample evaluation) and row i of the table holds N copies
        # (i*N + n = step i, sample n) -- 8x fewer launches than one row per (step, sample)
        t_u = t_steps.float().contiguous()
        embs, eos = [], []
        for r0 in range(0, S, 32):                        # the linear kernels take <= 32 rows per launch
            ctx = self.time_mlp(t_u[r0:r0 + 32].contiguous(), False, min(32, S - r0))
            embs.append(ctx.emb)
            eos.append(ctx.eo_all)

        def per_sample(x):
            return x[:, None, :].expand(S, N, x.shape[1]).reshape(S, -1)

        emb = per_sample(torch.cat(embs))
        eo = per_sample(torch.cat(eos)) if eos[0] is not None else None
        self._tt = dict(N=N, index=index, emb=emb, eo=eo, emb_cols=embs[0].shape[1],
                        eo_cols=eos[0].shape[1] if eo is not None else 0)

    def time_mlp(self, t, ctx_save, N, t_scale=1.0, t_trunc=False):
        m = self.m
        tt = getattr(self, "_tt", None)
        if tt is not None and not ctx_save and N == tt["N"] and t_scale == 1.0 and not t_trunc:
            emb = torch.empty((N, tt["emb_cols"]), device=tt["emb"].device, dtype=tt["emb"].dtype)
            ops.gather_row(tt["emb"], tt["index"], emb)
            ctx = Ctx(emb, False, N)
            if tt["eo"] is not None:
                ctx.eo_all = torch.empty((N, tt["eo_cols"]), device=emb.device, dtype=tt["eo"].dtype)
                ops.gather_row(tt["eo"], tt["index"], ctx.eo_all)
            return ctx
        if self.kind == "efficient":
            l1, l2 = m.time_embed[0], m.time_embed[2]
            feats = ops.timestep_embedding(t, m.model_channels, False, 0, t_scale=t_scale, t_trunc=t_trunc)
        else:
            l1, l2 = m.time_embedding.linear_1, m.time_embedding.linear_2
            feats = ops.timestep_embedding(t, m.time_proj_dim, m.flip_sin_to_cos, m.freq_shift, t_scale=t_scale,
                                           t_trunc=t_trunc)
        h1 = ops.linear(feats, l1.weight, l1.bias)
        emb = ops.linear(h1, l2.weight, l2.bias, in_silu=True)
        ctx = Ctx(emb, ctx_save, N)
        if self.gl is not None:
            ctx.eo_all = self.gl.forward(emb)
        if ctx.tape is not None:
            def bwd():
                dh1 = torch.empty_like(h1)
                ops.linear_bwd(h1, l2.weight, ctx.demb, l2.weight.grad, l2.bias.grad, dx=dh1, in_silu=True)
                ops.linear_bwd(feats, l1.weight, dh1, l1.weight.grad, l1.bias.grad)
            ctx.tape.append(bwd)
            if self.gl is not None:
                ctx.demb_all = torch.zeros_like(ctx.eo_all)

                def gbwd():   # runs after every ResBlock wrote its demb slice, before the time MLP backward
                    self.gl.backward(emb, ctx.demb_all, dx=ctx.demb, dx_acc=True)
                ctx.tape.append(gbwd)
        return ctx

    # ---------------------------------------------------------------- model
    def forward(self, xin: torch.Tensor, t: torch.Tensor, save: bool, t_scale: float = 1.0, t_trunc: bool = False,
                context_ca: Optional[torch.Tensor] = None):
        """xin: NHWC bf16 [N,H,W,CPAD] (channels past the model's in_channels are 0), t: [N] timesteps
        (``t*t_scale``, truncated to integers if ``t_trunc``).

        Returns (out fp32 NHWC [N,H,W,Kpad], ctx) -- ctx carries the backward tape when ``save``."""
        m = self.m
        N = xin.shape[0]
        if xin.dim() == 3:   # 1-D signal [N][L][C] -> an (L, 1) image
            xin = xin.unsqueeze(2)
        if getattr(m, "center_input_sample", False):   # x = 2 * cat(x, context) - 1 (unet_diffusers_nd.py:156-157)
            xin = ops.affine_channels(xin, m.conv_in.in_channels, 2.0, -1.0)
        ctx = self.time_mlp(t, save, N, t_scale, t_trunc)
        ctx.cca = context_ca
        x = Act(xin, need_grad=False)
        if self.kind == "efficient":
            hs = []
            h = x
            if m.pool_factor > 1:   # before the first encoder mark: its gradient lands in the last segment
                h = self.pool_layer(m.pool.down.conv, x, ctx)
            for blk in m.input_blocks:
                if ctx.tape is not None:
                    ctx.marks.append(len(ctx.tape))
                for layer in blk:
                    h = self._apply(layer, h, ctx)
                hs.append(h)
            if ctx.tape is not None:
                ctx.marks.append(len(ctx.tape))
            for layer in m.middle_block:
                h = self._apply(layer, h, ctx)
            if ctx.tape is not None:
                ctx.mark = len(ctx.tape)
            for blk in m.output_blocks:
                skip = hs.pop()
                layers = list(blk)
                h = self.res_block(layers[0], [h, skip], ctx)
                for layer in layers[1:]:
                    h = self._apply(layer, h, ctx)
            if m.pool_factor > 1:
                hb = self.head(m.out[0], m.out[2].conv, h, ctx, bf16_out=True)
                out = self.unpool_layer(m.unpool.up.convT, hb, ctx)
            else:
                out = self.head(m.out[0], m.out[2].conv, h, ctx)
        else:
            if ctx.tape is not None:
                ctx.marks.append(len(ctx.tape))
            h = self.conv_layer(m.conv_in, x, ctx)
            res = [h]
            for blk in m.down_blocks:
                if ctx.tape is not None:
                    ctx.marks.append(len(ctx.tape))
                for j, r in enumerate(blk.resnets):
                    h = self.res_block(r, [h], ctx)
                    if blk.attentions is not None:
                        h = self.attention(blk.attentions[j], h, ctx)
                    res.append(h)
                if blk.downsamplers is not None:
                    h = self._apply(blk.downsamplers[0], h, ctx)
                    res.append(h)
            if ctx.tape is not None:
                ctx.marks.append(len(ctx.tape))
            if m.mid_block is not None:
                h = self.res_block(m.mid_block.resnets[0], [h], ctx)
                if m.mid_block.attentions is not None:
                    h = self.attention(m.mid_block.attentions[0], h, ctx)
                h = self.res_block(m.mid_block.resnets[1], [h], ctx)
            if ctx.tape is not None:
                ctx.mark = len(ctx.tape)
            for blk in m.up_blocks:
                for j, r in enumerate(blk.resnets):
                    h = self.res_block(r, [h, res.pop()], ctx)
                    if blk.attentions is not None:
                        h = self.attention(blk.attentions[j], h, ctx)
                if blk.upsamplers is not None:
                    h = self._apply(blk.upsamplers[0], h, ctx)
            out = self.head(m.conv_norm_out, m.conv_out, h, ctx)
        return out, ctx

    def _apply(self, layer, h: Act, ctx: Ctx) -> Act:
        if isinstance(layer, ResBlockND):
            return self.res_block(layer, [h], ctx)
        if isinstance(layer, ConvND):
            return self.conv_layer(layer.conv, h, ctx)
        if isinstance(layer, DownsampleND):
            if not layer.use_conv:
                return self.resample_layer(h, ctx, up=False)
            return self.conv_layer(layer.op.conv, h, ctx, stride=2)
        if isinstance(layer, UpsampleND):
            if not layer.use_conv:
                return self.resample_layer(h, ctx, up=True)
            if self.dims1:   # nearest-x2 along the signal only, then the 3-tap conv
                return self.conv_layer(layer.conv.conv, self.resample_layer(h, ctx, up=True), ctx)
            return self.conv_layer(layer.conv.conv, h, ctx, upsample=True)
        if isinstance(layer, (SpatialSelfAttention, DiffusersAttentionND)):
            return self.attention(layer, h, ctx)
        if isinstance(layer, SpatialCrossAttention):
            return self.cross_attention(layer, h, ctx)
        raise NotImplementedError(type(layer).__name__)

    # Backward segments, in backward order: 0 = output head + decoder, 1 = middle block, then the encoder
    # stages deepest first (EfficientUNetND input_blocks / UNetDiffusersND conv_in + down_blocks), and last the
    # grouped ResBlock emb projections + time MLP.  The parameters of segment k (backward_param_groups()[k])
    # have their final gradients once segments 0..k ran, so a data-parallel step can all-reduce them while
    # the later segments run.
    def _stage_modules(self) -> List[List[torch.nn.Module]]:
        m = self.m
        if self.kind == "efficient":
            return [[blk] for blk in m.input_blocks]
        return [[m.conv_in]] + [[blk] for blk in m.down_blocks]

    def _late_ids(self) -> set:
        late = set()
        if self.gl is not None:
            for sub in self.m.modules():
                if isinstance(sub, ResBlockND) and id(sub) in self.gl_slot and sub.emb_layers is not None:
                    late.update(id(p) for p in sub.emb_layers.parameters())
        return late

    def backward_param_groups(self) -> List[List[torch.nn.Parameter]]:
        """Parameters per backward segment (see above); the last group holds every parameter not in an
        earlier one (time MLP, grouped emb projections, anything unused)."""
        m = self.m
        if self.kind == "efficient":
            head = [[m.output_blocks, m.out, m.unpool], [m.middle_block]]
        else:
            head = [[m.up_blocks, m.conv_norm_out, m.conv_out], [m.mid_block] if m.mid_block is not None else []]
        mods = head + list(reversed(self._stage_modules()))
        late = self._late_ids()
        seen, groups = set(), []
        for ms in mods:
            g = []
            for mod in ms:
                for p in mod.parameters():
                    if id(p) not in late and id(p) not in seen:
                        seen.add(id(p))
                        g.append(p)
            groups.append(g)
        groups.append([p for p in m.parameters() if id(p) not in seen])
        return groups

    @staticmethod
    def seg_ranges(ctx: Ctx) -> List[Tuple[int, int]]:
        """Tape ranges [lo, hi) of the backward segments (segment 0 additionally runs the output head)."""
        mk = ctx.marks
        out = [(ctx.mark, len(ctx.tape)), (mk[-1], ctx.mark)]
        for i in range(len(mk) - 1, 0, -1):
            out.append((mk[i - 1], mk[i]))
        out.append((0, mk[0]))
        return out

    def backward(self, ctx: Ctx, dpred: torch.Tensor, part: int = 0, segs: Optional[Tuple[int, int]] = None):
        """Run the written-out backward. ``dpred``: bf16 NHWC [N,H,W,Kpad] gradient of the output.

        ``segs`` = (first, last): run backward segments first..last (inclusive, see backward_param_groups);
        their parameter gradients (GroupNorm gamma/beta folds included) are final on return, and the tape is
        released after the last segment.  ``part`` (older interface): 1 = segment 0 (head + decoder), 2 = the
        rest, 0 = everything."""
        nseg = len(ctx.marks) + 2
        if segs is None:
            segs = {0: (0, nseg - 1), 1: (0, 0), 2: (1, nseg - 1)}[part]
        lo, hi = segs
        ranges = self.seg_ranges(ctx)
        ops.gb_defer()   # GroupNorm gamma/beta folds: batched launches
        try:
            for k in range(lo, hi + 1):
                if k == 0:
                    self._head_bwd(dpred)
                a, b = ranges[k]
                for fn in reversed(ctx.tape[a:b]):
                    fn()
        finally:
            ops.gb_flush()
        self._join()   # every weight gradient of these segments has landed before anyone reads .grad
        if hi == nseg - 1:
            ctx.tape = None
            self._head_bwd = None

    def decoder_params(self) -> List[torch.nn.Parameter]:
        """Parameters whose gradients are final after ``backward(part=1)``: the decoder blocks and the
        output head, minus the ResBlock emb projections (their gradients come from the grouped linear
        backward, which runs last)."""
        return self.backward_param_groups()[0]

    # ----------------------------------------------------------- utilities
    def stage_input(self, x: torch.Tensor, context: Optional[torch.Tensor]):
        """NC(D)HW fp32 (x, optional concat context) -> N(D)HWC bf16 with CPAD-padded channels."""
        Cin = x.shape[1] + (context.shape[1] if context is not None else 0)
        Cp = max(CPAD, -(-Cin // 8) * 8)
        return ops.noise_prepare(None, x.float().contiguous(), None, None,
                                 context.float().contiguous() if context is not None else None, Cp)

    def params(self):
        return [p for p in self.m.parameters()]

    def ensure_grads(self):
        for p in self.m.parameters():
            if p.grad is None:
                p.grad = torch.zeros_like(p)


def get_engine(model) -> UNetEngine:
    eng = getattr(model, "_fmd_engine", None)
    if eng is None:
        eng = UNetEngine(model)
        object.__setattr__(model, "_fmd_engine", eng)
    return eng


class _UNetFunction(torch.autograd.Function):
    @staticmethod
    def forward(fctx, x, t, context, context_ca, engine, *params):
        xin = engine.stage_input(x, context)
        out, ctx = engine.forward(xin, t, save=True, context_ca=context_ca)
        fctx.engine = engine
        fctx.ctx = ctx
        fctx.kpad = out.shape[-1]
        y = ops.nhwc_to_nchw(out, engine.m_out_channels)
        return y.squeeze(-1) if engine.dims1 else y

    @staticmethod
    def backward(fctx, gout):
        eng = fctx.engine
        eng.ensure_grads()
        dpred = ops.nchw_to_nhwc(gout.contiguous(), fctx.kpad)
        if eng.dims1:
            dpred = dpred.unsqueeze(2)
        eng.backward(fctx.ctx, dpred)
        fctx.ctx = None
        return (None, None, None, None, None) + tuple(None for _ in eng.params())


def unet_apply(model, x: torch.Tensor, t: torch.Tensor, context: Optional[torch.Tensor],
               context_ca: Optional[torch.Tensor] = None):
    """Module-level entry: NCHW fp32 in -> NCHW fp32 out, differentiable w.r.t. the parameters."""
    ops._need_cuda(x, type(model).__name__)
    eng = get_engine(model)
    eng.m_out_channels = model.conv_out.out_channels if eng.kind == "diffusers" else int(model.out_channels)
    params = eng.params()
    if torch.is_grad_enabled() and any(p.requires_grad for p in params):
        return _UNetFunction.apply(x, t, context, context_ca, eng, *params)
    xin = eng.stage_input(x, context)
    out, _ = eng.forward(xin, t, save=False, context_ca=context_ca)
    y = ops.nhwc_to_nchw(out, eng.m_out_channels)
    return y.squeeze(-1) if eng.dims1 else y
