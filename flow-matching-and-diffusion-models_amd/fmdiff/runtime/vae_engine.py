"""Fused HIP execution of the AutoencoderKL encoder / decoder (config D: encode -> denoise -> decode).

Walks the reference module trees (``src/nn/modules/vae/encoder.py:139-158``,
``decoder.py:133-160``, ``src/models/vae/kl.py:116-128``) with the UNet engine's layer
implementations (``fmdiff.runtime.engine``): ResBlocks as two fused implicit-GEMM / halo convs
with GroupNorm+SiLU in the gather and skip + residual in the epilogue, stride-2 / nearest-x2
resampling inside the convs, the mid-block SpatialSelfAttention on the attention kernels, and
GroupNorm -> SiLU -> conv_out on the head kernels.  ``quant_conv`` (1x1, pointwise after conv_out) is
folded into conv_out's weights, so ``encode`` ends in one head launch; ``post_quant_conv`` runs as a
1x1 conv before the decoder (folding it into conv_in would be wrong at the zero-padded border).
Forward / inference only: VAE training is outside the hot path.
"""
from __future__ import annotations

import weakref

import torch

from . import ops
from .engine import CPAD, Act, Ctx, UNetEngine, WeightCache
from ..nn.params import Conv, Identity

F32 = torch.float32


class VAEEngine(UNetEngine):
    def __init__(self, module):
        self._model = weakref.ref(module)
        self.kind = "vae"
        self.wc = WeightCache()
        self._tt = None
        self.gl, self.gl_slot = None, {}
        self._fold = None
        self._fold_key = None
        self._head_bwd = None
        self.dims1 = False   # the VAE engine runs 2-D models only (spatial_dims checked on entry)

    def _ctx(self, part, N, dev):
        emb = None
        if part.emb_channels is not None:   # the reference feeds zeros (encoder.py:141-144)
            emb = torch.zeros((N, part.emb_channels), device=dev, dtype=F32)
        return Ctx(emb, False, N)

    def _stage(self, x):
        """NCHW fp32 -> NHWC bf16 with CPAD-padded channels."""
        ops._need_cuda(x, "AutoencoderKL")
        Cp = max(CPAD, -(-x.shape[1] // 8) * 8)
        return ops.noise_prepare(None, x.float().contiguous(), None, None, None, Cp)

    def _mid(self, part, h, ctx):
        h = self.res_block(part.mid_block1, [h], ctx)
        if not isinstance(part.mid_attn, Identity):
            h = self.attention(part.mid_attn, h, ctx)
        return self.res_block(part.mid_block2, [h], ctx)

    def _encoder_trunk(self, enc, x):
        if enc.spatial_dims != 2:
            raise NotImplementedError("fmdiff VAE engine: spatial_dims=2")
        ctx = self._ctx(enc, x.shape[0], x.device)
        h = self.conv_layer(enc.conv_in.conv, Act(self._stage(x), need_grad=False), ctx)
        for stage in enc.downs:
            for i, blk in enumerate(stage.blocks):
                h = self.res_block(blk, [h], ctx)
                if i < len(stage.attns):
                    h = self.attention(stage.attns[i], h, ctx)
            if hasattr(stage, "down"):
                h = self._apply(stage.down, h, ctx)
        return self._mid(enc, h, ctx), ctx

    def _decoder_trunk(self, dec, hin: Act, ctx):
        if dec.tanh_out:
            raise NotImplementedError("fmdiff VAE engine: tanh_out decoders")
        h = self.conv_layer(dec.conv_in.conv, hin, ctx)
        h = self._mid(dec, h, ctx)
        for stage in reversed(dec.ups):
            for i, blk in enumerate(stage.blocks):
                h = self.res_block(blk, [h], ctx)
                if i < len(stage.attns):
                    h = self.attention(stage.attns[i], h, ctx)
            if hasattr(stage, "up"):
                h = self._apply(stage.up, h, ctx)
        return self.head(dec.norm_out, dec.conv_out.conv, h, ctx)

    # ------------------------------------------------------------ entry points
    @torch.no_grad()
    def encoder_forward(self, x):
        """Encoder.forward: NCHW fp32 -> NCHW fp32 moments before quant_conv."""
        enc = self.m
        h, ctx = self._encoder_trunk(enc, x)
        out = self.head(enc.norm_out, enc.conv_out.conv, h, ctx)
        return ops.nhwc_to_nchw(out, enc.conv_out.conv.out_channels)

    def _folded_out(self, vae) -> Conv:
        """conv_out followed by the 1x1 quant_conv as one 3x3 conv: W = Wq . Wout, b = Wq bout + bq
        (exact: quant_conv is pointwise after conv_out)."""
        co, qc = vae.encoder.conv_out.conv, vae.quant_conv.conv
        key = tuple((t._version, t.data_ptr()) for t in (co.weight, co.bias, qc.weight, qc.bias))
        if key != self._fold_key:
            if self._fold is None:
                self._fold = Conv(2, co.in_channels, qc.out_channels, 3, padding=1).to(co.weight.device)
            wq = qc.weight.detach().reshape(qc.out_channels, -1)
            self._fold.weight.data.copy_(torch.einsum("oz,zchw->ochw", wq, co.weight.detach()))
            self._fold.bias.data.copy_(wq @ co.bias.detach() + qc.bias.detach())
            self._fold_key = key
        return self._fold

    @torch.no_grad()
    def encode_moments(self, x):
        """AutoencoderKL.encode up to the DiagonalGaussian parameters: NCHW fp32 -> [B, 2*embed_dim, h, w]."""
        vae = self.m
        h, ctx = self._encoder_trunk(vae.encoder, x)
        fold = self._folded_out(vae)
        out = self.head(vae.encoder.norm_out, fold, h, ctx)
        return ops.nhwc_to_nchw(out, fold.out_channels)

    @torch.no_grad()
    def decoder_forward(self, z):
        dec = self.m
        ctx = self._ctx(dec, z.shape[0], z.device)
        out = self._decoder_trunk(dec, Act(self._stage(z), need_grad=False), ctx)
        return ops.nhwc_to_nchw(out, dec.conv_out.conv.out_channels)

    @torch.no_grad()
    def decode(self, z):
        """AutoencoderKL.decode (denorm handled by the caller): post_quant_conv, then the decoder."""
        vae = self.m
        dec, pq = vae.decoder, vae.post_quant_conv.conv
        zin = self._stage(z)
        Kp = max(CPAD, -(-pq.out_channels // 8) * 8)
        hz, _ = ops.conv(zin, Kp, self.wc.get(pq.weight, 0, Kp, zin.shape[-1]), ks=1, pad=0,
                         bias=self.wc.padded(pq.bias, Kp))
        ctx = self._ctx(dec, z.shape[0], z.device)
        out = self._decoder_trunk(dec, Act(hz, need_grad=False), ctx)
        return ops.nhwc_to_nchw(out, dec.conv_out.conv.out_channels)


def get_vae_engine(module) -> VAEEngine:
    eng = getattr(module, "_fmd_vae_engine", None)
    if eng is None:
        eng = VAEEngine(module)
        object.__setattr__(module, "_fmd_vae_engine", eng)
    return eng
