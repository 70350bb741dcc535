"""Calling a single block outside a UNet.

The fused engine executes whole UNets (``fmdiff.runtime.engine``).  A lone
``Conv`` runs through the same implicit-GEMM kernel (forward only).  A lone
``ResBlockND`` / ``SpatialSelfAttention`` / ``SpatialCrossAttention`` /
``DiffusersAttentionND`` runs through the same engine layer methods (the fused
HIP kernels of the UNet path) on a one-block engine, differentiable w.r.t. its
input, its time embedding and its parameters -- the reference's block
self-tests call the blocks this way (``src/nn/blocks/residual.py:160-215``,
``attention.py:277-341``).
"""
from __future__ import annotations

import weakref

import torch

from . import ops


def conv_forward(conv, x: torch.Tensor) -> torch.Tensor:
    """NCHW fp32 -> NCHW fp32 through csrc/conv.hip (no autograd)."""
    ops._need_cuda(x, "Conv")
    if conv.dims != 2 and not (conv.dims == 1 and conv.kernel_size == (1,)):
        raise NotImplementedError("standalone Conv: 2-D convs and 1x1 Conv1d only")
    if x.dim() == 3:   # Conv1d k=1 over tokens: treat as [N, C, T, 1]
        x4 = x.unsqueeze(-1)
    else:
        x4 = x
    Cin = x4.shape[1]
    Cp = -(-Cin // 8) * 8
    K = conv.out_channels
    Kp = -(-K // 8) * 8
    xin = ops.nchw_to_nhwc(x4, Cp)
    w = ops.prep_weights(conv.weight.detach(), 0, Kp, Cp)
    ks = conv.kernel_size[0]
    bias = None
    if conv.bias is not None:
        bias = torch.zeros(Kp, device=x.device, dtype=torch.float32)
        bias[:K].copy_(conv.bias.detach())
    out, _ = ops.conv(xin, Kp, w, ks=ks, stride=conv.stride[0], pad=conv.padding[0], bias=bias, out_f32=True)
    y = ops.nhwc_to_nchw(out, K)
    return y.squeeze(-1) if x.dim() == 3 else y


def linear_forward(lin, x: torch.Tensor) -> torch.Tensor:
    ops._need_cuda(x, "Linear")
    if x.dim() != 2 or x.shape[0] > 32:
        raise NotImplementedError("standalone Linear: [B<=32, in] inputs (time-embedding path)")
    return ops.linear(x.float().contiguous(), lin.weight.detach(), lin.bias.detach() if lin.bias is not None else None)


def _block_engine_cls():
    from .engine import UNetEngine, WeightCache

    class BlockEngine(UNetEngine):
        """One-block engine: the UNet engine's layer methods (res_block / attention / cross_attention) on a
        lone block module (no grouped emb projections, no time MLP)."""

        def __init__(self, block):   # UNetEngine.__init__'s UNet-model checks do not apply
            self._model = weakref.ref(block)
            self.kind = "block"
            self.wc = WeightCache()
            self._tt = None
            self.gl, self.gl_slot = None, {}
            self._head_bwd = None
            self.dims1 = False

    return BlockEngine


def _block_engine(block):
    eng = getattr(block, "_fmd_block_engine", None)
    if eng is None:
        eng = _block_engine_cls()(block)
        object.__setattr__(block, "_fmd_block_engine", eng)
    return eng


def _run_block(eng, block, x_nhwc, emb, context, save):
    from ..nn.blocks.attention import DiffusersAttentionND, SpatialCrossAttention, SpatialSelfAttention
    from ..nn.blocks.residual import ResBlockND
    from .engine import Act, Ctx
    N = x_nhwc.shape[0]
    e = emb.float().contiguous() if emb is not None else torch.zeros((N, 1), device=x_nhwc.device)
    ctx = Ctx(e, save, N)
    ctx.cca = context
    xa = Act(x_nhwc, need_grad=save)
    if isinstance(block, ResBlockND):
        if block.uses_embedding and emb is None:
            raise ValueError("ResBlockND with emb_channels needs the time embedding")
        y = eng.res_block(block, [xa], ctx)
    elif isinstance(block, (SpatialSelfAttention, DiffusersAttentionND)):
        y = eng.attention(block, xa, ctx)
    elif isinstance(block, SpatialCrossAttention):
        y = eng.cross_attention(block, xa, ctx)
    else:
        raise NotImplementedError(type(block).__name__)
    return xa, y, ctx


class _BlockFunction(torch.autograd.Function):
    @staticmethod
    def forward(fctx, x, emb, context, block, *params):
        eng = _block_engine(block)
        xin = ops.nchw_to_nhwc(x.unsqueeze(-1) if x.dim() == 3 else x)   # 1-D signal: an (L, 1) image
        xa, y, ctx = _run_block(eng, block, xin, emb, context, True)
        fctx.state = (eng, xa, y, ctx, x.shape[1], emb is not None, x.dim() == 3)
        out = ops.nhwc_to_nchw(y.t, y.C)
        return out.squeeze(-1) if x.dim() == 3 else out

    @staticmethod
    def backward(fctx, gout):
        eng, xa, y, ctx, C, has_emb, d1 = fctx.state
        fctx.state = None
        for p in eng.m.parameters():
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        y.grad = ops.nchw_to_nhwc(gout.contiguous().unsqueeze(-1) if d1 else gout.contiguous())
        ops.gb_defer()
        try:
            for fn in reversed(ctx.tape):
                fn()
        finally:
            ops.gb_flush()
        eng._join()
        dx = ops.nhwc_to_nchw(xa.grad, C) if xa.grad is not None else None
        if d1 and dx is not None:
            dx = dx.squeeze(-1)
        demb = ctx.demb.clone() if has_emb else None
        return (dx, demb, None, None) + tuple(None for _ in eng.m.parameters())


def block_forward(block, x, emb, context=None):
    """NC(D)HW fp32 -> NC(D)HW fp32 through the fused HIP layer kernels; channels must be multiples of 8.
    Gradients flow to ``x``, ``emb`` and the block's parameters (accumulated into ``.grad``), not to
    ``context``."""
    ops._need_cuda(x, type(block).__name__)
    if x.shape[1] % 8:
        raise NotImplementedError(f"{type(block).__name__}: standalone execution needs channels % 8 == 0")
    ctxt = context.float().contiguous() if context is not None else None
    params = list(block.parameters())
    if torch.is_grad_enabled() and (x.requires_grad or (emb is not None and emb.requires_grad)
                                    or any(p.requires_grad for p in params)):
        return _BlockFunction.apply(x.float(), emb, ctxt, block, *params)
    eng = _block_engine(block)
    _, y, _ = _run_block(eng, block, ops.nchw_to_nhwc(x.unsqueeze(-1) if x.dim() == 3 else x), emb, ctxt, False)
    out = ops.nhwc_to_nchw(y.t, y.C)
    return out.squeeze(-1) if x.dim() == 3 else out
