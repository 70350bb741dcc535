"""Functional fp32 CPU forward of the reference UNets (TEST INFRASTRUCTURE ONLY).

Every function here evaluates the reference's module semantics from a
state_dict (keys exactly as the reference module tree names them) with the
same sequence of ``torch.nn.functional`` ops, so on CPU fp32 it reproduces the
reference bit-for-bit (pinned by ``tests/golden``).  Citations are to
``/root/reference/src``.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch
import torch.nn.functional as F

from . import spec as S

SD = Dict[str, torch.Tensor]


# --------------------------------------------------------------------- ops
def conv_nd(dims: int, x, w, b, stride=1, padding=0):
    """``ConvND`` -> nn.Conv{1,2,3}d (``nn/ops/convolution.py:8-54``)."""
    fn = {1: F.conv1d, 2: F.conv2d, 3: F.conv3d}[dims]
    return fn(x, w, b, stride=stride, padding=padding)


def timestep_embedding(t, dim, max_period=10000, flip_sin_to_cos=True, freq_shift=0):
    """Sinusoidal features (``nn/ops/time_embedding.py:4-32``)."""
    half = dim // 2
    expo = -math.log(max_period) * torch.arange(0, half, dtype=torch.float32)
    expo = expo / max(half - freq_shift, 1)
    args = t[:, None].float() * torch.exp(expo)[None, :]
    emb = torch.cat([torch.sin(args), torch.cos(args)], dim=-1)
    if flip_sin_to_cos:
        emb = torch.cat([emb[:, half:], emb[:, :half]], dim=-1)
    if dim % 2:
        emb = torch.cat([emb, torch.zeros_like(emb[:, :1])], dim=-1)
    return emb


def normalize_timesteps(t, x):
    """``BaseUNetND._normalize_timesteps`` (``models/unet/base.py:15-20``)."""
    if not torch.is_tensor(t):
        t = torch.tensor([t], dtype=torch.long)
    if t.ndim == 0:
        t = t[None]
    return t.expand(x.shape[0])


def resblock(sd: SD, L: dict, x, emb, dims, drop=None):
    """``ResBlockND.forward`` (``nn/blocks/residual.py:84-120``).  ``drop=(p, keep)``: the out_layers
    nn.Dropout (``residual.py:117``) in training mode with a given keep mask (NC(D)HW bool) --
    F.dropout's h * keep / (1 - p)."""
    p = L["prefix"]
    g1 = S.gn_groups(L["cin"], L["groups"])
    g2 = S.gn_groups(L["cout"], L["groups"])
    h = F.group_norm(x, g1, sd[f"{p}.norm1.weight"], sd[f"{p}.norm1.bias"], L["eps"])
    h = F.silu(h)
    h = conv_nd(dims, h, sd[f"{p}.conv1.conv.weight"], sd[f"{p}.conv1.conv.bias"], padding=1)
    e = F.silu(emb) if L["emb_act"] else emb
    e = F.linear(e, sd[f"{p}.emb_layers.weight"], sd[f"{p}.emb_layers.bias"]).type(h.dtype)
    e = e.view(*e.shape, *([1] * (h.ndim - e.ndim)))
    if L["scale_shift"]:
        scale, shift = torch.chunk(e, 2, dim=1)
    elif L["add_emb"]:
        h = h + e
    h = F.group_norm(h, g2, sd[f"{p}.norm2.weight"], sd[f"{p}.norm2.bias"], L["eps"])
    if L["scale_shift"]:
        h = h * (1 + scale) + shift
    h = F.silu(h)
    if drop is not None:
        h = h * drop[1].to(h.dtype) / (1.0 - drop[0])
    h = conv_nd(dims, h, sd[f"{p}.conv2.conv.weight"], sd[f"{p}.conv2.conv.bias"], padding=1)
    if L["cin"] == L["cout"]:
        skip = x
    else:
        k = 3 if L["use_conv"] else 1
        skip = conv_nd(dims, x, sd[f"{p}.skip_connection.conv.weight"], sd[f"{p}.skip_connection.conv.bias"],
                       padding=k // 2)
    return skip + h


def _sdpa(q, k, v):
    return F.scaled_dot_product_attention(q, k, v, dropout_p=0.0, is_causal=False)


def _linear_attention(q, k, v, eps=1e-6):
    """``LinearQKVAttention`` (``nn/blocks/attention.py:53-70``)."""
    ks = F.softmax(k, dim=-2)
    qs = F.softmax(q, dim=-1)
    ctx = torch.einsum("...nd,...ne->...de", ks, v)
    ctx = ctx / (ks.sum(dim=-2, keepdim=False).unsqueeze(-1) + eps)
    return torch.einsum("...nd,...de->...ne", qs, ctx)


def self_attention(sd: SD, L: dict, x):
    """``SpatialSelfAttention`` incl. the raw-reshape head split (``attention.py:82-117``)."""
    p = L["prefix"]
    b, c, *sp = x.shape
    inner = L["heads"] * L["dim_head"]
    xf = x.reshape(b, c, -1)
    hn = F.group_norm(xf, S.attn_groups(c), sd[f"{p}.norm.weight"], sd[f"{p}.norm.bias"], 1e-5)
    qkv = F.conv1d(hn, sd[f"{p}.qkv.weight"], sd[f"{p}.qkv.bias"])
    qkv = qkv.reshape(b, L["heads"], qkv.shape[-1], -1)
    q, k, v = qkv.chunk(3, dim=-1)
    h = _linear_attention(q, k, v) if L["linear"] else _sdpa(q, k, v)
    h = h.reshape(b, inner, -1)
    h = F.conv1d(h, sd[f"{p}.proj_out.weight"], sd[f"{p}.proj_out.bias"])
    return (xf + h).reshape(b, c, *sp)


def cross_attention(sd: SD, L: dict, x, context):
    """``SpatialCrossAttention`` (``attention.py:120-189``)."""
    p = L["prefix"]
    b, c, *sp = x.shape
    inner = L["heads"] * L["dim_head"]
    xf = x.reshape(b, c, -1)
    cd = L["ctx"]
    if context.dim() == 3:
        ctx = context if context.shape[1] == cd else context.transpose(1, 2)
    else:
        ctx = context.reshape(context.shape[0], context.shape[1], -1)
    q = F.conv1d(F.group_norm(xf, S.attn_groups(c), sd[f"{p}.norm.weight"], sd[f"{p}.norm.bias"], 1e-5),
                 sd[f"{p}.q_proj.weight"], sd[f"{p}.q_proj.bias"])
    kv = F.conv1d(F.group_norm(ctx, S.attn_groups(cd), sd[f"{p}.context_norm.weight"], sd[f"{p}.context_norm.bias"], 1e-5),
                  sd[f"{p}.kv_proj.weight"], sd[f"{p}.kv_proj.bias"])
    q = q.reshape(b, L["heads"], q.shape[-1], -1)
    kv = kv.reshape(b, L["heads"], kv.shape[-1], -1)
    k, v = kv.chunk(2, dim=-1)
    h = _linear_attention(q, k, v) if L["linear"] else _sdpa(q, k, v)
    h = F.conv1d(h.reshape(b, inner, -1), sd[f"{p}.proj_out.weight"], sd[f"{p}.proj_out.bias"])
    return (xf + h).reshape(b, c, *sp)


def diffusers_attention(sd: SD, L: dict, x, context=None):
    """``DiffusersAttentionND`` (``attention.py:192-274``)."""
    p = L["prefix"]
    b, c = x.shape[:2]
    sp = x.shape[2:]
    heads = L["heads"]
    hd = c // heads
    xf = x.reshape(b, c, -1)
    xn = F.group_norm(xf, S.attn_groups(c, L["groups"]), sd[f"{p}.group_norm.weight"], sd[f"{p}.group_norm.bias"],
                      L["eps"]).transpose(1, 2)
    q = F.linear(xn, sd[f"{p}.to_q.weight"], sd[f"{p}.to_q.bias"])
    if L["ctx"] is None:
        src = xn
    else:
        cd = L["ctx"]
        if context.dim() == 3:
            ctx = context if context.shape[1] == cd else context.transpose(1, 2)
        else:
            ctx = context.reshape(context.shape[0], context.shape[1], -1)
        src = F.group_norm(ctx, S.attn_groups(cd, L["groups"]), sd[f"{p}.context_norm.weight"],
                           sd[f"{p}.context_norm.bias"], L["eps"]).transpose(1, 2)
    k = F.linear(src, sd[f"{p}.to_k.weight"], sd[f"{p}.to_k.bias"])
    v = F.linear(src, sd[f"{p}.to_v.weight"], sd[f"{p}.to_v.bias"])
    q = q.view(b, -1, heads, hd).transpose(1, 2)
    k = k.view(b, -1, heads, hd).transpose(1, 2)
    v = v.view(b, -1, heads, hd).transpose(1, 2)
    o = _sdpa(q, k, v)
    o = o.transpose(1, 2).reshape(b, -1, c)
    o = F.linear(o, sd[f"{p}.to_out.0.weight"], sd[f"{p}.to_out.0.bias"])
    return o.transpose(1, 2).reshape(b, c, *sp) + x


def downsample(sd: SD, L: dict, x, dims):
    """``DownsampleND`` (``nn/ops/upsampling.py:32-62``)."""
    if L["use_conv"]:
        return conv_nd(dims, x, sd[f"{L['prefix']}.op.conv.weight"], sd[f"{L['prefix']}.op.conv.bias"],
                       stride=2, padding=1)
    fn = {1: F.avg_pool1d, 2: F.avg_pool2d, 3: F.avg_pool3d}[dims]
    return fn(x, kernel_size=2, stride=2)


def upsample(sd: SD, L: dict, x, dims):
    """``UpsampleND`` nearest x2 then 3x3 conv (``nn/ops/upsampling.py:8-30``)."""
    x = F.interpolate(x, scale_factor=2, mode="nearest")
    if L["use_conv"]:
        x = conv_nd(dims, x, sd[f"{L['prefix']}.conv.conv.weight"], sd[f"{L['prefix']}.conv.conv.bias"], padding=1)
    return x


def _apply(sd, L, h, emb, ctx, dims):
    k = L["kind"]
    if k == "res":
        return resblock(sd, L, h, emb, dims)
    if k == "conv":
        return conv_nd(dims, h, sd[f"{L['prefix']}.weight"], sd[f"{L['prefix']}.bias"], stride=L["stride"], padding=L["pad"])
    if k == "self_attn":
        return self_attention(sd, L, h)
    if k == "cross_attn":
        return cross_attention(sd, L, h, ctx)
    if k == "dattn":
        return diffusers_attention(sd, L, h, ctx)
    if k == "down":
        return downsample(sd, L, h, dims)
    if k == "up":
        return upsample(sd, L, h, dims)
    raise ValueError(k)


# ------------------------------------------------------------------ models
def efficient_unet(sd: SD, spec: dict, x, t, context=None, context_ca=None):
    """EfficientUNetND forward (``models/unet/unet.py:295-326`` + ``base.py:41-53``)."""
    dims = spec["dims"]
    if context is not None:
        x = torch.cat([x, context], dim=1)
    t = normalize_timesteps(t, x)
    feats = timestep_embedding(t, spec["model_channels"], flip_sin_to_cos=False, freq_shift=0)
    emb = F.linear(feats, sd["time_embed.0.weight"], sd["time_embed.0.bias"])
    emb = F.linear(F.silu(emb), sd["time_embed.2.weight"], sd["time_embed.2.bias"])
    lay = S.efficient_layout(spec)
    pf = lay["pool"]
    if pf > 1:   # PoolND: ConvND(kernel = stride = pool_factor, padding 0) (nn/ops/pooling.py:10-30, unet.py:124-126)
        x = conv_nd(dims, x, sd["pool.down.conv.weight"], sd["pool.down.conv.bias"], stride=pf, padding=0)
    hs = []
    h = x
    for block in lay["inputs"]:
        for L in block:
            h = _apply(sd, L, h, emb, context_ca, dims)
        hs.append(h)
    for L in lay["middle"]:
        h = _apply(sd, L, h, emb, context_ca, dims)
    for block in lay["outputs"]:
        h = torch.cat([h, hs.pop()], dim=1)
        for L in block:
            h = _apply(sd, L, h, emb, context_ca, dims)
    h = F.group_norm(h, S.gn_groups(lay["out_ch"], 32), sd["out.0.weight"], sd["out.0.bias"], 1e-5)
    h = F.silu(h)
    h = conv_nd(dims, h, sd["out.2.conv.weight"], sd["out.2.conv.bias"], padding=1)
    if pf > 1:   # UnPoolND: ConvTransposeND(kernel = stride = pool_factor) (pooling.py:87-105, unet.py:280-287)
        fn = {1: F.conv_transpose1d, 2: F.conv_transpose2d, 3: F.conv_transpose3d}[dims]
        h = fn(h, sd["unpool.up.convT.weight"], sd["unpool.up.convT.bias"], stride=pf)
    return h


def diffusers_unet(sd: SD, spec: dict, x, t, context=None, context_ca=None):
    """UNetDiffusersND forward (``models/unet/unet_diffusers_nd.py:151-191``)."""
    dims = spec["dims"]
    if context is not None:
        x = torch.cat([x, context], dim=1)
    if spec["center_input_sample"]:
        x = 2 * x - 1.0
    t = normalize_timesteps(t, x)
    c0 = spec["block_out_channels"][0]
    feats = timestep_embedding(t, c0, max_period=10000, flip_sin_to_cos=spec["flip_sin_to_cos"],
                               freq_shift=spec["freq_shift"]).to(dtype=x.dtype)
    emb = F.linear(feats, sd["time_embedding.linear_1.weight"], sd["time_embedding.linear_1.bias"])
    emb = F.linear(F.silu(emb), sd["time_embedding.linear_2.weight"], sd["time_embedding.linear_2.bias"])
    lay = S.diffusers_layout(spec)
    h = conv_nd(dims, x, sd["conv_in.weight"], sd["conv_in.bias"], padding=1)
    res = [h]
    for blk in lay["downs"]:
        for j, R in enumerate(blk["res"]):
            h = resblock(sd, R, h, emb, dims)
            if blk["attn"]:
                h = diffusers_attention(sd, blk["attn"][j], h, context_ca)
            res.append(h)
        if blk["down"] is not None:
            h = downsample(sd, blk["down"], h, dims)
            res.append(h)
    if lay["mid"] is not None:
        h = resblock(sd, lay["mid"]["res"][0], h, emb, dims)
        if lay["mid"]["attn"]:
            h = diffusers_attention(sd, lay["mid"]["attn"][0], h, context_ca)
        h = resblock(sd, lay["mid"]["res"][1], h, emb, dims)
    for blk in lay["ups"]:
        for j, R in enumerate(blk["res"]):
            h = torch.cat([h, res.pop()], dim=1)
            h = resblock(sd, R, h, emb, dims)
            if blk["attn"]:
                h = diffusers_attention(sd, blk["attn"][j], h, context_ca)
        if blk["up"] is not None:
            h = upsample(sd, blk["up"], h, dims)
    g = S.gn_groups(c0, spec["norm_num_groups"])
    h = F.group_norm(h, g, sd["conv_norm_out.weight"], sd["conv_norm_out.bias"], spec["norm_eps"])
    h = F.silu(h)
    return conv_nd(dims, h, sd["conv_out.weight"], sd["conv_out.bias"], padding=1)


def unet_forward(sd: SD, spec: dict, x, t, context=None, context_ca=None):
    if spec["impl"] == "diffusers_nd":
        return diffusers_unet(sd, spec, x, t, context, context_ca)
    return efficient_unet(sd, spec, x, t, context, context_ca)


# ---------------------------------------------------------- state helpers
def param_shapes(spec: dict) -> Dict[str, tuple]:
    """Every parameter name -> shape, in the reference's state_dict order."""
    shapes: Dict[str, tuple] = {}
    dims = spec["dims"]
    ks = (3,) * dims

    def conv(p, cin, cout, k=ks):
        shapes[f"{p}.weight"] = (cout, cin, *k)
        shapes[f"{p}.bias"] = (cout,)

    def norm(p, c):
        shapes[f"{p}.weight"] = (c,)
        shapes[f"{p}.bias"] = (c,)

    def lin(p, i, o):
        shapes[f"{p}.weight"] = (o, i)
        shapes[f"{p}.bias"] = (o,)

    def layer(L, emb_dim):
        k = L["kind"]
        p = L["prefix"]
        if k == "res":
            norm(f"{p}.norm1", L["cin"])
            conv(f"{p}.conv1.conv", L["cin"], L["cout"])
            lin(f"{p}.emb_layers", emb_dim, 2 * L["cout"] if L["scale_shift"] else L["cout"])
            norm(f"{p}.norm2", L["cout"])
            conv(f"{p}.conv2.conv", L["cout"], L["cout"])
            if L["cin"] != L["cout"]:
                conv(f"{p}.skip_connection.conv", L["cin"], L["cout"], ks if L["use_conv"] else (1,) * dims)
        elif k == "conv":
            conv(p, L["cin"], L["cout"])
        elif k == "self_attn":
            inner = L["heads"] * L["dim_head"]
            norm(f"{p}.norm", L["ch"])
            conv(f"{p}.qkv", L["ch"], 3 * inner, (1,))
            conv(f"{p}.proj_out", inner, L["ch"], (1,))
        elif k == "cross_attn":
            inner = L["heads"] * L["dim_head"]
            norm(f"{p}.norm", L["ch"])
            norm(f"{p}.context_norm", L["ctx"])
            conv(f"{p}.q_proj", L["ch"], inner, (1,))
            conv(f"{p}.kv_proj", L["ctx"], 2 * inner, (1,))
            conv(f"{p}.proj_out", inner, L["ch"], (1,))
        elif k == "dattn":
            c = L["ch"]
            norm(f"{p}.group_norm", c)
            lin(f"{p}.to_q", c, c)
            if L["ctx"] is None:
                lin(f"{p}.to_k", c, c)
                lin(f"{p}.to_v", c, c)
            else:
                norm(f"{p}.context_norm", L["ctx"])
                lin(f"{p}.to_k", L["ctx"], c)
                lin(f"{p}.to_v", L["ctx"], c)
            lin(f"{p}.to_out.0", c, c)
        elif k == "down":
            if L["use_conv"]:
                conv(f"{p}.op.conv", L["ch"], L["ch"])
        elif k == "up":
            if L["use_conv"]:
                conv(f"{p}.conv.conv", L["ch"], L["ch"])

    if spec["impl"] == "diffusers_nd":
        c0 = spec["block_out_channels"][0]
        ed = 4 * c0
        lay = S.diffusers_layout(spec)
        conv("conv_in", spec["in_channels"], c0)
        lin("time_embedding.linear_1", c0, ed)
        lin("time_embedding.linear_2", ed, ed)
        # registration order (unet_diffusers_nd.py:75-76 create both ModuleLists
        # before mid_block is assigned): conv_in, time_embedding, down_blocks,
        # up_blocks, mid_block, head
        for blk in lay["downs"]:
            for R in blk["res"]:
                layer(R, ed)
            for A in blk["attn"]:
                layer(A, ed)
            if blk["down"]:
                layer(blk["down"], ed)
        for blk in lay["ups"]:
            for R in blk["res"]:
                layer(R, ed)
            for A in blk["attn"]:
                layer(A, ed)
            if blk["up"]:
                layer(blk["up"], ed)
        if lay["mid"]:
            for R in lay["mid"]["res"]:
                layer(R, ed)
            for A in lay["mid"]["attn"]:
                layer(A, ed)
        norm("conv_norm_out", c0)
        conv("conv_out", c0, spec["out_channels"])
        return shapes
    mc = spec["model_channels"]
    ed = 4 * mc
    lay = S.efficient_layout(spec)
    pf = lay["pool"]
    lin("time_embed.0", mc, ed)
    lin("time_embed.2", ed, ed)
    if pf > 1:
        conv("pool.down.conv", spec["in_channels"], mc, (pf,) * dims)
    for block in lay["inputs"]:
        for L in block:
            layer(L, ed)
    for L in lay["middle"]:
        layer(L, ed)
    for block in lay["outputs"]:
        for L in block:
            layer(L, ed)
    norm("out.0", lay["out_ch"])
    conv("out.2.conv", mc, mc if pf > 1 else spec["out_channels"])
    if pf > 1:   # ConvTranspose weight layout [in, out, *k]
        shapes["unpool.up.convT.weight"] = (mc, spec["out_channels"], *((pf,) * dims))
        shapes["unpool.up.convT.bias"] = (spec["out_channels"],)
    return shapes


def seeded_tensors(shapes: Dict[str, tuple], seed: int, scale: float = 1.0) -> SD:
    """Deterministic non-zero tensors for a name -> shape map (order matters).

    For entry number ``i`` a CPU generator seeded with ``seed + i`` draws
    ``randn``; weights (ndim >= 2) are scaled by ``scale / sqrt(fan_in)``, 1-D
    ``*.bias`` entries are ``0.1*randn`` and other 1-D entries (norm weights)
    ``1 + 0.1*randn``.  Zero-initialised reference layers are therefore
    non-zero, so they cannot hide bugs.
    """
    out: SD = {}
    for i, (name, shp) in enumerate(shapes.items()):
        g = torch.Generator().manual_seed(seed + i)
        r = torch.randn(shp, generator=g, dtype=torch.float32)
        if name.endswith(".bias"):
            out[name] = 0.1 * r
        elif len(shp) == 1:
            out[name] = 1.0 + 0.1 * r
        else:
            fan_in = int(torch.tensor(shp[1:]).prod().item())
            out[name] = r * (scale / math.sqrt(fan_in))
    return out


def seeded_state_dict(spec: dict, seed: int, scale: float = 1.0) -> SD:
    """``seeded_tensors`` over the full UNet parameter list of ``spec``."""
    return seeded_tensors(param_shapes(spec), seed, scale)
