"""Functional fp32 CPU forward of the reference AutoencoderKL (TEST INFRASTRUCTURE ONLY).

Restates ``src/nn/modules/vae/encoder.py:19-158``, ``decoder.py:19-160`` and
``src/models/vae/kl.py:22-140`` (encode -> moments, ``DiagonalGaussian.mode``, decode) from a
state_dict with the same ``torch.nn.functional`` op sequence; pinned against outputs of the reference
modules themselves (``tests/golden/make_vae_golden.py`` -> ``tests/golden/vae_golden.pt``).
Only the tests, ``__graft_entry__.smoke()`` and ``bench.py``'s CPU leg may import this module.
"""
from __future__ import annotations

import math
from typing import Dict

import torch
import torch.nn.functional as F

SD = Dict[str, torch.Tensor]


def _gcd_groups(c: int, norm_groups=None) -> int:
    return norm_groups if norm_groups is not None else max(1, math.gcd(c, 32))


def _rb_groups(c: int, groups: int = 32) -> int:
    """make_group_norm (nn/ops/normalization.py:11-19): largest divisor of C that is <= 32."""
    g = min(groups, c)
    while c % g:
        g -= 1
    return g


def resblock(sd: SD, p: str, x, cin: int, cout: int):
    """ResBlockND without a time embedding (residual.py:84-120, emb_channels=None)."""
    h = F.silu(F.group_norm(x, _rb_groups(cin), sd[f"{p}.norm1.weight"], sd[f"{p}.norm1.bias"], 1e-5))
    h = F.conv2d(h, sd[f"{p}.conv1.conv.weight"], sd[f"{p}.conv1.conv.bias"], padding=1)
    h = F.silu(F.group_norm(h, _rb_groups(cout), sd[f"{p}.norm2.weight"], sd[f"{p}.norm2.bias"], 1e-5))
    h = F.conv2d(h, sd[f"{p}.conv2.conv.weight"], sd[f"{p}.conv2.conv.bias"], padding=1)
    skip = x if cin == cout else F.conv2d(x, sd[f"{p}.skip_connection.conv.weight"],
                                          sd[f"{p}.skip_connection.conv.bias"])
    return skip + h


def attention(sd: SD, p: str, x, heads: int, dim_head: int):
    """SpatialSelfAttention, softmax, raw head split (attention.py:104-117)."""
    b, c, *sp = x.shape
    xf = x.reshape(b, c, -1)
    hn = F.group_norm(xf, max(1, math.gcd(c, 32)), sd[f"{p}.norm.weight"], sd[f"{p}.norm.bias"], 1e-5)
    qkv = F.conv1d(hn, sd[f"{p}.qkv.weight"], sd[f"{p}.qkv.bias"])
    qkv = qkv.reshape(b, heads, qkv.shape[-1], -1)
    q, k, v = qkv.chunk(3, dim=-1)
    h = F.scaled_dot_product_attention(q, k, v)
    h = F.conv1d(h.reshape(b, heads * dim_head, -1), sd[f"{p}.proj_out.weight"], sd[f"{p}.proj_out.bias"])
    return (xf + h).reshape(b, c, *sp)


def _channels(cfg):
    if cfg.get("down_channels") is not None:
        return tuple(cfg["down_channels"])
    return tuple(cfg.get("base_ch", 128) * m for m in cfg.get("ch_mult", (1, 2, 4, 4)))


def _attn_shape(cfg, channels):
    heads = cfg.get("attn_heads", 4)
    heads = heads if heads is not None else 1
    dh = cfg.get("attn_dim_head", 64)
    if dh is None:
        dh = channels if heads == 1 else max(1, channels // heads)
    return heads, dh


def encoder(sd: SD, cfg: dict, x, prefix="encoder"):
    """Encoder.forward (encoder.py:139-158)."""
    chans = _channels(cfg)
    nrb = cfg.get("num_res_blocks", 2)
    attn_res = tuple(cfg.get("attn_resolutions", ()))
    use_attn = cfg.get("use_attention", True)
    res = cfg.get("resolution", 256)
    h = F.conv2d(x, sd[f"{prefix}.conv_in.conv.weight"], sd[f"{prefix}.conv_in.conv.bias"], padding=1)
    cin = cfg.get("base_ch", 128)
    for i, cout in enumerate(chans):
        for j in range(nrb):
            h = resblock(sd, f"{prefix}.downs.{i}.blocks.{j}", h, cin, cout)
            cin = cout
            if use_attn and res in attn_res:
                h = attention(sd, f"{prefix}.downs.{i}.attns.{j}", h, *_attn_shape(cfg, cin))
        if i != len(chans) - 1:
            h = F.conv2d(h, sd[f"{prefix}.downs.{i}.down.op.conv.weight"], sd[f"{prefix}.downs.{i}.down.op.conv.bias"],
                         stride=2, padding=1)
            res //= 2
    h = resblock(sd, f"{prefix}.mid_block1", h, cin, cin)
    if use_attn:
        h = attention(sd, f"{prefix}.mid_attn", h, *_attn_shape(cfg, cin))
    h = resblock(sd, f"{prefix}.mid_block2", h, cin, cin)
    h = F.silu(F.group_norm(h, _gcd_groups(cin, cfg.get("norm_groups")), sd[f"{prefix}.norm_out.weight"],
                            sd[f"{prefix}.norm_out.bias"], 1e-5))
    return F.conv2d(h, sd[f"{prefix}.conv_out.conv.weight"], sd[f"{prefix}.conv_out.conv.bias"], padding=1)


def decoder(sd: SD, cfg: dict, z, prefix="decoder"):
    """Decoder.forward (decoder.py:133-160), tanh_out=False."""
    chans = _channels(cfg)
    nrb = cfg.get("num_res_blocks", 2)
    attn_res = tuple(cfg.get("attn_resolutions", ()))
    use_attn = cfg.get("use_attention", True)
    res = cfg.get("resolution", 256) // (2 ** (len(chans) - 1))
    cin = chans[-1]
    h = F.conv2d(z, sd[f"{prefix}.conv_in.conv.weight"], sd[f"{prefix}.conv_in.conv.bias"], padding=1)
    h = resblock(sd, f"{prefix}.mid_block1", h, cin, cin)
    if use_attn:
        h = attention(sd, f"{prefix}.mid_attn", h, *_attn_shape(cfg, cin))
    h = resblock(sd, f"{prefix}.mid_block2", h, cin, cin)
    # construction order: ups.insert(0, stage) for idx over reversed(channels); forward walks reversed(ups)
    n = len(chans)
    for idx, cout in enumerate(reversed(chans)):
        s = n - 1 - idx
        for j in range(nrb + 1):
            h = resblock(sd, f"{prefix}.ups.{s}.blocks.{j}", h, cin, cout)
            cin = cout
            if use_attn and res in attn_res:
                h = attention(sd, f"{prefix}.ups.{s}.attns.{j}", h, *_attn_shape(cfg, cin))
        if idx != n - 1:
            h = F.interpolate(h, scale_factor=2, mode="nearest")
            h = F.conv2d(h, sd[f"{prefix}.ups.{s}.up.conv.conv.weight"], sd[f"{prefix}.ups.{s}.up.conv.conv.bias"],
                         padding=1)
            res *= 2
    h = F.silu(F.group_norm(h, _gcd_groups(cin, cfg.get("norm_groups")), sd[f"{prefix}.norm_out.weight"],
                            sd[f"{prefix}.norm_out.bias"], 1e-5))
    return F.conv2d(h, sd[f"{prefix}.conv_out.conv.weight"], sd[f"{prefix}.conv_out.conv.bias"], padding=1)


def encode_moments(sd: SD, cfg: dict, x):
    """AutoencoderKL.encode up to the DiagonalGaussian parameters (kl.py:116-122)."""
    return F.conv2d(encoder(sd, cfg, x), sd["quant_conv.conv.weight"], sd["quant_conv.conv.bias"])


def decode(sd: SD, cfg: dict, z):
    """AutoencoderKL.decode (kl.py:124-128), denorm=False."""
    return decoder(sd, cfg, F.conv2d(z, sd["post_quant_conv.conv.weight"], sd["post_quant_conv.conv.bias"]))
