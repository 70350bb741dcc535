"""Config -> architecture rules for the oracle (TEST INFRASTRUCTURE ONLY).

Restates ``DiffusionUNetFactory`` (reference
``src/models/generators/diffusionfactory.py:35-130``) as plain data: the
result is a nested description of every layer with the state_dict prefix the
reference module tree gives it, so ``oracle.unet`` can evaluate the network
functionally from a state_dict.
"""
from __future__ import annotations

import math
from typing import Any, Dict, List, Optional, Sequence, Tuple


def _as_tuple(value, default: Tuple[int, ...]) -> Tuple[int, ...]:
    # diffusionfactory.py:10-15
    if value is None:
        return tuple(default)
    if isinstance(value, int):
        return (value,)
    return tuple(value)


def gn_groups(channels: int, groups: int = 32) -> int:
    """``make_group_norm`` group rule (reference ``src/nn/ops/normalization.py:11-19``)."""
    g = min(groups, channels)
    while channels % g != 0 and g > 1:
        g -= 1
    return g


def attn_groups(channels: int, groups: int = 32) -> int:
    """Attention norms use ``gcd(C, 32)`` (reference ``src/nn/blocks/attention.py:97,210``)."""
    return max(1, math.gcd(channels, groups))


def resolve_channels(training_cfg: Dict[str, Any], model_cfg: Dict[str, Any]) -> int:
    """``channels = training.channels or unet.out_channels or 1`` (``diffusion_utils.py:113``)."""
    unet = model_cfg.get("unet", {}) or {}
    return int(training_cfg.get("channels") or unet.get("out_channels") or 1)


def derive_spec(model_cfg: Dict[str, Any], conditioning: Optional[str], channels: Optional[int]) -> Dict[str, Any]:
    """Map a ``model.unet`` config block to a flat spec dict (diffusionfactory.py:35-40)."""
    cfg = dict(model_cfg or {})
    impl = str(cfg.get("unet_impl", "efficient_nd")).lower()
    if impl in {"diffusers_nd", "diffusers_exact_nd", "exact_nd", "diffusers"}:
        return _derive_diffusers(cfg, conditioning, channels)
    return _derive_efficient(cfg, conditioning, channels)


def _derive_efficient(cfg, conditioning, channels) -> Dict[str, Any]:
    # diffusionfactory.py:42-83
    boc = _as_tuple(cfg.get("block_out_channels"), (128, 128, 256, 256, 512, 512))
    model_channels = int(cfg.get("model_channels", boc[0] if boc else 128))
    in_ch = cfg.get("in_channels", channels or 1)
    cond_ch = cfg.get("conditioning_channels", channels or in_ch)
    mode = (conditioning or "").lower()
    if mode == "concatenate":
        in_ch = in_ch + cond_ch
    out_ch = cfg.get("out_channels", channels or 1)
    nrb = int(cfg.get("num_res_blocks", cfg.get("layers_per_block", 2)))
    base = model_channels or boc[0]
    inferred = tuple(max(1, int(c // base)) for c in boc) if boc else ()
    mult = _as_tuple(cfg.get("channel_mult"), inferred)
    attn_res = _as_tuple(cfg.get("attention_resolutions"), (1,))
    xres = cfg.get("cross_attention_resolutions")
    x_mid = bool(cfg.get("cross_attention_in_middle", False))
    if xres is None and mode == "attention":
        xres = attn_res
        if "cross_attention_in_middle" not in cfg:
            x_mid = True
    return dict(
        impl="efficient_nd",
        dims=int(cfg.get("spatial_dims", 2)),
        in_channels=int(in_ch),
        model_channels=model_channels,
        out_channels=int(out_ch),
        num_res_blocks=nrb,
        channel_mult=tuple(mult) or (1, 2, 3, 4),
        attention_resolutions=tuple(attn_res),
        cross_attention_resolutions=tuple(xres) if xres is not None else (),
        cross_attention_in_middle=x_mid,
        cross_attention_dim=int(cfg.get("cross_attention_dim", cond_ch)),
        dropout=float(cfg.get("dropout", 0.0)),
        conv_resample=bool(cfg.get("conv_resample", True)),
        dim_head=int(cfg.get("dim_head", 64)),
        num_heads=int(cfg.get("num_heads", 4)),
        use_linear_attn=bool(cfg.get("use_linear_attn", True)),
        use_scale_shift_norm=bool(cfg.get("use_scale_shift_norm", True)),
        emb_act_before_proj=bool(cfg.get("emb_activation_before_proj", False)),
        pool_factor=int(cfg.get("pool_factor", 1)),
    )


def _derive_diffusers(cfg, conditioning, channels) -> Dict[str, Any]:
    # diffusionfactory.py:85-130
    mode = (conditioning or "").lower()
    in_ch = int(cfg.get("in_channels", channels or 1))
    cond_ch = int(cfg.get("conditioning_channels", channels or in_ch))
    if mode == "concatenate" and not bool(cfg.get("in_channels_already_conditioned", False)):
        in_ch += cond_ch
    if mode == "attention":
        dd = ("CrossAttnDownBlock2D", "CrossAttnDownBlock2D", "CrossAttnDownBlock2D", "DownBlock2D")
        du = ("UpBlock2D", "CrossAttnUpBlock2D", "CrossAttnUpBlock2D", "CrossAttnUpBlock2D")
        dm = "UNetMidBlock2DCrossAttn"
    else:
        dd = ("DownBlock2D", "AttnDownBlock2D", "AttnDownBlock2D", "AttnDownBlock2D")
        du = ("AttnUpBlock2D", "AttnUpBlock2D", "AttnUpBlock2D", "UpBlock2D")
        dm = "UNetMidBlock2D"
    return dict(
        impl="diffusers_nd",
        dims=int(cfg.get("spatial_dims", 2)),
        in_channels=in_ch,
        out_channels=int(cfg.get("out_channels", channels or 1)),
        center_input_sample=bool(cfg.get("center_input_sample", False)),
        freq_shift=int(cfg.get("freq_shift", 0)),
        flip_sin_to_cos=bool(cfg.get("flip_sin_to_cos", True)),
        down_block_types=tuple(cfg.get("down_block_types", dd)),
        mid_block_type=cfg.get("mid_block_type", dm),
        up_block_types=tuple(cfg.get("up_block_types", du)),
        block_out_channels=_as_tuple(cfg.get("block_out_channels"), (224, 448, 672, 896)),
        layers_per_block=int(cfg.get("layers_per_block", 2)),
        attention_head_dim=int(cfg.get("attention_head_dim", 8)),
        norm_num_groups=int(cfg.get("norm_num_groups", 32)),
        norm_eps=float(cfg.get("norm_eps", 1e-5)),
        scale_shift=str(cfg.get("resnet_time_scale_shift", "default")) == "scale_shift",
        add_attention=bool(cfg.get("add_attention", True)),
        cross_attention_dim=int(cfg.get("cross_attention_dim", cond_ch)) if mode == "attention" else None,
    )


# ---------------------------------------------------------------------------
# layer layout: every layer with its state_dict prefix, in execution order
# ---------------------------------------------------------------------------

def res_layer(prefix, cin, cout, *, scale_shift, emb_act, add_emb, groups=32, eps=1e-5, use_conv=False):
    return dict(kind="res", prefix=prefix, cin=cin, cout=cout, scale_shift=scale_shift,
                emb_act=emb_act, add_emb=add_emb, groups=groups, eps=eps, use_conv=use_conv)


def efficient_layout(spec: Dict[str, Any]) -> Dict[str, Any]:
    """Layer list of EfficientUNetND (reference ``src/models/unet/unet.py:70-293``)."""
    mc = spec["model_channels"]
    ss = spec["use_scale_shift_norm"]
    ea = spec["emb_act_before_proj"]
    attn = set(spec["attention_resolutions"])
    xattn = set(spec["cross_attention_resolutions"])
    pool = spec["pool_factor"]

    def attn_layers(prefix, j, ch, ds, linear):
        out = []
        if ds in attn:
            out.append(dict(kind="self_attn", prefix=f"{prefix}.{j}", ch=ch, heads=spec["num_heads"],
                            dim_head=spec["dim_head"], linear=linear))
            j += 1
        if ds in xattn:
            out.append(dict(kind="cross_attn", prefix=f"{prefix}.{j}", ch=ch, heads=spec["num_heads"],
                            dim_head=spec["dim_head"], linear=linear, ctx=spec["cross_attention_dim"]))
            j += 1
        return out, j

    start = mc if pool > 1 else spec["in_channels"]
    inputs: List[List[dict]] = [[dict(kind="conv", prefix="input_blocks.0.0.conv", cin=start, cout=mc, k=3, stride=1, pad=1)]]
    chans = [mc]
    ch = mc
    ds = 1
    for level, m in enumerate(spec["channel_mult"]):
        for _ in range(spec["num_res_blocks"]):
            p = f"input_blocks.{len(inputs)}"
            layers = [res_layer(f"{p}.0", ch, m * mc, scale_shift=ss, emb_act=ea, add_emb=False)]
            ch = m * mc
            extra, _ = attn_layers(p, 1, ch, ds, spec["use_linear_attn"])
            inputs.append(layers + extra)
            chans.append(ch)
        if level != len(spec["channel_mult"]) - 1:
            p = f"input_blocks.{len(inputs)}.0"
            inputs.append([dict(kind="down", prefix=p, ch=ch, use_conv=spec["conv_resample"])])
            chans.append(ch)
            ds *= 2
    middle = [res_layer("middle_block.0", ch, ch, scale_shift=ss, emb_act=ea, add_emb=False),
              dict(kind="self_attn", prefix="middle_block.1", ch=ch, heads=spec["num_heads"],
                   dim_head=spec["dim_head"], linear=False)]
    j = 2
    if spec["cross_attention_in_middle"] or ds in xattn:
        middle.append(dict(kind="cross_attn", prefix="middle_block.2", ch=ch, heads=spec["num_heads"],
                           dim_head=spec["dim_head"], linear=False, ctx=spec["cross_attention_dim"]))
        j = 3
    middle.append(res_layer(f"middle_block.{j}", ch, ch, scale_shift=ss, emb_act=ea, add_emb=False))
    outputs: List[List[dict]] = []
    for level, m in list(enumerate(spec["channel_mult"]))[::-1]:
        for i in range(spec["num_res_blocks"] + 1):
            p = f"output_blocks.{len(outputs)}"
            skip = chans.pop()
            layers = [res_layer(f"{p}.0", ch + skip, mc * m, scale_shift=ss, emb_act=ea, add_emb=False)]
            layers[0]["skip_ch"] = skip
            ch = mc * m
            extra, j = attn_layers(p, 1, ch, ds, spec["use_linear_attn"])
            layers += extra
            if level and i == spec["num_res_blocks"]:
                layers.append(dict(kind="up", prefix=f"{p}.{j}", ch=ch, use_conv=spec["conv_resample"]))
                ds //= 2
            outputs.append(layers)
    return dict(inputs=inputs, middle=middle, outputs=outputs, out_ch=ch, pool=pool)


def diffusers_layout(spec: Dict[str, Any]) -> Dict[str, Any]:
    """Layer list of UNetDiffusersND (reference ``unet_diffusers_nd.py:19-191``, ``legacy_unet.py``)."""
    boc = spec["block_out_channels"]
    g = spec["norm_num_groups"]
    eps = spec["norm_eps"]
    ss = spec["scale_shift"]
    hd = max(spec["attention_head_dim"], 1)
    downs = []
    out_c = boc[0]
    for i, t in enumerate(spec["down_block_types"]):
        in_c = out_c
        out_c = boc[i]
        final = i == len(boc) - 1
        with_attn = t in {"AttnDownBlock2D", "CrossAttnDownBlock2D"}
        ctx = spec["cross_attention_dim"] if t == "CrossAttnDownBlock2D" else None
        res, att = [], []
        c = in_c
        for j in range(spec["layers_per_block"]):
            res.append(res_layer(f"down_blocks.{i}.resnets.{j}", c, out_c, scale_shift=ss, emb_act=True,
                                 add_emb=True, groups=g, eps=eps))
            if with_attn:
                att.append(dict(kind="dattn", prefix=f"down_blocks.{i}.attentions.{j}", ch=out_c,
                                heads=max(1, out_c // hd), groups=g, eps=eps, ctx=ctx))
            c = out_c
        down = None if final else dict(kind="down", prefix=f"down_blocks.{i}.downsamplers.0", ch=out_c, use_conv=True)
        downs.append(dict(res=res, attn=att, down=down))
    mid = None
    if spec["mid_block_type"] is not None:
        c = boc[-1]
        ctx = spec["cross_attention_dim"] if spec["mid_block_type"] == "UNetMidBlock2DCrossAttn" else None
        mid = dict(
            res=[res_layer(f"mid_block.resnets.{j}", c, c, scale_shift=ss, emb_act=True, add_emb=True, groups=g, eps=eps)
                 for j in range(2)],
            attn=[dict(kind="dattn", prefix="mid_block.attentions.0", ch=c, heads=max(1, c // hd), groups=g,
                       eps=eps, ctx=ctx)] if spec["add_attention"] else [],
        )
    rev = list(reversed(boc))
    ups = []
    out_c = rev[0]
    for i, t in enumerate(spec["up_block_types"]):
        prev = out_c
        out_c = rev[i]
        in_c = rev[min(i + 1, len(boc) - 1)]
        final = i == len(boc) - 1
        with_attn = t in {"AttnUpBlock2D", "CrossAttnUpBlock2D"}
        ctx = spec["cross_attention_dim"] if t == "CrossAttnUpBlock2D" else None
        nl = spec["layers_per_block"] + 1
        res, att = [], []
        for j in range(nl):
            skip = in_c if j == nl - 1 else out_c
            rin = prev if j == 0 else out_c
            r = res_layer(f"up_blocks.{i}.resnets.{j}", rin + skip, out_c, scale_shift=ss, emb_act=True,
                          add_emb=True, groups=g, eps=eps)
            r["skip_ch"] = skip
            res.append(r)
            if with_attn:
                att.append(dict(kind="dattn", prefix=f"up_blocks.{i}.attentions.{j}", ch=out_c,
                                heads=max(1, out_c // hd), groups=g, eps=eps, ctx=ctx))
        up = None if final else dict(kind="up", prefix=f"up_blocks.{i}.upsamplers.0", ch=out_c, use_conv=True)
        ups.append(dict(res=res, attn=att, up=up))
    return dict(downs=downs, mid=mid, ups=ups)
