"""``DiffusionUNetFactory`` (reference ``src/models/generators/diffusionfactory.py:25-130``).

Maps a JSON ``model.unet`` block to an EfficientUNetND / UNetDiffusersND with
the reference's defaulting rules, so ``configs/*.json`` are drop-in."""
from __future__ import annotations

from typing import Any, Dict, Iterable, Sequence

from ..unet import EfficientUNetND, UNetDiffusersND

__all__ = ["DiffusionUNetFactory"]


def _to_tuple(value: Iterable[int] | int | None, default: tuple) -> tuple:
    if value is None:
        return default
    if isinstance(value, int):
        return (value,)
    return tuple(value)


def _infer_channel_mult(block_out_channels: Sequence[int], base_channels: int) -> tuple:
    if not block_out_channels:
        return ()
    base = base_channels or block_out_channels[0]
    return tuple(max(1, int(ch // base)) for ch in block_out_channels)


class DiffusionUNetFactory:
    DEFAULT_BLOCK_CHANNELS = (128, 128, 256, 256, 512, 512)
    DIFFUSERS_IMPLS = {"diffusers_nd", "diffusers_exact_nd", "exact_nd", "diffusers"}

    def build(self, model_cfg: Dict[str, Any], conditioning: str | None = None, channels: int | None = None):
        cfg = dict(model_cfg or {})
        impl = str(cfg.get("unet_impl", "efficient_nd")).lower()
        if impl in self.DIFFUSERS_IMPLS:
            return self._build_diffusers_nd(cfg, conditioning, channels)
        return self._build_efficient_nd(cfg, conditioning, channels)

    def _build_efficient_nd(self, cfg, conditioning=None, channels=None):
        boc = _to_tuple(cfg.get("block_out_channels"), self.DEFAULT_BLOCK_CHANNELS)
        mc = int(cfg.get("model_channels", boc[0] if boc else 128))
        in_ch = cfg.get("in_channels", channels or 1)
        cond_ch = cfg.get("conditioning_channels", channels or in_ch)
        mode = (conditioning or "").lower()
        if mode == "concatenate":
            in_ch = in_ch + cond_ch
        attn = _to_tuple(cfg.get("attention_resolutions"), (1,))
        xres = cfg.get("cross_attention_resolutions")
        x_mid = bool(cfg.get("cross_attention_in_middle", False))
        if xres is None and mode == "attention":
            xres = attn
            if "cross_attention_in_middle" not in cfg:
                x_mid = True
        return EfficientUNetND(
            spatial_dims=int(cfg.get("spatial_dims", 2)), in_channels=in_ch, model_channels=mc,
            out_channels=cfg.get("out_channels", channels or 1),
            num_res_blocks=int(cfg.get("num_res_blocks", cfg.get("layers_per_block", 2))),
            attention_resolutions=attn, cross_attention_resolutions=xres,
            cross_attention_dim=int(cfg.get("cross_attention_dim", cond_ch)), cross_attention_in_middle=x_mid,
            dropout=float(cfg.get("dropout", 0.0)),
            channel_mult=_to_tuple(cfg.get("channel_mult"), _infer_channel_mult(boc, mc)) or (1, 2, 3, 4),
            conv_resample=bool(cfg.get("conv_resample", True)), dim_head=int(cfg.get("dim_head", 64)),
            num_heads=int(cfg.get("num_heads", 4)), use_linear_attn=bool(cfg.get("use_linear_attn", True)),
            use_scale_shift_norm=bool(cfg.get("use_scale_shift_norm", True)),
            emb_activation_before_proj=bool(cfg.get("emb_activation_before_proj", False)),
            pool_factor=int(cfg.get("pool_factor", 1)))

    def _build_diffusers_nd(self, cfg, conditioning=None, channels=None):
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
        return UNetDiffusersND(
            spatial_dims=int(cfg.get("spatial_dims", 2)), sample_size=cfg.get("sample_size"), in_channels=in_ch,
            out_channels=int(cfg.get("out_channels", channels or 1)),
            center_input_sample=bool(cfg.get("center_input_sample", False)),
            time_embedding_type=str(cfg.get("time_embedding_type", "positional")),
            freq_shift=int(cfg.get("freq_shift", 0)), flip_sin_to_cos=bool(cfg.get("flip_sin_to_cos", True)),
            down_block_types=cfg.get("down_block_types", dd), mid_block_type=cfg.get("mid_block_type", dm),
            up_block_types=cfg.get("up_block_types", du),
            block_out_channels=_to_tuple(cfg.get("block_out_channels"), (224, 448, 672, 896)),
            layers_per_block=int(cfg.get("layers_per_block", 2)),
            downsample_padding=int(cfg.get("downsample_padding", 1)), dropout=float(cfg.get("dropout", 0.0)),
            attention_head_dim=int(cfg.get("attention_head_dim", 8)),
            norm_num_groups=int(cfg.get("norm_num_groups", 32)), norm_eps=float(cfg.get("norm_eps", 1e-5)),
            resnet_time_scale_shift=str(cfg.get("resnet_time_scale_shift", "default")),
            add_attention=bool(cfg.get("add_attention", True)),
            cross_attention_dim=int(cfg.get("cross_attention_dim", cond_ch)) if mode == "attention" else None)
