"""``AutoencoderKL`` (reference ``src/models/vae/kl.py:22-140``): same constructor, attributes and state_dict
keys.  ``encode`` / ``decode`` run the encoder (+ quant_conv folded into its output conv) and the
decoder (post_quant_conv, then the decoder) through the fused HIP engine (``fmdiff.runtime.vae_engine``);
the inference path of config D: encode -> latent denoise -> decode."""
from __future__ import annotations

import os
import warnings
from typing import Optional, Tuple, Union

import torch

from ...nn.modules.vae import Decoder, DiagonalGaussian, Encoder
from ...nn.ops.convolution import ConvND
from .base import BaseVAE

LATENT_SCALE: float = 0.18215


class AutoencoderKL(BaseVAE):
    def __init__(self, in_channels: int = 3, out_channels: int = 3, resolution: int = 256, base_ch: int = 128,
                 ch_mult: Tuple[int, ...] = (1, 2, 4, 4), down_channels: Tuple[int, ...] | None = None,
                 num_res_blocks: int = 2, attn_resolutions: Tuple[int, ...] = (), z_channels: int = 4,
                 embed_dim: int = 4, dropout: float = 0.0, use_attention: bool = True, attn_heads: int = 4,
                 attn_dim_head: int = 64, spatial_dims: int = 2, emb_channels: Optional[int] = None,
                 use_scale_shift_norm: bool = False, norm_groups: Optional[int] = None,
                 codebook_size: Optional[int] = None, num_embeddings: Optional[int] = None,
                 ckpt_path: Optional[str] = None, double_z: bool = True, block_factory=None) -> None:
        super().__init__()
        self.spatial_dims = spatial_dims
        common = dict(base_ch=base_ch, ch_mult=ch_mult, down_channels=down_channels, num_res_blocks=num_res_blocks,
                      attn_resolutions=attn_resolutions, resolution=resolution, z_channels=z_channels,
                      dropout=dropout, use_attention=use_attention, attn_heads=attn_heads,
                      attn_dim_head=attn_dim_head, spatial_dims=spatial_dims, emb_channels=emb_channels,
                      use_scale_shift_norm=use_scale_shift_norm, norm_groups=norm_groups,
                      block_factory=block_factory)
        self.encoder = Encoder(in_channels=in_channels, double_z=double_z, **common)
        self.decoder = Decoder(out_ch=out_channels, tanh_out=False, **common)
        self.quant_conv = ConvND(spatial_dims, 2 * z_channels, 2 * embed_dim, 1, padding=0)
        self.post_quant_conv = ConvND(spatial_dims, embed_dim, z_channels, 1, padding=0)
        self.embed_dim = embed_dim
        self.num_embeddings = num_embeddings
        self.codebook_size = codebook_size
        if ckpt_path:
            if not os.path.exists(ckpt_path):
                raise FileNotFoundError(f"Checkpoint not found: {ckpt_path}")
            self.load_state_dict(torch.load(ckpt_path, map_location="cpu", weights_only=True))
        else:
            warnings.warn("[AutoencoderKL] No checkpoint provided. Random initialization.")

    def encode(self, x: torch.Tensor, normalize: bool = False) -> Union[DiagonalGaussian, torch.Tensor]:
        from ...runtime.vae_engine import get_vae_engine
        moments = get_vae_engine(self).encode_moments(x)
        posterior = DiagonalGaussian(moments)
        if normalize:
            return posterior.mode() * LATENT_SCALE
        return posterior

    def decode(self, z: torch.Tensor, denorm: bool = False) -> torch.Tensor:
        from ...runtime.vae_engine import get_vae_engine
        if denorm:
            z = z / LATENT_SCALE
        return get_vae_engine(self).decode(z)

    def forward(self, x: torch.Tensor, sample_posterior: bool = True):
        posterior = self.encode(x, normalize=False)
        z = posterior.sample() if sample_posterior else posterior.mode()
        return self.decode(z, denorm=False), posterior
