"""Latent helpers of config D: the reference's ``encode_vae_batch`` /
``decode_vae_batch`` (``src/utils/model_utils/vae_utils.py:54-85``) and the encode -> denoise -> decode
composition the reference performs across ``encode_vae_batch`` + ``sample_with_scheduler`` +
``decode_vae_batch`` (it has no single pipeline object).  The VAE runs on the fused HIP engine
(``fmdiff.runtime.vae_engine``), the latent sampler on ``FusedFlowSampler``."""
from __future__ import annotations

from typing import Optional

import torch


def encode_vae_batch(model, inputs: torch.Tensor) -> torch.Tensor:
    """Image batch in [0, 1] -> latent ``posterior.mode()`` (vae_utils.py:54-68)."""
    posterior = model.encode(model.image_to_model_range(inputs), normalize=False)
    return posterior.mode()


def decode_vae_batch(model, latents: torch.Tensor, recon_type: str = "l1") -> torch.Tensor:
    """Latent batch -> images in [0, 1] (vae_utils.py:71-85)."""
    return model.raw_output_to_image(model.decode(latents, denorm=False), recon_type=recon_type)


@torch.no_grad()
def latent_flow_sample(vae, sampler, cond_images: torch.Tensor, noise: Optional[torch.Tensor] = None,
                       use_graph: bool = True) -> torch.Tensor:
    """encode the conditioning images -> FM-Euler sampling in latent space (concatenate conditioning) ->
    decode.  ``sampler`` is a ``FusedFlowSampler`` over a latent UNet whose in_channels = 2 * embed_dim."""
    cond = encode_vae_batch(vae, cond_images).contiguous()
    if noise is None:
        noise = torch.randn_like(cond)
    lat = sampler.sample(noise, cond, use_graph=use_graph)
    return decode_vae_batch(vae, lat)
