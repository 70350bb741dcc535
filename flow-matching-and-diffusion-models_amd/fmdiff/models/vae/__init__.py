"""VAE models (reference ``src/models/vae/__init__.py``).  ``VQVAE`` (codebook training) is out of scope."""
from .base import BaseVAE
from .kl import LATENT_SCALE, AutoencoderKL

__all__ = ["BaseVAE", "AutoencoderKL", "LATENT_SCALE"]
