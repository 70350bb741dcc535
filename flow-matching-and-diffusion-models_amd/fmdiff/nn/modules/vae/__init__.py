"""VAE modules (reference ``src/nn/modules/vae/__init__.py``): encoder, decoder, diagonal Gaussian.

The codebooks and discriminators of the reference (VQ-VAE / GAN training) are outside the hot path
(DESIGN.md section 7)."""
from .decoder import Decoder
from .encoder import Encoder
from .reparameterizer import DiagonalGaussian

__all__ = ["Encoder", "Decoder", "DiagonalGaussian"]
