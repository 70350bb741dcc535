"""``BaseVAE`` (reference ``src/models/vae/base.py:12-26``)."""
from __future__ import annotations

import abc

from ..autoencoder import BaseAutoencoder


class BaseVAE(BaseAutoencoder, metaclass=abc.ABCMeta):
    def make_discriminator(self):
        raise NotImplementedError("GAN discriminators (VAE training) are outside the fmdiff hot path")
