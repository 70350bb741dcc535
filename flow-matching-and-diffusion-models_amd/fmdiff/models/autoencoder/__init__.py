from .base import BaseAutoencoder

__all__ = ["BaseAutoencoder"]
