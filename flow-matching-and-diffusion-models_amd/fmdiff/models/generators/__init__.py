from .diffusionfactory import DiffusionUNetFactory

__all__ = ["DiffusionUNetFactory"]
