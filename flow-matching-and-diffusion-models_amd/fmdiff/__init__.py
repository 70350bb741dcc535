"""fmdiff: MI355X-native (gfx950) flow-matching / diffusion UNet train + sample engine.

Mirrors the reference's ``src/nn``, ``src/models``, ``src/pipelines`` APIs; the
compute runs in hand-written HIP kernels (``csrc/``) behind a C ABI
(``include/fmdiff.h``)."""
__version__ = "0.1.0"
