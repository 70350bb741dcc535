"""Low-level model modules (reference ``src/nn/modules``)."""
