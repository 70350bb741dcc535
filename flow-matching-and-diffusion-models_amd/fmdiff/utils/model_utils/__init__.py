"""Model construction / sampling helpers (reference ``src/utils/model_utils``)."""
from .diffusion_utils import (build_diffusion_model, decode_diffusion_batch, encode_diffusion_batch,  # noqa: F401
                              prepare_diffusion_visual_batch, select_visual_indices,
                              warn_attention_conditioning_shape)
