"""Input pipeline: LDCT tensor-cache datasets and the pinned-host -> side-stream device prefetcher."""
from .prefetch import DevicePrefetcher  # noqa: F401
from .tensor_cache import (LDCTAttentionCacheDataset, LDCTCacheDataset, TensorPairDataset,  # noqa: F401
                           cache_path_for_entry, save_tensor_cache)
