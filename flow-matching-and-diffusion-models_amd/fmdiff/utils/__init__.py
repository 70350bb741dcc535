"""Run-level helpers mirroring the reference's ``src/utils`` (training_utils, model_utils)."""
from .training_utils import (allocate_run_dir, get_rank, get_world_size, is_distributed, is_main_process,  # noqa: F401
                             load_json_config, maybe_load_checkpoint, resolve_batch_size, resolve_device,
                             save_checkpoint, save_json_config, set_seed, setup_distributed)
