"""DDPM trainer entry point (reference ``src/pipelines/train/diffusion_lib.py:34``).

``train(dataset, json_path, val_dataset=None, resume=None)``: ``timesteps ~ randint(0, N)``,
``noisy = scheduler.add_noise(x0, eps, timesteps)`` (folded into the model-input kernel), target ``eps``
-- one FusedTrainStep(objective="ddpm") per batch; loop as ``loop.run_training``.  Checkpoints:
``diff_last.pt`` / ``diff_best.pt``."""
from __future__ import annotations

from .loop import run_training


def train(dataset, json_path, val_dataset=None, resume=None, **kw) -> None:
    run_training(dataset, json_path, val_dataset, resume, objective="ddpm", **kw)
