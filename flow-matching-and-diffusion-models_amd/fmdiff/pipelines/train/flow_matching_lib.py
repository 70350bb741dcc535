"""Flow-matching trainer entry point (reference ``src/pipelines/train/flow_matching_lib.py:33``).

``train(dataset, json_path, val_dataset=None, resume=None)``: ``x_t = (1 - t) x0 + t eps``,
``timesteps = (t * (N - 1)).long()``, target ``eps - x0`` -- one FusedTrainStep per batch; the loop,
sharding, checkpoints and metrics are ``loop.run_training``.  Checkpoints: ``flow_last.pt`` /
``flow_best.pt``."""
from __future__ import annotations

from .loop import run_training


def train(dataset, json_path, val_dataset=None, resume=None, **kw) -> None:
    run_training(dataset, json_path, val_dataset, resume, objective="flow_matching", **kw)
