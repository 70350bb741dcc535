"""Run-level helpers of the trainers (reference: ``src/utils/training_utils.py``).

Same names, arguments and behaviour as the reference's helpers the FM / DDPM trainers call:
config I/O with the ``__config_path__`` marker (``:39-55``), ``_runN`` run directories
(``:57-74``), seeding (``:77-85``), device resolution honouring ``LOCAL_RANK`` (``:88-98``), the
``train_batch_size`` -> ``batch_size`` fallback (``:101-109``), checkpoint save / resume
(``:198-202``, ``:235-256``) and the env:// process-group bring-up (``:209-232``).  One deliberate
difference: ``resolve_device`` also makes the chosen GPU current (``torch.cuda.set_device``), which
the reference never does, so every HIP launch of a rank lands on its own GPU.
"""
from __future__ import annotations

import json
import logging
import os
import random
import re
from pathlib import Path
from typing import Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

__all__ = ["load_json_config", "save_json_config", "allocate_run_dir", "set_seed", "resolve_device",
           "resolve_batch_size", "save_checkpoint", "maybe_load_checkpoint", "setup_distributed",
           "is_distributed", "is_main_process", "get_rank", "get_world_size"]


def load_json_config(path) -> dict:
    """JSON config as a dict, with ``__config_path__`` recording where it came from."""
    path = Path(path)
    if not path.exists():
        raise FileNotFoundError(f"Config not found: {path}")
    cfg = json.loads(path.read_text())
    if isinstance(cfg, dict):
        cfg["__config_path__"] = str(path)
    return cfg


def save_json_config(path, cfg: dict) -> None:
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    path.write_text(json.dumps(cfg, indent=2))


def allocate_run_dir(base) -> Path:
    """Next free ``<base>_runN`` sibling of ``base`` (N = 1 + the largest existing)."""
    base = Path(base)
    base.parent.mkdir(parents=True, exist_ok=True)
    rx = re.compile(rf"^{re.escape(base.name)}_run(\d+)$")
    taken = [int(m.group(1)) for e in base.parent.iterdir() if e.is_dir() for m in [rx.match(e.name)] if m]
    return base.parent / f"{base.name}_run{max(taken, default=0) + 1}"


def set_seed(seed) -> None:
    if seed is None:
        return
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def resolve_device(value, default: torch.device) -> torch.device:
    """``training.manual_device`` if set, else ``cuda:LOCAL_RANK`` under torchrun, else ``default``."""
    if value is None or (isinstance(value, str) and value.lower() == "none"):
        local = os.environ.get("LOCAL_RANK")
        dev = torch.device("cuda", int(local)) if (local is not None and torch.cuda.is_available()) else default
    else:
        dev = value if isinstance(value, torch.device) else torch.device(value)
    if dev.type == "cuda" and torch.cuda.is_available():
        torch.cuda.set_device(dev if dev.index is not None else torch.device("cuda", 0))
    return dev


def resolve_batch_size(training_cfg: dict, key: str, fallback) -> int:
    """``train_batch_size`` falls back to ``batch_size`` (the key without ``train_``), then to ``fallback``."""
    value = training_cfg.get(key)
    if value is None:
        value = training_cfg.get(key[len("train_"):] if key.startswith("train_") else key, fallback)
    return int(value)


def save_checkpoint(state: dict, path) -> None:
    """Write ``state`` with torch.save (atomic: temporary file + rename, so a crash never leaves half a file)."""
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    tmp = path.with_name(path.name + ".tmp")
    torch.save(state, tmp)
    os.replace(tmp, path)


def setup_distributed(backend: Optional[str] = None) -> bool:
    """env:// process group when ``WORLD_SIZE`` > 1 (torchrun); ``nccl`` (RCCL on ROCm) on GPUs, else gloo."""
    if not dist.is_available():
        return False
    if dist.is_initialized():
        return True
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return False
    dist.init_process_group(backend=backend or ("nccl" if torch.cuda.is_available() else "gloo"))
    return True


def is_distributed() -> bool:
    return dist.is_available() and dist.is_initialized()


def is_main_process() -> bool:
    return not is_distributed() or dist.get_rank() == 0


def get_rank() -> int:
    return dist.get_rank() if is_distributed() else 0


def get_world_size() -> int:
    return dist.get_world_size() if is_distributed() else 1


def maybe_load_checkpoint(path, prefix: str, model, optimizer=None, scheduler=None, scaler=None) -> Tuple[int, float]:
    """Restore ``model`` (and the optimizer / LR scheduler / scaler objects given) from a trainer checkpoint;
    returns (start_epoch, best_metric) = (saved epoch + 1, saved best), or (1, inf) if there is none.

    ``optimizer`` may be a fused train step (anything with ``load_optimizer_state_dict``): then the AdamW
    moments and the step count come from the checkpoint's torch-format ``optimizer`` / ``lr_scheduler``
    entries, whichever trainer wrote them."""
    if path is None:
        return 1, float("inf")
    path = Path(path)
    if not path.exists():
        logging.warning("%s checkpoint not found: %s", prefix, path)
        return 1, float("inf")
    payload = torch.load(path, map_location="cpu", weights_only=True)
    model.load_state_dict(payload["model"])
    if optimizer is not None and payload.get("optimizer"):
        if hasattr(optimizer, "load_optimizer_state_dict"):
            optimizer.load_optimizer_state_dict(payload["optimizer"], payload.get("lr_scheduler"))
        else:
            optimizer.load_state_dict(payload["optimizer"])
    if scheduler is not None and payload.get("lr_scheduler"):
        scheduler.load_state_dict(payload["lr_scheduler"])
    if scaler is not None and payload.get("scaler"):
        scaler.load_state_dict(payload["scaler"])
    start = int(payload.get("epoch", 0)) + 1
    best = payload.get("best_metric", float("inf"))
    logging.info("Resumed %s trainer from %s (epoch %d)", prefix, path, start - 1)
    return start, float(best)
