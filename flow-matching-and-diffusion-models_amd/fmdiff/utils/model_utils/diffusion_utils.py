"""Model factory and sampling entry points of the trainers / samplers
(reference: ``src/utils/model_utils/diffusion_utils.py``).

* ``build_diffusion_model`` (``:93-144``): config -> ``DiffusionUNetFactory`` model on the device, optional
  checkpoint (torch ``{"model": ...}`` payload, bare state_dict or ``.safetensors``), with the legacy
  diffusers key remap (``:15-90``) either on request (``unet.load_legacy``) or as the fallback when the
  plain load fails.  Checkpoints are read with ``weights_only=True`` only.
* ``decode_diffusion_batch`` (``:165-245``): scheduler from the config (+ ``run_model --scheduler``
  override), tail selection, optional noised-reference init, then ``sample_with_scheduler`` on the HIP
  engine.  On an fmdiff UNet with any scheduler that has a HIP step (FlowMatchEuler, DDPM, DDIM,
  DPM-Solver(++), UniPC) the loop -- whole schedule or its selected tail -- is the graph-replayed
  ``FusedSampler`` (the generic loop's arithmetic, one host launch per step; DDPM's variance noise drawn
  up front), unless ``use_fused=False``.
* ``encode_diffusion_batch`` (``:147-162``), ``prepare_diffusion_visual_batch`` (``:273-300``),
  ``select_visual_indices`` (``src/utils/indexing_utils.py:6-28``), ``warn_attention_conditioning_shape``.
"""
from __future__ import annotations

import logging
import random
from typing import Dict, Optional

import torch

from ...models.generators import DiffusionUNetFactory
from ...pipelines.utils import (build_scheduler, resolve_conditioning_mode, resolve_scheduler_override,
                                sample_with_scheduler, select_timesteps)

# diffusers / legacy UNet parameter names -> this model tree's names (reference diffusion_utils.py:15-43)
_LEGACY_RENAMES = (
    (".query.", ".to_q."), (".key.", ".to_k."), (".value.", ".to_v."), (".proj_attn.", ".to_out.0."),
    (".conv1.weight", ".conv1.conv.weight"), (".conv1.bias", ".conv1.conv.bias"),
    (".conv2.weight", ".conv2.conv.weight"), (".conv2.bias", ".conv2.conv.bias"),
    (".time_emb_proj.weight", ".emb_layers.weight"), (".time_emb_proj.bias", ".emb_layers.bias"),
    (".conv_shortcut.weight", ".skip_connection.conv.weight"), (".conv_shortcut.bias", ".skip_connection.conv.bias"),
    (".downsamplers.0.conv.weight", ".downsamplers.0.op.conv.weight"),
    (".downsamplers.0.conv.bias", ".downsamplers.0.op.conv.bias"),
    (".upsamplers.0.conv.weight", ".upsamplers.0.conv.conv.weight"),
    (".upsamplers.0.conv.bias", ".upsamplers.0.conv.conv.bias"),
)


def _remap_legacy_unet_keys(state_dict: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """Rename diffusers-style keys (every rule applied in order to every key; shapes untouched)."""
    out = {}
    for key, value in state_dict.items():
        for old, new in _LEGACY_RENAMES:
            key = key.replace(old, new)
        out[key] = value
    return out


def _load_legacy_unet_state(model: torch.nn.Module, state: Dict[str, torch.Tensor], strict_shapes: bool = True):
    """Load a remapped legacy state: exact-shape tensors only; with ``strict_shapes`` any shape mismatch or
    missing / unexpected key is an error naming the counts (reference ``:46-90``)."""
    state = _remap_legacy_unet_keys(state)
    own = model.state_dict()
    matched, bad_shape = {}, []
    for k, v in state.items():
        if k not in own:
            continue
        if tuple(v.shape) != tuple(own[k].shape):
            bad_shape.append(f"{k}: ckpt={tuple(v.shape)} model={tuple(own[k].shape)}")
        else:
            matched[k] = v
    unexpected = [k for k in state if k not in own]
    missing = [k for k in own if k not in matched]
    if strict_shapes and bad_shape:
        msg = "Legacy load failed due to shape mismatches:\n" + "\n".join(bad_shape[:20])
        if len(bad_shape) > 20:
            msg += f"\n... and {len(bad_shape) - 20} more"
        raise RuntimeError(msg)
    model.load_state_dict(matched, strict=False)
    if strict_shapes and (missing or unexpected):
        parts = ([f"missing={len(missing)}"] if missing else []) + ([f"unexpected={len(unexpected)}"] if unexpected
                                                                     else [])
        raise RuntimeError("Legacy load key mismatch after conversion (" + ", ".join(parts) + "). "
                           "Architecture/config likely differs from the source checkpoint.")


def _read_state(ckpt_path: str, device) -> Dict[str, torch.Tensor]:
    if ckpt_path.endswith(".safetensors"):
        from safetensors.torch import load_file
        return load_file(ckpt_path, device="cpu")
    payload = torch.load(ckpt_path, map_location="cpu", weights_only=True)
    return payload["model"] if isinstance(payload, dict) and "model" in payload else payload


def build_diffusion_model(cfg: dict, device, ckpt_path=None, set_eval: bool = True):
    """UNet of ``cfg["model"]["unet"]`` (conditioning from the training block, channels =
    ``training.channels`` or ``unet.out_channels`` or 1) on ``device``, optionally loaded from a checkpoint."""
    tr = cfg["training"]
    unet_cfg = cfg["model"].get("unet", {})
    mode = resolve_conditioning_mode(tr.get("conditioning") or cfg["model"].get("conditioning"))
    channels = int(tr.get("channels", unet_cfg.get("out_channels", 1)) or 1)
    model = DiffusionUNetFactory().build(unet_cfg, mode, channels).to(device)
    if ckpt_path is not None:
        state = _read_state(str(ckpt_path), device)
        strict = bool(unet_cfg.get("legacy_strict_shapes", True))
        if bool(unet_cfg.get("load_legacy", False)):
            _load_legacy_unet_state(model, state, strict_shapes=strict)
        else:
            try:
                model.load_state_dict(state)
            except RuntimeError:   # external diffusers-style checkpoint: same shapes, other names
                _load_legacy_unet_state(model, state, strict_shapes=strict)
    if set_eval:
        model.eval()
    return model


def encode_diffusion_batch(scheduler, targets: torch.Tensor, timesteps: torch.Tensor) -> torch.Tensor:
    """Forward-noise ``targets`` at ``timesteps`` (scheduler.add_noise with fresh Gaussian noise)."""
    return scheduler.add_noise(targets, torch.randn_like(targets), timesteps)


def _fused_ok(model, scheduler, use_fused) -> bool:
    """The graph-replayed sampler (FusedSampler) serves every scheduler with a HIP step on an fmdiff UNet."""
    from ...models.unet.base import BaseUNetND
    from ...pipelines.schedulers import (DDIMScheduler, DDPMScheduler, DPMSolverMultistepScheduler,
                                         FlowMatchEulerDiscreteScheduler, UniPCMultistepScheduler)
    if isinstance(scheduler, UniPCMultistepScheduler) and int(scheduler.config.solver_order) > 3:
        return False   # the table step (fmd_sched_step) holds <= 3 history coefficients; the eager step any order
    return use_fused and isinstance(model, BaseUNetND) and isinstance(scheduler, (
        FlowMatchEulerDiscreteScheduler, DDPMScheduler, DDIMScheduler, DPMSolverMultistepScheduler,
        UniPCMultistepScheduler))


def decode_diffusion_batch(model, training_cfg: dict, model_cfg: dict, device, batch_shape,
                           conditioning_batch: Optional[torch.Tensor] = None, timing: Optional[dict] = None,
                           num_inference_steps: Optional[int] = None, start_step: Optional[int] = None,
                           last_n_steps: Optional[int] = None, reference_batch: Optional[torch.Tensor] = None,
                           init_from_reference: bool = False, scheduler_override: Optional[str] = None,
                           use_fused: bool = True) -> torch.Tensor:
    """Sample a batch with the model's configured scheduler (reference ``diffusion_utils.py:165-245``)."""
    sch_cfg = dict(model_cfg.get("scheduler", {}))
    ov = resolve_scheduler_override(scheduler_override)
    if ov is not None:
        sch_cfg["name"] = ov["name"]
        sch_cfg["params"] = {**dict(sch_cfg.get("params", {})), **dict(ov.get("params", {}))}
    scheduler, n_inf = build_scheduler(sch_cfg, training_cfg)
    if num_inference_steps is not None:
        n_inf = int(num_inference_steps)
    scheduler.set_timesteps(n_inf)
    selected = scheduler.timesteps
    if start_step is not None:
        selected = selected[selected <= int(start_step)]
    if last_n_steps is not None:
        selected = selected[-int(last_n_steps):]
    init = None
    if init_from_reference and reference_batch is not None:
        if selected.numel() == 0:
            raise ValueError("No timesteps selected after applying start_step/last_n_steps.")
        if hasattr(scheduler, "add_noise"):
            ts = selected[0].expand(reference_batch.size(0)).to(reference_batch.device)
            init = scheduler.add_noise(reference_batch, torch.randn_like(reference_batch), ts).to(device)
        else:
            logging.warning("Requested init_from_reference but scheduler '%s' has no add_noise; falling back to "
                            "random init.", scheduler.__class__.__name__)
    mode = resolve_conditioning_mode(training_cfg.get("conditioning") or model_cfg.get("conditioning"))
    latent_norm = training_cfg.get("latent_norm")
    if _fused_ok(model, scheduler, use_fused) and mode in (None, "concatenate", "attention"):
        start = len(scheduler.timesteps) - len(select_timesteps(scheduler.timesteps, start_step, last_n_steps))
        return _fused_decode(model, scheduler, n_inf, batch_shape, device, mode, conditioning_batch, latent_norm,
                             init, start, timing)
    return sample_with_scheduler(model, scheduler, n_inf, batch_shape, device, conditioning_mode=mode,
                                 conditioning_batch=conditioning_batch, latent_norm=latent_norm, timing=timing,
                                 start_step=start_step, last_n_steps=last_n_steps, init_sample=init)


def _fused_decode(model, scheduler, n_inf, batch_shape, device, mode, cond, latent_norm, init, start, timing):
    """The schedule (or its selected tail, from step ``start``) as one graph-replayed step (FusedSampler): the
    generic loop's arithmetic with the conditioning aligned / normalised the same way, one host launch per
    step; ``timing`` gets the loop's model_seconds / model_calls."""
    from ...pipelines.train.fused import FusedSampler
    from ...pipelines.utils import _align_conditioning, normalize_latent_conditioning
    init = init.to(device) if init is not None else torch.randn(batch_shape, device=device)
    cond = _align_conditioning(cond, init.size(0))
    cat = cca = None
    if mode == "concatenate" and cond is not None:
        cat = cond.to(device)
    elif mode == "attention" and cond is not None:
        cca = normalize_latent_conditioning(cond.to(device), latent_norm)
    sampler = FusedSampler(model, scheduler, n_inf, start=start)
    return sampler.sample(init, cat, use_graph=True, context_ca=cca, timing=timing)


def warn_attention_conditioning_shape(conditioning_batch: Optional[torch.Tensor], model_cfg: dict) -> bool:
    """Warn (and return True) when the attention conditioning's channels differ from unet.cross_attention_dim."""
    if conditioning_batch is None or conditioning_batch.dim() < 2:
        return False
    expected = (model_cfg.get("unet", {}) if isinstance(model_cfg, dict) else {}).get("cross_attention_dim")
    if expected is None or int(conditioning_batch.shape[1]) == int(expected):
        return False
    logging.warning("Attention conditioning has %d channels, but model unet.cross_attention_dim is %d. This often "
                    "means the evaluation split is pointing at pixel conditioning instead of the expected latent "
                    "conditioning.", int(conditioning_batch.shape[1]), int(expected))
    return True


def select_visual_indices(ds, count: int, seed: Optional[int] = None) -> list:
    """One random slice per case for up to ``count`` cases (rows with a Case / case / case_id), else a random
    subset (reference ``src/utils/indexing_utils.py:6-28``)."""
    total = len(ds)
    if total <= 0:
        return []
    rng = random.Random(seed)
    picked = []
    rows = getattr(ds, "data", None)
    if isinstance(rows, list):
        by_case = {}
        for i, row in enumerate(rows):
            cid = row.get("Case") or row.get("case") or row.get("case_id")
            if cid is not None:
                by_case.setdefault(cid, []).append(i)
        if by_case:
            ids = list(by_case)
            rng.shuffle(ids)
            picked = [rng.choice(by_case[c]) for c in ids[:count]]
    if not picked:
        picked = list(range(total))
        rng.shuffle(picked)
        picked = picked[:count]
    return picked


def prepare_diffusion_visual_batch(dataset, count: int, device, seed: Optional[int] = None):
    """(targets, conditioning or None) stacked from ``select_visual_indices`` samples."""
    items = [dataset[i] for i in select_visual_indices(dataset, count, seed=seed)]
    targets = torch.stack([it["target"] for it in items]).to(device)
    conds = [it.get("image") for it in items]
    cond = torch.stack(conds).to(device) if conds and all(c is not None for c in conds) else None
    return targets, cond
