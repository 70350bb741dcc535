"""The FM / DDPM trainer loop shared by ``flow_matching_lib.train`` and ``diffusion_lib.train``.

Reference: ``src/pipelines/train/flow_matching_lib.py:33-248`` and ``diffusion_lib.py:34-250`` (the two
differ only in the objective, checkpoint prefix and log wording).  Kept from the reference:

* config parsing with its fallbacks (``train_batch_size`` -> ``batch_size`` -> 4, ``num_epochs`` ->
  ``epochs`` -> 1, ``lr_warmup_steps`` 500, ``gradient_accumulation_steps``, ``conditioning`` from the
  training or model block, ``latent_norm``), ``_runN`` run directories and ``train_config.json``;
* ``setup_distributed`` + ``DistributedSampler(shuffle=True)`` with ``set_epoch(epoch)`` each epoch, and
  the LR horizon ``epochs * ceil(len(dataset) / batch_size)`` (the GLOBAL dataset length, as upstream);
* the per-chunk loss bookkeeping ``epoch_loss += loss * chunk_size`` and the two epoch-end SUM
  all-reduces (loss, sample count) that give every rank the global mean;
* ``{prefix}_last.pt`` / ``{prefix}_best.pt`` / ``epochs/epochNNNN/epoch.pt`` checkpoints with the
  ``{model, optimizer, lr_scheduler, scaler, epoch, best_metric}`` payload (torch AdamW / LambdaLR
  state-dict formats, so either trainer resumes the other's checkpoint), ``metrics.csv``
  (``epoch,train_loss``), rank-0-only I/O, ``resume`` / ``training.resume``;
* visual grids every ``save_images_every`` epochs (``decode_diffusion_batch`` of ``visual_samples`` images).

Changed, MI355X-first: the step is ``FusedTrainStep`` (HIP UNet forward/backward, fused AdamW +
cosine LR on the device, gradients all-reduced over RCCL -- the reference has no gradient sync, SURVEY
§0.4), replayed from a hipGraph for full batches; the epoch loss accumulates on the device (no per-chunk
``loss.item()`` host sync); batches arrive through ``DevicePrefetcher`` (pinned host -> side stream).
"""
from __future__ import annotations

import logging
import math
from pathlib import Path
from typing import Callable, Optional

import torch
import torch.distributed as dist
from torch.utils.data import DataLoader
from torch.utils.data.distributed import DistributedSampler

from ... import utils as U
from ...utils.model_utils import build_diffusion_model, decode_diffusion_batch, prepare_diffusion_visual_batch
from ..utils import (_prepare_attention_context, build_scheduler, normalize_latent_conditioning,
                     resolve_conditioning_mode)

_KIND = {  # objective -> (model_type, checkpoint prefix, default output dir, log name)
    "flow_matching": ("flow_matching", "flow", "checkpoints/flow_matching", "FlowMatch"),
    "ddpm": ("diffusion", "diff", "checkpoints/diffusion", "Diffusion"),
}


def default_step_factory(model, **kw):
    from .fused import FusedTrainStep
    return FusedTrainStep(model, **kw)


def _broadcast_path(path: Optional[Path]) -> Path:
    """Rank 0's run directory on every rank (each rank allocating its own ``_runN`` could disagree)."""
    if not U.is_distributed():
        return path
    box = [str(path) if path is not None else None]
    dist.broadcast_object_list(box, src=0)
    return Path(box[0])


def _save_grid(t: torch.Tensor, path: Path) -> None:
    """Square-ish PNG grid of [N, C, H, W] images in [0, 1] (reference evaluation_utils.make_grid/save_image)."""
    import numpy as np
    from PIL import Image
    n = t.shape[0]
    rows = max(1, int(math.sqrt(n)))
    cols = max(1, n // rows)
    x = t[: rows * cols].detach().float().clamp(0, 1).cpu()
    if x.shape[1] == 1:
        x = x.expand(-1, 3, -1, -1)
    c, h, w = x.shape[1:]
    grid = x.reshape(rows, cols, c, h, w).permute(2, 0, 3, 1, 4).reshape(c, rows * h, cols * w)
    path.parent.mkdir(parents=True, exist_ok=True)
    Image.fromarray((grid.numpy() * 255.0).clip(0, 255).astype(np.uint8).transpose(1, 2, 0)).save(path)


def run_training(dataset, json_path, val_dataset=None, resume: Optional[str] = None, *, objective: str,
                 step_factory: Optional[Callable] = None, use_graph: Optional[bool] = None):
    """Train on ``dataset`` (items: dicts with ``target`` [C,*S] and ``image`` (conditioning or = target))."""
    model_type = _KIND[objective][0]
    logging.basicConfig(level=logging.INFO, format="%(asctime)s | %(levelname)s | %(message)s", force=True)
    cfg = U.load_json_config(json_path)
    if "model" not in cfg:
        raise ValueError("Config does not declare a 'model' section.")
    mblock = cfg["model"]
    mt = str(mblock.get("model_type", "")).lower()
    if mt != model_type:
        raise ValueError(f"Expected model_type '{model_type}', got '{mt}'.")
    tr = cfg["training"]

    U.setup_distributed(tr.get("dist_backend"))
    U.set_seed(tr.get("seed"))
    device = U.resolve_device(tr.get("manual_device"), torch.device("cuda" if torch.cuda.is_available() else "cpu"))
    if device.type == "cuda" and torch.cuda.current_stream(device) == torch.cuda.default_stream(device):
        # the whole loop (prefetch hand-off, graph replays, epoch reductions) on a created stream: collectives
        # next to graph replays on the legacy null stream were measured to corrupt data (fused.py _own_stream)
        work = torch.cuda.Stream(device)
        work.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(work):
            out = _train_loop(dataset, val_dataset, resume, cfg, tr, mblock, objective, step_factory, use_graph, device)
        torch.cuda.current_stream(device).wait_stream(work)
        return out
    return _train_loop(dataset, val_dataset, resume, cfg, tr, mblock, objective, step_factory, use_graph, device)


def _train_loop(dataset, val_dataset, resume, cfg, tr, mblock, objective, step_factory, use_graph, device):
    model_type, prefix, default_out, log_name = _KIND[objective]
    batch_size = U.resolve_batch_size(tr, "train_batch_size", tr.get("batch_size", 4))
    num_workers = int(tr.get("num_workers", 4))
    epochs = int(tr.get("num_epochs", tr.get("epochs", 1)))
    lr = float(tr.get("learning_rate", 1e-4))
    weight_decay = float(tr.get("weight_decay", 0.0))
    mode = resolve_conditioning_mode(tr.get("conditioning") or mblock.get("conditioning"))
    save_every = int(tr.get("save_model_epochs", tr.get("save_every", 5)))
    grad_accum = max(1, int(tr.get("gradient_accumulation_steps", 1)))
    warmup = int(tr.get("lr_warmup_steps", 500))
    latent_norm = tr.get("latent_norm")

    base_out = Path(tr.get("output_dir", default_out))
    out_dir = _broadcast_path(U.allocate_run_dir(base_out) if (resume is None and U.is_main_process())
                              else base_out)
    tr["output_dir"] = str(out_dir)
    if U.is_main_process():
        out_dir.mkdir(parents=True, exist_ok=True)
        if not (out_dir / "train_config.json").exists():
            U.save_json_config(out_dir / "train_config.json", cfg)

    model = build_diffusion_model(cfg, device, ckpt_path=None, set_eval=False)
    scheduler, _ = build_scheduler(mblock.get("scheduler", {}), tr)
    n_train = int(scheduler.config.num_train_timesteps)
    total_steps = epochs * math.ceil(len(dataset) / batch_size)
    make = step_factory or default_step_factory
    step = make(model, objective=objective, lr=lr, weight_decay=weight_decay, warmup=warmup, total_steps=total_steps,
                num_train_timesteps=n_train, grad_accum=grad_accum,
                ddpm_scheduler=scheduler if objective == "ddpm" else None,
                process_group=dist.group.WORLD if U.is_distributed() else None)

    sampler = DistributedSampler(dataset, shuffle=True) if U.is_distributed() else None
    loader = DataLoader(dataset, batch_size=batch_size, shuffle=sampler is None, sampler=sampler,
                        num_workers=num_workers, pin_memory=False)   # pinning is the prefetcher's job
    cuda = device.type == "cuda"
    graphs = cuda if use_graph is None else (bool(use_graph) and cuda)

    vis_on = bool(tr.get("save_images", False))
    vis_every = int(tr.get("save_images_every", 10))
    vis_t = vis_c = None
    if vis_on and U.is_main_process():
        vis_t, vis_c = prepare_diffusion_visual_batch(val_dataset if val_dataset is not None else dataset,
                                                      int(tr.get("visual_samples", 8)), device, seed=tr.get("seed"))

    metrics = out_dir / "metrics.csv"
    if U.is_main_process() and not metrics.exists():
        metrics.write_text("epoch,train_loss\n")

    rflag = Path(resume) if resume else None
    if rflag is None and isinstance(tr.get("resume"), str) and tr["resume"].lower() != "none":
        rflag = Path(tr["resume"])
    start_epoch, best = U.maybe_load_checkpoint(rflag, prefix, model, step) if rflag else (1, float("inf"))

    captured = False
    for epoch in range(start_epoch, epochs + 1):
        if sampler is not None:
            sampler.set_epoch(epoch)
        model.train()
        n_seen = 0
        step.epoch_loss_sum(reset=True)
        if cuda:
            from ...data.prefetch import DevicePrefetcher
            batches = DevicePrefetcher(loader, device)
        else:
            batches = loader
        for batch in batches:
            clean = batch["target"].to(device)
            cond = batch.get("image")
            cond = cond.to(device) if torch.is_tensor(cond) else None
            ldct, cca = None, None
            if mode == "concatenate" and cond is not None:
                ldct = cond
            elif mode == "attention" and cond is not None:
                cca = _prepare_attention_context(normalize_latent_conditioning(cond, latent_norm))
            bs = clean.shape[0]
            if graphs and bs == batch_size:
                if not captured:
                    step.capture(clean, ldct, warmup_iters=2, context_ca=cca)
                    captured = True
                step.replay(clean=clean, ldct=ldct, context_ca=cca)
            else:   # a ragged last batch (or no graphs): the same step, eagerly
                step.step(clean, ldct, context_ca=cca)
            n_seen += bs

        loss_t = step.epoch_loss_sum(reset=True).to(device=device, dtype=torch.float32).reshape(())
        count_t = torch.tensor(n_seen, device=device)
        if U.is_distributed():
            dist.all_reduce(loss_t)
            dist.all_reduce(count_t)
        avg = (loss_t / count_t.clamp(min=1)).item()
        if U.is_main_process():
            logging.info("%s Epoch %03d | loss %.6f", log_name, epoch, avg)

        state = {"model": {k: v.detach().cpu() for k, v in model.state_dict().items()},
                 "optimizer": step.optimizer_state_dict(), "lr_scheduler": step.lr_scheduler_state_dict(),
                 "scaler": None, "epoch": epoch, "best_metric": best}
        if U.is_main_process():
            U.save_checkpoint(state, out_dir / f"{prefix}_last.pt")
            if avg < best:
                best = avg
                state["best_metric"] = best
                U.save_checkpoint(state, out_dir / f"{prefix}_best.pt")
                logging.info("New best %s loss %.6f -> %s", log_name, best, out_dir / f"{prefix}_best.pt")
            if epoch % save_every == 0 or epoch == epochs:
                U.save_checkpoint(state, out_dir / "epochs" / f"epoch{epoch:04d}" / "epoch.pt")
        best = min(best, avg)

        if vis_on and U.is_main_process() and vis_t is not None and (epoch % vis_every == 0 or epoch == epochs):
            model.eval()
            with torch.no_grad():
                outs = decode_diffusion_batch(model, tr, mblock, device, tuple(vis_t.shape),
                                              vis_c if mode in {"concatenate", "attention"} else None)
            vis_dir = out_dir / "visuals"
            _save_grid(vis_c if vis_c is not None else vis_t, vis_dir / f"epoch{epoch:04d}_input.png")
            _save_grid(outs.clamp(0.0, 1.0), vis_dir / f"epoch{epoch:04d}_output.png")
            _save_grid(vis_t, vis_dir / f"epoch{epoch:04d}_target.png")
            model.train()

        if U.is_main_process():
            with metrics.open("a") as fh:
                fh.write(f"{epoch},{avg:.6f}\n")
    return out_dir
