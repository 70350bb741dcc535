"""Golden fixture for the BENCHED configuration: config B at its bench resolution.

Run in the build container only (the reference never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_b256.py

Builds the reference's own EfficientUNetND from ``configs/flow_matching/ldct_flow_matching.json``
(113,008,257 parameters, concatenate conditioning) by importing ``/root/reference/src``, fills
the parameters with ``oracle.unet.seeded_state_dict`` and records, at 256x256 and batch 2:

* ``fwd/*``   one forward (x, cond, t -> y);
* ``step/*``  one FM train step exactly as ``src/pipelines/train/flow_matching_lib.py:150-182``
  runs it (t, eps injected; ``timesteps = (t * 999).long()``; ``x_t = (1-t) x0 + t eps``;
  ``input = cat([x_t, ldct])``; ``loss = mse(pred, eps - x0)``; backward; ``torch.optim.AdamW``
  (lr 1e-4, wd 0) stepped under ``transformers.get_cosine_schedule_with_warmup`` (the formula
  diffusers' helper implements; warmup 0 so this first step moves the weights, total 1000)):
  the loss, per-parameter gradient sums / sums of squares, the full gradients of every
  parameter with <= 4096 elements, and per-parameter sums before and after the AdamW update;
  plus order-sensitive fingerprints (tests/golden/projections.py) of every gradient and every AdamW
  parameter delta: 8 seeded Rademacher projections per tensor and every 397th element of the concatenation.

Output: ``tests/golden/golden_b256.pt`` (tensors only; ``weights_only=True``) + ``golden_b256.json``.
"""
from __future__ import annotations

import json
import os
import sys

import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REF, "src"))

from models.generators import DiffusionUNetFactory  # noqa: E402  (reference)
from transformers.optimization import get_cosine_schedule_with_warmup  # noqa: E402

from oracle import spec as S  # noqa: E402
from oracle import unet as U  # noqa: E402

sys.path.insert(0, HERE)
import projections as P  # noqa: E402

torch.set_num_threads(8)
CFG = "configs/flow_matching/ldct_flow_matching.json"
IMG, B, SEED = 256, 2, 4242
LR, WARMUP, TOTAL = 1e-4, 0, 1000
SMALL = 4096


def main():
    cfg = json.load(open(os.path.join(REF, CFG)))
    tr, mc = cfg["training"], cfg["model"]
    ch = S.resolve_channels(tr, mc)
    model = DiffusionUNetFactory().build(mc["unet"], tr.get("conditioning"), ch)
    spec = S.derive_spec(mc["unet"], tr.get("conditioning"), ch)
    sd = U.seeded_state_dict(spec, SEED)
    model.load_state_dict(sd)
    out, meta = {}, {}
    g = torch.Generator().manual_seed(SEED)

    # ---- forward
    x = torch.randn(B, 1, IMG, IMG, generator=g)
    cond = torch.rand(B, 1, IMG, IMG, generator=g)
    t = torch.tensor([3, 871])
    with torch.no_grad():
        y = model(torch.cat([x, cond], 1), t)
    out.update({"fwd/x": x, "fwd/cond": cond, "fwd/t": t, "fwd/y": y})
    print("fwd", tuple(y.shape), float(y.abs().mean()))

    # ---- one FM train step (flow_matching_lib.py:150-182)
    clean = torch.rand(B, 1, IMG, IMG, generator=g)
    ldct = (clean + 0.05 * torch.randn(B, 1, IMG, IMG, generator=g)).clamp(0, 1)
    noise = torch.randn(B, 1, IMG, IMG, generator=g)
    tt = torch.rand(B, generator=g)
    N = int(mc["scheduler"]["num_train_timesteps"])
    timesteps = (tt * (N - 1)).long()
    x_t = (1.0 - tt[:, None, None, None]) * clean + tt[:, None, None, None] * noise
    opt = torch.optim.AdamW(model.parameters(), lr=LR, weight_decay=float(tr["weight_decay"]))
    sched = get_cosine_schedule_with_warmup(opt, num_warmup_steps=WARMUP, num_training_steps=TOTAL)
    names = [k for k, _ in model.named_parameters()]
    before = torch.stack([p.detach().double().sum() for _, p in model.named_parameters()])
    p_before = [p.detach().clone() for _, p in model.named_parameters()]
    opt.zero_grad(set_to_none=True)
    pred = model(torch.cat([x_t, ldct], 1), timesteps)
    loss = F.mse_loss(pred, noise - clean)
    loss.backward()
    grads = {k: p.grad.detach().clone() for k, p in model.named_parameters()}
    opt.step()
    sched.step()
    after = torch.stack([p.detach().double().sum() for _, p in model.named_parameters()])
    deltas = [p.detach().double() - b.double() for (_, p), b in zip(model.named_parameters(), p_before)]
    glist = [grads[k] for k in names]
    out.update({"step/proj_grad": P.projections(glist, SEED), "step/sample_grad": P.strided_sample(glist).float(),
                "step/proj_delta": P.projections(deltas, SEED + 1),
                "step/sample_delta": P.strided_sample(deltas).float()})
    out.update({"step/clean": clean, "step/ldct": ldct, "step/noise": noise, "step/t": tt,
                "step/loss": loss.detach(), "step/param_sum_before": before, "step/param_sum_after": after,
                "step/grad_sum": torch.stack([grads[k].double().sum() for k in names]),
                "step/grad_sq": torch.stack([grads[k].double().pow(2).sum() for k in names]),
                "step/grad_l1": torch.stack([grads[k].double().abs().sum() for k in names])})
    small = [k for k in names if grads[k].numel() <= SMALL]
    for k in small:
        out[f"step/grad/{k}"] = grads[k]
    meta = dict(config=CFG, unet=mc["unet"], training=dict(conditioning=tr.get("conditioning"), channels=ch),
                seed=SEED, img=IMG, batch=B, lr=LR, warmup=WARMUP, total=TOTAL, num_train_timesteps=N,
                weight_decay=float(tr["weight_decay"]), param_names=names, small_grads=small,
                numel=[int(p.numel()) for _, p in model.named_parameters()])
    print("step loss", float(loss), "params", sum(meta["numel"]))
    torch.save(out, os.path.join(HERE, "golden_b256.pt"))
    with open(os.path.join(HERE, "golden_b256.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote", sum(v.numel() * v.element_size() for v in out.values()) / 1e6, "MB")


if __name__ == "__main__":
    main()
