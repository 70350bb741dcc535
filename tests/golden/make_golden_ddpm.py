"""Golden fixtures for the DDPM train step on the configurations that use it (configs A and C).

Run in the build container only (the reference never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_ddpm.py

For each case the reference's own model is built by importing ``/root/reference/src`` (its
``DiffusionUNetFactory`` from the config's ``model.unet`` block), the parameters are filled with
``oracle.unet.seeded_state_dict``, and ONE DDPM train step is run exactly as
``src/pipelines/train/diffusion_lib.py:153-185`` runs it, with the random draws injected:

    noisy = scheduler.add_noise(clean, eps, timesteps)   # integer timesteps, config betas
    pred  = model(cat([noisy, ldct]), timesteps)          # concatenate conditioning
    loss  = mse(pred, eps); backward
    torch.optim.AdamW(lr, wd) under get_cosine_schedule_with_warmup(warmup 0, total 1000); one step

``scheduler.add_noise`` is diffusers' DDPMScheduler, which is not installed here: the fixture uses the
oracle's restatement (``oracle/schedulers.py::DDPM``, pinned by its closed-form KATs), which
``fmd_add_noise`` reproduces bit-exactly (tests/test_gpu_ddpm.py::test_add_noise_bit_exact).

Cases: ``c256`` = ``configs/diffusion/ldct_ddpm.json`` (config C's 113 M EfficientUNetND) at 256x256,
batch 2; ``mnist`` = ``configs/MNIST/mnist_ddpm_diffusers_nd.json`` (config A's UNetDiffusersND) at its
32x32 ``img_size``, batch 2.

Stored per case: inputs, loss, per-parameter gradient sums / sums of squares, full gradients of tensors
with <= 4096 elements, per-parameter sums before / after AdamW, and the order-sensitive fingerprints of
tests/golden/projections.py for every gradient and every AdamW delta.

Output: ``tests/golden/golden_ddpm.pt`` (tensors only; ``weights_only=True``) + ``golden_ddpm.json``.
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
sys.path.insert(0, HERE)

from models.generators import DiffusionUNetFactory  # noqa: E402  (reference)
from transformers.optimization import get_cosine_schedule_with_warmup  # noqa: E402

import projections as P  # noqa: E402
from oracle import schedulers as OS  # noqa: E402
from oracle import spec as S  # noqa: E402
from oracle import unet as U  # noqa: E402

torch.set_num_threads(8)
CASES = [  # name, config, image size, batch, seed, timesteps
    ("c256", "configs/diffusion/ldct_ddpm.json", 256, 2, 5151, [37, 842]),
    ("mnist", "configs/MNIST/mnist_ddpm_diffusers_nd.json", 32, 2, 6262, [5, 611]),
]
WARMUP, TOTAL = 0, 1000
SMALL = 4096


def run_case(name, path, img, B, seed, ts_list):
    cfg = json.load(open(os.path.join(REF, path)))
    tr, mc = cfg["training"], cfg["model"]
    ch = S.resolve_channels(tr, mc)
    model = DiffusionUNetFactory().build(mc["unet"], tr.get("conditioning"), ch)
    spec = S.derive_spec(mc["unet"], tr.get("conditioning"), ch)
    model.load_state_dict(U.seeded_state_dict(spec, seed))
    sp = mc["scheduler"]
    n_train = int(sp.get("num_train_timesteps", tr.get("num_train_timesteps", 1000)))
    sched = OS.DDPM(n_train, **sp.get("params", {}))
    lr, wd = float(tr["learning_rate"]), float(tr.get("weight_decay", 0.0))

    g = torch.Generator().manual_seed(seed)
    clean = torch.rand(B, ch, img, img, generator=g)
    ldct = (clean + 0.05 * torch.randn(B, ch, img, img, generator=g)).clamp(0, 1)
    noise = torch.randn(B, ch, img, img, generator=g)
    ts = torch.tensor(ts_list, dtype=torch.long)
    noisy = sched.add_noise(clean, noise, ts)

    names = [k for k, _ in model.named_parameters()]
    before = torch.stack([p.detach().double().sum() for _, p in model.named_parameters()])
    p_before = [p.detach().clone() for _, p in model.named_parameters()]
    opt = torch.optim.AdamW(model.parameters(), lr=lr, weight_decay=wd)
    lrs = get_cosine_schedule_with_warmup(opt, num_warmup_steps=WARMUP, num_training_steps=TOTAL)
    opt.zero_grad(set_to_none=True)
    pred = model(torch.cat([noisy, ldct], 1), ts)
    loss = F.mse_loss(pred, noise)
    loss.backward()
    grads = [p.grad.detach().clone() for _, p in model.named_parameters()]
    opt.step()
    lrs.step()
    after = torch.stack([p.detach().double().sum() for _, p in model.named_parameters()])
    deltas = [p.detach().double() - b.double() for (_, p), b in zip(model.named_parameters(), p_before)]

    out = {f"{name}/{k}": v for k, v in dict(
        clean=clean, ldct=ldct, noise=noise, t=ts, noisy=noisy, loss=loss.detach(),
        param_sum_before=before, param_sum_after=after,
        grad_sum=torch.stack([gg.double().sum() for gg in grads]),
        grad_sq=torch.stack([gg.double().pow(2).sum() for gg in grads]),
        grad_l1=torch.stack([gg.double().abs().sum() for gg in grads]),
        proj_grad=P.projections(grads, seed), sample_grad=P.strided_sample(grads).float(),
        proj_delta=P.projections(deltas, seed + 1), sample_delta=P.strided_sample(deltas).float()).items()}
    small = [k for k, gg in zip(names, grads) if gg.numel() <= SMALL]
    for k, gg in zip(names, grads):
        if gg.numel() <= SMALL:
            out[f"{name}/grad/{k}"] = gg
    meta = dict(config=path, unet=mc["unet"], training=dict(conditioning=tr.get("conditioning"), channels=ch),
                scheduler=sp, seed=seed, img=img, batch=B, lr=lr, weight_decay=wd, warmup=WARMUP, total=TOTAL,
                num_train_timesteps=n_train, param_names=names, small_grads=small,
                numel=[int(p.numel()) for _, p in model.named_parameters()], proj_seed_grad=seed,
                proj_seed_delta=seed + 1)
    print(name, "loss", float(loss), "params", sum(meta["numel"]))
    return out, meta


def main():
    out, meta = {}, {}
    for case in CASES:
        o, m = run_case(*case)
        out.update(o)
        meta[case[0]] = m
    torch.save(out, os.path.join(HERE, "golden_ddpm.pt"))
    with open(os.path.join(HERE, "golden_ddpm.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote", sum(v.numel() * v.element_size() for v in out.values()) / 1e6, "MB")


if __name__ == "__main__":
    main()
