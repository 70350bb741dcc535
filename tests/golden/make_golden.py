"""Generate the committed golden fixtures from the reference itself.

Run in the build container only (the reference never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports the reference's own ``src/nn`` + ``src/models`` from
``/root/reference/src`` (pure PyTorch, CPU, fp32), fills every parameter with
the deterministic rule ``oracle.unet.seeded_state_dict`` (so only seeds, inputs
and outputs need to be stored), runs forwards / one train step, and writes
``tests/golden/golden.pt`` (tensors only; load with ``weights_only=True``).
Model configs are the reference's ``configs/**.json`` ``model.unet`` blocks,
recorded inline in the fixture as JSON text.
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
from nn.blocks.attention import SpatialSelfAttention  # noqa: E402  (reference)
from nn.blocks.residual import ResBlockND  # noqa: E402  (reference)
from nn.ops.time_embedding import timestep_embedding  # noqa: E402  (reference)

from oracle import spec as S  # noqa: E402
from oracle import unet as U  # noqa: E402

torch.set_num_threads(8)

# (fixture name, reference config path, image size, batch)
MODEL_CASES = [
    ("ldct_fm_test", "configs/LDCT/LDCT_flow_matching_test.json", 32, 2),
    ("mnist_ddpm_diffusers", "configs/MNIST/mnist_ddpm_diffusers_nd.json", 32, 2),
    ("mnist_fm_compvis", "configs/MNIST/mnist_flow_matching_compvis.json", 32, 2),
    ("ldct_fm_b64", "configs/flow_matching/ldct_flow_matching.json", 64, 2),
    ("ldct_fm_diffusers_b64", "configs/flow_matching/ldct_flow_matching_diffusers_nd.json", 64, 2),
]


def build(cfg_path):
    cfg = json.load(open(os.path.join(REF, cfg_path)))
    tr, mc = cfg["training"], cfg["model"]
    ch = S.resolve_channels(tr, mc)
    model = DiffusionUNetFactory().build(mc["unet"], tr.get("conditioning"), ch)
    spec = S.derive_spec(mc["unet"], tr.get("conditioning"), ch)
    return cfg, model, spec


def main():
    out = {}
    meta = {}
    for name, path, img, B in MODEL_CASES:
        cfg, model, spec = build(path)
        seed = 1000 + len(meta)
        sd = U.seeded_state_dict(spec, seed)
        model.load_state_dict(sd)
        g = torch.Generator().manual_seed(seed)
        cin = spec["in_channels"] - (1 if cfg["training"].get("conditioning") == "concatenate" else 0)
        x = torch.randn(B, cin, img, img, generator=g)
        cond = torch.rand(B, 1, img, img, generator=g) if cfg["training"].get("conditioning") == "concatenate" else None
        t = torch.randint(0, 1000, (B,), generator=g)
        with torch.no_grad():
            y = model(x, t, context=cond)
        out[f"{name}/x"] = x
        if cond is not None:
            out[f"{name}/cond"] = cond
        out[f"{name}/t"] = t
        out[f"{name}/y"] = y
        meta[name] = dict(config=path, unet=cfg["model"]["unet"], training=dict(
            conditioning=cfg["training"].get("conditioning"), channels=cfg["training"].get("channels")),
            seed=seed, img=img, batch=B)
        print(name, tuple(y.shape), float(y.abs().mean()))

    # ---- one FM train step on the tiny LDCT config (flow_matching_lib.py:150-182)
    cfg, model, spec = build("configs/LDCT/LDCT_flow_matching_test.json")
    seed = 77
    sd = U.seeded_state_dict(spec, seed)
    model.load_state_dict(sd)
    g = torch.Generator().manual_seed(seed)
    B, img = 2, 32
    clean = torch.rand(B, 1, img, img, generator=g)
    ldct = (clean + 0.05 * torch.randn(B, 1, img, img, generator=g)).clamp(0, 1)
    noise = torch.randn(B, 1, img, img, generator=g)
    t = torch.rand(B, generator=g)
    N = cfg["model"]["scheduler"]["num_train_timesteps"]
    timesteps = (t * (N - 1)).long()
    x_t = (1.0 - t[:, None, None, None]) * clean + t[:, None, None, None] * noise
    pred = model(torch.cat([x_t, ldct], 1), timesteps)
    loss = F.mse_loss(pred, noise - clean)
    loss.backward()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3, weight_decay=0.0)
    grads = {k: p.grad.detach().clone() for k, p in model.named_parameters()}
    opt.step()
    for k in ("clean", "ldct", "noise", "t"):
        out[f"fm_step/{k}"] = locals()[k]
    out["fm_step/loss"] = loss.detach()
    names = list(grads)
    out["fm_step/grad_sum"] = torch.stack([grads[k].double().sum() for k in names])
    out["fm_step/grad_sq"] = torch.stack([grads[k].double().pow(2).sum() for k in names])
    out["fm_step/param_sum_after"] = torch.stack([p.detach().double().sum() for _, p in model.named_parameters()])
    meta["fm_step"] = dict(config="configs/LDCT/LDCT_flow_matching_test.json", unet=cfg["model"]["unet"],
                           training=dict(conditioning="concatenate", channels=1), seed=seed, lr=1e-3,
                           num_train_timesteps=N, param_names=names)
    print("fm_step loss", float(loss))

    # ---- module cases: raw-reshape self-attention (attention.py:82-117) and ResBlock variants
    att = SpatialSelfAttention(512, heads=4, dim_head=64, use_linear=False, use_efficient_attn=True)
    att.load_state_dict(U.seeded_tensors({k: tuple(v.shape) for k, v in att.state_dict().items()}, 500))
    xa = torch.randn(2, 512, 8, 8, generator=torch.Generator().manual_seed(501))
    with torch.no_grad():
        out["attn/y"] = att(xa)
    out["attn/x"] = xa
    meta["attn"] = dict(dim=512, heads=4, dim_head=64, seed=500)
    for i, (cin, cout, ss, act, add) in enumerate([(128, 128, True, False, False), (384, 256, True, False, False),
                                                   (64, 128, False, True, True)]):
        rb = ResBlockND(channels=cin, emb_channels=512, dropout=0.0, out_channels=cout, use_scale_shift_norm=ss,
                        emb_activation_before_proj=act, add_embedding_to_hidden=add, zero_init_last_conv=False)
        rb.load_state_dict(U.seeded_tensors({k: tuple(v.shape) for k, v in rb.state_dict().items()}, 600 + 10 * i))
        g = torch.Generator().manual_seed(601 + 10 * i)
        xr = torch.randn(2, cin, 16, 16, generator=g)
        er = torch.randn(2, 512, generator=g)
        with torch.no_grad():
            out[f"res{i}/y"] = rb(xr, er)
        out[f"res{i}/x"] = xr
        out[f"res{i}/emb"] = er
        meta[f"res{i}"] = dict(cin=cin, cout=cout, scale_shift=ss, emb_act=act, add_emb=add, seed=600 + 10 * i,
                               names=list(rb.state_dict().keys()))
    tt = torch.tensor([0.0, 1.0, 17.0, 999.0, 1000.0, 979.6122436523438])
    out["temb/t"] = tt
    out["temb/flip"] = timestep_embedding(tt, 128, flip_sin_to_cos=True)
    out["temb/noflip"] = timestep_embedding(tt, 128, flip_sin_to_cos=False)
    out["temb/odd"] = timestep_embedding(tt, 33, flip_sin_to_cos=False, freq_shift=1)

    torch.save(out, os.path.join(HERE, "golden.pt"))
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote", sum(v.numel() * v.element_size() for v in out.values()) / 1e6, "MB")


if __name__ == "__main__":
    main()
