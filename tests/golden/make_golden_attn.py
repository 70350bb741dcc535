"""Generate reference fixtures for the attention-conditioning blocks (build container only; the reference never
travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_attn.py

Imports the reference's own ``SpatialCrossAttention`` and ``DiffusersAttentionND`` (``/root/reference/src/nn/
blocks/attention.py``), fills every parameter with ``oracle.unet.seeded_tensors`` (only seeds, inputs and
outputs are stored), and for a channel-major (b, c_ctx, tokens) context and a tokens-last (b, tokens, c_ctx)
one records the forward output and the gradients of x and of every parameter for a seeded output
cotangent.  Writes ``tests/golden/golden_attn.pt`` (tensors only; ``weights_only=True``) + ``golden_attn.json``.
"""
from __future__ import annotations

import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REF, "src"))

from nn.blocks.attention import DiffusersAttentionND, SpatialCrossAttention  # noqa: E402  (reference)

from oracle import unet as U  # noqa: E402

torch.set_num_threads(8)

# (name, builder kwargs, x shape, context channels, context tokens, seed)
CASES = [
    ("spatial_cross", dict(kind="spatial", dim=64, context_dim=4, heads=2, dim_head=32), (2, 64, 16, 16), 4, 64, 700),
    ("diffusers_cross", dict(kind="diffusers", channels=64, heads=8, context_dim=4, norm_num_groups=16),
     (2, 64, 16, 16), 4, 64, 710),
]


def build(kw):
    kw = dict(kw)
    kind = kw.pop("kind")
    if kind == "spatial":
        return SpatialCrossAttention(kw["dim"], context_dim=kw["context_dim"], heads=kw["heads"],
                                     dim_head=kw["dim_head"], use_linear=False)
    return DiffusersAttentionND(kw["channels"], heads=kw["heads"], context_dim=kw["context_dim"],
                                norm_num_groups=kw["norm_num_groups"])


def main():
    out, meta = {}, {}
    for name, kw, xs, cc, ct, seed in CASES:
        mod = build(kw)
        shapes = {k: tuple(v.shape) for k, v in mod.state_dict().items()}
        mod.load_state_dict(U.seeded_tensors(shapes, seed))
        g = torch.Generator().manual_seed(seed + 1)
        x0 = torch.randn(*xs, generator=g)
        ctx_bct = torch.randn(xs[0], cc, ct, generator=g)
        gout = torch.randn(*xs, generator=g)
        out[f"{name}/x"] = x0
        out[f"{name}/ctx"] = ctx_bct
        out[f"{name}/gout"] = gout
        for layout in ("bct", "btc"):
            ctx = ctx_bct if layout == "bct" else ctx_bct.transpose(1, 2).contiguous()
            mod.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_()
            y = mod(x, ctx)
            y.backward(gout)
            out[f"{name}/{layout}/y"] = y.detach()
            out[f"{name}/{layout}/dx"] = x.grad.detach()
            for k, p in mod.named_parameters():
                out[f"{name}/{layout}/grad/{k}"] = p.grad.detach().clone()
        meta[name] = dict(kw, seed=seed, x_shape=list(xs), ctx_channels=cc, ctx_tokens=ct,
                          params=[k for k, _ in mod.named_parameters()])
    torch.save(out, os.path.join(HERE, "golden_attn.pt"))
    with open(os.path.join(HERE, "golden_attn.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote", sum(v.numel() * v.element_size() for v in out.values()) / 1e6, "MB")


if __name__ == "__main__":
    main()
