"""Diagnostics for the MFMA attention kernels (GPU box): pack layout, forward on canonical planes, special inputs."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "flow-matching-and-diffusion-models_amd")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from fmdiff import _lib  # noqa: E402
from fmdiff.runtime import ops  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)


def canon_fwd(q, k, v, dh):
    BH, Tq, D = q.shape
    co = torch.empty_like(q)
    lse = torch.empty((BH, Tq), device=dev, dtype=torch.float32)
    _lib.call("fmd_attn_mfma_fwd", q.data_ptr(), k.data_ptr(), v.data_ptr(), BH, Tq, k.shape[1], dh, co.data_ptr(),
              lse.data_ptr(), ops.stream())
    torch.cuda.synchronize()
    return co, lse


def ref(q, k, v, dh):
    qf, kf, vf = q[..., :dh].float(), k[..., :dh].float(), v[..., :dh].float()
    s = qf @ kf.transpose(1, 2) / dh ** 0.5
    return torch.softmax(s, -1) @ vf, torch.logsumexp(s, -1)


def rep(name, got, want):
    err = (got.float() - want.float()).abs().max().item()
    print(f"{name:40s} max err {err:.3e} (scale {want.abs().max().item():.3e})", flush=True)


for (T, dh) in [(32, 64), (64, 64), (32, 32), (32, 16)]:
    D = int(_lib.lib().fmd_attn_head_pad(dh))
    BH = 2
    q = torch.zeros(BH, T, D, device=dev, dtype=torch.bfloat16)
    k = torch.zeros_like(q)
    v = torch.zeros_like(q)
    # 1: q = 0 -> uniform attention, O = mean(V)
    v[..., :dh] = torch.randn(BH, T, dh, device=dev).to(torch.bfloat16)
    co, lse = canon_fwd(q, k, v, dh)
    o_ref, l_ref = ref(q, k, v, dh)
    rep(f"T{T} dh{dh} uniform O", co[..., :dh], o_ref)
    rep(f"T{T} dh{dh} uniform lse", lse, l_ref)
    # 2: V = one-hot(key) in d (T <= D): O[q][d] = P[q][key d]
    if T <= D:
        v.zero_()
        for kk in range(T):
            v[:, kk, kk] = 1
        q[..., :dh] = torch.randn(BH, T, dh, device=dev).to(torch.bfloat16)
        k[..., :dh] = torch.randn(BH, T, dh, device=dev).to(torch.bfloat16)
        co, lse = canon_fwd(q, k, v, dh)
        o_ref, l_ref = ref(q, k, v, dh)
        rep(f"T{T} dh{dh} onehot-V O (=P)", co[..., :dh], o_ref)
        rep(f"T{T} dh{dh} onehot-V lse", lse, l_ref)
        if (co[..., :dh].float() - o_ref).abs().max() > 0.05:
            print("got P rows 0..3 (first 8 keys):\n", co[0, :4, :8].float().cpu())
            print("want:\n", o_ref[0, :4, :8].cpu())
    # 3: random
    q[..., :dh] = torch.randn(BH, T, dh, device=dev).to(torch.bfloat16)
    k[..., :dh] = torch.randn(BH, T, dh, device=dev).to(torch.bfloat16)
    v[..., :dh] = torch.randn(BH, T, dh, device=dev).to(torch.bfloat16)
    co, lse = canon_fwd(q, k, v, dh)
    o_ref, l_ref = ref(q, k, v, dh)
    rep(f"T{T} dh{dh} random O", co[..., :dh], o_ref)
    rep(f"T{T} dh{dh} random lse", lse, l_ref)

# pack layout (raw self-attention)
B, T, heads, dh = 2, 64, 4, 64
inner = heads * dh
qkv = torch.randn(B, T, 3 * inner, device=dev).to(torch.bfloat16)
flat = qkv.transpose(1, 2).reshape(B, heads, T, 3 * dh)
qr, kr, vr = (x.reshape(B * heads, T, dh) for x in flat.chunk(3, dim=-1))
cq, ck, cv = (torch.empty(B * heads, T, 64, device=dev, dtype=torch.bfloat16) for _ in range(3))
ops._attn_pack(qkv, qkv, B, T, T, heads, dh, 1, 0, 0, 2, cq, ck, cv)
torch.cuda.synchronize()
rep("pack raw q", cq, qr)
rep("pack raw k", ck, kr)
rep("pack raw v", cv, vr)
