"""The forward-only GroupNorm fold inside the halo conv (csrc/conv_halo9.hip, fmd_conv_desc.fold_*): each workgroup
computes its sample's GN affine from the producers' statistics slabs instead of reading gn_prep's a/b
(reference: ResBlockND's GroupNorm + SiLU -> 3x3 conv, src/nn/blocks/residual.py:84-120, normalization.py:11-19,
convolution.py:8-54).  Checked against the two-launch form (fmd_gn_prep -> fmd_conv with pro=(a, b)) and against an
fp32 torch reference, on the config D 32^2 level: concatenated inputs with 64-pixel slab rows, a single input with
16-pixel rows (the split-K combine's) and the scale-shift embedding; and the fallback where the halo path declines."""
import os
import sys

import pytest
import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "flow-matching-and-diffusion-models_amd")]

pytestmark = pytest.mark.gpu
DEV = "cuda"

# name: (N, H, C0, C1, K, rows, scale-shift)
CASES = {
    "concat_rows64": (8, 32, 128, 128, 128, 64, False),
    "single_rows16_ss": (8, 32, 128, 0, 128, 16, True),
    "single_rows64_256": (8, 32, 256, 0, 256, 64, False),
}


def _inputs(name):
    N, H, C0, C1, K, rows, ss = CASES[name]
    g = torch.Generator().manual_seed(sum(map(ord, name)))
    x0 = (torch.randn(N, H, H, C0, generator=g) * 1.2 + 0.3).to(torch.bfloat16).to(DEV)
    x1 = (torch.randn(N, H, H, C1, generator=g) * 0.8 - 0.2).to(torch.bfloat16).to(DEV) if C1 else None
    C = C0 + C1
    w = (torch.randn(K, C, 3, 3, generator=g) / (3 * C ** 0.5)).to(DEV)
    gamma = (1 + 0.2 * torch.randn(C, generator=g)).to(DEV)
    beta = (0.1 * torch.randn(C, generator=g)).to(DEV)
    emb = (0.3 * torch.randn(N, 2 * C, generator=g)).to(DEV) if ss else None
    return x0, x1, w, gamma, beta, emb, rows


def _fold_dict(ops, x0, x1, gamma, beta, emb, rows):
    return dict(st0=ops.channel_stats(x0, rows=rows), st1=ops.channel_stats(x1, rows=rows) if x1 is not None else None,
                groups=32, eps=1e-6, gamma=gamma, beta=beta, emb=emb, emb_stride=emb.shape[1] if emb is not None else 0)


@pytest.mark.parametrize("name", list(CASES))
def test_halo_fold_matches_gn_prep_path_and_torch(name, monkeypatch):
    from fmdiff.runtime import ops
    monkeypatch.setattr(ops, "HALO_FOLD", True)
    x0, x1, w, gamma, beta, emb, rows = _inputs(name)
    N, H, C0 = x0.shape[0], x0.shape[1], x0.shape[-1]
    C1 = x1.shape[-1] if x1 is not None else 0
    K = w.shape[0]
    assert ops.halo_eligible(N, H, H, H, K, Cin=C0 + C1, pro=True)
    wk = ops.prep_weights(w, 0)
    f = _fold_dict(ops, x0, x1, gamma, beta, emb, rows)
    got, _ = ops.conv(x0, K, wk, src1=x1, pro_fold=f)
    a, b, _ = ops.gn_prep(f["st0"], f["st1"], N, H * H, C0, C1, 32, 1e-6, gamma, beta, emb=emb,
                          emb_stride=f["emb_stride"], emb_mode=1 if emb is not None else 0)
    ref2, _ = ops.conv(x0, K, wk, src1=x1, pro=(a, b, True))
    torch.cuda.synchronize()
    err2 = (got.float() - ref2.float()).abs().max().item()
    scale = ref2.float().abs().max().item()
    # the two folds differ only in summation order (fp32 channel totals, fp64 group sums): a bf16 step at most
    assert err2 <= 8e-3 * scale, (err2, scale)
    # fp32 torch
    x = torch.cat([x0, x1], -1) if x1 is not None else x0
    xf = x.float().permute(0, 3, 1, 2)
    xg = xf.reshape(N, 32, -1)
    z = ((xg - xg.mean(-1, keepdim=True)) / torch.sqrt(xg.var(-1, unbiased=False, keepdim=True) + 1e-6)).reshape_as(xf)
    z = z * gamma[None, :, None, None] + beta[None, :, None, None]
    if emb is not None:
        C = C0 + C1
        z = z * (1 + emb[:, :C, None, None]) + emb[:, C:, None, None]
    z = F.silu(z).to(torch.bfloat16).float()
    ref = F.conv2d(z, w.to(torch.bfloat16).float(), padding=1).permute(0, 2, 3, 1)
    err = (got.float() - ref).abs().max().item()
    print(f"[halo fold] {name}: vs gn_prep path {err2 / scale:.2e}, vs torch {err / ref.abs().max().item():.2e}")
    assert err <= 1.5e-2 * ref.abs().max().item()


def test_halo_fold_falls_back_where_the_halo_path_declines(monkeypatch):
    """Too few rows per slab row block for the fold, or a generic-path problem: pro_fold is folded by gn_prep first
    and the result equals the pro=(a, b) call bit for bit."""
    from fmdiff.runtime import ops
    monkeypatch.setattr(ops, "HALO_FOLD", True)
    x0, x1, w, gamma, beta, emb, rows = _inputs("single_rows16_ss")
    N, H, C0 = x0.shape[0], x0.shape[1], x0.shape[-1]
    K = w.shape[0]
    wk = ops.prep_weights(w, 0)
    f = _fold_dict(ops, x0, None, gamma, beta, emb, rows)
    a, b, _ = ops.gn_prep(f["st0"], None, N, H * H, C0, 0, 32, 1e-6, gamma, beta, emb=emb,
                          emb_stride=f["emb_stride"], emb_mode=1)
    for kw in (dict(force_generic=True), {}):
        if not kw:
            monkeypatch.setattr(ops, "HALO_FOLD_MAX_ROWS", 8)   # 64 rows per image: above the cap
        got, _ = ops.conv(x0, K, wk, pro_fold=f, **kw)
        ref, _ = ops.conv(x0, K, wk, pro=(a, b, True), **kw)
        torch.cuda.synchronize()
        assert torch.equal(got, ref), kw
