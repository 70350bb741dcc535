"""The split-K halo conv combined inside its own launch (csrc/conv_halo9.hip, fmd_conv_desc.tickets; runtime/ops.py
HALO_TICKET): every part stores its fp32 accumulators, the part that draws the tile's last ticket sums them in part
order and runs the unsplit epilogue (bias, per-sample bias, the 1x1 skip segment, residual, data-gradient SiLU',
statistics with 64-pixel rows).  Against the two-launch form (partials + splitk_reduce_rows) on the small levels the
latent UNet and the config B sampler split (reference: ConvND, src/nn/ops/convolution.py:8-54, inside ResBlockND,
src/nn/blocks/residual.py:84-120): outputs within a bf16 step, statistics equal to the fp64 sums of the kernel's own
bf16 outputs, results bit-identical across repeats (the part order fixes the sum), the tickets left at zero."""
import os
import sys

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "flow-matching-and-diffusion-models_amd")]

pytestmark = pytest.mark.gpu
DEV = "cuda"

# name: (N, H, C0, C1, K, up, extras)
CASES = {
    "latent32_concat_pro": (8, 32, 128, 128, 128, False, ("pro", "bias_nc")),
    "latent32_skip": (8, 32, 256, 0, 128, False, ("pro", "seg2")),
    "b16_pro_stats": (8, 16, 512, 0, 512, False, ("pro",)),
    "up32_from16": (8, 32, 256, 0, 256, True, ("pro",)),
    "dgrad_ep": (4, 32, 512, 0, 256, False, ("ep",)),
    "resid": (4, 32, 256, 256, 256, False, ("pro", "resid")),
}


def _args(name, O):
    N, H, C0, C1, K, up, ex = CASES[name]
    g = torch.Generator().manual_seed(sum(map(ord, name)))
    Hs = H // 2 if up else H

    def r(*s, sc=1.0):
        return (torch.randn(*s, generator=g) * sc).to(DEV)

    x0 = r(N, Hs, Hs, C0).to(torch.bfloat16)
    x1 = r(N, Hs, Hs, C1).to(torch.bfloat16) if C1 else None
    w = O.prep_weights(r(K, C0 + C1, 3, 3, sc=1 / (3 * (C0 + C1) ** 0.5)), 0)
    kw = dict(src1=x1, bias=r(K, sc=0.1), upsample=up)
    if "pro" in ex:
        kw["pro"] = ((torch.rand(N, C0 + C1, generator=g) + 0.5).to(DEV), r(N, C0 + C1, sc=0.2), True)
    if "bias_nc" in ex:
        kw["bias_nc"] = r(N, K, sc=0.1)
    if "seg2" in ex:
        kw.update(src2=r(N, H, H, C0).to(torch.bfloat16), wgt2=O.prep_weights(r(K, C0, 1, 1, sc=1 / C0 ** 0.5), 0),
                  bias2=r(K, sc=0.1))
    if "resid" in ex:
        kw["resid"] = r(N, H, H, K).to(torch.bfloat16)
    if "ep" in ex:
        kw["ep"] = (r(N, H, H, K).to(torch.bfloat16), None, (torch.rand(N, K, generator=g) + 0.5).to(DEV),
                    r(N, K, sc=0.2))
    return x0, w, kw, (N, H, C0 + C1, K)


@pytest.mark.parametrize("name", list(CASES))
def test_halo_ticket_combine_matches_combine_launch(name, monkeypatch):
    from fmdiff.runtime import ops as O
    x0, w, kw, (N, H, C, K) = _args(name, O)
    up = kw["upsample"]
    sp = O.halo_splits(N, H, H, K, C)
    assert sp > 1 and O.halo_eligible(N, H // 2 if up else H, H, H, K, upsample=up, Cin=C, pro="pro" in kw)
    monkeypatch.setattr(O, "HALO_TICKET", True)
    a, sa = O.conv(x0, K, w, want_stats=True, **kw)
    a2, sa2 = O.conv(x0, K, w, want_stats=True, **kw)
    monkeypatch.setattr(O, "HALO_TICKET", False)
    b, sb = O.conv(x0, K, w, want_stats=True, **kw)
    torch.cuda.synchronize()
    assert sa.rows == 64 and sb.rows == O.SPLIT_STATS_ROWS
    # the part order fixes the sum: bit-identical across repeats
    assert torch.equal(a, a2) and torch.equal(sa.slab, sa2.slab)
    # vs the two-launch combine: the same fp32 parts summed in another order, one bf16 rounding each
    af, bf = a.float(), b.float()
    err = (af - bf).abs().max().item()
    assert err <= 8e-3 * bf.abs().max().item(), (name, err)
    # statistics: per sample, the fp64 sums of the kernel's own bf16 outputs (or of out * x for the data gradient)
    y = a.double().reshape(N, -1, K)
    q = y * kw["ep"][0].double().reshape(N, -1, K) if "ep" in kw else y * y
    tot = sa.slab.double().reshape(N, -1, K, 2).sum(1)
    for c, t in ((0, y), (1, q)):
        assert ((tot[..., c] - t.sum(1)).abs() <= 1e-5 * t.abs().sum(1) + 1e-6).all(), (name, c)
    # the tickets are left at zero for the next launch
    assert int(O._small_workspace(a.device)[1].abs().sum()) == 0


def test_halo_ticket_combine_under_uneven_load(monkeypatch):
    """The parts of a tile arrive in an order a concurrent GEMM on a second stream perturbs; the result must not
    move (30 launches bit-equal to the solo one)."""
    from fmdiff.runtime import ops as O
    monkeypatch.setattr(O, "HALO_TICKET", True)
    x0, w, kw, (N, H, C, K) = _args("latent32_skip", O)
    ref, sref = O.conv(x0, K, w, want_stats=True, **kw)
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    A = torch.randn(8192, 8192, device=DEV, dtype=torch.bfloat16)
    for i in range(30):
        if i % 3 == 0:
            with torch.cuda.stream(side):
                A @ A
        got, sgot = O.conv(x0, K, w, want_stats=True, **kw)
        assert torch.equal(got, ref) and torch.equal(sgot.slab, sref.slab), i
    torch.cuda.synchronize()


# implicit-GEMM problems that run split-K (csrc/conv.hip conv_igemm): name -> (N, Hs, C, K, ks, stride, transposed,
# extras); every one with whole tiles, so ticketed (statistics one row per wave: bpx / 2 pixels, 64 for K <= 64)
GEN = {
    "s2_32to16": (8, 32, 256, 256, 3, 2, False, ("pro",)),
    "pw_8": (8, 8, 512, 512, 1, 1, False, ("resid",)),
    "s1_4_tiny": (8, 4, 512, 512, 3, 1, False, ("pro", "bias_nc")),
    "k64_16": (8, 16, 256, 64, 3, 1, False, ("pro", "generic")),
    "generic_32_resid": (8, 32, 256, 256, 3, 1, False, ("pro", "resid", "generic")),
    "dgrad_t_16": (8, 16, 512, 256, 3, 1, True, ("ep",)),
}


def _gen_args(name, O):
    N, Hs, C, K, ks, st, tr, ex = GEN[name]
    g = torch.Generator().manual_seed(sum(map(ord, name)) + 7)
    Ho = Hs // st if ks == 3 and st == 2 else Hs

    def r(*s, sc=1.0):
        return (torch.randn(*s, generator=g) * sc).to(DEV)

    x0 = r(N, Hs, Hs, C).to(torch.bfloat16)
    wt = r(K, C, ks, ks, sc=1 / (ks * C ** 0.5))
    w = O.prep_weights(wt.transpose(0, 1).contiguous(), 1) if tr else O.prep_weights(wt, 0)
    kw = dict(ks=ks, stride=st, pad=ks // 2, transposed=tr, bias=r(K, sc=0.1), force_generic="generic" in ex)
    if tr:   # data gradient of a stride-1 3x3 conv over K -> C: the weights of its forward, transposed gather
        kw["bias"] = None
    if "pro" in ex:
        kw["pro"] = ((torch.rand(N, C, generator=g) + 0.5).to(DEV), r(N, C, sc=0.2), True)
    if "bias_nc" in ex:
        kw["bias_nc"] = r(N, K, sc=0.1)
    if "resid" in ex:
        kw["resid"] = r(N, Ho, Ho, K).to(torch.bfloat16)
    if "ep" in ex:
        kw["ep"] = (r(N, Ho, Ho, K).to(torch.bfloat16), None, (torch.rand(N, K, generator=g) + 0.5).to(DEV),
                    r(N, K, sc=0.2))
    return x0, w, kw, (N, Ho, K)


@pytest.mark.parametrize("name", list(GEN))
def test_split_ticket_combine_implicit_gemm(name, monkeypatch):
    from fmdiff.runtime import ops as O
    x0, w, kw, (N, Ho, K) = _gen_args(name, O)
    K_out = K
    monkeypatch.setattr(O, "SPLIT_TICKET", True)
    a, sa = O.conv(x0, K_out, w, want_stats=True, **kw)
    a2, sa2 = O.conv(x0, K_out, w, want_stats=True, **kw)
    monkeypatch.setattr(O, "SPLIT_TICKET", False)
    b, sb = O.conv(x0, K_out, w, want_stats=True, **kw)
    torch.cuda.synchronize()
    assert torch.equal(a, a2) and torch.equal(sa.slab, sa2.slab)
    af, bf = a.float(), b.float()
    err = (af - bf).abs().max().item()
    assert err <= 8e-3 * bf.abs().max().item(), (name, err)
    if (Ho * Ho) % 64 == 0:   # statistics from the kernel (else a separate channel_stats pass, not under test)
        # the off run took the two-launch split (16-pixel rows), the on run the ticketed one (one row per wave)
        assert sb.rows == O.SPLIT_STATS_ROWS and sa.rows in (32, 64), (sa.rows, sb.rows)
        y = a.double().reshape(N, -1, K_out)
        q = y * kw["ep"][0].double().reshape(N, -1, K_out) if "ep" in kw else y * y
        tot = sa.slab.double().reshape(N, -1, K_out, 2).sum(1)
        for c, t in ((0, y), (1, q)):
            assert ((tot[..., c] - t.sum(1)).abs() <= 1e-5 * t.abs().sum(1) + 1e-6).all(), (name, c)
    assert int(O._small_workspace(a.device)[1].abs().sum()) == 0


# problems whose 8-row halo grid is under one round of the chip: 4-row tiles (fmd_halo_set_th4_max_workgroups)
TH4 = {
    "latent32_c128": (8, 32, 128, 0, 128, False, ("pro", "bias_nc")),
    "latent32_skip_c128": (8, 32, 128, 0, 128, False, ("pro", "seg2")),
    "up32_c128": (8, 32, 128, 0, 128, True, ("pro",)),
    "b16_k256": (8, 16, 256, 0, 256, False, ("pro", "resid")),
}


@pytest.mark.parametrize("name", list(TH4))
def test_halo_4row_tiles_match_8row(name, monkeypatch):
    """4-row tiles accumulate every output element over the same (chunk, tap, k-half) sequence as 8-row tiles and
    the split parts own the same chunks: outputs bit-identical, statistics rows the same 64-pixel blocks (permuted),
    per-sample totals equal."""
    from fmdiff import _lib
    from fmdiff.runtime import ops as O, tuning
    CASES[name] = TH4[name]
    try:
        x0, w, kw, (N, H, C, K) = _args(name, O)
    finally:
        del CASES[name]
    L = _lib.lib()
    outs = []
    try:
        for th4 in (tuning.get("HALO_TH4_MAX_WG"), 0):
            assert L.fmd_halo_set_th4_max_workgroups(th4) == 0
            outs.append(O.conv(x0, K, w, want_stats=True, **kw))
            torch.cuda.synchronize()
    finally:
        L.fmd_halo_set_th4_max_workgroups(tuning.get("HALO_TH4_MAX_WG"))
    (a, sa), (b, sb) = outs
    assert torch.equal(a, b), name
    ta = sa.slab.double().reshape(N, -1, K, 2).sum(1)
    tb = sb.slab.double().reshape(N, -1, K, 2).sum(1)
    assert torch.allclose(ta, tb, rtol=1e-12, atol=1e-9), name
