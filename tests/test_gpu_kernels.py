"""Per-kernel numerics on the GPU: each HIP kernel vs a plain PyTorch fp32 reference of the same op.

Inputs are bf16-rounded before the reference sees them, so the only expected
differences are fp32 accumulation order and the final bf16 rounding of the
kernel output (tolerance: 1.5e-2 x max|ref| for bf16 outputs, 1e-4 for fp32).
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def ops():
    from fmdiff.runtime import ops as O
    return O


def _close(got, ref, rel=1.5e-2):
    ref = ref.float().cpu()
    got = got.float().cpu()
    err = (got - ref).abs().max().item()
    scale = max(ref.abs().max().item(), 1e-6)
    assert err <= rel * scale, f"max err {err:.3e} vs scale {scale:.3e}"


def _rand_nhwc(N, H, W, C, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(N, H, W, C, generator=g) * scale).to(torch.bfloat16)


def _w(K, C, ks, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(K, C, ks, ks, generator=g) / math.sqrt(C * ks * ks)


def _to_nchw(x):
    return x.float().permute(0, 3, 1, 2).contiguous()


def _bfw(w):
    return w.to(torch.bfloat16).float()


@pytest.mark.parametrize("case", [
    dict(N=2, H=16, W=16, C=128, K=128, ks=3, stride=1),
    dict(N=2, H=16, W=16, C=64, K=128, ks=3, stride=2),
    dict(N=1, H=8, W=8, C=256, K=64, ks=1, stride=1),
    dict(N=2, H=32, W=32, C=8, K=128, ks=3, stride=1),
    dict(N=2, H=16, W=16, C=128, K=8, ks=3, stride=1),
])
def test_conv_forward(case):
    O = ops()
    N, H, W, C, K, ks, s = (case[k] for k in ("N", "H", "W", "C", "K", "ks", "stride"))
    x = _rand_nhwc(N, H, W, C, 1)
    w = _w(K, C, ks, 2)
    b = torch.randn(K) * 0.1
    pad = ks // 2
    out, _ = O.conv(x.to(DEV), K, O.prep_weights(w.to(DEV), 0), ks=ks, stride=s, pad=pad, bias=b.to(DEV))
    ref = F.conv2d(_to_nchw(x), _bfw(w), b, stride=s, padding=pad).permute(0, 2, 3, 1)
    _close(out, ref)


def test_conv_prologue_concat_upsample_skip_resid_stats():
    O = ops()
    N, H, W, C0, C1, K = 2, 8, 8, 64, 32, 128
    x0, x1 = _rand_nhwc(N, H, W, C0, 3), _rand_nhwc(N, H, W, C1, 4)
    a = torch.rand(N, C0 + C1) + 0.5
    bb = torch.randn(N, C0 + C1) * 0.2
    w = _w(K, C0 + C1, 3, 5)
    bias = torch.randn(K) * 0.1
    # upsample + concat + GN-affine/SiLU prologue, stats epilogue
    out, st = O.conv(x0.to(DEV), K, O.prep_weights(w.to(DEV), 0), src1=x1.to(DEV), upsample=True,
                     pro=(a.to(DEV), bb.to(DEV), True), bias=bias.to(DEV), want_stats=True)
    xc = torch.cat([_to_nchw(x0), _to_nchw(x1)], 1)
    z = F.silu(xc * a[:, :, None, None] + bb[:, :, None, None]).to(torch.bfloat16).float()
    ref = F.conv2d(F.interpolate(z, scale_factor=2, mode="nearest"), _bfw(w), bias, padding=1).permute(0, 2, 3, 1)
    _close(out, ref)
    s = st.slab.cpu().view(N, -1, K, 2).sum(1)
    o = out.float().cpu()
    torch.testing.assert_close(s[..., 0], o.sum((1, 2)), rtol=2e-3, atol=2e-2)
    torch.testing.assert_close(s[..., 1], (o * o).sum((1, 2)), rtol=2e-3, atol=2e-2)
    # 1x1 skip second segment over the concat + residual-free epilogue
    h = _rand_nhwc(N, H, W, K, 6)
    w2 = _w(K, K, 3, 7)
    ws = _w(K, C0 + C1, 1, 8)
    bs = torch.randn(K) * 0.1
    out2, _ = O.conv(h.to(DEV), K, O.prep_weights(w2.to(DEV), 0), src2=x0.to(DEV), src3=x1.to(DEV),
                     wgt2=O.prep_weights(ws.to(DEV), 0), bias=bias.to(DEV), bias2=bs.to(DEV))
    ref2 = (F.conv2d(_to_nchw(h), _bfw(w2), bias, padding=1)
            + F.conv2d(torch.cat([_to_nchw(x0), _to_nchw(x1)], 1), _bfw(ws), bs)).permute(0, 2, 3, 1)
    _close(out2, ref2)
    # identity residual
    out3, _ = O.conv(h.to(DEV), K, O.prep_weights(w2.to(DEV), 0), resid=h.to(DEV))
    ref3 = (F.conv2d(_to_nchw(h), _bfw(w2), padding=1) + _to_nchw(h)).permute(0, 2, 3, 1)
    _close(out3, ref3)


def test_conv_splitk_matches():
    O = ops()
    x = _rand_nhwc(2, 8, 8, 512, 9)
    w = _w(256, 512, 3, 10)
    wp = O.prep_weights(w.to(DEV), 0)
    a, _ = O.conv(x.to(DEV), 256, wp, splits=1)
    b, _ = O.conv(x.to(DEV), 256, wp, splits=6)
    _close(b, a.float(), rel=8e-3)


@pytest.mark.parametrize("ep", [False, True])
def test_conv_splitk_fused_stats(ep):
    """Split-K combine with the channel statistics fused (splitk_reduce_rows): output and (sum v, sum v^2)
    / (sum v, sum v*x) slab rows vs fmd_channel_stats of the same output, plus bias / per-sample bias /
    SiLU'-epilogue handling vs the unsplit conv."""
    O = ops()
    N, H, W, C, K = 2, 16, 16, 256, 192
    x = _rand_nhwc(N, H, W, C, 41).to(DEV)
    wp = O.prep_weights(_w(K, C, 3, 42).to(DEV), 0)
    g = torch.Generator().manual_seed(43)
    bias = (torch.randn(K, generator=g) * 0.1).to(DEV)
    bnc = (torch.randn(N, K, generator=g) * 0.1).to(DEV)
    kw = dict(bias=bias, bias_nc=bnc, want_stats=True, force_generic=True)
    if ep:
        xe = _rand_nhwc(N, H, W, K, 44).to(DEV)
        kw.update(ep=(xe, None, (torch.rand(N, K, generator=g) + 0.5).to(DEV),
                      (torch.randn(N, K, generator=g) * 0.2).to(DEV)))
    a, sa = O.conv(x, K, wp, splits=1, **kw)
    b, sb = O.conv(x, K, wp, splits=4, **kw)
    _close(b, a.float(), rel=8e-3)
    assert sb.rows == O.SPLIT_STATS_ROWS
    ref = O.channel_stats(b, rows=sb.rows, y=(kw["ep"][0], None, K) if ep else None)
    torch.testing.assert_close(sb.slab, ref.slab, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("case", ["8x8_k512_ss", "16x16_k128", "4x4_k256_resid", "1x1_k512", "3d_k128",
                                  "8x8_k64_cb64", "8x8_k128_cb32", "halo_16x16_c256_pro"])
def test_conv_gn_fused_combine(case, monkeypatch):
    """fmd_conv_gn: a split-K conv whose combine also runs the GroupNorm(+scale/shift)+SiLU of its output, vs the
    same conv through fmd_conv + fmd_gn_fused_apply on that output (a, b, mean/rstd, t).  ``_cb64`` / ``_cb32``: 64 /
    32 channels per combine block with 2- / 4-channel groups (32 / 8 groups in one block); ``halo_``: the production
    route -- halo-kernel split-K partials (GN+SiLU prologue) into combine_gn_kernel, not the generic conv."""
    O = ops()
    from fmdiff import _lib
    monkeypatch.setattr(O, "CONV_GN_MIN_BLOCKS", 0)
    g = torch.Generator().manual_seed(len(case))
    d3 = case.startswith("3d")
    halo = case.startswith("halo")
    N, H, C, K = {"8x8_k512_ss": (8, 8, 512, 512), "16x16_k128": (4, 16, 128, 128), "4x4_k256_resid": (8, 4, 256, 256),
                  "1x1_k512": (8, 1, 512, 512), "3d_k128": (1, 8, 128, 128), "8x8_k64_cb64": (8, 8, 64, 64),
                  "8x8_k128_cb32": (8, 8, 128, 128), "halo_16x16_c256_pro": (8, 16, 256, 128)}[case]
    G = 32
    cb = 64 if case.endswith("cb64") else 32 if case.endswith("cb32") else 4
    if cb != 4:
        monkeypatch.setattr(O, "CONV_GN_CB", cb)
        _lib.call("fmd_conv_gn_set_block_channels", cb)
    shape = (N, H, H, H, C) if d3 else (N, H, H, C)
    x = (torch.randn(*shape, generator=g) * 0.5).to(torch.bfloat16).to(DEV)
    ks = 1 if H == 1 else 3
    w = torch.randn(K, C, 3, 3, 3, generator=g) / math.sqrt(C * 27) if d3 else _w(K, C, ks, 91)
    wp = O.prep_weights(w.to(DEV), 0)
    kw = dict(bias=(torch.randn(K, generator=g) * 0.1).to(DEV), bias_nc=(torch.randn(N, K, generator=g) * 0.1).to(DEV),
              splits=5, force_generic=True, ks=ks, pad=ks // 2)
    if halo:   # halo_splits picks the split count (2 images x 1 tile: split-K over the 4 chunks), GN+SiLU prologue
        kw.update(splits=None, force_generic=False,
                  pro=((torch.rand(N, C, generator=g) + 0.5).to(DEV), (torch.randn(N, C, generator=g) * 0.1).to(DEV), True))
        assert O.halo_eligible(N, H, H, H, K, Cin=C, pro=True) and O.halo_splits(N, H, H, K, C) > 1
    if case.endswith("resid"):
        kw["resid"] = (torch.randn(*shape[:-1], K, generator=g)).to(torch.bfloat16).to(DEV)
    gamma, beta = (torch.rand(K, generator=g) + 0.5).to(DEV), (torch.randn(K, generator=g) * 0.1).to(DEV)
    emb = (torch.randn(N, 2 * K, generator=g) * 0.2).to(DEV) if case.endswith("ss") else None
    req = dict(groups=G, eps=1e-5, gamma=gamma, beta=beta, emb=emb, emb_stride=2 * K if emb is not None else 0,
               emb_mode=1 if emb is not None else 0)
    out, st = O.conv(x, K, wp, gn=req, **kw)
    assert "res" in req and st is None
    a, b, mr, t = req["res"]
    ref, _ = O.conv(x, K, wp, **kw)
    _close(out, ref.float(), rel=1e-2)
    if (K // G) % 4 == 0:
        ra, rb, rmr, rt = O.gn_fused_apply(out, None, G, 1e-5, gamma, beta, emb=emb,
                                           emb_stride=2 * K if emb is not None else 0,
                                           emb_mode=1 if emb is not None else 0)
    else:   # fmd_gn_fused_apply takes groups of 4k channels only: GroupNorm of the same bf16 output in fp64 torch
        assert emb is None
        o = out.double().reshape(N, -1, G, K // G)
        mean = o.mean(dim=(1, 3))
        var = (o * o).mean(dim=(1, 3)) - mean * mean
        rstd = (var + 1e-5).rsqrt()
        ra = (gamma.double()[None] * rstd.repeat_interleave(K // G, dim=1)).float()
        rb = (beta.double()[None] - mean.repeat_interleave(K // G, dim=1) * ra.double()).float()
        rmr = torch.stack([mean, rstd], dim=-1).float()
        y = out.float() * ra.reshape(N, *([1] * (out.dim() - 2)), K) + rb.reshape(N, *([1] * (out.dim() - 2)), K)
        rt = y * torch.sigmoid(y)
    torch.testing.assert_close(mr, rmr, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(a, ra, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(b, rb, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(t.float(), rt.float(), rtol=1e-2, atol=1e-2)
    if halo:   # the split halo conv itself against the unsplit generic conv of the same prologue
        ref_g, _ = O.conv(x, K, wp, **dict(kw, splits=1, force_generic=True))
        _close(out, ref_g.float(), rel=1e-2)
    if cb != 4:
        _lib.call("fmd_conv_gn_set_block_channels", 4)


@pytest.mark.parametrize("N,splits", [(1, None), (3, None), (3, 1)])
def test_conv_1x1_stats_unsplit_tile(N, splits):
    """A 1x1 (transposed) conv with K > 64 that runs unsplit on a small image: the host must pick the kernel's
    128-pixel tile for the fused-statistics test (M = 64 / 192 pixels is not a multiple of it), so the statistics
    come from the separate pass instead of a kernel error; output and statistics vs torch."""
    O = ops()
    H = W = 8
    Cin = K = 128
    dy = _rand_nhwc(N, H, W, Cin, 81)
    w = _w(Cin, K, 1, 82)   # forward weight [Cin_fwd=Cin][K][1][1] of the conv whose data gradient this is
    got, st = O.conv(dy.to(DEV), K, O.prep_weights(w.to(DEV), 1), ks=1, pad=0, transposed=True, out_hw_=(H, W),
                     want_stats=True, splits=splits)
    ref = torch.einsum("nhwc,ck->nhwk", dy.float(), _bfw(w)[:, :, 0, 0])
    _close(got, ref)
    refst = O.channel_stats(got, rows=st.rows)
    torch.testing.assert_close(st.slab, refst.slab, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("mode", ["s1", "s2", "up", "1x1", "s2_split"])
def test_conv_data_gradient(mode):
    """Data gradients through the generic implicit GEMM; s2 runs the parity-class decomposition of the
    stride-2 transposed gather (csrc/conv.hip ``par``), s2_split the same with split-K partial slabs."""
    O = ops()
    split = mode.endswith("_split")
    mode = mode.replace("_split", "")
    N, H, W, C, K = 2, 16, 16, 64, 128
    ks, s, up = (1, 1, False) if mode == "1x1" else (3, 2 if mode == "s2" else 1, mode == "up")
    pad = ks // 2
    x = _to_nchw(_rand_nhwc(N, H, W, C, 11)).requires_grad_()
    w = _w(K, C, ks, 12)
    xin = F.interpolate(x, scale_factor=2, mode="nearest") if up else x
    y = F.conv2d(xin, _bfw(w), stride=s, padding=pad)
    dy = torch.randn_like(y).to(torch.bfloat16).float()
    y.backward(dy)
    dyn = dy.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).to(DEV)
    if up:
        got, _ = O.conv(dyn, C, O.prep_weights(w.to(DEV), 2), ks=4, stride=2, pad=1, out_hw_=(H, W))
    else:
        got, _ = O.conv(dyn, C, O.prep_weights(w.to(DEV), 1), ks=ks, stride=s, pad=pad, transposed=True,
                        out_hw_=(H, W), splits=3 if split else None)
    _close(got, x.grad.permute(0, 2, 3, 1))


@pytest.mark.parametrize("mode", ["s1", "s2", "up", "1x1", "pro", "s1_generic", "pro_generic", "up_generic",
                                  "stem", "stem_pro", "stem_s2"])
def test_wgrad(mode):
    """16x16, C=64, K=128: the 3x3 stride-1 modes run the halo kernel (csrc/wgrad_halo.hip) unless *_generic.
    stem*: C=8 (the padded 2-channel conv_in): the generic kernel's merged (tap, cin) column tile."""
    O = ops()
    generic = mode.endswith("_generic")
    mode = mode.replace("_generic", "")
    N, H, W, C, K = 2, 16, 16, 64, 128
    if mode.startswith("stem"):
        C, K = 8, 96
        mode = {"stem": "s1", "stem_pro": "pro", "stem_s2": "s2"}[mode]
    ks, s, up = (1, 1, False) if mode == "1x1" else (3, 2 if mode == "s2" else 1, mode == "up")
    pad = ks // 2
    xb = _rand_nhwc(N, H, W, C, 13)
    x = _to_nchw(xb)
    pro = None
    if mode == "pro":
        a = torch.rand(N, C) + 0.5
        b = torch.randn(N, C) * 0.2
        x = F.silu(x * a[:, :, None, None] + b[:, :, None, None]).to(torch.bfloat16).float()
        pro = (a.to(DEV), b.to(DEV), True)
    w = _w(K, C, ks, 14).requires_grad_()
    bias = torch.zeros(K, requires_grad=True)
    xin = F.interpolate(x, scale_factor=2, mode="nearest") if up else x
    y = F.conv2d(xin, w, bias, stride=s, padding=pad)
    dy = torch.randn_like(y).to(torch.bfloat16).float()
    y.backward(dy)
    dw = torch.zeros(K, C, ks, ks, device=DEV)
    db = torch.zeros(K, device=DEV)
    O.wgrad(xb.to(DEV), dy.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).to(DEV), dw, ks=ks, stride=s,
            pad=pad, upsample=up, pro=pro, db=db, force_generic=generic)
    torch.testing.assert_close(dw.cpu(), w.grad, rtol=2e-2, atol=2e-2 * w.grad.abs().max().item())
    torch.testing.assert_close(db.cpu(), bias.grad, rtol=1e-3, atol=1e-3 * bias.grad.abs().max().item())


@pytest.mark.parametrize("splits,generic", [(3, False), (20, False), (64, False), (37, True)])
def test_wgrad_split_combine(splits, generic):
    """The weight-gradient split-K combine (wgrad_reduce2): wide splits (more than 16 slab lanes), accumulate into
    dW/db, vs torch; repeated runs are bit-identical (fixed summation order)."""
    O = ops()
    N, H, W, C, K = 4, 32, 32, 64, 128
    xb = _rand_nhwc(N, H, W, C, 61)
    w = _w(K, C, 3, 62).requires_grad_()
    bias = torch.zeros(K, requires_grad=True)
    y = F.conv2d(_to_nchw(xb), w, bias, padding=1)
    dy = torch.randn_like(y).to(torch.bfloat16).float()
    y.backward(dy)
    dyn = dy.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).to(DEV)
    g = torch.Generator().manual_seed(63)
    dw0, db0 = torch.randn(K, C, 3, 3, generator=g), torch.randn(K, generator=g)
    outs = []
    for _ in range(2):
        dw, db = dw0.clone().to(DEV), db0.clone().to(DEV)
        O.wgrad(xb.to(DEV), dyn, dw, db=db, accumulate=True, splits=splits, force_generic=generic)
        outs.append((dw.cpu(), db.cpu()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    torch.testing.assert_close(outs[0][0] - dw0, w.grad, rtol=2e-2, atol=2e-2 * w.grad.abs().max().item())
    torch.testing.assert_close(outs[0][1] - db0, bias.grad, rtol=1e-3, atol=1e-3 * bias.grad.abs().max().item())


@pytest.mark.parametrize("case", ["concat_pro", "wide_dy_offset", "many_tiles"])
def test_wgrad_halo_vs_torch(case):
    """Halo-tiled wgrad on multi-tile / multi-split problems: two-source concat with GN+SiLU prologue,
    a dY that is a channel slice of a wider tensor (ldy/dy_offset), and many tiles per split."""
    O = ops()
    N, H, W, C0, C1, K = 2, 32, 32, 64, 128, 128
    if case == "wide_dy_offset":
        C1, K = 0, 256
    if case == "many_tiles":
        N, H, W, C1 = 4, 64, 64, 0
    C = C0 + C1
    assert O.wgrad_halo_eligible(H, W, H, W, K, C, C0)
    x0 = _rand_nhwc(N, H, W, C0, 31)
    x1 = _rand_nhwc(N, H, W, C1, 32) if C1 else None
    x = _to_nchw(torch.cat([x0, x1], -1) if C1 else x0)
    a = torch.rand(N, C) + 0.5
    b = torch.randn(N, C) * 0.2
    xt = F.silu(x * a[:, :, None, None] + b[:, :, None, None]).to(torch.bfloat16).float()
    w = _w(K, C, 3, 33).requires_grad_()
    bias = torch.zeros(K, requires_grad=True)
    y = F.conv2d(xt, w, bias, padding=1)
    dy = torch.randn_like(y).to(torch.bfloat16).float()
    y.backward(dy)
    dyn = dy.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    off = 0
    if case == "wide_dy_offset":   # dY lives at channels [64, 64+K) of a 384-channel tensor
        wide = torch.zeros(N, H, W, 384, dtype=torch.bfloat16)
        wide[..., 64:64 + K] = dyn
        dyn, off = wide, 64
    dw = torch.zeros(K, C, 3, 3, device=DEV)
    db = torch.zeros(K, device=DEV)
    O.wgrad(x0.to(DEV), dyn.to(DEV), dw, src1=x1.to(DEV) if C1 else None, pro=(a.to(DEV), b.to(DEV), True),
            db=db, dy_offset=off)
    torch.testing.assert_close(dw.cpu(), w.grad, rtol=2e-2, atol=2e-2 * w.grad.abs().max().item())
    torch.testing.assert_close(db.cpu(), bias.grad, rtol=1e-3, atol=1e-3 * bias.grad.abs().max().item())


@pytest.mark.parametrize("case", ["plain", "pro_concat"])
def test_wgrad_halo_stride2_vs_torch(case):
    """Halo weight gradient of a 2-D stride-2 3x3 conv (the space-to-depth planes as chunks: DownsampleND's conv,
    csrc/wgrad_halo.hip S2D) vs torch autograd on the bf16-rounded operands, and vs the generic kernel on the same
    inputs; the second case with a GN+SiLU prologue over a two-source concat."""
    O = ops()
    g = torch.Generator().manual_seed(97)
    N, H, W, C0, K = 4, 64, 64, 64, 128
    C1 = 64 if case == "pro_concat" else 0
    x0 = _rand_nhwc(N, H, W, C0, 98)
    x1 = _rand_nhwc(N, H, W, C1, 99) if C1 else None
    x = _to_nchw(torch.cat([x0, x1], -1) if C1 else x0)
    C = C0 + C1
    pro = None
    if case == "pro_concat":
        a = torch.rand(N, C, generator=g) + 0.5
        b = torch.randn(N, C, generator=g) * 0.2
        pro = (a.to(DEV), b.to(DEV), True)
        x = F.silu(x * a[:, :, None, None] + b[:, :, None, None]).to(torch.bfloat16).float()
    w = (torch.randn(K, C, 3, 3, generator=g) / math.sqrt(C * 9)).requires_grad_()
    bias = torch.zeros(K, requires_grad=True)
    y = F.conv2d(x, w, bias, stride=2, padding=1)
    dy = torch.randn_like(y).to(torch.bfloat16).float()
    y.backward(dy)
    dyn = dy.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).to(DEV)
    assert O.wgrad_halo_eligible(H, W, H // 2, W // 2, K, C, C0, 3, 2)
    res = []
    for generic in (False, True):
        dw = torch.zeros(K, C, 3, 3, device=DEV)
        db = torch.zeros(K, device=DEV)
        O.wgrad(x0.to(DEV), dyn, dw, src1=x1.to(DEV) if C1 else None, pro=pro, ks=3, stride=2, pad=1, db=db,
                force_generic=generic)
        res.append((dw.cpu(), db.cpu()))
    for dw, db in res:
        torch.testing.assert_close(dw, w.grad, rtol=2e-2, atol=2e-2 * w.grad.abs().max().item())
        torch.testing.assert_close(db, bias.grad, rtol=1e-3, atol=1e-3 * bias.grad.abs().max().item())
    rel = ((res[0][0] - res[1][0]).norm() / res[1][0].norm()).item()
    assert rel < 5e-3, rel


@pytest.mark.parametrize("C,rows_img,N", [(128, 32768, 1), (384, 4096, 2), (1030, 512, 1), (6, 256, 3)])
def test_stats_fold(C, rows_img, N):
    """fmd_stats_fold: 128 consecutive slab rows summed (row-lane chains + fixed-order lane combine) vs torch."""
    O = ops()
    g = torch.Generator().manual_seed(C)
    slab = torch.randn(N * rows_img, C, 2, generator=g).to(DEV)
    st = O.fold_stats(O.Stats(slab, 64), rows_img * 64) if rows_img >= O.STATS_FOLD_MIN else None
    out = torch.empty(N * rows_img // 128, C, 2, device=DEV)
    from fmdiff import _lib
    _lib.call("fmd_stats_fold", slab.data_ptr(), N * rows_img, C, 128, out.data_ptr(), O.stream())
    ref = slab.view(-1, 128, C, 2).double().sum(1).float()
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-4)
    if st is not None:
        assert st.rows == 64 * 128 and torch.equal(st.slab, out)


@pytest.mark.parametrize("fold", [False, True])
def test_groupnorm_forward_backward(fold, monkeypatch):
    """GroupNorm forward / backward through the slab statistics path; ``fold`` runs the slabs through
    fmd_stats_fold first (forced on this small problem)."""
    O = ops()
    if fold:
        monkeypatch.setattr(O, "STATS_FOLD_MIN", 2)
        monkeypatch.setattr(O, "STATS_FOLD", 2)
    N, H, W, C, G = 2, 16, 16, 96, 32
    xb = _rand_nhwc(N, H, W, C, 15, 2.0) .float().add(0.5).to(torch.bfloat16)
    x = _to_nchw(xb).requires_grad_()
    gamma = (torch.rand(C) + 0.5).requires_grad_()
    beta = (torch.randn(C) * 0.1).requires_grad_()
    emb = torch.randn(N, 2 * C) * 0.3
    scale, shift = emb[:, :C], emb[:, C:]
    z = F.group_norm(x, G, gamma, beta, 1e-5) * (1 + scale[:, :, None, None]) + shift[:, :, None, None]
    dz = torch.randn_like(z).to(torch.bfloat16).float()
    z.backward(dz)
    st = O.channel_stats(xb.to(DEV))
    a, b, mr = O.gn_prep(st, None, N, H * W, C, 0, G, 1e-5, gamma.detach().to(DEV), beta.detach().to(DEV),
                         emb=emb.to(DEV), emb_stride=2 * C, emb_mode=1)
    zk = xb.float().to(DEV) * a[:, None, None, :] + b[:, None, None, :]
    _close(zk, z.detach().permute(0, 2, 3, 1), rel=1e-4)
    dzn = dz.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).to(DEV)
    s12 = O.channel_stats(dzn, y=(xb.to(DEV), None, C))
    dg = torch.zeros(C, device=DEV)
    dbt = torch.zeros(C, device=DEV)
    demb = torch.zeros(N, 2 * C, device=DEV)
    P, Q, R = O.gn_bwd_prep(s12, N, H * W, C, G, mr, gamma.detach().to(DEV), beta.detach().to(DEV), dg, dbt,
                            emb=emb.to(DEV), emb_stride=2 * C, emb_mode=1, demb=demb, demb_stride=2 * C)
    dx = torch.empty_like(dzn)
    O.gn_bwd_apply(dzn, xb.to(DEV), None, P, Q, R, None, dx, 0)
    _close(dx, x.grad.permute(0, 2, 3, 1))
    torch.testing.assert_close(dg.cpu(), gamma.grad, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(dbt.cpu(), beta.grad, rtol=1e-3, atol=1e-3)
    ref_ds = (dz * F.group_norm(x.detach(), G, gamma.detach(), beta.detach(), 1e-5)).sum((2, 3))
    torch.testing.assert_close(demb[:, :C].cpu(), ref_ds, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(demb[:, C:].cpu(), dz.sum((2, 3)), rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("H,W,C0,C1,G,ss", [(8, 8, 512, 0, 32, True), (16, 16, 256, 256, 32, False),
                                             (4, 4, 512, 512, 32, True), (32, 32, 128, 0, 32, False),
                                             (1, 1, 512, 0, 32, True), (2, 2, 96, 32, 8, False)])
def test_gn_fused_apply_vs_torch(H, W, C0, C1, G, ss):
    """fmd_gn_fused_apply (small-level GroupNorm forward in one launch, statistics straight from x0|x1) vs
    F.group_norm (+ scale/shift) + SiLU in fp32, and its a/b/mean_rstd vs the slab path (channel_stats +
    gn_prep) that the backward also accepts."""
    O = ops()
    N = 3
    C = C0 + C1
    g = torch.Generator().manual_seed(H * 1000 + C)
    x = (torch.randn(N, C, H, W, generator=g) * 1.5 + 0.3).to(torch.bfloat16)
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g) * 0.1
    emb = torch.randn(N, 2 * C, generator=g) * 0.3 if ss else None
    z = F.group_norm(x.float(), G, gamma, beta, 1e-5)
    if ss:
        z = z * (1 + emb[:, :C, None, None]) + emb[:, C:, None, None]
    ref = F.silu(z).permute(0, 2, 3, 1)
    xn = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    x0, x1 = xn[..., :C0].contiguous(), (xn[..., C0:].contiguous() if C1 else None)
    a, b, mr, t = O.gn_fused_apply(x0, x1, G, 1e-5, gamma.to(DEV), beta.to(DEV),
                                   emb=emb.to(DEV) if ss else None, emb_stride=2 * C if ss else 0,
                                   emb_mode=1 if ss else 0)
    _close(t.float(), ref, rel=1.5e-2)
    st0 = O.channel_stats(x0)
    st1 = O.channel_stats(x1) if C1 else None
    a2, b2, mr2 = O.gn_prep(st0, st1, N, H * W, C0, C1, G, 1e-5, gamma.to(DEV), beta.to(DEV),
                            emb=emb.to(DEV) if ss else None, emb_stride=2 * C if ss else 0, emb_mode=1 if ss else 0)
    torch.testing.assert_close(a.cpu(), a2.cpu(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(b.cpu(), b2.cpu(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(mr.cpu(), mr2.cpu(), rtol=1e-4, atol=1e-5)


def test_groupnorm_deferred_gamma_beta_fold():
    """gb_defer/gb_flush (fmd_gn_gb_fold, one launch for many GroupNorms, incl. > FMD_GB_MAX jobs and
    dgamma-only jobs) == the per-call fold of fmd_gn_bwd_prep, bit for bit."""
    O = ops()
    N, HW, G = 2, 64, 8
    shapes = [(32 + 16 * (i % 5)) for i in range(70)]
    g = torch.Generator().manual_seed(5)
    cases = []
    for i, Cc in enumerate(shapes):
        slab = torch.randn(N * HW // 64, Cc, 2, generator=g).to(DEV)
        mr = torch.stack([torch.randn(N, G, generator=g), torch.rand(N, G, generator=g) + 0.5], -1).to(DEV)
        gamma = (torch.rand(Cc, generator=g) + 0.5).to(DEV)
        beta = torch.randn(Cc, generator=g).to(DEV)
        init = torch.randn(2, Cc, generator=g).to(DEV)
        cases.append((O.Stats(slab, 64), Cc, mr, gamma, beta, init, i % 7 == 3))
    ref, got = [], []
    for st, Cc, mr, gamma, beta, init, no_beta in cases:
        dg, db = init[0].clone(), init[1].clone()
        O.gn_bwd_prep(st, N, HW, Cc, G, mr, gamma, beta, dg, None if no_beta else db)
        ref.append((dg, db))
    O.gb_defer()
    for st, Cc, mr, gamma, beta, init, no_beta in cases:
        dg, db = init[0].clone(), init[1].clone()
        O.gn_bwd_prep(st, N, HW, Cc, G, mr, gamma, beta, dg, None if no_beta else db)
        got.append((dg, db))
    O.gb_flush()
    torch.cuda.synchronize()
    for (a0, b0), (a1, b1) in zip(ref, got):
        assert torch.equal(a0, a1) and torch.equal(b0, b1)


@pytest.mark.parametrize("raw,T,heads,dh", [(1, 64, 4, 64), (0, 256, 16, 8), (0, 64, 8, 32), (1, 64, 2, 16),
                                         (1, 1024, 4, 64), (0, 300, 2, 40), (1, 100, 3, 24), (0, 17, 2, 64),
                                         (0, 1000, 1, 12), (1, 4096, 2, 32)])
def test_attention(raw, T, heads, dh):
    O = ops()
    B = 2
    inner = heads * dh
    qkv = (torch.randn(B, T, 3 * inner) * 0.5).to(torch.bfloat16)
    f = qkv.float().requires_grad_()
    if raw:
        flat = f.transpose(1, 2).reshape(B, heads, T, 3 * dh)   # (B, 3*inner, T) read raw
        q, k, v = flat.chunk(3, dim=-1)
    else:
        q, k, v = (f[..., i * inner:(i + 1) * inner].view(B, T, heads, dh).transpose(1, 2) for i in range(3))
    o = F.scaled_dot_product_attention(q, k, v)
    if raw:
        o_tok = o.reshape(B, inner, T).transpose(1, 2)          # raw reinterpretation as (inner, T)
    else:
        o_tok = o.transpose(1, 2).reshape(B, T, inner)
    do = torch.randn_like(o_tok).to(torch.bfloat16).float()
    o_tok.backward(do)
    og, lse = O.attention_fwd(qkv.to(DEV), T, heads, dh, raw)
    _close(og, o_tok.detach())
    dq = O.attention_bwd(qkv.to(DEV), og, do.contiguous().to(torch.bfloat16).to(DEV), lse, T, heads, dh, raw)
    _close(dq, f.grad, rel=2e-2)
    if hasattr(lse, "lse"):   # MFMA path: the backward from a bare lse re-packs q, k, v, o -- same result
        dq2 = O.attention_bwd(qkv.to(DEV), og, do.contiguous().to(torch.bfloat16).to(DEV), lse.lse, T, heads, dh, raw)
        assert torch.equal(dq, dq2)


@pytest.mark.parametrize("raw,T,heads,dh", [(1, 256, 4, 64), (1, 4160, 2, 64), (0, 777, 2, 32), (1, 100, 3, 24)])
def test_linear_attention(raw, T, heads, dh):
    """LinearQKVAttention (oracle/unet.py _linear_attention, reference attention.py:53-70) vs fp32 autograd;
    T > 1024 splits the token reductions over several chunks."""
    from oracle.unet import _linear_attention
    O = ops()
    B = 2
    inner = heads * dh
    qkv = (torch.randn(B, T, 3 * inner) * 0.7).to(torch.bfloat16)
    f = qkv.float().requires_grad_()
    if raw:
        q, k, v = f.transpose(1, 2).reshape(B, heads, T, 3 * dh).chunk(3, dim=-1)
    else:
        q, k, v = (f[..., i * inner:(i + 1) * inner].view(B, T, heads, dh).transpose(1, 2) for i in range(3))
    o = _linear_attention(q, k, v)
    o_tok = o.reshape(B, inner, T).transpose(1, 2) if raw else o.transpose(1, 2).reshape(B, T, inner)
    do = torch.randn_like(o_tok).to(torch.bfloat16).float()
    o_tok.backward(do)
    og, state = O.linear_attention_fwd(qkv.to(DEV), T, heads, dh, raw)
    _close(og, o_tok.detach())
    dq = O.linear_attention_bwd(qkv.to(DEV), do.contiguous().to(torch.bfloat16).to(DEV), state, T, heads, dh, raw)
    _close(dq, f.grad, rel=2e-2)


@pytest.mark.parametrize("linear,Tq,Tk,heads,dh", [(0, 256, 1024, 4, 64), (0, 70, 33, 2, 32), (0, 1, 300, 2, 16),
                                                  (0, 600, 5, 3, 48), (1, 256, 1024, 4, 64),
                                                  (1, 1500, 2100, 2, 24)])
def test_cross_attention(linear, Tq, Tk, heads, dh):
    """SpatialCrossAttention core (reference attention.py:179-184: raw q / kv reshapes, chunk(2)) vs fp32 autograd,
    softmax and LinearQKVAttention."""
    from oracle.unet import _linear_attention
    O = ops()
    B = 2
    inner = heads * dh
    qb = (torch.randn(B, Tq, inner) * 0.7).to(torch.bfloat16)
    kvb = (torch.randn(B, Tk, 2 * inner) * 0.7).to(torch.bfloat16)
    qf, kvf = qb.float().requires_grad_(), kvb.float().requires_grad_()
    q = qf.transpose(1, 2).reshape(B, heads, Tq, dh)
    k, v = kvf.transpose(1, 2).reshape(B, heads, Tk, 2 * dh).chunk(2, dim=-1)
    o = _linear_attention(q, k, v) if linear else F.scaled_dot_product_attention(q, k, v)
    o_tok = o.reshape(B, inner, Tq).transpose(1, 2)
    do = torch.randn_like(o_tok).to(torch.bfloat16).float()
    o_tok.backward(do)
    eps = 1e-6 if linear else None
    og, saved = O.cross_attention_fwd(qb.to(DEV), kvb.to(DEV), Tq, Tk, heads, dh, eps)
    _close(og, o_tok.detach())
    dq, dkv = O.cross_attention_bwd(qb.to(DEV), kvb.to(DEV), og, do.contiguous().to(torch.bfloat16).to(DEV), saved,
                                    Tq, Tk, heads, dh, eps)
    _close(dq, qf.grad, rel=2e-2)
    _close(dkv, kvf.grad, rel=2e-2)


def test_time_embedding_and_linear():
    O = ops()
    from oracle.unet import timestep_embedding
    t = torch.tensor([0.0, 1.0, 17.0, 999.0, 1000.0, 979.6122436523438])
    for dim, flip, shift in [(128, False, 0), (128, True, 0), (33, False, 1)]:
        got = O.timestep_embedding(t.to(DEV), dim, flip, shift)
        torch.testing.assert_close(got.cpu(), timestep_embedding(t, dim, flip_sin_to_cos=flip, freq_shift=shift),
                                   rtol=2e-5, atol=2e-4)
    for Bf, If in ((1, 128), (5, 200), (20, 512), (32, 64)):   # fmd_linear's 8- and 32-row instances, ragged I
        xf = torch.randn(Bf, If)
        wf = torch.randn(300, If) * 0.05
        bf = torch.randn(300) * 0.1
        for silu in (False, True):
            got = O.linear(xf.to(DEV), wf.to(DEV), bf.to(DEV), in_silu=silu)
            torch.testing.assert_close(got.cpu(), F.linear(F.silu(xf) if silu else xf, wf, bf), rtol=1e-4, atol=1e-4)
    x = torch.randn(8, 128, requires_grad=True)
    w = torch.randn(512, 128) * 0.05
    b = torch.randn(512) * 0.1
    for silu in (False, True):
        y = F.linear(F.silu(x) if silu else x, w, b)
        got = O.linear(x.detach().to(DEV), w.to(DEV), b.to(DEV), in_silu=silu)
        torch.testing.assert_close(got.cpu(), y.detach(), rtol=1e-4, atol=1e-4)
        dy = torch.randn_like(y)
        x.grad = None
        wr = w.clone().requires_grad_()
        br = b.clone().requires_grad_()
        F.linear(F.silu(x) if silu else x, wr, br).backward(dy)
        dw = torch.zeros_like(w, device=DEV)
        db = torch.zeros_like(b, device=DEV)
        dx = torch.empty(8, 128, device=DEV)
        O.linear_bwd(x.detach().to(DEV), w.to(DEV), dy.to(DEV), dw, db, dx=dx, in_silu=silu)
        torch.testing.assert_close(dw.cpu(), wr.grad, rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(db.cpu(), br.grad, rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(dx.cpu(), x.grad, rtol=1e-4, atol=1e-4)
        # dx accumulation, and the 512 x 512 layer of the time MLP (I = O = 512, 8 column blocks x 8 batch rows)
        dx2 = dx.clone()
        O.linear_bwd(x.detach().to(DEV), w.to(DEV), dy.to(DEV), dw, db, dx=dx2, dx_acc=True, in_silu=silu)
        torch.testing.assert_close(dx2.cpu(), 2 * x.grad, rtol=1e-4, atol=1e-4)
        x5 = torch.randn(8, 512)
        w5 = torch.randn(512, 512) * 0.05
        dy5 = torch.randn(8, 512)
        dx5 = torch.empty(8, 512, device=DEV)
        O.linear_bwd(x5.to(DEV), w5.to(DEV), dy5.to(DEV), None, None, dx=dx5, in_silu=silu)
        ref5 = dy5 @ w5
        if silu:
            ref5 = ref5 * torch.sigmoid(x5) * (1 + x5 * (1 - torch.sigmoid(x5)))
        torch.testing.assert_close(dx5.cpu(), ref5, rtol=1e-4, atol=1e-4)


def test_adamw_matches_torch():
    O = ops()
    torch.manual_seed(0)
    p0 = torch.randn(10000)
    ref = p0.clone().requires_grad_()
    opt = torch.optim.AdamW([ref], lr=1e-3, weight_decay=0.01, foreach=False)
    p, m, v = p0.clone().to(DEV), torch.zeros(10000, device=DEV), torch.zeros(10000, device=DEV)
    for step in range(1, 4):
        g = torch.randn(10000)
        ref.grad = g.clone()
        opt.step()
        O.adamw(p, g.to(DEV), m, v, 1e-3, 0.9, 0.999, 1e-8, 0.01, step)
    torch.testing.assert_close(p.cpu(), ref.detach(), rtol=1e-6, atol=1e-7)


def _conv3x3_ref64(z, w, bias=None):
    """fp64 3x3 pad-1 conv of NCHW ``z`` (any float dtype) with ``w`` [K][C][3][3]: im2col + matmul in fp64 on the
    device (no fp64 path in MIOpen), returns NHWC fp64."""
    N, C, H, W = z.shape
    cols = F.unfold(z.double(), 3, padding=1)                              # [N][C*9][H*W]
    y = torch.einsum("kc,ncp->npk", w.double().reshape(w.shape[0], -1), cols)
    if bias is not None:
        y = y + bias.double()
    return y.reshape(N, H, W, -1)


@pytest.mark.parametrize("case", ["plain", "pro_concat_stats", "upsample", "skip_seg2", "skip_wide", "dgrad_ep",
                                  "k64", "k256_pro_nosilu"])
def test_halo_conv_matches_generic(case):
    """csrc/conv_halo9.hip (halo staged once per chunk) vs the per-tap implicit GEMM (csrc/conv.hip), and both against
    an fp64 reference of the same op, for three fixed seeds.

    N=8 at 64x64 = 128 tiles: the smallest problem the halo path accepts (fmd_conv_halo), so every case runs it.
    Every input -- activations, weights, bias, prologue affine, data-gradient epilogue -- comes from a local
    generator seeded per (case, seed), so neither test order nor the global RNG changes what is compared.

    Statistics (the GroupNorm-forward sums (sum y, sum y^2), or the data-gradient epilogue's GroupNorm-backward sums
    (sum dz, sum dz*x) with dz = conv(dy) * SiLU'(a x + b), reference residual.py:84-120 via normalization.py:11-19),
    per (sample, channel), for each path, two bounds derived from the summands t_p, not fixed constants:
      (1) the slab equals the fp64 sum of the path's OWN bf16 outputs within 1e-5 ||t||_1 (fp32 summation error):
          catches a lost, doubled or mis-paired pixel exactly, whatever the rounding;
      (2) it equals the fp64 sum of the exact (unrounded) terms within 6 * 2^-8 ||t||_2: each summand carries one
          zero-mean round-to-nearest error of at most 2^-8 |t|, so the Hoeffding bound is exceeded with probability
          <= 3e-8 per sum.

    Round 5's scratch failure of the dgrad_ep case (0.168 vs the old fixed 3e-2 between the two paths) came from the
    halo v10 development build, whose data-gradient epilogue took SiLU' in fp16 (reproduced in round 6 on the v10
    tree)."""
    O = ops()
    N, H, W = 8, 64, 64
    C0, C1, K = 64, 0, 128
    if case == "pro_concat_stats":
        C1 = 96
    if case == "k64":
        K = 64
    if case == "k256_pro_nosilu":
        C0, K = 192, 256
    up = case == "upsample"
    Hs, Ws = (H // 2, W // 2) if up else (H, W)
    Cin = C0 + C1
    assert O.halo_eligible(N, Hs, H, W, K, upsample=up)
    for seed in (0, 1, 2):
        g = torch.Generator().manual_seed(1000 * seed + sum(map(ord, case)))

        def rnd(*s, scale=1.0):
            return torch.randn(*s, generator=g) * scale

        x0 = rnd(N, Hs, Ws, C0).to(torch.bfloat16).to(DEV)
        x1 = rnd(N, Hs, Ws, C1).to(torch.bfloat16).to(DEV) if C1 else None
        wf = rnd(K, Cin, 3, 3, scale=1.0 / math.sqrt(Cin * 9))
        w = O.prep_weights(wf.to(DEV), 0)
        bias = rnd(K, scale=0.1)
        kw = dict(bias=bias.to(DEV))
        pro = None
        if case in ("pro_concat_stats", "upsample", "skip_wide", "k256_pro_nosilu"):
            pro = (torch.rand(N, Cin, generator=g) + 0.5, rnd(N, Cin, scale=0.2), case != "k256_pro_nosilu")
            kw["pro"] = (pro[0].to(DEV), pro[1].to(DEV), pro[2])
        skip = None
        if case in ("skip_seg2", "skip_wide"):
            c2, c3 = (96, 32) if case == "skip_seg2" else (256, 128)
            s2 = rnd(N, H, W, c2).to(torch.bfloat16).to(DEV)
            s3 = rnd(N, H, W, c3).to(torch.bfloat16).to(DEV)
            w2f = rnd(K, c2 + c3, 1, 1, scale=1.0 / math.sqrt(c2 + c3))
            b2 = rnd(K, scale=0.1)
            skip = (s2, s3, w2f, b2)
            kw.update(src2=s2, src3=s3, wgt2=O.prep_weights(w2f.to(DEV), 0), bias2=b2.to(DEV), resid=None)
        ep = None
        if case == "dgrad_ep":
            ep = (rnd(N, H, W, K).to(torch.bfloat16).to(DEV), torch.rand(N, K, generator=g) + 0.5,
                  rnd(N, K, scale=0.2))
            kw["ep"] = (ep[0], None, ep[1].to(DEV), ep[2].to(DEV))
        want = case in ("pro_concat_stats", "dgrad_ep", "upsample")
        a, sa = O.conv(x0, K, w, src1=x1, upsample=up, want_stats=want, **kw)
        b, sb = O.conv(x0, K, w, src1=x1, upsample=up, want_stats=want, force_generic=True, **kw)

        # fp64 reference (the conv operand rounded to bf16 where the kernels round it: the staged prologue output)
        xc = torch.cat([x0, x1], -1) if x1 is not None else x0
        z = xc.double().permute(0, 3, 1, 2)
        if pro is not None:
            pa, pb = pro[0].double().to(DEV)[:, :, None, None], pro[1].double().to(DEV)[:, :, None, None]
            z = z * pa + pb
            if pro[2]:
                z = F.silu(z)
            z = z.to(torch.bfloat16).double()
        if up:
            z = F.interpolate(z, scale_factor=2, mode="nearest")
        y = _conv3x3_ref64(z, wf.to(torch.bfloat16).to(DEV), bias.to(DEV))
        if skip is not None:
            s = torch.cat([skip[0], skip[1]], -1).double()
            y = y + s @ skip[2].reshape(K, -1).to(torch.bfloat16).to(DEV).double().t() + skip[3].to(DEV).double()
        if ep is not None:
            xe = ep[0].double()
            zz = ep[1].double().to(DEV)[:, None, None, :] * xe + ep[2].double().to(DEV)[:, None, None, :]
            sg = torch.sigmoid(zz)
            y = y * (sg * (1 + zz * (1 - sg)))
        scale = y.abs().max().item()
        for got in (a, b):
            err = (got.double() - y).abs().max().item()
            assert err <= 1e-2 * scale, f"{case} seed {seed}: output max err {err:.3e} vs scale {scale:.3e}"
        torch.testing.assert_close(a.float(), b.float(), rtol=1e-2, atol=1e-2 * b.float().abs().max().item())
        if want:
            xe = ep[0].double().reshape(N, -1, K) if ep is not None else None

            def terms(v):   # the two summands per (sample, channel): (v, v*x) or (v, v^2), fp64, [N][HW][K] each
                v = v.double().reshape(N, -1, K)
                return v, (v * xe if xe is not None else v * v)

            def sums(tt):
                return torch.stack([tt[0].sum(1), tt[1].sum(1)], -1)                # [N][K][2]

            def norm(tt, p):
                return torch.stack([tt[0].norm(p=p, dim=1), tt[1].norm(p=p, dim=1)], -1)

            te = terms(y)
            ref, l2, l1e = sums(te), norm(te, 2), norm(te, 1)
            report = []
            for name, out, st in (("halo", a, sa), ("generic", b, sb)):
                tot = st.slab.double().view(N, -1, K, 2).sum(1)
                # (1) the slab is the sum of the path's OWN bf16 outputs, up to fp32 summation error
                to = terms(out)
                own, l1 = sums(to), norm(to, 1)
                r1 = ((tot - own).abs() / (1e-5 * l1 + 1e-6)).max().item()
                # (2) against the exact fp64 sums: every summand carries one zero-mean round-to-nearest error of at
                # most 2^-8 |t| (2^-9 for the linear terms, 2 x 2^-9 for the squares), so by Hoeffding
                # P(|err| > 6 * 2^-8 ||t||_2) <= 2 exp(-18) = 3e-8 per sum
                r2 = ((tot - ref).abs() / (6 * 2.0 ** -8 * l2 + 1e-6 * l1e)).max().item()
                report.append(f"{name} own {r1:.3f} exact {r2:.3f}")
                assert r1 <= 1, f"{case} seed {seed}: {name} statistics are not the sums of its outputs ({r1:.2f})"
                assert r2 <= 1, f"{case} seed {seed}: {name} statistics exceed the rounding bound ({r2:.2f})"
            print(f"[halo_vs_generic] {case} seed {seed}: worst |err| / bound: {'; '.join(report)}")


@pytest.mark.parametrize("case", ["pro_stats", "resid", "upsample_pro", "skip_seg2", "dgrad_ep", "split_k", "depth3d"])
def test_halo_conv_8_row_tiles_match_16_row_tiles(case):
    """conv3x3_halo9b with 8-row tiles (the default for grids under 1024 workgroups, fmd_halo_set_th8_max_workgroups)
    against the 16-row form on the same problem: outputs bit-identical (same per-pixel summation order), statistics
    equal as per-sample totals (their rows are the same 64-pixel blocks in another order)."""
    from fmdiff import _lib
    O = ops()
    L = _lib.lib()
    N, H, W, C0, K = 8, 64, 64, 64, 128
    d3 = case == "depth3d"
    up = case == "upsample_pro"
    Hs, Ws = (H // 2, W // 2) if up else (H, W)
    if d3:
        N, D, H, W = 2, 8, 32, 32
        Hs, Ws = H, W
        x0 = _rand_ndhwc(N, D, H, W, C0, 41).to(DEV)
        wf = (torch.randn(K, C0, 3, 3, 3) / math.sqrt(C0 * 27)).to(DEV)
    else:
        x0 = _rand_nhwc(N, Hs, Ws, C0, 41).to(DEV)
    kw = dict(bias=(torch.randn(K) * 0.1).to(DEV))
    if case in ("pro_stats", "upsample_pro", "split_k"):
        kw["pro"] = ((torch.rand(N, C0) + 0.5).to(DEV), (torch.randn(N, C0) * 0.2).to(DEV), True)
    if case == "resid":
        kw["resid"] = _rand_nhwc(N, H, W, K, 42).to(DEV)
    if case == "skip_seg2":
        kw.update(src2=_rand_nhwc(N, H, W, 96, 43).to(DEV), src3=_rand_nhwc(N, H, W, 32, 44).to(DEV),
                  wgt2=O.prep_weights(_w(K, 128, 1, 45).to(DEV), 0), bias2=(torch.randn(K) * 0.1).to(DEV))
    if case == "dgrad_ep":
        kw["ep"] = (_rand_nhwc(N, H, W, K, 46).to(DEV), None, (torch.rand(N, K) + 0.5).to(DEV),
                    (torch.randn(N, K) * 0.2).to(DEV))
    if case == "split_k":
        kw["splits"] = 2
    want = case in ("pro_stats", "upsample_pro", "dgrad_ep", "depth3d")
    res = []
    try:
        for lim in (1 << 30, 0):   # 8-row tiles for every grid, then never
            L.fmd_halo_set_th8_max_workgroups(lim)
            if d3:
                from fmdiff.runtime.engine import WeightCache
                out, st = O.conv(x0, K, None, ks=3, want_stats=want, wgt_tiled=WeightCache().dtiled(wf, 0), **kw)
            else:
                w = O.prep_weights(_w(K, C0, 3, 47).to(DEV), 0)
                out, st = O.conv(x0, K, w, upsample=up, want_stats=want, **kw)
            torch.cuda.synchronize()
            res.append((out.clone(), None if st is None else st.slab.clone()))
    finally:
        from fmdiff.runtime import tuning   # the configured value (an FMD_TUNE override included), not the default
        L.fmd_halo_set_th8_max_workgroups(tuning.get("HALO_TH8_MAX_WG"))
    assert torch.equal(res[0][0], res[1][0])
    if want:
        ta = res[0][1].double().view(N, -1, K, 2).sum(1)
        tb = res[1][1].double().view(N, -1, K, 2).sum(1)
        torch.testing.assert_close(ta, tb, rtol=1e-6, atol=1e-4)


@pytest.mark.parametrize("case", ["s2d_pro_stats", "s2d_updgrad", "d2s", "s2d_3d", "d2s_3d"])
def test_halo_stride2_8_row_tiles_match_16_row_tiles(case):
    """fmd_conv_s2d / fmd_conv_d2s with 8-row tiles (grids under 1024 workgroups) against the 16-row form on the same
    problem: outputs bit-identical, statistics equal as per-sample totals."""
    from fmdiff import _lib
    O = ops()
    L = _lib.lib()
    g = torch.Generator().manual_seed(101)
    d3 = case.endswith("_3d")
    kw = {}
    if case.startswith("s2d_pro") or case == "s2d_3d":
        N, C, K = (2 if d3 else 8), 64, 128
        sp = (8, 128, 128) if d3 else (128, 128)
        x = (_rand_ndhwc(N, *sp, C, 102) if d3 else _rand_nhwc(N, *sp, C, 102)).to(DEV)
        w = torch.randn(K, C, *([3] * len(sp)), generator=g) / math.sqrt(C * 27)
        tiled = O.s2d_tile_weights(w.to(DEV), 0)
        if not d3:
            kw["pro"] = ((torch.rand(N, C, generator=g) + 0.5).to(DEV), (torch.randn(N, C, generator=g) * 0.2).to(DEV),
                         True)

        def run():
            return O.conv(x, K, None, ks=3, stride=2, pad=1, bias=(torch.ones(K) * 0.1).to(DEV), want_stats=True,
                          s2d_tiled=tiled, **kw)
    elif case == "s2d_updgrad":
        N, Cin, K, Hl = 8, 128, 64, 64
        w = torch.randn(K, Cin, 3, 3, generator=g) / math.sqrt(Cin * 9)
        dy = _rand_nhwc(N, 2 * Hl, 2 * Hl, K, 103).to(DEV)
        tiled = O.s2d_tile_weights(w.to(DEV), 1)

        def run():
            return O.conv(dy, Cin, None, ks=4, stride=2, pad=1, out_hw_=(Hl, Hl), s2d_tiled=tiled)
    else:
        N, C, K = (1 if d3 else 8), 128, 128
        sp = (8, 64, 64) if d3 else (64, 64)
        w = torch.randn(K, C, *([3] * len(sp)), generator=g) / math.sqrt(C * 27)
        dy = (_rand_ndhwc(N, *[v // 2 for v in sp], K, 104) if d3 else _rand_nhwc(N, *[v // 2 for v in sp], K, 104)).to(DEV)
        tiled = O.s2d_tile_weights(w.to(DEV), 2)

        def run():
            return O.conv(dy, C, None, ks=3, stride=2, pad=1, transposed=True, out_hw_=sp, s2d_tiled=tiled)
    res = []
    try:
        for lim in (1 << 30, 0):
            L.fmd_halo_set_th8_max_workgroups(lim)
            out, st = run()
            torch.cuda.synchronize()
            res.append((out.clone(), None if st is None else st.slab.clone()))
    finally:
        from fmdiff.runtime import tuning   # the configured value (an FMD_TUNE override included), not the default
        L.fmd_halo_set_th8_max_workgroups(tuning.get("HALO_TH8_MAX_WG"))
    assert torch.equal(res[0][0], res[1][0])
    if res[0][1] is not None:
        Kk = res[0][0].shape[-1]
        ta = res[0][1].double().view(N, -1, Kk, 2).sum(1)
        tb = res[1][1].double().view(N, -1, Kk, 2).sum(1)
        torch.testing.assert_close(ta, tb, rtol=1e-6, atol=1e-4)


@pytest.mark.parametrize("case", ["fwd_pro_stats", "dgrad_ep_stats"])
def test_halo_conv_bench_problem_vs_torch(case):
    """The bench's roofline kernel on the bench's own problem -- non-split conv3x3_halo at 8x256^2, 128 -> 128
    channels -- vs an fp32 torch conv of the same op (computed on the GPU, TF32 off):

    * fwd_pro_stats: y = conv3x3(bf16(SiLU(a*x + b))) + bias, with the fused channel statistics;
    * dgrad_ep_stats: the ResBlock data gradient dz = conv_transpose3x3(dy) * SiLU'(a*x + b) (flipped-tap
      weights, mode 3) with the GroupNorm-backward sums (sum dz, sum dz*x).

    Tolerance: max |err| <= 1.5e-2 * max|ref| and relative L2 <= 5e-3 (bf16 output rounding + fp32
    accumulation order); statistics rtol 2e-3."""
    O = ops()
    N, H, W, C, K = 8, 256, 256, 128, 128
    torch.backends.cudnn.allow_tf32 = False
    g = torch.Generator(device=DEV).manual_seed(61)
    x = torch.randn(N, H, W, C, device=DEV, generator=g).to(torch.bfloat16)
    w = torch.randn(K, C, 3, 3, device=DEV, generator=g) / math.sqrt(C * 9)
    a = torch.rand(N, C, device=DEV, generator=g) + 0.5
    b = torch.randn(N, C, device=DEV, generator=g) * 0.2
    wb = w.to(torch.bfloat16).float()
    assert O.halo_eligible(N, H, H, W, K, Cin=C, pro=True) and O.halo_splits(N, H, W, K, C) == 1
    if case == "fwd_pro_stats":
        bias = torch.randn(K, device=DEV, generator=g) * 0.1
        wt = O.tile_weights(O.prep_weights(w, 0))
        out, st = O.conv(x, K, None, pro=(a, b, True), bias=bias, want_stats=True, wgt_tiled=wt)
        z = F.silu(x.float() * a[:, None, None, :] + b[:, None, None, :]).to(torch.bfloat16).float()
        ref = F.conv2d(z.permute(0, 3, 1, 2), wb, bias, padding=1).permute(0, 2, 3, 1)
        xs = None
    else:
        dy = torch.randn(N, H, W, K, device=DEV, generator=g).to(torch.bfloat16)
        wt = O.tile_weights(O.prep_weights(w, 3))
        out, st = O.conv(dy, C, None, ks=3, pad=1, out_hw_=(H, W), wgt_tiled=wt, ep=(x, None, a, b),
                         want_stats=True)
        dx = F.conv_transpose2d(dy.float().permute(0, 3, 1, 2), wb, padding=1).permute(0, 2, 3, 1)
        zz = x.float() * a[:, None, None, :] + b[:, None, None, :]
        s = torch.sigmoid(zz)
        ref = dx * (s * (1 + zz * (1 - s)))
        xs = x.float()
    got = out.float()
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item()
    rel = ((got - ref).norm() / ref.norm()).item()
    print(f"{case}: max err {err:.3e} (scale {scale:.3e}), rel L2 {rel:.3e}")
    assert err <= 1.5e-2 * scale and rel <= 5e-3
    sums = st.slab.view(N, -1, out.shape[-1], 2).sum(1)
    torch.testing.assert_close(sums[..., 0], got.sum((1, 2)), rtol=2e-3, atol=2e-1)
    torch.testing.assert_close(sums[..., 1], (got * (xs if xs is not None else got)).sum((1, 2)), rtol=2e-3,
                               atol=2e-1)


@pytest.mark.parametrize("B,I", [(8, 512), (3, 128), (20, 256), (1, 1024)])
@pytest.mark.parametrize("in_silu", [False, True])
def test_grouped_linear_vs_torch(in_silu, B, I):
    """fmd_grouped_linear(_bwd): several emb projections (O = 256, 1024, 100) in one launch each way; batches
    below, at and above the 8-row kernel instance (B = 20 runs the 32-row one), a ragged last row block."""
    O = ops()
    torch.manual_seed(5)
    lins = [torch.nn.Linear(I, n).to(DEV) for n in (256, 1024, 100)]
    x = torch.randn(B, I, device=DEV)
    gl = O.GroupedLinear(lins, in_silu)
    y = gl.forward(x)
    xr = x.clone().requires_grad_()
    xin = F.silu(xr) if in_silu else xr
    refs = [l(xin) for l in lins]
    torch.testing.assert_close(y, torch.cat(refs, 1), rtol=1e-4, atol=1e-4)
    dy = torch.randn_like(y)
    torch.autograd.backward(refs, [dy[:, o:o + n] for o, n in zip(gl.off, gl.O)])
    want_w = [l.weight.grad.clone() for l in lins]
    want_b = [l.bias.grad.clone() for l in lins]
    for l in lins:
        l.weight.grad = torch.full_like(l.weight, 0.5)   # backward accumulates
        l.bias.grad = torch.full_like(l.bias, 0.25)
    dx = torch.ones(B, I, device=DEV)
    gl.backward(x, dy, dx=dx, dx_acc=True)
    torch.testing.assert_close(dx, xr.grad + 1, rtol=1e-4, atol=1e-4)
    for l, w, b in zip(lins, want_w, want_b):
        torch.testing.assert_close(l.weight.grad, w + 0.5, rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(l.bias.grad, b + 0.25, rtol=1e-4, atol=1e-4)


def test_weight_cache_batched_refresh_matches_individual_preps():
    """fmd_prep_weights_batch (one launch, all layouts from the fp32 masters) == the per-weight
    fmd_prep_weights / fmd_tile_weights_halo results, bit for bit."""
    from fmdiff.runtime.engine import WeightCache
    torch.manual_seed(3)
    wc = WeightCache()
    ws = [torch.randn(128, 128, 3, 3, device=DEV), torch.randn(256, 384, 3, 3, device=DEV),
          torch.randn(1, 128, 3, 3, device=DEV), torch.randn(512, 256, 1, 1, device=DEV),
          torch.randn(256, 256, 3, 3, device=DEV), torch.randn(768, 512, 1, device=DEV)]
    want = {}
    reqs = [(0, 0, None, None), (0, 3, None, None), (0, 1, None, None), (1, 0, None, None), (1, 3, None, None),
            (2, 0, 8, None), (2, 3, 8, None), (3, 0, None, None), (3, 1, None, None), (4, 2, None, None),
            (4, 0, None, None), (5, 0, None, None)]
    for wi, mode, kp, cp in reqs:
        want[("b", wi, mode, kp)] = wc.get(ws[wi], mode, kp, cp).clone()
        if mode in (0, 3) and ws[wi].dim() == 4 and ws[wi].shape[-1] == 3:
            want[("t", wi, mode, kp)] = wc.tiled(ws[wi], mode, kp, cp).clone()
    for e in wc._c.values():
        e["buf"].zero_()
    wc.invalidate()
    torch.cuda.synchronize()
    for (kind, wi, mode, kp), ref in want.items():
        got = wc.get(ws[wi], mode, kp, None) if kind == "b" else wc.tiled(ws[wi], mode, kp, None)
        assert torch.equal(got, ref), (kind, wi, mode, kp)


def test_weight_cache_cubic_batched_refresh_matches_individual_preps():
    """fmd_prep_weights_batch_cubic (3x3x3 masters: base layouts with 27 taps, and the depth-tap halo tiles
    of WeightCache.dtiled, kind 2) == the per-weight fmd_prep_weights_t / fp32 depth-packed view +
    fmd_tile_weights_halo first fills, bit for bit; channel counts off the 16 / 32 tiles included."""
    from fmdiff.runtime.engine import WeightCache
    torch.manual_seed(4)
    wc = WeightCache()
    ws = [torch.randn(128, 128, 3, 3, 3, device=DEV), torch.randn(136, 72, 3, 3, 3, device=DEV),
          torch.randn(64, 8, 3, 3, 3, device=DEV), torch.randn(8, 128, 3, 3, 3, device=DEV)]
    want = {}
    for wi in range(len(ws)):
        for mode in (0, 1, 3):
            want[("b", wi, mode)] = wc.get(ws[wi], mode).clone()
        for mode in (0, 3):
            want[("d", wi, mode)] = wc.dtiled(ws[wi], mode).clone()
    for e in wc._c.values():
        e["buf"].zero_()
    wc.invalidate()
    torch.cuda.synchronize()
    for (kind, wi, mode), ref in want.items():
        got = wc.get(ws[wi], mode) if kind == "b" else wc.dtiled(ws[wi], mode)
        assert torch.equal(got, ref), (kind, wi, mode)


@pytest.mark.parametrize("K,C", [(1, 64), (3, 64), (1, 160), (8, 512)])
def test_head_kernels_vs_torch(K, C):
    """csrc/head.hip: GN-affine+SiLU -> 3x3 conv to K <= 8 channels (fp32 out, Kp = 8), its data gradient
    (SiLU' epilogue + GN-backward sums) and weight/bias gradients, vs torch fp32 autograd on the same
    bf16-rounded inputs.  Tolerance: 1e-2 x max|ref| (bf16 transformed activations / bf16 dz).  12 tiles: from
    C = 128 the forward runs as 4 chunk groups per workgroup (C = 160: 5 chunks, groups idle in the second round;
    C = 512, K = 8: the VAE encoder's head shape)."""
    O = ops()
    N, H, W = 2, 32, 48
    g = torch.Generator().manual_seed(11)
    h = _rand_nhwc(N, H, W, C, 12)
    a = torch.rand(N, C, generator=g) + 0.5
    b = torch.randn(N, C, generator=g) * 0.2
    w = torch.randn(K, C, 3, 3, generator=g) / math.sqrt(C * 9)
    bias = torch.randn(K, generator=g) * 0.1
    dpred = (torch.randn(N, H, W, 8, generator=g) * 0.5).to(torch.bfloat16)
    dpred[..., K:] = 0
    hd, ad, bd = h.to(DEV), a.to(DEV), b.to(DEV)
    out = O.head_fwd(hd, (ad, bd), w.to(DEV), bias.to(DEV), K)
    # reference
    x = _to_nchw(h).requires_grad_()
    z = x * a[:, :, None, None] + b[:, :, None, None]
    t = F.silu(z)
    wr = w.clone().requires_grad_()
    br = bias.clone().requires_grad_()
    ref = F.conv2d(t, wr, br, padding=1)
    _close(out[..., :K], ref.permute(0, 2, 3, 1), rel=1e-2)
    if K < out.shape[-1]:
        assert out[..., K:].abs().max().item() == 0.0
    dref = _to_nchw(dpred)[:, :K]
    ref.backward(dref)
    dw = torch.zeros(K, C, 3, 3, device=DEV)
    db = torch.zeros(K, device=DEV)
    O.head_wgrad(dpred.to(DEV), K, hd, (ad, bd), dw, db)
    _close(dw, wr.grad, rel=1e-2)
    _close(db, br.grad, rel=1e-2)
    dz, st = O.head_dgrad(dpred.to(DEV), w.to(DEV), K, hd, (ad, bd))
    # dz = dL/dz of the pre-activation (the GN-backward input)
    zr = z.detach().requires_grad_()
    F.conv2d(F.silu(zr), w, bias, padding=1).backward(dref)
    dz_ref = zr.grad.permute(0, 2, 3, 1)
    _close(dz, dz_ref, rel=1e-2)
    s = st.slab.double().cpu().view(N, -1, C, 2).sum(1)
    xs = h.double().view(N, -1, C)
    dzd = dz.double().cpu().view(N, -1, C)
    torch.testing.assert_close(s[..., 0], dzd.sum(1), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(s[..., 1], (dzd * xs).sum(1), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("K,C", [(1, 64), (2, 64), (1, 160)])
def test_head_kernels_3d_vs_torch(K, C):
    """csrc/head.hip with depth (D > 0): GN-affine+SiLU -> 3x3x3 conv (zero depth padding) to K <= 2
    channels, its data gradient + GN-backward sums and its weight/bias gradients, vs torch fp32 conv3d
    autograd on the same bf16 inputs (the ConvND(dims=3) head of src/models/unet/unet.py:286-293).
    Tolerance: 1e-2 x max|ref| as in the 2-D test."""
    O = ops()
    N, D, H, W = 2, 5, 16, 32
    g = torch.Generator().manual_seed(21)
    h = (torch.randn(N, D, H, W, C, generator=g)).to(torch.bfloat16)
    a = torch.rand(N, C, generator=g) + 0.5
    b = torch.randn(N, C, generator=g) * 0.2
    w = torch.randn(K, C, 3, 3, 3, generator=g) / math.sqrt(C * 27)
    bias = torch.randn(K, generator=g) * 0.1
    dpred = (torch.randn(N, D, H, W, 8, generator=g) * 0.5).to(torch.bfloat16)
    dpred[..., K:] = 0
    hd, ad, bd = h.to(DEV), a.to(DEV), b.to(DEV)
    out = O.head_fwd(hd, (ad, bd), w.to(DEV), bias.to(DEV), K)
    bc = (slice(None), slice(None), None, None, None)
    z = h.float().permute(0, 4, 1, 2, 3) * a[bc] + b[bc]
    wr = w.clone().requires_grad_()
    br = bias.clone().requires_grad_()
    zr = z.clone().requires_grad_()
    ref = F.conv3d(F.silu(zr), wr, br, padding=1)
    _close(out[..., :K], ref.permute(0, 2, 3, 4, 1), rel=1e-2)
    assert out[..., K:].abs().max().item() == 0.0
    ref.backward(dpred.float().permute(0, 4, 1, 2, 3)[:, :K])
    dw = torch.zeros(K, C, 3, 3, 3, device=DEV)
    db = torch.zeros(K, device=DEV)
    O.head_wgrad(dpred.to(DEV), K, hd, (ad, bd), dw, db)
    _close(dw, wr.grad, rel=1e-2)
    _close(db, br.grad, rel=1e-2)
    dz, st = O.head_dgrad(dpred.to(DEV), w.to(DEV), K, hd, (ad, bd))
    _close(dz, zr.grad.permute(0, 2, 3, 4, 1), rel=1e-2)
    s = st.slab.double().cpu().view(N, -1, C, 2).sum(1)
    xs = h.double().view(N, -1, C)
    dzd = dz.double().cpu().view(N, -1, C)
    torch.testing.assert_close(s[..., 0], dzd.sum(1), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(s[..., 1], (dzd * xs).sum(1), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("C0,C1,Kd", [(128, 128, 128), (64, 0, 256), (256, 128, 128)])
def test_conv1x1_gn_apply_vs_torch(C0, C1, Kd):
    """fmd_conv_gn_apply: the ResBlock skip-conv data gradient (dy @ W_skip) fused into the GroupNorm
    backward apply dx = P*dz + Q*x + R + extra (+ dx), over a two-source concat, vs torch fp32."""
    O = ops()
    N, H, W = 2, 16, 16
    C = C0 + C1
    g = torch.Generator().manual_seed(21)
    dy = _rand_nhwc(N, H, W, Kd, 22)
    w = torch.randn(Kd, C, 1, 1, generator=g) / math.sqrt(Kd)
    dz = _rand_nhwc(N, H, W, C, 23)
    x = _rand_nhwc(N, H, W, C, 24)
    P, Q, R = (torch.randn(N, C, generator=g) * s for s in (1.0, 0.3, 0.1))
    old0 = _rand_nhwc(N, H, W, C0, 25)
    ref = (dy.float().view(N, -1, Kd) @ _bfw(w).view(Kd, C)).view(N, H, W, C)
    ref = ref + P[:, None, None] * dz.float() + Q[:, None, None] * x.float() + R[:, None, None]
    ref[..., :C0] += old0.float()
    d0 = old0.to(DEV).contiguous()
    d1 = torch.empty(N, H, W, C1, device=DEV, dtype=torch.bfloat16) if C1 else None
    x0 = x[..., :C0].contiguous().to(DEV)
    x1 = x[..., C0:].contiguous().to(DEV) if C1 else None
    O.conv1x1_gn_apply(dy.to(DEV), O.prep_weights(w.to(DEV), 1), dz.to(DEV), x0, x1, P.to(DEV), Q.to(DEV),
                       R.to(DEV), d0, 1, d1, 0)
    got = torch.cat([d0, d1], -1) if C1 else d0
    _close(got, ref)


@pytest.mark.parametrize("case", ["pro_stats", "skip_seg2", "dgrad_ep", "concat_resid"])
def test_halo_conv_split_k_matches_generic(case):
    """Small levels (32x32, 4 images): the halo kernel splits its channel chunks over blockIdx.y, writes fp32
    partial slabs and splitk_reduce applies the epilogue (bias, per-sample bias, skip, residual, SiLU'),
    with channel statistics from a separate pass; vs the per-tap implicit GEMM."""
    O = ops()
    N, H, W = 4, 32, 32
    C0, C1, K = 512, 0, 256
    if case == "concat_resid":
        C0, C1 = 256, 256
    x0 = _rand_nhwc(N, H, W, C0, 31).to(DEV)
    x1 = _rand_nhwc(N, H, W, C1, 32).to(DEV) if C1 else None
    w = O.prep_weights(_w(K, C0 + C1, 3, 33).to(DEV), 0)
    kw = dict(bias=(torch.randn(K) * 0.1).to(DEV))
    if case in ("pro_stats", "concat_resid"):
        kw["pro"] = ((torch.rand(N, C0 + C1) + 0.5).to(DEV), (torch.randn(N, C0 + C1) * 0.2).to(DEV), True)
        kw["bias_nc"] = (torch.randn(N, K) * 0.1).to(DEV)
    if case == "skip_seg2":
        s2 = _rand_nhwc(N, H, W, 256, 34).to(DEV)
        s3 = _rand_nhwc(N, H, W, 256, 35).to(DEV)
        kw.update(src2=s2, src3=s3, wgt2=O.prep_weights(_w(K, 512, 1, 36).to(DEV), 0),
                  bias2=(torch.randn(K) * 0.1).to(DEV))
    if case == "concat_resid":
        kw["resid"] = _rand_nhwc(N, H, W, K, 37).to(DEV)
    if case == "dgrad_ep":
        xe = _rand_nhwc(N, H, W, K, 38).to(DEV)
        kw["ep"] = (xe, None, (torch.rand(N, K) + 0.5).to(DEV), (torch.randn(N, K) * 0.2).to(DEV))
    sp = O.halo_splits(N, H, W, K, C0 + C1)
    assert sp > 1 and O.halo_eligible(N, H, H, W, K, Cin=C0 + C1, pro="pro" in kw)
    want = case != "skip_seg2"
    a, sa = O.conv(x0, K, w, src1=x1, want_stats=want, **kw)
    b, sb = O.conv(x0, K, w, src1=x1, want_stats=want, force_generic=True, **kw)
    torch.testing.assert_close(a.float(), b.float(), rtol=1e-2, atol=1e-2 * b.float().abs().max().item())
    if want:
        ta = sa.slab.view(N, -1, K, 2).sum(1)
        tb = sb.slab.view(N, -1, K, 2).sum(1)
        torch.testing.assert_close(ta, tb, rtol=2e-3, atol=2e-2)


@pytest.mark.parametrize("case", ["pro_stats", "skip_seg2", "dgrad_ep", "upsample", "split", "concat_pro"])
def test_halo_conv_matches_generic_implicit_gemm(case):
    """The halo-tiled 3x3 conv (csrc/conv_halo.hip: unrolled 9-tap chunk pipeline, chunk-invariant staging
    geometry) against the generic implicit GEMM (csrc/conv.hip, force_generic) on every epilogue / prologue
    variant the UNet uses: GN+SiLU prologue with statistics, the ResBlock skip 1x1 segment, the dgrad
    SiLU' epilogue with GN-backward sums, nearest-x2 upsample gather, split-K, two-source concat.  Two
    independent kernels, fp32 accumulation in different orders: outputs within bf16 rounding (relative L2
    < 4e-3), statistics within 1e-2 relative."""
    O = ops()
    N, H, W, C, K = 4, 128, 128, 128, 128
    if case == "split":
        N, H, W, C, K = 4, 32, 32, 512, 256
    x = _rand_nhwc(N, H // 2 if case == "upsample" else H, W // 2 if case == "upsample" else W, C, 51).to(DEV)
    w = O.prep_weights(_w(K, C if case != "concat_pro" else 2 * C, 3, 52).to(DEV), 0)
    kw = dict(bias=(torch.randn(K) * 0.1).to(DEV), want_stats=case != "split")
    Ct = 2 * C if case == "concat_pro" else C
    if case in ("pro_stats", "upsample", "split", "concat_pro"):
        kw["pro"] = ((torch.rand(N, Ct) + 0.5).to(DEV), (torch.randn(N, Ct) * 0.2).to(DEV), True)
    if case == "concat_pro":
        kw["src1"] = _rand_nhwc(N, H, W, C, 56).to(DEV)
    if case == "upsample":
        kw["upsample"] = True
    if case == "skip_seg2":
        kw.update(src2=_rand_nhwc(N, H, W, 64, 53).to(DEV), wgt2=O.prep_weights(_w(K, 64, 1, 54).to(DEV), 0))
    if case == "dgrad_ep":
        kw["ep"] = (_rand_nhwc(N, H, W, K, 55).to(DEV), None, (torch.rand(N, K) + 0.5).to(DEV),
                    (torch.randn(N, K) * 0.2).to(DEV))
    assert O.halo_eligible(N, x.shape[1], H, W, K, upsample=case == "upsample", Cin=Ct, pro="pro" in kw)
    wt = O.tile_weights(w)
    w2t = O.tile_weights(kw["wgt2"]) if "wgt2" in kw else None
    oh, sh = O.conv(x, K, w, wgt_tiled=wt, wgt2_tiled=w2t, **kw)
    og, sg = O.conv(x, K, w, force_generic=True, **kw)
    err = ((oh.float() - og.float()).norm() / og.float().norm()).item()
    print(f"{case}: halo vs generic rel L2 {err:.3e}")
    assert err < 4e-3
    if sh is not None:
        a = sh.slab.view(N, -1, K, 2).sum(1)
        b = sg.slab.view(N, -1, K, 2).sum(1)
        serr = ((a - b).norm() / b.norm()).item()
        print(f"{case}: statistics rel L2 {serr:.3e}")
        assert serr < 1e-2


@pytest.mark.parametrize("kind,order,variant,betas", [
    ("dpm", 1, "dpmsolver++", "default"), ("dpm", 2, "dpmsolver++", "default"), ("dpm", 3, "dpmsolver++", "ldct"),
    ("dpm", 2, "heun", "default"), ("dpm", 2, "dpmsolver", "ldct"), ("unipc", 1, "bh2", "default"),
    ("unipc", 2, "bh2", "ldct"), ("unipc", 3, "bh2", "default"), ("unipc", 2, "bh1", "default")])
def test_multistep_schedulers_vs_oracle(kind, order, variant, betas):
    """DPMSolverMultistepScheduler / UniPCMultistepScheduler (host coefficients + fmd_lincomb) vs the CPU
    restatement in oracle/schedulers.py over a 12-step loop with arbitrary model outputs.  ldct betas =
    configs/diffusion/ldct_ddpm.json (linear 0.00085 -> 0.012).  Tolerance 1e-5 relative (fp32 with the
    scalar products folded in a different order)."""
    from oracle import schedulers as OS
    from fmdiff.pipelines.schedulers import DPMSolverMultistepScheduler, UniPCMultistepScheduler
    bk = dict(beta_start=0.00085, beta_end=0.012) if betas == "ldct" else {}
    if kind == "dpm":
        algo = "dpmsolver" if variant == "dpmsolver" else "dpmsolver++"
        kw = dict(solver_order=order, algorithm_type=algo, final_sigmas_type="sigma_min" if algo == "dpmsolver"
                  else "zero", solver_type="heun" if variant == "heun" else "midpoint", **bk)
        ref, got = OS.DPMSolverMultistep(1000, **kw), DPMSolverMultistepScheduler(1000, **kw)
    else:
        kw = dict(solver_order=order, solver_type=variant, **bk)
        ref, got = OS.UniPCMultistep(1000, **kw), UniPCMultistepScheduler(1000, **kw)
    ref.set_timesteps(12)
    got.set_timesteps(12)
    g = torch.Generator().manual_seed(4)
    xr = torch.randn(2, 1, 16, 16, generator=g)
    xg = xr.clone().to(DEV)
    for t in ref.timesteps:
        eps = torch.randn(2, 1, 16, 16, generator=g) * 0.8 + 0.1 * xr
        xr = ref.step(eps, t, xr).prev_sample
        xg = got.step(eps.to(DEV), t, xg).prev_sample
        torch.testing.assert_close(xg.cpu(), xr, rtol=1e-5, atol=1e-5 * xr.abs().max().item())



def _to_ncdhw(x):
    return x.float().permute(0, 4, 1, 2, 3).contiguous()


def _rand_ndhwc(N, D, H, W, C, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(N, D, H, W, C, generator=g) * scale).to(torch.bfloat16)


@pytest.mark.parametrize("mode", ["s1_pro_stats", "s2", "up_concat", "1x1"])
def test_conv3d_forward_vs_torch(mode):
    """3-D implicit GEMM (NDHWC, 3x3x3 / 1x1x1, config E's EfficientUNetND(spatial_dims=3) convs) vs F.conv3d."""
    O = ops()
    N, D, H, W, C0, C1, K = 2, 6, 8, 8, 32, 0, 48
    if mode == "up_concat":
        C1 = 16
    ks, s = (1, 1) if mode == "1x1" else (3, 2 if mode == "s2" else 1)
    pad = ks // 2
    x0 = _rand_ndhwc(N, D, H, W, C0, 61)
    x1 = _rand_ndhwc(N, D, H, W, C1, 62) if C1 else None
    g = torch.Generator().manual_seed(63)
    w = torch.randn(K, C0 + C1, ks, ks, ks, generator=g) / math.sqrt((C0 + C1) * ks ** 3)
    b = torch.randn(K, generator=g) * 0.1
    kw = dict(bias=b.to(DEV), ks=ks, stride=s, pad=pad)
    x = _to_ncdhw(torch.cat([x0, x1], -1) if C1 else x0)
    if mode == "s1_pro_stats":
        a = torch.rand(N, C0) + 0.5
        bb = torch.randn(N, C0) * 0.2
        kw["pro"] = (a.to(DEV), bb.to(DEV), True)
        x = F.silu(x * a[:, :, None, None, None] + bb[:, :, None, None, None]).to(torch.bfloat16).float()
        kw["want_stats"] = True
    if mode == "up_concat":
        kw["upsample"] = True
        x = F.interpolate(x, scale_factor=2, mode="nearest")
    out, st = O.conv(x0.to(DEV), K, O.prep_weights(w.to(DEV), 0), src1=x1.to(DEV) if C1 else None, **kw)
    ref = F.conv3d(x, _bfw(w), b, stride=s, padding=pad).permute(0, 2, 3, 4, 1)
    _close(out, ref)
    if st is not None:
        o = out.float().cpu()
        tot = st.slab.cpu().view(N, -1, K, 2).sum(1)
        torch.testing.assert_close(tot[..., 0], o.sum((1, 2, 3)), rtol=2e-3, atol=2e-2)


@pytest.mark.parametrize("mode", ["s1", "s2", "up"])
def test_conv3d_data_gradient_vs_torch(mode):
    """3-D data gradients: stride 1 = forward gather with reversed taps (mode-3 weights); stride 2 = transposed
    gather; nearest-x2 upsample = high-resolution data gradient + 2x2x2 sum pool (fmd_sum_pool2_3d)."""
    O = ops()
    N, D, H, W, C, K = 2, 4, 8, 8, 32, 48
    s = 2 if mode == "s2" else 1
    x = _to_ncdhw(_rand_ndhwc(N, D, H, W, C, 71)).requires_grad_()
    g = torch.Generator().manual_seed(72)
    w = torch.randn(K, C, 3, 3, 3, generator=g) / math.sqrt(C * 27)
    xin = F.interpolate(x, scale_factor=2, mode="nearest") if mode == "up" else x
    y = F.conv3d(xin, _bfw(w), stride=s, padding=1)
    dy = torch.randn_like(y).to(torch.bfloat16).float()
    y.backward(dy)
    dyn = dy.permute(0, 2, 3, 4, 1).contiguous().to(torch.bfloat16).to(DEV)
    if mode == "s2":
        got, _ = O.conv(dyn, C, O.prep_weights(w.to(DEV), 1), stride=2, transposed=True, out_hw_=(D, H, W))
    else:
        hi = (2 * D, 2 * H, 2 * W) if mode == "up" else (D, H, W)
        g1, _ = O.conv(dyn, C, O.prep_weights(w.to(DEV), 3), out_hw_=hi)
        if mode == "up":
            got = torch.empty(N, D, H, W, C, device=DEV, dtype=torch.bfloat16)
            O.sum_pool2_3d(g1, got)
        else:
            got = g1
    _close(got, x.grad.permute(0, 2, 3, 4, 1), rel=2e-2)


@pytest.mark.parametrize("mode", ["s1_pro", "s2", "up"])
def test_wgrad3d_vs_torch(mode):
    O = ops()
    N, D, H, W, C, K = 2, 4, 8, 8, 32, 48
    s, up = (2 if mode == "s2" else 1), mode == "up"
    xb = _rand_ndhwc(N, D, H, W, C, 81)
    x = _to_ncdhw(xb)
    pro = None
    if mode == "s1_pro":
        a = torch.rand(N, C) + 0.5
        bb = torch.randn(N, C) * 0.2
        x = F.silu(x * a[:, :, None, None, None] + bb[:, :, None, None, None]).to(torch.bfloat16).float()
        pro = (a.to(DEV), bb.to(DEV), True)
    g = torch.Generator().manual_seed(82)
    w = (torch.randn(K, C, 3, 3, 3, generator=g) / math.sqrt(C * 27)).requires_grad_()
    bias = torch.zeros(K, requires_grad=True)
    xin = F.interpolate(x, scale_factor=2, mode="nearest") if up else x
    y = F.conv3d(xin, w, bias, stride=s, padding=1)
    dy = torch.randn_like(y).to(torch.bfloat16).float()
    y.backward(dy)
    dw = torch.zeros(K, C, 3, 3, 3, device=DEV)
    db = torch.zeros(K, device=DEV)
    O.wgrad(xb.to(DEV), dy.permute(0, 2, 3, 4, 1).contiguous().to(torch.bfloat16).to(DEV), dw, stride=s,
            upsample=up, pro=pro, db=db)
    torch.testing.assert_close(dw.cpu(), w.grad, rtol=2e-2, atol=2e-2 * w.grad.abs().max().item())
    torch.testing.assert_close(db.cpu(), bias.grad, rtol=1e-3, atol=1e-3 * bias.grad.abs().max().item())


@pytest.mark.parametrize("case", ["fwd_concat_stats", "fwd_skip", "fwd_resid", "fwd_pro", "dgrad_ep_stats",
                                  "dgrad_acc", "fwd_split", "fwd_up"])
def test_conv3d_depth_halo_matches_generic(case):
    """3x3x3 s1 conv on the halo kernel with (depth tap, channel block) chunks vs the generic 3-D implicit GEMM
    (itself checked against F.conv3d above); N = 2 so the depth-boundary zeros between samples are exercised."""
    O = ops()
    from fmdiff.runtime.engine import WeightCache
    wc = WeightCache()
    N, D, H, W = 2, 66, 16, 16                       # 132 slices x 1 tile: halo-eligible without split
    if case == "fwd_split":
        D = 24                                       # 48 slices: split-K over (kz, channel block) chunks
    C0, C1, K = 64, (32 if case in ("fwd_concat_stats", "fwd_pro") else 0), 128
    dgrad = case.startswith("dgrad")
    up = case == "fwd_up"                            # nearest-x2 source: (D/2, H/2, W/2)
    x0 = _rand_ndhwc(N, D // 2, H // 2, W // 2, C0, 71).to(DEV) if up else _rand_ndhwc(N, D, H, W, C0, 71).to(DEV)
    x1 = _rand_ndhwc(N, D, H, W, C1, 72).to(DEV) if C1 else None
    g = torch.Generator().manual_seed(73)
    Cin = C0 + C1
    w = (torch.randn(K, Cin if not dgrad else C0, 3, 3, 3, generator=g) / math.sqrt(Cin * 27)).to(DEV)
    if dgrad:   # data gradient of a C0 -> K conv: dy has K channels, the result C0
        src, Kout, mode = _rand_ndhwc(N, D, H, W, K, 74).to(DEV), C0, 3
    else:
        src, Kout, mode = x0, K, 0
    b = (torch.randn(Kout, generator=g) * 0.1).to(DEV)
    kw, extra = {}, {}
    if case in ("fwd_concat_stats", "fwd_split"):
        kw = dict(bias=b, bias_nc=(torch.randn(N, Kout, generator=g) * 0.1).to(DEV), want_stats=True)
    elif case == "fwd_pro":
        a_ = (torch.rand(N, Cin, generator=g) + 0.5).to(DEV)
        b_ = (torch.randn(N, Cin, generator=g) * 0.2).to(DEV)
        kw = dict(bias=b, pro=(a_, b_, True), want_stats=True)
    elif case == "fwd_skip":
        ws_ = (torch.randn(K, C0, 1, 1, 1, generator=g) / 8).to(DEV)
        x2 = _rand_ndhwc(N, D, H, W, C0, 75).to(DEV)
        kw = dict(bias=b, bias2=(torch.randn(K, generator=g) * 0.1).to(DEV), want_stats=True, src2=x2)
        extra = dict(wgt2=wc.get(ws_, 0), wgt2_tiled=wc.tiled(ws_, 0))
    elif case == "fwd_up":
        kw = dict(bias=b, want_stats=True, upsample=True)
    elif case == "fwd_resid":
        kw = dict(bias=b, resid=_rand_ndhwc(N, D, H, W, K, 76).to(DEV), want_stats=True)
    elif case == "dgrad_ep_stats":
        xe = _rand_ndhwc(N, D, H, W, C0, 77).to(DEV)
        kw = dict(ep=(xe, None, (torch.rand(N, C0, generator=g) + 0.5).to(DEV),
                      (torch.randn(N, C0, generator=g) * 0.2).to(DEV)), want_stats=True)
    else:
        base = _rand_ndhwc(N, D, H, W, C0, 78).to(DEV)
    src1 = x1 if not dgrad else None
    halo_ok = O.halo_eligible(N * D, H // 2 if up else H, H, W, Kout, upsample=up,
                              Cin=src.shape[-1] + (C1 if not dgrad else 0), pro="pro" in kw, ztaps=3)
    assert halo_ok
    if case == "dgrad_acc":
        kw_g, kw_r = dict(out=base.clone(), accumulate=True), dict(out=base.clone(), accumulate=True)
    else:
        kw_g = kw_r = kw
    got, st = O.conv(src, Kout, None, ks=3, stride=1, pad=1, src1=src1, wgt_tiled=wc.dtiled(w, mode),
                     **{k: v for k, v in extra.items() if k == "wgt2_tiled"}, **kw_g)
    ref, rst = O.conv(src, Kout, wc.get(w, mode), ks=3, stride=1, pad=1, src1=src1, force_generic=True,
                      **{k: v for k, v in extra.items() if k == "wgt2"}, **kw_r)
    _close(got, ref, rel=1e-2)
    if kw.get("want_stats"):
        t1 = st.slab.double().view(N, -1, Kout, 2).sum(1)
        t2 = rst.slab.double().view(N, -1, Kout, 2).sum(1)
        _close(t1, t2, rel=1e-2)


def test_conv_combine_matches_torch():
    """fmd_conv_combine: sum of fp32 split slabs + bias + residual -> bf16, with fused statistics."""
    O = ops()
    g = torch.Generator().manual_seed(81)
    N, D, H, W, K = 2, 4, 8, 8, 64
    M = N * D * H * W
    ws = torch.randn(3, M, K, generator=g).to(DEV)
    b = (torch.randn(K, generator=g) * 0.1).to(DEV)
    r = _rand_ndhwc(N, D, H, W, K, 82).to(DEV)
    out, st = O.conv_combine(ws, K, (N, D, H, W), bias=b, resid=r, want_stats=True)
    ref = (ws.sum(0).view(N, D, H, W, K) + b + r.float()).to(torch.bfloat16)
    _close(out, ref, rel=1e-2)
    s = st.slab.double().view(N, -1, K, 2).sum(1)
    rf = ref.double().view(N, -1, K)
    _close(s[..., 0], rf.sum(1), rel=1e-3)
    _close(s[..., 1], (rf * rf).sum(1), rel=1e-3)


@pytest.mark.parametrize("pro,concat,up", [(True, False, False), (False, True, False), (True, False, True)])
def test_wgrad3d_depth_halo_matches_generic(pro, concat, up):
    """3x3x3 weight gradient on the halo kernel with (depth tap, 64-channel block) input chunks vs the generic
    3-D weight-gradient GEMM (checked against autograd of F.conv3d above); N = 2 exercises the sample
    boundaries of the depth taps."""
    O = ops()
    N, D, H, W, C0, K = 2, 5, 8, 16, 64, 128
    C1 = 64 if concat else 0
    sd, sh, sw = (D // 2 + 1, H // 2, W // 2) if up else (D, H, W)
    if up:
        D = 2 * sd
    assert O.wgrad_halo_eligible(sh, sw, H, W, K, C0 + C1, C0, upsample=up)
    x0 = _rand_ndhwc(N, sd, sh, sw, C0, 91).to(DEV)
    x1 = _rand_ndhwc(N, sd, sh, sw, C1, 92).to(DEV) if C1 else None
    dy = _rand_ndhwc(N, D, H, W, K, 93).to(DEV)
    g = torch.Generator().manual_seed(94)
    pk = (((torch.rand(N, C0 + C1, generator=g) + 0.5).to(DEV), (torch.randn(N, C0 + C1, generator=g) * 0.2).to(DEV),
           True) if pro else None)
    outs = []
    for generic in (False, True):
        dw = torch.zeros(K, C0 + C1, 3, 3, 3, device=DEV)
        db = torch.zeros(K, device=DEV)
        O.wgrad(x0, dy, dw, src1=x1, pro=pk, db=db, force_generic=generic, upsample=up)
        outs.append((dw, db))
    _close(outs[0][0], outs[1][0], rel=1e-2)
    _close(outs[0][1], outs[1][1], rel=1e-3)


@pytest.mark.parametrize("n,offset", [(10001, 0), (4096, 1)])
def test_adamw_sched_matches_torch_with_cosine_warmup(n, offset):
    """fmd_adamw_sched (device-side step counter, get_cosine_schedule_with_warmup LR) vs torch.optim.AdamW +
    transformers' schedule, on a length with a tail and on a misaligned (element-offset) buffer."""
    from transformers import get_cosine_schedule_with_warmup
    O = ops()
    torch.manual_seed(1)
    p0 = torch.randn(n)
    ref = p0.clone().requires_grad_()
    opt = torch.optim.AdamW([ref], lr=2e-3, weight_decay=0.01, foreach=False)
    sch = get_cosine_schedule_with_warmup(opt, 2, 6)
    buf = lambda t: torch.cat([torch.zeros(offset), t]).to(DEV)[offset:]
    p, m, v = buf(p0), buf(torch.zeros(n)), buf(torch.zeros(n))
    ctr = torch.zeros(1, dtype=torch.int32, device=DEV)
    for _ in range(5):
        g = torch.randn(n)
        ref.grad = g.clone()
        opt.step()
        sch.step()
        O.adamw_sched(p, buf(g), m, v, ctr, 2e-3, 2, 6, wd=0.01)
        O.counter_add(ctr)
    torch.testing.assert_close(p.cpu(), ref.detach(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("case", ["plain", "concat", "upsample", "split", "affine", "d3", "d3_up"])
def test_halo_conv_gout_side_output(case):
    """fmd_conv_desc.gout: the halo kernel copies its prologue's output G = SiLU(a*x+b) (or the affine alone)
    for the tile's own pixels out of each staged halo image.  Checks: (1) the conv output agrees with the
    plain call's (another kernel generation: within a bf16 step); (2) every element of G is written (NaN-filled beforehand) and equals
    the fp32 torch transform rounded to bf16 within one bf16 ulp (the kernel's SiLU uses v_exp / v_rcp);
    (3) the weight gradient from G (no prologue) is bit-identical to the one that recomputes GN + SiLU."""
    O = ops()
    d3 = case.startswith("d3")
    up = case in ("upsample", "d3_up")
    if d3:
        N, D, H, W, C0, C1, K = 2, 66, 16, 16, 64, 32, 128
        Ds, Hs, Ws = (D // 2, H // 2, W // 2) if up else (D, H, W)
        C1 = 0 if up else C1
        x0 = _rand_ndhwc(N, Ds, Hs, Ws, C0, 91).to(DEV)
        x1 = _rand_ndhwc(N, Ds, Hs, Ws, C1, 92).to(DEV) if C1 else None
    else:
        N, H, W, C0, C1, K = 4, 128, 128, 128, 0, 128
        if case == "split":
            N, H, W, C0, K = 4, 32, 32, 512, 256
        if case == "concat":
            C1 = 128
        Hs, Ws = (H // 2, W // 2) if up else (H, W)
        x0 = _rand_nhwc(N, Hs, Ws, C0, 91).to(DEV)
        x1 = _rand_nhwc(N, Hs, Ws, C1, 92).to(DEV) if C1 else None
    Ct = C0 + C1
    g = torch.Generator().manual_seed(93)
    a = (torch.rand(N, Ct, generator=g) + 0.5).to(DEV)
    b = (torch.randn(N, Ct, generator=g) * 0.3).to(DEV)
    silu = case != "affine"
    wf = (torch.randn(K, Ct, *((3,) * (3 if d3 else 2)), generator=g) / math.sqrt(Ct * 9)).to(DEV)
    from fmdiff.runtime.engine import WeightCache
    wc = WeightCache()
    wt = wc.dtiled(wf, 0) if d3 else O.tile_weights(O.prep_weights(wf, 0))
    kw = dict(src1=x1, pro=(a, b, silu), bias=(torch.randn(K, generator=g) * 0.1).to(DEV), upsample=up,
              want_stats=case != "split", wgt_tiled=wt)
    if d3:
        kw["out_hw_"] = (D, H, W)
    gout = torch.full((*x0.shape[:-1], Ct), float("nan"), device=DEV, dtype=torch.bfloat16)
    y0, _ = O.conv(x0, K, None, **kw)
    y1, _ = O.conv(x0, K, None, gout=gout, **kw)
    # a gout call runs the round-3 halo kernel, a plain one the v9 kernel (bias as the accumulators' start value):
    # equal up to fp32 summation order, i.e. within a bf16 step
    torch.testing.assert_close(y1.float(), y0.float(), rtol=1e-2, atol=1e-2 * y0.float().abs().max().item())
    xf = torch.cat([x0, x1], -1).float() if x1 is not None else x0.float()
    shp = (N,) + (1,) * (xf.dim() - 2) + (Ct,)
    z = xf * a.view(shp) + b.view(shp)
    ref = (F.silu(z) if silu else z).to(torch.bfloat16).float()
    got = gout.float()
    assert not torch.isnan(got).any(), f"{torch.isnan(got).sum().item()} elements of G never written"
    err = (got - ref).abs()
    print(f"{case}: G max err {err.max().item():.3e}, {(err > 0).float().mean().item():.2e} of elements differ")
    assert (err <= ref.abs() * 2.0 ** -7 + 1e-6).all()
    if case in ("split", "affine"):
        return
    dy = (_rand_ndhwc(N, D, H, W, K, 94) if d3 else _rand_nhwc(N, H, W, K, 94)).to(DEV)
    dw0 = torch.zeros(K, Ct, *((3,) * (3 if d3 else 2)), device=DEV)
    dw1 = torch.zeros_like(dw0)
    O.wgrad(x0, dy, dw0, src1=x1, pro=(a, b, True), upsample=up)
    O.wgrad(gout, dy, dw1, upsample=up)
    rel = ((dw1 - dw0).norm() / dw0.norm()).item()
    print(f"{case}: wgrad from G vs recomputed prologue rel L2 {rel:.3e} (bit-identical: {torch.equal(dw0, dw1)})")
    assert rel < 1e-3


@pytest.mark.parametrize("hw", [32, 64])
def test_conv_s2_dgrad_parity_classes_with_fused_stats(hw):
    """Stride-2 data gradient with the SiLU' epilogue and fused GroupNorm-backward statistics (the
    DownsampleND backward whose input feeds a GroupNorm): the parity-class launch (one z-slice per output
    parity, only the 1/2/2/4 taps that reach it) writes its statistics in image-major rows.  Output vs torch
    (conv_transpose2d then SiLU'), statistics per (image, channel) vs the split-K path's independent reduce."""
    O = ops()
    N, H, W, C, K = 2, hw, hw, 64, 128
    g = torch.Generator().manual_seed(61)
    w = _w(K, C, 3, 62)
    dy = _rand_nhwc(N, H // 2, W // 2, K, 63)
    xe = _rand_nhwc(N, H, W, C, 64)
    a = torch.rand(N, C, generator=g) + 0.5
    b = torch.randn(N, C, generator=g) * 0.2
    wk = O.prep_weights(w.to(DEV), 1)
    kw = dict(ks=3, stride=2, pad=1, transposed=True, out_hw_=(H, W), want_stats=True,
              ep=(xe.to(DEV), None, a.to(DEV), b.to(DEV)))
    got, st = O.conv(dy.to(DEV), C, wk, splits=1, **kw)
    ref2, st2 = O.conv(dy.to(DEV), C, wk, splits=3, **kw)
    dx = F.conv_transpose2d(_to_nchw(dy), _bfw(w), stride=2, padding=1, output_padding=1)
    z = _to_nchw(xe) * a[:, :, None, None] + b[:, :, None, None]
    sg = torch.sigmoid(z)
    ref = (dx * sg * (1 + z * (1 - sg))).permute(0, 2, 3, 1)
    _close(got, ref)
    assert st.rows == 64
    t1 = st.slab.double().view(N, -1, C, 2).sum(1)
    t2 = st2.slab.double().view(N, -1, C, 2).sum(1)
    rel = ((t1 - t2).norm() / t2.norm()).item()
    print(f"hw={hw}: parity-class statistics vs split-K reduce rel L2 {rel:.3e}")
    assert rel < 1e-2


def test_conv3d_s2_dgrad_parity_classes_with_fused_stats():
    """3-D stride-2 data gradient with the SiLU' epilogue and fused statistics: 8 parity classes, image-major
    slab rows (class c owns the c-th eighth of each image's rows).  Output vs torch conv_transpose3d then
    SiLU'; statistics per (image, channel) vs the split-K path's independent reduce."""
    O = ops()
    N, D, H, W, C, K = 2, 16, 16, 16, 64, 128
    g = torch.Generator().manual_seed(71)
    w = torch.randn(K, C, 3, 3, 3, generator=g) / math.sqrt(C * 27)
    dy = _rand_ndhwc(N, D // 2, H // 2, W // 2, K, 72)
    xe = _rand_ndhwc(N, D, H, W, C, 73)
    a = torch.rand(N, C, generator=g) + 0.5
    b = torch.randn(N, C, generator=g) * 0.2
    wk = O.prep_weights(w.to(DEV), 1)
    kw = dict(ks=3, stride=2, pad=1, transposed=True, out_hw_=(D, H, W), want_stats=True,
              ep=(xe.to(DEV), None, a.to(DEV), b.to(DEV)))
    got, st = O.conv(dy.to(DEV), C, wk, splits=1, **kw)
    _, st2 = O.conv(dy.to(DEV), C, wk, splits=3, **kw)
    dyc = dy.float().permute(0, 4, 1, 2, 3)
    dx = F.conv_transpose3d(dyc, _bfw(w), stride=2, padding=1, output_padding=1)
    z = xe.float().permute(0, 4, 1, 2, 3) * a[:, :, None, None, None] + b[:, :, None, None, None]
    sg = torch.sigmoid(z)
    ref = (dx * sg * (1 + z * (1 - sg))).permute(0, 2, 3, 4, 1)
    _close(got, ref)
    t1 = st.slab.double().view(N, -1, C, 2).sum(1)
    t2 = st2.slab.double().view(N, -1, C, 2).sum(1)
    rel = ((t1 - t2).norm() / t2.norm()).item()
    print(f"3-D parity-class statistics vs split-K reduce rel L2 {rel:.3e}")
    assert rel < 1e-2


@pytest.mark.parametrize("case", ["down", "down_pro_stats", "updgrad", "updgrad_acc"])
def test_s2d_halo_conv_vs_torch(case):
    """fmd_conv_s2d (csrc/conv_halo9.hip): stride-2 convs as 2x2 convs over the space-to-depth view on the halo
    kernel, vs fp32 torch on the bf16-rounded operands.  down: DownsampleND's 3x3 stride-2 conv (+ bias; the
    _pro_stats case with a GroupNorm-affine + SiLU prologue and fused statistics); updgrad: the data gradient of
    conv3x3(nearest_x2(x)) through the 4x4 stride-2 gather the copy folds into (the _acc case adds into the
    existing gradient)."""
    O = ops()
    g = torch.Generator().manual_seed(50)
    if case.startswith("down"):
        N, H, W, C, K = 8, 128, 128, 64, 128
        x = _rand_nhwc(N, H, W, C, 51)
        w = _w(K, C, 3, 52)
        b = torch.randn(K, generator=g) * 0.1
        pro = None
        xin = x.float()
        if case == "down_pro_stats":
            pa, pb = torch.rand(N, C, generator=g) + 0.5, torch.randn(N, C, generator=g) * 0.2
            pro = (pa.to(DEV), pb.to(DEV), True)
            xin = F.silu(pa[:, None, None, :] * xin + pb[:, None, None, :]).to(torch.bfloat16).float()
        got, st = O.conv(x.to(DEV), K, None, ks=3, stride=2, pad=1, bias=b.to(DEV), pro=pro,
                         want_stats=case == "down_pro_stats", s2d_tiled=O.s2d_tile_weights(w.to(DEV), 0))
        ref = F.conv2d(_to_nchw(xin), _bfw(w), b, stride=2, padding=1).permute(0, 2, 3, 1)
        _close(got, ref)
        if st is not None:
            gf = got.float().cpu()
            sums = st.slab.view(N, -1, K, 2).sum(1).cpu()
            torch.testing.assert_close(sums[..., 0], gf.sum((1, 2)), rtol=5e-3, atol=3e-2)
            torch.testing.assert_close(sums[..., 1], (gf * gf).sum((1, 2)), rtol=5e-3, atol=3e-2)
    else:
        N, Hl, Wl, Cin, K = 8, 64, 64, 128, 128
        w = _w(K, Cin, 3, 53)
        dy = _rand_nhwc(N, 2 * Hl, 2 * Wl, K, 54)
        xl = torch.zeros(N, Cin, Hl, Wl, requires_grad=True)
        y = F.conv2d(F.interpolate(xl, scale_factor=2, mode="nearest"), _bfw(w), padding=1)
        y.backward(_to_nchw(dy))
        ref = xl.grad.permute(0, 2, 3, 1)
        out = None
        if case == "updgrad_acc":
            prev = _rand_nhwc(N, Hl, Wl, Cin, 55)
            out = prev.to(DEV).clone()
            ref = ref + prev.float()
        got, _ = O.conv(dy.to(DEV), Cin, None, ks=4, stride=2, pad=1, out_hw_=(Hl, Wl), out=out,
                        accumulate=case == "updgrad_acc", s2d_tiled=O.s2d_tile_weights(w.to(DEV), 1))
        _close(got, ref)


@pytest.mark.parametrize("case", ["plain", "acc"])
def test_d2s_halo_dgrad_vs_torch(case):
    """fmd_conv_d2s (csrc/conv_halo9.hip): the data gradient of DownsampleND's stride-2 3x3 conv as a 2x2 conv onto
    the depth-to-space view of the output, vs torch autograd of F.conv2d(stride=2) on the bf16-rounded operands (the
    acc case adds into the existing gradient)."""
    O = ops()
    N, H, W, C, K = 8, 128, 128, 128, 256   # input x [N, H, W, C] -> y [N, H/2, W/2, K]
    w = _w(K, C, 3, 61)
    dy = _rand_nhwc(N, H // 2, W // 2, K, 62)
    x = torch.zeros(N, C, H, W, requires_grad=True)
    F.conv2d(x, _bfw(w), stride=2, padding=1).backward(_to_nchw(dy))
    ref = x.grad.permute(0, 2, 3, 1)
    out = None
    if case == "acc":
        prev = _rand_nhwc(N, H, W, C, 63)
        out = prev.to(DEV).clone()
        ref = ref + prev.float()
    assert O.d2s_eligible(N, H // 2, W // 2, H, W, C, K)
    got, _ = O.conv(dy.to(DEV), C, None, ks=3, stride=2, pad=1, transposed=True, out_hw_=(H, W), out=out,
                    accumulate=case == "acc", s2d_tiled=O.s2d_tile_weights(w.to(DEV), 2))
    _close(got, ref)


@pytest.mark.parametrize("case", ["down", "down_pro_stats", "updgrad", "updgrad_acc", "d2s", "d2s_acc"])
def test_s2d_d2s_halo_3d_vs_torch(case):
    """3-D stride-2 convs on the halo kernel (csrc/conv_halo9.hip, depth taps as chunks) vs torch autograd of
    F.conv3d on the bf16-rounded operands: down = DownsampleND's Conv3d(stride 2) forward (fmd_conv_s2d; the
    _pro_stats case with a GroupNorm-affine + SiLU prologue and fused statistics); updgrad = the data gradient of
    Conv3d(nearest_x2(x)) as the 4x4x4 stride-2 gather; d2s = the data gradient of the stride-2 Conv3d onto 8
    output classes (fmd_conv_d2s).  The _acc cases add into an existing gradient.  Depth sizes cover both the
    zero-padded first slice and the last."""
    O = ops()
    g = torch.Generator().manual_seed(90)
    if case.startswith("down"):
        N, D, H, W, C, K = 2, 8, 128, 128, 64, 128
        assert O.s2d_eligible(N, H, W, H // 2, W // 2, K, C, 3, D, D // 2)
        x = _rand_ndhwc(N, D, H, W, C, 91)
        w = torch.randn(K, C, 3, 3, 3, generator=g) / math.sqrt(C * 27)
        b = torch.randn(K, generator=g) * 0.1
        xin, pro = _to_ncdhw(x), None
        if case == "down_pro_stats":
            pa, pb = torch.rand(N, C, generator=g) + 0.5, torch.randn(N, C, generator=g) * 0.2
            pro = (pa.to(DEV), pb.to(DEV), True)
            xin = F.silu(pa[:, :, None, None, None] * xin + pb[:, :, None, None, None]).to(torch.bfloat16).float()
        got, st = O.conv(x.to(DEV), K, None, ks=3, stride=2, pad=1, bias=b.to(DEV), pro=pro,
                         want_stats=case == "down_pro_stats", s2d_tiled=O.s2d_tile_weights(w.to(DEV), 0))
        ref = F.conv3d(xin, _bfw(w), b, stride=2, padding=1).permute(0, 2, 3, 4, 1)
        _close(got, ref)
        if st is not None:
            gf = got.float().cpu()
            sums = st.slab.view(N, -1, K, 2).sum(1).cpu()
            torch.testing.assert_close(sums[..., 0], gf.sum((1, 2, 3)), rtol=5e-3, atol=5e-2)
            torch.testing.assert_close(sums[..., 1], (gf * gf).sum((1, 2, 3)), rtol=5e-3, atol=5e-2)
        return
    if case.startswith("updgrad"):
        N, D, H, W, Cin, K = 2, 4, 64, 64, 128, 64       # low-resolution x; dy at 2D x 2H x 2W
        w = torch.randn(K, Cin, 3, 3, 3, generator=g) / math.sqrt(Cin * 27)
        dy = _rand_ndhwc(N, 2 * D, 2 * H, 2 * W, K, 92)
        xl = torch.zeros(N, Cin, D, H, W, requires_grad=True)
        F.conv3d(F.interpolate(xl, scale_factor=2, mode="nearest"), _bfw(w), padding=1).backward(_to_ncdhw(dy))
        ref = xl.grad.permute(0, 2, 3, 4, 1)
        out = None
        if case == "updgrad_acc":
            prev = _rand_ndhwc(N, D, H, W, Cin, 93)
            out = prev.to(DEV).clone()
            ref = ref + prev.float()
        assert O.s2d_eligible(N, 2 * H, 2 * W, H, W, Cin, K, 4, 2 * D, D)
        got, _ = O.conv(dy.to(DEV), Cin, None, ks=4, stride=2, pad=1, out_hw_=(D, H, W), out=out,
                        accumulate=case == "updgrad_acc", s2d_tiled=O.s2d_tile_weights(w.to(DEV), 1))
        _close(got, ref)
        return
    N, D, H, W, C, K = 1, 8, 64, 64, 128, 128            # x [N, C, D, H, W] -> y [N, K, D/2, H/2, W/2]
    w = torch.randn(K, C, 3, 3, 3, generator=g) / math.sqrt(C * 27)
    dy = _rand_ndhwc(N, D // 2, H // 2, W // 2, K, 94)
    x = torch.zeros(N, C, D, H, W, requires_grad=True)
    F.conv3d(x, _bfw(w), stride=2, padding=1).backward(_to_ncdhw(dy))
    ref = x.grad.permute(0, 2, 3, 4, 1)
    out = None
    if case == "d2s_acc":
        prev = _rand_ndhwc(N, D, H, W, C, 95)
        out = prev.to(DEV).clone()
        ref = ref + prev.float()
    assert O.d2s_eligible(N, H // 2, W // 2, H, W, C, K, D // 2, D)
    got, _ = O.conv(dy.to(DEV), C, None, ks=3, stride=2, pad=1, transposed=True, out_hw_=(D, H, W), out=out,
                    accumulate=case == "d2s_acc", s2d_tiled=O.s2d_tile_weights(w.to(DEV), 2))
    _close(got, ref)
