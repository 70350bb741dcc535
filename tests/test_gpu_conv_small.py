"""fmd_conv_small (csrc/conv_small.hip): the one-launch small-level conv against a plain PyTorch fp32 reference of
the same ops, and against the multi-launch path it replaces (fmd_gn_fused_apply / fmd_gn_prep + fmd_conv).

Reference ops: ResBlockND's GroupNorm(+scale/shift)+SiLU -> 3x3 conv (+ time-embedding add, 1x1 skip conv,
residual) (src/nn/blocks/residual.py:84-120, normalization.py:11-19, convolution.py:8-54), DownsampleND's stride-2
conv and UpsampleND's nearest-x2 + conv (src/nn/ops/upsampling.py:8-62).  Inputs are bf16-rounded before the
reference sees them and the GN+SiLU operand is rounded to bf16 where the kernel rounds it, so what remains is fp32
accumulation order and the final bf16 rounding: tolerance 1.5e-2 x max|ref| (the per-kernel bound of
tests/test_gpu_kernels.py).  The statistics slab must equal the fp64 sums of the kernel's own bf16 outputs within
fp32 summation error (1e-5 ||t||_1).
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"

# name: (N, Hs, C0, C1, K, mode, gn, emb(scale-shift), skip, bias_nc, resid)
CASES = {
    "s1_32_cat_skip": (8, 32, 128, 128, 128, "s1", True, False, True, False, False),
    "s1_16_cat_skip_embadd": (8, 16, 128, 128, 128, "s1", True, False, True, True, False),
    "s1_8_ss_resid": (8, 8, 256, 0, 256, "s1", True, True, False, False, True),
    "s1_8_conv2_skip": (8, 8, 256, 0, 256, "s1", True, True, "other", False, False),
    "s1_16_conv2_skip": (8, 16, 128, 0, 128, "s1", True, True, "other", False, False),
    "point_1_conv2_skip": (8, 1, 512, 0, 512, "point", True, True, "other", False, False),
    "s1_8_cat_skip": (8, 8, 256, 256, 256, "s1", True, False, True, False, False),
    "s1_4_cat_skip": (8, 4, 256, 256, 256, "s1", True, False, True, True, False),
    "s1_4_ragged_n3": (3, 4, 256, 0, 256, "s1", True, True, False, False, True),
    "s1_2_cat": (8, 2, 512, 512, 512, "s1", True, False, False, False, False),
    "s1_2_conv2_skip": (8, 2, 512, 0, 512, "s1", True, True, "other", False, False),
    "point_1_cat_skip": (8, 1, 512, 512, 512, "point", True, False, True, True, False),
    "point_1_ss_resid": (8, 1, 512, 0, 512, "point", True, True, False, False, True),
    "s2_32": (8, 32, 128, 0, 128, "s2", False, False, False, False, False),
    "s2_16": (8, 16, 128, 0, 128, "s2", False, False, False, False, False),
    "s2_8": (8, 8, 256, 0, 256, "s2", False, False, False, False, False),
    "up_8": (8, 8, 256, 0, 256, "up", False, False, False, False, False),
    "up_1": (8, 1, 512, 0, 512, "up", False, False, False, False, False),
    "up_16": (8, 16, 128, 0, 128, "up", False, False, False, False, False),
}


@pytest.fixture(autouse=True)
def _small_conv_on(monkeypatch):
    """The kernel under test, whatever the SMALL_CONV defaults of runtime/tuning.py (the level cap is a speed
    choice; the kernel takes 32^2 too)."""
    from fmdiff.runtime import ops
    monkeypatch.setattr(ops, "SMALL_CONV", True)
    monkeypatch.setattr(ops, "SMALL_CONV_MAX_HW", 1024)
    monkeypatch.setattr(ops, "SMALL_CONV_MAX_WORK", 1 << 30)


def _bf(t):
    return t.to(torch.bfloat16).float()


def _make(name, seed=0):
    from fmdiff.runtime import ops
    N, Hs, C0, C1, K, mode, gn, ss, skip, addemb, resid = CASES[name]
    g = torch.Generator().manual_seed(seed + sum(map(ord, name)))
    C = C0 + C1
    G = 32
    Ho = Hs // 2 if mode == "s2" else 2 * Hs if mode == "up" else Hs
    x0 = (torch.randn(N, Hs, Hs, C0, generator=g) * 1.3 + 0.2).to(torch.bfloat16)
    x1 = (torch.randn(N, Hs, Hs, C1, generator=g) * 0.7 - 0.1).to(torch.bfloat16) if C1 else None
    ks = 1 if mode == "point" else 3
    w = torch.randn(K, C, ks, ks, generator=g) / math.sqrt(C * ks * ks)
    p = dict(N=N, Hs=Hs, C0=C0, C1=C1, K=K, mode=mode, Ho=Ho, x0=x0, x1=x1, w=w, G=G,
             bias=torch.randn(K, generator=g) * 0.1)
    if gn:
        p["gamma"] = 1 + 0.2 * torch.randn(C, generator=g)
        p["beta"] = 0.1 * torch.randn(C, generator=g)
        if ss:
            p["emb"] = 0.3 * torch.randn(N, 2 * C, generator=g)
    if skip:   # the skip sources: the conv's own input (True), or a separate block input (ResBlock conv2: "other")
        if skip == "other":
            # the deepest levels: a 512 + 512 up-block input (the 1x1 segment's largest case, 4 chunks per wave)
            p["xs0"] = torch.randn(N, Ho, Ho, 512 if C >= 512 else 256 if C >= 256 else 96, generator=g).to(
                torch.bfloat16)
            p["xs1"] = torch.randn(N, Ho, Ho, 512 if C >= 512 else 160, generator=g).to(torch.bfloat16)
        else:
            p["xs0"], p["xs1"] = x0, x1
        Cs = p["xs0"].shape[-1] + (p["xs1"].shape[-1] if p["xs1"] is not None else 0)
        p["skip_w"] = torch.randn(K, Cs, 1, 1, generator=g) / math.sqrt(Cs)
        p["bias2"] = torch.randn(K, generator=g) * 0.1
    if addemb:
        p["bias_nc_full"] = torch.randn(N, K + 64, generator=g) * 0.5   # a view with row stride K + 64
    if resid:
        p["resid"] = torch.randn(N, Ho, Ho, K, generator=g).to(torch.bfloat16)
    p["gn"] = gn
    p["ops"] = ops
    return p


def _reference(p):
    """fp32 torch of the same ops, NHWC out."""
    x = torch.cat([p["x0"], p["x1"]], -1) if p["x1"] is not None else p["x0"]
    x = x.float().permute(0, 3, 1, 2)
    N, C = x.shape[:2]
    z = x
    if p["gn"]:
        G = p["G"]
        xg = x.reshape(N, G, -1)
        mean = xg.mean(-1, keepdim=True)
        var = xg.var(-1, unbiased=False, keepdim=True)
        z = ((xg - mean) / torch.sqrt(var + 1e-6)).reshape_as(x)
        z = z * p["gamma"][None, :, None, None] + p["beta"][None, :, None, None]
        if "emb" in p:
            sc, sh = p["emb"][:, :C], p["emb"][:, C:]
            z = z * (1 + sc[:, :, None, None]) + sh[:, :, None, None]
        z = _bf(F.silu(z))
    if p["mode"] == "up":
        z = F.interpolate(z, scale_factor=2, mode="nearest")
    stride = 2 if p["mode"] == "s2" else 1
    pad = 0 if p["mode"] == "point" else 1
    y = F.conv2d(z, _bf(p["w"]), p["bias"], stride=stride, padding=pad)
    if "skip_w" in p:
        xs = torch.cat([p["xs0"], p["xs1"]], -1) if p["xs1"] is not None else p["xs0"]
        y = y + F.conv2d(xs.float().permute(0, 3, 1, 2), _bf(p["skip_w"]), p["bias2"])
    if "bias_nc_full" in p:
        y = y + p["bias_nc_full"][:, :p["K"], None, None]
    y = y.permute(0, 2, 3, 1)
    if "resid" in p:
        y = y + p["resid"].float()
    return y


def _run_small(p, split=None, x0=None, check_only=False):
    ops = p["ops"]
    x0 = p["x0"].to(DEV) if x0 is None else x0
    x1 = p["x1"].to(DEV) if p["x1"] is not None else None
    wk = ops.prep_weights(p["w"].to(DEV), 0)
    gn = None
    if p["gn"]:
        gn = dict(st0=ops.channel_stats(x0), st1=ops.channel_stats(x1) if x1 is not None else None, groups=p["G"],
                  eps=1e-6, gamma=p["gamma"].to(DEV), beta=p["beta"].to(DEV))
        if "emb" in p:
            gn["emb"] = p["emb"].to(DEV)
    kw = dict(bias=p["bias"].to(DEV))
    skip = None
    if "skip_w" in p:
        kw["skip_wgt"] = ops.prep_weights(p["skip_w"].to(DEV), 0)
        kw["bias2"] = p["bias2"].to(DEV)
        kw["src2"] = p["xs0"].to(DEV)
        kw["src3"] = p["xs1"].to(DEV) if p["xs1"] is not None else None
        skip = (p["xs0"].shape[-1], p["xs1"].shape[-1] if p["xs1"] is not None else 0)
    if "bias_nc_full" in p:
        kw["bias_nc"] = p["bias_nc_full"].to(DEV)[:, :p["K"]]
    if "resid" in p:
        kw["resid"] = p["resid"].to(DEV)
    ok = ops.conv_small_ok(tuple(x0.shape), p["K"], C1=p["C1"], mode=p["mode"], gn=gn, skip=skip, split=split)
    if check_only:
        return ok
    assert ok
    return ops.conv_small(x0, p["K"], wk, src1=x1, mode=p["mode"], gn=gn, split=split, **kw)


@pytest.mark.parametrize("split", [0, 1])
@pytest.mark.parametrize("name", list(CASES))
def test_conv_small_vs_torch(name, split):
    """split 0: the plan's parts (the in-launch combine wherever the grid is small), 1: one workgroup per tile."""
    p = _make(name)
    if split == 1 and not _run_small(p, 1, check_only=True):
        pytest.skip("the plan takes this problem only as parts of the reduction")   # the 1x1 segment's registers
    ref = _reference(p)
    out, st = _run_small(p, split)
    torch.cuda.synchronize()
    got = out.float().cpu()
    assert got.shape == ref.shape
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item()
    print(f"[conv_small] {name} split={split}: max err {err:.3e} / max |ref| {scale:.3e} = {err / scale:.2e}")
    assert err <= 1.5e-2 * scale
    # statistics: the fp64 sums of the kernel's own bf16 outputs, per slab row
    N, Ho, K = p["N"], p["Ho"], p["K"]
    rows = st.rows
    t = got.double().reshape(-1, rows, K)
    own = torch.stack([t.sum(1), (t * t).sum(1)], -1)
    l1 = torch.stack([t.abs().sum(1), (t * t).sum(1)], -1)
    slab = st.slab.double().cpu()
    assert slab.shape == own.shape
    assert ((slab - own).abs() <= 1e-5 * l1 + 1e-6).all(), (slab - own).abs().max().item()


@pytest.mark.parametrize("name", ["s1_16_cat_skip_embadd", "s1_8_ss_resid", "s1_2_conv2_skip", "s1_8_conv2_skip"])
def test_conv_small_vs_split_path(name):
    """Against the launches it replaces: GroupNorm via fmd_gn_prep (+ scale/shift) + fmd_gn_apply_fwd, then
    fmd_conv (split-K implicit GEMM) with the same bias / skip / residual epilogue."""
    p = _make(name, seed=5)
    ops = p["ops"]
    x0 = p["x0"].to(DEV)
    x1 = p["x1"].to(DEV) if p["x1"] is not None else None
    N, Hs, C0, C1, K = p["N"], p["Hs"], p["C0"], p["C1"], p["K"]
    emb = p["emb"].to(DEV) if "emb" in p else None
    a, b, _ = ops.gn_prep(ops.channel_stats(x0), ops.channel_stats(x1) if x1 is not None else None, N, Hs * Hs, C0,
                          C1, p["G"], 1e-6, p["gamma"].to(DEV), p["beta"].to(DEV), emb=emb,
                          emb_stride=emb.shape[1] if emb is not None else 0, emb_mode=1 if emb is not None else 0)
    t = ops.gn_apply_fwd(x0, x1, a, b)
    kw = dict(bias=p["bias"].to(DEV))
    if "skip_w" in p:
        kw.update(src2=p["xs0"].to(DEV), src3=p["xs1"].to(DEV) if p["xs1"] is not None else None,
                  wgt2=ops.prep_weights(p["skip_w"].to(DEV), 0), bias2=p["bias2"].to(DEV))
    if "bias_nc_full" in p:
        kw["bias_nc"] = p["bias_nc_full"].to(DEV)[:, :K].contiguous()
    if "resid" in p:
        kw["resid"] = p["resid"].to(DEV)
    ref, _ = ops.conv(t, K, ops.prep_weights(p["w"].to(DEV), 0), force_generic=True, **kw)
    out, _ = _run_small(p)
    torch.cuda.synchronize()
    err = (out.float() - ref.float()).abs().max().item()
    scale = ref.float().abs().max().item()
    print(f"[conv_small vs split path] {name}: {err / scale:.2e}")
    assert err <= 1.5e-2 * scale


def test_conv_small_plan_rejects_what_it_cannot_take():
    """fmd_conv_small_plan is a host-side query: out-of-range problems are refused, never launched.  (Also in the CPU
    suite: tests/test_host.py.)"""
    from fmdiff.runtime import ops
    assert ops.conv_small_ok((8, 8, 8, 64), 64)
    assert not ops.conv_small_ok((8, 8, 8, 32), 64)          # C < 64
    assert not ops.conv_small_ok((8, 8, 8, 64), 24)          # K % 16
    assert not ops.conv_small_ok((8, 8, 12, 64), 64)         # 64 % Ho*Wo, Ho*Wo % 64
    assert not ops.conv_small_ok((1, 16, 16, 2048), 64, split=1)   # more than one CU's LDS unsplit ...
    assert ops.conv_small_ok((1, 16, 16, 2048), 64)               # ... fits as parts of the reduction
    assert not ops.conv_small_ok((8, 64, 64, 128), 128)      # above SMALL_CONV_MAX_HW
    # 3x3 over 1024 channels (36 weight fragments per wave) leaves no registers for a 1x1 segment, unless split
    assert ops.conv_small_ok((8, 2, 2, 512), 512, C1=512)
    assert not ops.conv_small_ok((8, 2, 2, 512), 512, C1=512, skip=(512, 512), split=1)
    assert ops.conv_small_ok((8, 2, 2, 512), 512, C1=512, skip=(512, 512), split=0)


@pytest.mark.parametrize("name", ["s1_2_cat", "s1_2_conv2_skip", "point_1_cat_skip", "s1_4_ragged_n3",
                                  "s1_16_cat_skip_embadd"])
def test_conv_small_split_combine(name):
    """The in-launch combine of a split reduction (csrc/conv_small.hip, (7)): every part count agrees with the
    unsplit result within fp32 reassociation; each is bit-identical across repeats whatever the arrival order of the
    parts; launches with different part counts and different inputs back to back on one stream (the tickets reset
    by every launch, the reducer's loads of a previous launch's slab lines) each reproduce their solo result."""
    p = _make(name, seed=3)
    ops = p["ops"]
    x0a = p["x0"].to(DEV)
    x0b = (x0a.float() * -0.7 + 0.3).to(torch.bfloat16)
    Ps = [P for P in (1, 2, 4, 8, 16) if _run_small(p, P, x0a, check_only=True)]
    assert len(Ps) >= 2, "fewer than two part counts qualify"
    base, _ = _run_small(p, Ps[0], x0a)   # the fewest parts the plan takes (1 where the registers allow)
    Ps = Ps[1:]
    solo = {}
    for P in Ps:
        outs = [_run_small(p, P, x)[0].clone() for x in (x0a, x0b)]
        solo[P] = outs
        err = (outs[0].float() - base.float()).abs().max().item()
        scale = base.float().abs().max().item()
        print(f"[conv_small split] {name} P={P}: vs the fewest parts {err / scale:.2e}")
        assert err <= 4e-3 * scale
    torch.cuda.synchronize()
    for rep in range(3):   # interleaved part counts and inputs, no synchronisation in between
        got = [(P, i, _run_small(p, P, x)[0]) for P in Ps[::-1] for i, x in enumerate((x0a, x0b))]
        torch.cuda.synchronize()
        for P, i, o in got:
            assert torch.equal(o, solo[P][i]), (rep, P, i)


def test_conv_small_split_combine_under_uneven_load():
    """The in-launch combine with the chip busy elsewhere (MI355X_MICROARCH.md: test hand-offs under UNEVEN load):
    a large GEMM runs on a second stream while the split convs are launched 30 times on this one, so the parts of a
    tile start and finish at scattered times and the reducer may be any of them; every output equals the solo
    result bit for bit."""
    p = _make("s1_2_cat", seed=7)
    x0 = p["x0"].to(DEV)
    solo, _ = _run_small(p, 8, x0)
    solo = solo.clone()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    a = torch.randn(8192, 8192, device=DEV, dtype=torch.bfloat16)
    outs = []
    with torch.cuda.stream(side):
        for _ in range(3):
            a = (a @ a).clamp_(-1, 1)
    for _ in range(30):
        outs.append(_run_small(p, 8, x0)[0])
    torch.cuda.synchronize()
    for i, o in enumerate(outs):
        assert torch.equal(o, solo), i
