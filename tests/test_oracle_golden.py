"""Pin the CPU oracle against fixtures produced by the reference itself (tests/golden/make_golden.py)."""
import math
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import schedulers as OS
from oracle import spec as S
from oracle import train_step as OT
from oracle import unet as U

MODEL_CASES = ["ldct_fm_test", "mnist_ddpm_diffusers", "mnist_fm_compvis", "ldct_fm_b64", "ldct_fm_diffusers_b64"]


def _spec(meta):
    tr = meta["training"]
    return S.derive_spec(meta["unet"], tr["conditioning"], tr["channels"] or 1)


def _params(spec, seed):
    # leaf tensors with requires_grad: matches nn.Parameter dispatch (bit-exact F.linear path)
    return {k: v.requires_grad_() for k, v in U.seeded_state_dict(spec, seed).items()}


@pytest.mark.parametrize("name", MODEL_CASES)
def test_unet_forward_bit_exact(golden, name):
    T, M = golden
    m = M[name]
    spec = _spec(m)
    sd = _params(spec, m["seed"])
    with torch.no_grad():
        y = U.unet_forward(sd, spec, T[f"{name}/x"], T[f"{name}/t"], context=T.get(f"{name}/cond"))
    assert y.shape == T[f"{name}/y"].shape
    assert torch.equal(y, T[f"{name}/y"]), (y - T[f"{name}/y"]).abs().max()


def test_fm_train_step(golden):
    T, M = golden
    m = M["fm_step"]
    spec = _spec(m)
    sd = _params(spec, m["seed"])
    loss, scaled = OT.fm_loss(sd, spec, T["fm_step/clean"], T["fm_step/ldct"], T["fm_step/noise"], T["fm_step/t"],
                              m["num_train_timesteps"])
    scaled.backward()
    assert torch.equal(loss.detach(), T["fm_step/loss"])
    names = m["param_names"]
    gs = torch.stack([sd[k].grad.double().sum() for k in names])
    gq = torch.stack([sd[k].grad.double().pow(2).sum() for k in names])
    torch.testing.assert_close(gs, T["fm_step/grad_sum"], rtol=1e-9, atol=1e-12)
    torch.testing.assert_close(gq, T["fm_step/grad_sq"], rtol=1e-9, atol=1e-12)
    OT.adamw_step(sd, m["lr"], 1, {})
    ps = torch.stack([sd[k].detach().double().sum() for k in names])
    torch.testing.assert_close(ps, T["fm_step/param_sum_after"], rtol=1e-7, atol=1e-7)


def test_b256_forward_bit_exact(golden_b256):
    """The benched configuration (config B, 256x256): the oracle reproduces the reference forward exactly."""
    T, m = golden_b256
    spec = _spec(m)
    sd = U.seeded_state_dict(spec, m["seed"])
    with torch.no_grad():
        y = U.unet_forward(sd, spec, T["fwd/x"], T["fwd/t"], context=T["fwd/cond"])
    assert torch.equal(y, T["fwd/y"]), (y - T["fwd/y"]).abs().max()


def test_b256_fm_train_step(golden_b256):
    """Config B at 256x256: oracle FM train step (loss, gradients) and AdamW + cosine LR vs the reference's."""
    T, m = golden_b256
    spec = _spec(m)
    sd = _params(spec, m["seed"])
    loss, scaled = OT.fm_loss(sd, spec, T["step/clean"], T["step/ldct"], T["step/noise"], T["step/t"],
                              m["num_train_timesteps"])
    scaled.backward()
    assert torch.equal(loss.detach(), T["step/loss"])
    names = m["param_names"]
    torch.testing.assert_close(torch.stack([sd[k].grad.double().sum() for k in names]), T["step/grad_sum"],
                               rtol=1e-9, atol=1e-12)
    torch.testing.assert_close(torch.stack([sd[k].grad.double().pow(2).sum() for k in names]), T["step/grad_sq"],
                               rtol=1e-9, atol=1e-12)
    for k in m["small_grads"]:
        assert torch.equal(sd[k].grad, T[f"step/grad/{k}"]), k
    lr = m["lr"] * OS.cosine_with_warmup(0, m["warmup"], m["total"])
    OT.adamw_step(sd, lr, 1, {}, weight_decay=m["weight_decay"])
    ps = torch.stack([sd[k].detach().double().sum() for k in names])
    torch.testing.assert_close(ps, T["step/param_sum_after"], rtol=1e-7, atol=1e-6)


def _fingerprints_match(T, prefix, vals, seed, what):
    """The fixture's order-sensitive fingerprints (tests/golden/projections.py) regenerate from the oracle's
    tensors: pins both the oracle and the fingerprint code the GPU tests use."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import projections as P
    pj = P.projections(vals, seed)
    ref = T[f"{prefix}/proj_{what}"]
    assert torch.allclose(pj, ref, rtol=1e-6, atol=1e-9 * ref.abs().max().item()), (pj - ref).abs().max()
    sm = P.strided_sample(vals).float()
    assert torch.allclose(sm, T[f"{prefix}/sample_{what}"], rtol=1e-6, atol=1e-12)


def test_b256_fingerprints(golden_b256):
    """Config B 256^2 FM step: the oracle's gradients reproduce the fixture's projections / strided sample."""
    T, m = golden_b256
    spec = _spec(m)
    sd = _params(spec, m["seed"])
    loss, scaled = OT.fm_loss(sd, spec, T["step/clean"], T["step/ldct"], T["step/noise"], T["step/t"],
                              m["num_train_timesteps"])
    scaled.backward()
    _fingerprints_match(T, "step", [sd[k].grad for k in m["param_names"]], m["seed"], "grad")


@pytest.mark.parametrize("case", ["c256", "mnist"])
def test_ddpm_train_step_vs_reference(golden_ddpm, case):
    """Configs C (256^2, 113 M EfficientUNetND) and A (MNIST UNetDiffusersND): the oracle's DDPM step
    (add_noise, loss, gradients, AdamW under the cosine schedule) vs the reference's
    (tests/golden/make_golden_ddpm.py; diffusion_lib.py:153-185)."""
    T, M = golden_ddpm
    m = M[case]
    spec = _spec(m)
    sd = _params(spec, m["seed"])
    before = {k: v.detach().clone() for k, v in sd.items()}
    sch = OS.DDPM(m["num_train_timesteps"], **m["scheduler"].get("params", {}))
    assert torch.equal(sch.add_noise(T[f"{case}/clean"], T[f"{case}/noise"], T[f"{case}/t"]), T[f"{case}/noisy"])
    loss, scaled = OT.ddpm_loss(sd, spec, sch, T[f"{case}/clean"], T[f"{case}/ldct"], T[f"{case}/noise"],
                                T[f"{case}/t"])
    scaled.backward()
    assert torch.equal(loss.detach(), T[f"{case}/loss"])
    names = m["param_names"]
    torch.testing.assert_close(torch.stack([sd[k].grad.double().sum() for k in names]), T[f"{case}/grad_sum"],
                               rtol=1e-9, atol=1e-12)
    for k in m["small_grads"]:
        assert torch.equal(sd[k].grad, T[f"{case}/grad/{k}"]), k
    _fingerprints_match(T, case, [sd[k].grad for k in names], m["proj_seed_grad"], "grad")
    lr = m["lr"] * OS.cosine_with_warmup(0, m["warmup"], m["total"])
    OT.adamw_step(sd, lr, 1, {}, weight_decay=m["weight_decay"])
    ps = torch.stack([sd[k].detach().double().sum() for k in names])
    torch.testing.assert_close(ps, T[f"{case}/param_sum_after"], rtol=1e-7, atol=1e-6)
    _fingerprints_match(T, case, [sd[k].detach().double() - before[k].double() for k in names],
                        m["proj_seed_delta"], "delta")


def test_self_attention_raw_reshape(golden):
    T, M = golden
    m = M["attn"]
    shapes = {"norm.weight": (512,), "norm.bias": (512,), "qkv.weight": (768, 512, 1), "qkv.bias": (768,),
              "proj_out.weight": (512, 256, 1), "proj_out.bias": (512,)}
    p = U.seeded_tensors(shapes, m["seed"])
    sd = {f"a.{k}": v for k, v in p.items()}
    L = dict(prefix="a", heads=4, dim_head=64, linear=False)
    with torch.no_grad():
        y = U.self_attention(sd, L, T["attn/x"])
    assert torch.equal(y, T["attn/y"])


@pytest.mark.parametrize("i", [0, 1, 2])
def test_resblock(golden, i):
    T, M = golden
    m = M[f"res{i}"]
    import oracle.unet as UU
    names = m["names"]
    shapes = {}
    cin, cout = m["cin"], m["cout"]
    for n in names:
        if n.startswith("norm1"):
            shapes[n] = (cin,)
        elif n.startswith("norm2"):
            shapes[n] = (cout,)
        elif n == "conv1.conv.weight":
            shapes[n] = (cout, cin, 3, 3)
        elif n == "conv2.conv.weight":
            shapes[n] = (cout, cout, 3, 3)
        elif n.endswith("conv.bias"):
            shapes[n] = (cout,)
        elif n == "emb_layers.weight":
            shapes[n] = (2 * cout if m["scale_shift"] else cout, 512)
        elif n == "emb_layers.bias":
            shapes[n] = (2 * cout if m["scale_shift"] else cout,)
        elif n == "skip_connection.conv.weight":
            shapes[n] = (cout, cin, 1, 1)
    p = UU.seeded_tensors(shapes, m["seed"])
    sd = {f"r.{k}": v.requires_grad_() for k, v in p.items()}
    L = S.res_layer("r", cin, cout, scale_shift=m["scale_shift"], emb_act=m["emb_act"], add_emb=m["add_emb"])
    with torch.no_grad():
        y = U.resblock(sd, L, T[f"res{i}/x"], T[f"res{i}/emb"], 2)
    assert torch.equal(y, T[f"res{i}/y"])


def test_timestep_embedding(golden):
    T, _ = golden
    t = T["temb/t"]
    assert torch.equal(U.timestep_embedding(t, 128, flip_sin_to_cos=True), T["temb/flip"])
    assert torch.equal(U.timestep_embedding(t, 128, flip_sin_to_cos=False), T["temb/noflip"])
    assert torch.equal(U.timestep_embedding(t, 33, flip_sin_to_cos=False, freq_shift=1), T["temb/odd"])


# ---- scheduler KATs (closed form): parity otherwise unpinned
def test_flowmatch_kat():
    s = OS.FlowMatchEuler(1000)
    assert s.sigma_min == 0.0010000000474974513
    s.set_timesteps(50)
    ts = s.timesteps
    assert ts.dtype == torch.float32
    assert ts[:3].tolist() == [1000.0, 979.6122436523438, 959.2244873046875]
    assert ts[-1].item() == 1.0
    assert s.sigmas[-1].item() == 0.0 and len(s.sigmas) == 51


def test_ddpm_kat():
    s = OS.DDPM(1000, beta_start=0.00085, beta_end=0.012)
    ac = s.alphas_cumprod
    assert abs(ac[0].item() - 0.99914998) < 1e-7
    assert abs(ac[499].item() - 0.16181217) < 1e-7
    assert abs(ac[999].item() - 0.00157896) < 1e-7
    s.set_timesteps(50)
    assert s.timesteps.tolist() == list(range(980, -1, -20))
    assert s.timesteps.dtype == torch.int64


def test_fm_train_timesteps_bitexact():
    t = torch.tensor([0.0, 0.5, 0.999999, 1e-7, 0.3333333])
    assert OT.fm_timesteps(t, 1000).tolist() == [0, 499, 998, 0, 332]


def test_cosine_schedule_matches_transformers():
    tf = pytest.importorskip("transformers.optimization")
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=1.0)
    sch = tf.get_cosine_schedule_with_warmup(opt, num_warmup_steps=5, num_training_steps=40)
    for step in range(40):
        assert math.isclose(opt.param_groups[0]["lr"], OS.cosine_with_warmup(step, 5, 40), rel_tol=1e-12)
        opt.step()
        sch.step()


def _vae_golden():
    import json
    import os
    G = torch.load(os.path.join(os.path.dirname(__file__), "golden", "vae_golden.pt"), weights_only=True)
    return G, json.loads(bytes(G["cfg_json"].tolist()).decode())


def test_vae_oracle_matches_reference_fixture():
    """oracle/vae.py (encode moments, decode) vs the reference AutoencoderKL's own outputs
    (tests/golden/make_vae_golden.py)."""
    from oracle import vae as V
    G, cfg = _vae_golden()
    sd = G["state"]
    with torch.no_grad():
        m = V.encode_moments(sd, cfg, G["x"] * 2.0 - 1.0)
        r = V.decode(sd, cfg, G["z"])
    mu, logvar = m.chunk(2, 1)
    torch.testing.assert_close(mu, G["mode"], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(logvar.clamp(-30.0, 20.0), G["moments"][:, 4:], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(r, G["rec"], rtol=1e-5, atol=1e-5)


def test_vae_module_state_dict_drop_in():
    """fmdiff AutoencoderKL: same constructor and state_dict keys/shapes as the reference."""
    import warnings
    from fmdiff.models.vae import AutoencoderKL
    G, cfg = _vae_golden()
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        vae = AutoencoderKL(**cfg)
    ref = G["state"]
    own = vae.state_dict()
    assert list(own.keys()) == list(ref.keys())
    assert all(own[k].shape == ref[k].shape for k in own)
    vae.load_state_dict(ref)


@pytest.mark.parametrize("name", ["spatial_cross", "diffusers_cross"])
@pytest.mark.parametrize("layout", ["bct", "btc"])
def test_cross_attention_blocks_vs_reference(golden_attn, name, layout):
    """oracle cross_attention / diffusers_attention (context_norm, raw vs view/transpose head split, both
    context layouts) vs the reference modules' own forward and autograd gradients (make_golden_attn.py)."""
    T, M = golden_attn
    m = M[name]
    import oracle.unet as UU
    from fmdiff.nn.blocks.attention import DiffusersAttentionND, SpatialCrossAttention
    if m["kind"] == "spatial":
        mod = SpatialCrossAttention(m["dim"], context_dim=m["context_dim"], heads=m["heads"], dim_head=m["dim_head"])
        L = dict(prefix="p", heads=m["heads"], dim_head=m["dim_head"], linear=False, ctx=m["context_dim"])
        fn = UU.cross_attention
    else:
        mod = DiffusersAttentionND(m["channels"], heads=m["heads"], context_dim=m["context_dim"],
                                   norm_num_groups=m["norm_num_groups"])
        L = dict(prefix="p", heads=m["heads"], groups=m["norm_num_groups"], eps=1e-5, ctx=m["context_dim"])
        fn = UU.diffusers_attention
    shapes = {k: tuple(v.shape) for k, v in mod.state_dict().items()}
    sd = {f"p.{k}": v.requires_grad_() for k, v in UU.seeded_tensors(shapes, m["seed"]).items()}
    ctx = T[f"{name}/ctx"] if layout == "bct" else T[f"{name}/ctx"].transpose(1, 2).contiguous()
    x = T[f"{name}/x"].clone().requires_grad_()
    y = fn(sd, L, x, ctx)
    torch.testing.assert_close(y, T[f"{name}/{layout}/y"], rtol=1e-5, atol=1e-6)
    y.backward(T[f"{name}/gout"])
    torch.testing.assert_close(x.grad, T[f"{name}/{layout}/dx"], rtol=1e-4, atol=1e-5)
    for k in m["params"]:
        torch.testing.assert_close(sd[f"p.{k}"].grad, T[f"{name}/{layout}/grad/{k}"], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("name", ["pool2_2d", "pool2_3d"])
def test_pool_factor_unet_vs_reference(name):
    """EfficientUNetND(pool_factor=2): PoolND patchify conv + UnPoolND transposed conv (oracle) vs the
    reference module's own forward (tests/golden/make_golden_pool.py), bit-exact."""
    import json
    d = os.path.join(os.path.dirname(__file__), "golden")
    T = torch.load(os.path.join(d, "golden_pool.pt"), weights_only=True)
    m = json.load(open(os.path.join(d, "golden_pool.json")))[name]
    spec = S.derive_spec(m["cfg"], None, 1)
    sd = U.seeded_state_dict(spec, m["seed"])
    with torch.no_grad():
        y = U.unet_forward(sd, spec, T[f"{name}/x"], T[f"{name}/t"])
    assert torch.equal(y, T[f"{name}/y"])


def test_vae_oracle_matches_config_d_fixture():
    """oracle/vae.py at config D's own architecture (configs/LDCT/LDCT_autoencoder_kl.json, 82.6 M parameters,
    reference VAEFactory; tests/golden/make_vae_golden_d.py) vs the reference's encode / decode outputs, with the
    weights regenerated by the fixture's name-seeded rule."""
    import json
    import os
    import sys
    import warnings
    from fmdiff.models.vae import AutoencoderKL
    from oracle import vae as V
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import seeded_params as SP
    G = torch.load(os.path.join(os.path.dirname(__file__), "golden", "vae_golden_d.pt"), weights_only=True)
    model = json.loads(bytes(G["cfg_json"].tolist()).decode())
    cfg = {k: v for k, v in model.items() if k not in ("latent_type", "model_type", "norm_type", "act")}
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        vae = AutoencoderKL(**cfg)
    sd = SP.fill_module(vae, 3131)
    assert sum(v.numel() for v in sd.values()) == int(G["nparam"])
    torch.set_num_threads(max(1, min(8, torch.get_num_threads())))
    with torch.no_grad():
        m = V.encode_moments(sd, cfg, G["x"] * 2.0 - 1.0)
        r = V.decode(sd, cfg, G["z"])
    mu, logvar = m.chunk(2, 1)
    torch.testing.assert_close(mu, G["mu"], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(logvar.clamp(-30.0, 20.0), G["logvar"], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(r, G["rec"], rtol=1e-4, atol=1e-4)


def test_unet_oracle_matches_config_e_fixture():
    """oracle/unet.py's 3-D EfficientUNetND at config E's own architecture (308 M parameters) reproduces the
    reference module's 64^3 forward (tests/golden/make_golden_e.py)."""
    import json
    import os
    from oracle import spec as S
    from oracle import unet as U
    d = os.path.join(os.path.dirname(__file__), "golden")
    T = torch.load(os.path.join(d, "golden_e.pt"), weights_only=True)
    m = json.load(open(os.path.join(d, "golden_e.json")))
    tr = m["training"]
    spec = S.derive_spec(m["unet"], tr["conditioning"], tr["channels"] or 1)
    sd = U.seeded_state_dict(spec, m["seed"])
    assert sum(v.numel() for v in sd.values()) == 308246913
    with torch.no_grad():
        y = U.unet_forward(sd, spec, torch.cat([T["fwd/x"], T["fwd/cond"]], 1), T["fwd/t"])
    torch.testing.assert_close(y, T["fwd/y"], rtol=1e-4, atol=1e-4)
