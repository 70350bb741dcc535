"""CPU tests of the host side: scheduler bookkeeping (bit-exact vs the oracle), the scheduler registry,
the model factory's state_dict surface, and the data-parallel gradient exchange over gloo (world 2)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fmdiff.models.generators import DiffusionUNetFactory
from fmdiff.pipelines import schedulers as FS
from fmdiff.pipelines import utils as PU
from fmdiff.runtime import dp
from oracle import schedulers as OS
from oracle import spec as S
from oracle import train_step as OT
from oracle import unet as U

MODEL_CASES = ["ldct_fm_test", "mnist_ddpm_diffusers", "mnist_fm_compvis", "ldct_fm_b64", "ldct_fm_diffusers_b64"]


# ------------------------------------------------------------------ schedulers (host tables)
@pytest.mark.parametrize("n", [1, 2, 10, 50, 999, 1000])
def test_flow_match_tables_bit_exact(n):
    a, o = FS.FlowMatchEulerDiscreteScheduler(1000), OS.FlowMatchEuler(1000)
    assert torch.equal(a.timesteps, o.timesteps) and torch.equal(a.sigmas, o.sigmas)
    assert a.sigma_min == o.sigma_min == 0.0010000000474974513
    a.set_timesteps(n)
    o.set_timesteps(n)
    assert a.timesteps.dtype == torch.float32
    assert torch.equal(a.timesteps, o.timesteps) and torch.equal(a.sigmas, o.sigmas)
    for t in a.timesteps[:3]:
        assert a.index_for_timestep(t) == o.index_for_timestep(t)


def test_flow_match_kat():
    s = FS.FlowMatchEulerDiscreteScheduler(1000)
    s.set_timesteps(50)
    assert s.timesteps[:3].tolist() == [1000.0, 979.6122436523438, 959.2244873046875]
    assert s.timesteps[-1].item() == 1.0 and s.sigmas[-1].item() == 0.0 and len(s.sigmas) == 51


@pytest.mark.parametrize("spacing", ["leading", "linspace", "trailing"])
@pytest.mark.parametrize("n", [1, 7, 50, 1000])
def test_ddpm_ddim_tables_bit_exact(spacing, n):
    kw = dict(beta_start=0.00085, beta_end=0.012, timestep_spacing=spacing)
    a, o = FS.DDPMScheduler(1000, **kw), OS.DDPM(1000, **kw)
    assert torch.equal(a.alphas_cumprod, o.alphas_cumprod)
    a.set_timesteps(n)
    o.set_timesteps(n)
    assert a.timesteps.dtype == torch.int64 and torch.equal(a.timesteps, o.timesteps)
    for t in a.timesteps[:4].tolist():
        c = a.coefficients(t)
        r = o.coefficients(t)
        want = torch.stack([r["sqrt_b"], r["sqrt_a"], r["c_x0"], r["c_xt"],
                            r["std"] if t > 0 else torch.tensor(0.0)]).float()
        assert torch.equal(c[:5], want)


def test_ddpm_leading_kat():
    s = FS.DDPMScheduler(1000)
    s.set_timesteps(50)
    assert s.timesteps.tolist() == list(range(980, -1, -20))


@pytest.mark.parametrize("sched", ["linear", "scaled_linear", "squaredcos_cap_v2"])
def test_beta_schedules(sched):
    a, o = FS.DDPMScheduler(1000, beta_schedule=sched), OS.DDPM(1000, beta_schedule=sched)
    assert torch.equal(a.betas, o.betas)


# ------------------------------------------------------------------ registry / loop host logic
@pytest.mark.parametrize("kind,order,variant", [
    ("dpm", 1, "dpmsolver++"), ("dpm", 2, "dpmsolver++"), ("dpm", 3, "dpmsolver++"), ("dpm", 2, "heun"),
    ("dpm", 2, "dpmsolver"), ("dpm", 3, "dpmsolver"), ("unipc", 1, "bh2"), ("unipc", 2, "bh2"),
    ("unipc", 3, "bh2"), ("unipc", 2, "bh1")])
def test_multistep_oracle_follows_exact_denoiser(kind, order, variant):
    """KAT for the restated DPM-Solver(++) / UniPC (parity otherwise unpinned: diffusers is absent): fed the
    exact epsilon of a fixed x0, every solver order integrates the probability-flow ODE exactly, so the final
    sample is alpha_T x0 + sigma_T eps0 (eps0 = the initial noise) to fp32 rounding."""
    from oracle import schedulers as OS
    if kind == "dpm":
        algo = "dpmsolver" if variant == "dpmsolver" else "dpmsolver++"
        fs = "sigma_min" if algo == "dpmsolver" else "zero"
        sch = OS.DPMSolverMultistep(solver_order=order, algorithm_type=algo, final_sigmas_type=fs,
                                    solver_type="heun" if variant == "heun" else "midpoint")
    else:
        sch = OS.UniPCMultistep(solver_order=order, solver_type=variant)
    sch.set_timesteps(20)
    g = torch.Generator().manual_seed(3)
    x0 = torch.rand(2, 1, 4, 4, generator=g) * 2 - 1
    e0 = torch.randn(2, 1, 4, 4, generator=g)
    a, sg = sch.alpha_sigma(sch.sigmas[0])
    x = a * x0 + sg * e0
    for i, t in enumerate(sch.timesteps):
        a, sg = sch.alpha_sigma(sch.sigmas[i])
        x = sch.step((x - a * x0) / sg, t, x).prev_sample
    a, sg = sch.alpha_sigma(sch.sigmas[-1])
    assert (x - (a * x0 + sg * e0)).abs().max().item() < 2e-6


def test_multistep_timesteps_kat():
    """linspace spacing (upstream default) for 50 steps over 1000: 999, 979, ..., 20; final sigma 0."""
    from oracle import schedulers as OS
    from fmdiff.pipelines.schedulers import DPMSolverMultistepScheduler, UniPCMultistepScheduler
    o = OS.DPMSolverMultistep()
    o.set_timesteps(50)
    assert o.timesteps[:3].tolist() == [999, 979, 959] and o.timesteps[-1].item() == 20
    assert o.sigmas[-1].item() == 0.0 and len(o.sigmas) == 51
    for cls in (DPMSolverMultistepScheduler, UniPCMultistepScheduler):
        sch = cls(1000)
        sch.set_timesteps(50)
        assert torch.equal(sch.timesteps, o.timesteps) and torch.equal(sch.sigmas, o.sigmas)
    with pytest.raises(ValueError):
        DPMSolverMultistepScheduler(1000, algorithm_type="dpmsolver")   # final_sigmas_type zero, like upstream


def test_build_scheduler_and_overrides():
    s, n = PU.build_scheduler({"name": "flow_match_euler", "params": {"shift": 1.0, "bogus": 3}}, {})
    assert isinstance(s, FS.FlowMatchEulerDiscreteScheduler) and n == 1000
    s, n = PU.build_scheduler({}, {"scheduler": "DDIM", "num_train_timesteps": 500, "num_inference_steps": 20})
    assert isinstance(s, FS.DDIMScheduler) and s.config.num_train_timesteps == 500 and n == 20
    s, _ = PU.build_scheduler(None, None)
    assert isinstance(s, FS.DDPMScheduler)
    with pytest.raises(ValueError, match="Unknown scheduler"):
        PU.build_scheduler({"name": "euler_a"}, {})
    assert PU.resolve_scheduler_override(None) is None
    assert PU.resolve_scheduler_override("  ") is None
    assert PU.resolve_scheduler_override("flowmatch") == {"name": "flow_match_euler"}
    assert PU.resolve_scheduler_override("dpmsolver++") == {
        "name": "dpm_multistep", "params": {"solver_order": 2, "algorithm_type": "dpmsolver++"}}
    with pytest.raises(ValueError, match="Unknown scheduler override"):
        PU.resolve_scheduler_override("heun")
    assert set(PU.SCHEDULER_REGISTRY) == {"ddpm", "ddim", "dpm_multistep", "dpm_sde", "unipc", "flow_match_euler",
                                          "flowmatch"}


def test_select_timesteps():
    ts = torch.tensor([980, 960, 500, 20, 0])
    assert PU.select_timesteps(ts, start_step=500).tolist() == [500, 20, 0]
    assert PU.select_timesteps(ts, last_n_steps=2).tolist() == [20, 0]
    assert PU.select_timesteps(ts, 960, 10).tolist() == [960, 500, 20, 0]
    with pytest.raises(ValueError):
        PU.select_timesteps(ts, start_step=-1)
    with pytest.raises(ValueError):
        PU.select_timesteps(ts, last_n_steps=0)
    with pytest.raises(ValueError, match="No timesteps"):
        PU.select_timesteps(torch.tensor([980, 960]), start_step=10)


def test_align_and_normalize_conditioning():
    c = torch.arange(2 * 1 * 2 * 2, dtype=torch.float32).view(2, 1, 2, 2)
    assert PU._align_conditioning(c, 5).shape[0] == 5
    assert torch.equal(PU._align_conditioning(c, 5)[2], c[0])
    z = PU.normalize_latent_conditioning(c, "standardize")
    assert torch.allclose(z.mean(dim=(2, 3)), torch.zeros(2, 1), atol=1e-6)
    m = PU.normalize_latent_conditioning(c, "minmax")
    assert m.amax().item() <= 1.0 and m.amin().item() >= 0.0
    assert PU.normalize_latent_conditioning(c, "off") is c
    with pytest.raises(ValueError):
        PU.normalize_latent_conditioning(c, "zscore")


# ------------------------------------------------------------------ factory surface
@pytest.mark.parametrize("name", MODEL_CASES)
def test_factory_state_dict_matches_reference_order(golden, name):
    _, M = golden
    m = M[name]
    tr = m["training"]
    spec = S.derive_spec(m["unet"], tr["conditioning"], tr["channels"] or 1)
    model = DiffusionUNetFactory().build(m["unet"], tr["conditioning"], tr["channels"] or 1)
    got = [(k, tuple(v.shape)) for k, v in model.state_dict().items()]
    want = list(U.param_shapes(spec).items())
    assert got == want


# ------------------------------------------------------------------ data parallel (gloo, world 2)
def test_bucket_bounds():
    assert dp.bucket_bounds(10, 4) == [(0, 3), (3, 6), (6, 9), (9, 10)]
    assert dp.bucket_bounds(3, 8) == [(0, 1), (1, 2), (2, 3)]
    assert dp.bucket_bounds(0, 4) == []
    b = dp.bucket_bounds(113_008_257, 4)
    assert b[0][0] == 0 and b[-1][1] == 113_008_257 and all(x[1] == y[0] for x, y in zip(b, b[1:]))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_worker(rank, world, port, meta, tensors, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    try:
        spec = S.derive_spec(meta["unet"], meta["training"]["conditioning"], meta["training"]["channels"] or 1)
        sd = {k: v.requires_grad_() for k, v in U.seeded_state_dict(spec, meta["seed"]).items()}
        B = tensors["clean"].shape[0]
        sl = slice(rank * B // world, (rank + 1) * B // world)        # DistributedSampler-style shard
        _, sc = OT.fm_loss(sd, spec, tensors["clean"][sl], tensors["ldct"][sl], tensors["noise"][sl],
                           tensors["t"][sl], meta["num_train_timesteps"])
        sc.backward()
        flat = torch.cat([p.grad.reshape(-1) for p in sd.values()])
        # the trainer's overlapped form: the front (decoder) part async, the rest blocking, then wait
        k = flat.numel() // 3
        works = dp.bucketed_allreduce_async(flat[:k], buckets=2)
        dp.bucketed_allreduce(flat[k:], buckets=3)
        for w in works:
            w.wait()
        flat /= world                                                     # grad_scale folded into AdamW on GPU
        if rank == 0:
            q.put(flat.numpy().copy())   # plain bytes: a shared-memory tensor dies with this process
    finally:
        dist.destroy_process_group()


def test_dp_allreduce_equals_global_batch(golden):
    """N-rank step with the bucketed all-reduce == one process on the concatenated batch."""
    T, M = golden
    meta = M["fm_step"]
    tensors = {k: T[f"fm_step/{k}"] for k in ("clean", "ldct", "noise", "t")}
    if tensors["clean"].shape[0] % 2:
        pytest.skip("fixture batch not divisible by 2")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, meta, tensors, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = torch.from_numpy(q.get(timeout=300))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    spec = S.derive_spec(meta["unet"], meta["training"]["conditioning"], meta["training"]["channels"] or 1)
    sd = {k: v.requires_grad_() for k, v in U.seeded_state_dict(spec, meta["seed"]).items()}
    _, sc = OT.fm_loss(sd, spec, tensors["clean"], tensors["ldct"], tensors["noise"], tensors["t"],
                       meta["num_train_timesteps"])
    sc.backward()
    want = torch.cat([p.grad.reshape(-1) for p in sd.values()])
    torch.testing.assert_close(got, want, rtol=1e-4, atol=1e-6)


def test_model_throughput_fields_match_reference_formulas():
    """pipelines.utils.model_throughput: the evaluate-side fields of diffusion_like.py:287-313."""
    from fmdiff.pipelines.utils import model_throughput
    row = model_throughput({"model_seconds": 2.0, "model_calls": 100}, 8)
    assert row == {"samples": 8, "model_seconds": "2.000000", "model_samples_per_second": "4.000000",
                   "model_seconds_per_sample": "0.25000000", "model_calls": 100}
    empty = model_throughput({}, 0)
    assert empty["model_samples_per_second"] == "0.000000" and empty["model_seconds_per_sample"] == "0.00000000"


# ------------------------------------------------------------------ bench.py's roofline traffic lookup
def test_bench_pmc_traffic_matches_timed_kernel_only():
    """bench.py reports ``roofline.traffic`` only from a committed PMC summary of the very kernel(s) it times
    (profiles/r*_traffic.json ``kernel_id``), the newest round first; any other kernel gets None."""
    import importlib.util
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(repo, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    fwd = bench.pmc_traffic("conv3x3_halo9b<false, 2, 0, 16>")
    assert fwd is not None and fwd["file"].startswith("profiles/r5_")
    assert 2.5e8 < fwd["bytes"] < 4e8   # ~1.05x the 276.8 MB algorithmic bytes of the 8x256^2x128 problem
    wg = bench.pmc_traffic(["wgrad_reduce2", "wgrad_halo_kernel<2, false>"])   # order-free set of kernels
    assert wg is not None and wg["file"].endswith("r5_wgrad_traffic.json")
    assert bench.pmc_traffic("conv3x3_halo<false, 2, false>") is None   # round 3's kernel: not the timed one
    assert bench.pmc_traffic(["wgrad_halo_kernel<2, false>"]) is None   # a subset is not the timed pair
    assert bench.pmc_traffic("conv3x3_halo9b<false, 2, 0, 8>") is None   # the 8-row instance: not the timed one


def test_tuning_table_and_override(monkeypatch):
    """runtime/tuning.py: every dispatch constant in one table, FMD_TUNE the only override; unknown names raise
    (a typo must not silently measure the default)."""
    import importlib
    from fmdiff.runtime import tuning
    try:
        monkeypatch.setenv("FMD_TUNE", "HALO_MIN_WG=64, SPLIT_CAP=8")
        t = importlib.reload(tuning)
        assert t.get("HALO_MIN_WG") == 64 and t.get("SPLIT_CAP") == 8 and t.overridden("SPLIT_CAP")
        assert t.get("HALO_SPLIT_WG") == t.TABLE["HALO_SPLIT_WG"][0] and not t.overridden("HALO_SPLIT_WG")
        monkeypatch.setenv("FMD_TUNE", "HALO_MIN_WGS=64")
        with pytest.raises(ValueError):
            importlib.reload(tuning)
        monkeypatch.delenv("FMD_TUNE")
        # a retired per-switch variable (round-4 A/B scripts set these) raises instead of measuring the default
        for stale in ("FMD_HALO_MIN_WG", "FMD_WGRAD_REDUCE", "FMD_HALO9"):
            monkeypatch.setenv(stale, "1")
            with pytest.raises(ValueError, match=stale):
                importlib.reload(tuning)
            monkeypatch.delenv(stale)
        tuning.check_environment({"FMD_LIB": "x", "FMD_TUNE": ""})   # the two live variables pass
    finally:
        monkeypatch.delenv("FMD_TUNE", raising=False)
        importlib.reload(tuning)
    assert not tuning._over


def test_conv_small_plan_is_a_host_query(monkeypatch):
    """fmd_conv_small_plan (csrc/conv_small.hip) decides eligibility on the host without a launch: the config-D latent
    UNet's small-level problems are taken, out-of-range ones refused (LDS, channel multiples, tile geometry)."""
    from fmdiff import _lib
    from fmdiff.runtime import ops
    try:
        _lib.lib()
    except (OSError, RuntimeError) as e:
        pytest.skip(f"library not loadable here: {e}")
    monkeypatch.setattr(ops, "SMALL_CONV", True)
    monkeypatch.setattr(ops, "SMALL_CONV_MAX_HW", 1024)
    monkeypatch.setattr(ops, "SMALL_CONV_MAX_WORK", 1 << 30)
    st64, st16 = ops.Stats(None, 64), ops.Stats(None, 16)
    gn = dict(st0=st64, st1=st64, groups=32, eps=1e-6)
    assert ops.conv_small_ok((8, 16, 16, 256), 128, C1=128, gn=gn, skip=(256, 128))      # 16^2 decoder concat
    assert ops.conv_small_ok((8, 4, 4, 512), 256, C1=256, gn=dict(gn, st0=st16, st1=st16), skip=(512, 256))
    assert ops.conv_small_ok((8, 1, 1, 512), 512, C1=512, mode="point", gn=dict(gn, st0=ops.Stats(None, 1),
                                                                                 st1=ops.Stats(None, 1)), skip=(512, 512))
    assert ops.conv_small_ok((8, 32, 32, 128), 128, mode="s2")
    assert not ops.conv_small_ok((8, 8, 8, 32), 64)          # C < 64
    assert not ops.conv_small_ok((8, 8, 8, 64), 24)          # K % 16
    assert not ops.conv_small_ok((8, 8, 12, 64), 64)         # Ho*Wo neither a multiple nor a divisor of 64
    assert not ops.conv_small_ok((1, 16, 16, 2048), 64, split=1)   # more than one CU's LDS unsplit ...
    assert ops.conv_small_ok((1, 16, 16, 2048), 64)               # ... fits as parts of the reduction
    assert not ops.conv_small_ok((8, 64, 64, 128), 128)      # above SMALL_CONV_MAX_HW
    # the in-launch split: parts until the grid has 256 workgroups, whole GroupNorm groups and >= 64 channels per
    # part; none where the grid already fills the chip; forced values validated
    gn2 = dict(gn, st0=ops.Stats(None, 4), st1=ops.Stats(None, 4))
    assert ops.conv_small_split((8, 2, 2, 512), 512, C1=512, gn=gn2, split=0) == 8        # 32 tiles -> 256
    assert ops.conv_small_split((8, 2, 2, 512), 512, C1=512, gn=gn2, split=1) == 1
    assert ops.conv_small_split((8, 2, 2, 512), 512, C1=512, gn=gn2, split=4) == 4
    assert ops.conv_small_split((8, 2, 2, 512), 512, C1=512, gn=gn2, split=3) < 0         # not a power of two
    assert ops.conv_small_split((8, 32, 32, 128), 128, mode="s2", split=0) == 1             # 32 x 8 16-cout tiles
    assert ops.conv_small_split((8, 16, 16, 128), 128, C1=128, gn=gn, skip=(128, 128), split=0) == 1
    assert ops.conv_small_split((8, 8, 8, 256), 256, gn=gn, split=0) == 2                   # 8 x 16 tiles -> 256


def test_small_level_caps_and_fold_descriptor(monkeypatch):
    """Host logic of the round-6 forward paths: the fmd_conv_small level caps of runtime/tuning.py (pixels, and
    pixels x input channels: config D's 16^2 level in, config B's 512-channel 16^2 level out), and the halo fold's
    descriptor fields (set from a pro_fold dict, cleared for the gn_prep fallback)."""
    from fmdiff import _lib
    from fmdiff.runtime import ops, tuning
    try:
        _lib.lib()
    except (OSError, RuntimeError) as e:
        pytest.skip(f"library not loadable here: {e}")
    assert tuning.get("SMALL_CONV_MAX_HW") == 256 and tuning.get("SMALL_CONV_MAX_WORK") == 65536
    monkeypatch.setattr(ops, "SMALL_CONV", True)
    st = ops.Stats(None, 64)
    gn = dict(st0=st, st1=st, groups=32, eps=1e-6)
    assert ops.conv_small_ok((8, 16, 16, 128), 128, C1=128, gn=gn)            # 256 px x 256 ch: D's 16^2 concat
    assert not ops.conv_small_ok((8, 16, 16, 512), 512, gn=dict(gn, st1=None))  # 256 x 512: B's 16^2 level
    assert ops.conv_small_ok((8, 8, 8, 256), 256, C1=256, gn=gn)              # 64 x 512
    assert not ops.conv_small_ok((8, 32, 32, 128), 128, gn=dict(gn, st1=None))  # 1,024 px: above the pixel cap
    d = _lib.ConvDesc()
    slab0, slab1 = torch.zeros(4), torch.zeros(4)
    f = dict(st0=ops.Stats(slab0, 64), st1=ops.Stats(slab1, 16), groups=32, eps=1e-5, gamma=None, beta=None,
             emb=torch.zeros(8, 512), silu=True)
    ops._set_fold(d, f)
    assert d.fold_st0 == slab0.data_ptr() and d.fold_rows0 == 64 and d.fold_rows1 == 16 and d.fold_G == 32
    assert abs(d.fold_eps - 1e-5) < 1e-12 and d.fold_emb_stride == 512 and d.pro_silu == 1
    ops._clear_fold(d)
    assert not d.fold_st0 and not d.fold_st1 and not d.fold_emb and d.fold_G == 0 and d.fold_rows0 == 0


def test_split_ticket_decision_mirrors_the_kernels(monkeypatch):
    """runtime/ops.split_ticket: which split-K convs combine inside their launch and the statistics rows they then
    write (the kernels return -14 otherwise, tests/test_gpu_halo_ticket.py): the halo kernel on whole 128-cout tiles
    with 64-pixel rows, never with a G side output, a residual + data-gradient epilogue, 3-D or fp32 / accumulating
    outputs; the implicit GEMM (opt-in, SPLIT_TICKET) on whole tiles without parity classes, one row per wave."""
    from fmdiff.runtime import ops
    monkeypatch.setattr(ops, "HALO_TICKET", True)
    monkeypatch.setattr(ops, "SPLIT_TICKET", False)
    st = ops.split_ticket
    assert st(True, 2, 128, 8192, 256, 128) == (True, 64)             # latent 32^2 ResBlock conv
    assert st(True, 1, 128, 8192, 256, 128) == (False, 0)             # unsplit: nothing to combine
    assert st(True, 2, 64, 8192, 256, 64)[0] is False                 # partial 128-cout tile
    assert st(True, 2, 128, 8192, 256, 128, gout=True)[0] is False    # G side output (the round-3 kernel)
    assert st(True, 2, 128, 8192, 256, 128, resid_and_ep=True)[0] is False
    assert st(True, 2, 128, 8192, 256, 128, d3=True)[0] is False
    assert st(True, 4, 256, 8192, 256, 128, out_f32=True)[0] is False
    assert st(False, 16, 256, 2048, 64, 128)[0] is False               # implicit GEMM: off by default
    monkeypatch.setattr(ops, "SPLIT_TICKET", True)
    assert st(False, 16, 256, 2048, 64, 128) == (True, 32)            # 64-pixel tiles: 32-pixel rows per wave
    assert st(False, 4, 64, 2048, 128, 64) == (True, 64)
    assert st(False, 4, 16, 4096, 256, 16) == (True, 64)              # K <= 16: 4 waves across 256 pixels
    assert st(False, 8, 256, 2000, 64, 128)[0] is False                # ragged pixel tile
    assert st(False, 8, 256, 2048, 64, 128, transposed=True, stride=2, ks=3, pad=1, Ho=32, Wo=32)[0] is False
    assert st(False, 8, 256, 2048, 64, 128, transposed=True, stride=1, ks=3, pad=1, Ho=16, Wo=16)[0] is True
    monkeypatch.setattr(ops, "HALO_TICKET", False)
    assert st(True, 2, 128, 8192, 256, 128)[0] is False
