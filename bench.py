"""Headline benchmark: LDCT 256x256 flow-matching UNet, train images/s + 50-step sampler, on MI355X.

Workload (BASELINE.json configs[1]): EfficientUNetND built
from the reference's ``configs/flow_matching/ldct_flow_matching.json`` ``model.unet``
block (113,008,257 params), concatenate conditioning (2 input channels), batch 8
per GPU, 256x256, synthetic LDCT-shaped tensors (clean in [0,1], ldct = clamp(clean
+ 0.05 N(0,1))), random init.  One "step" = one full FM train step (noise/t draw,
x_t, forward, MSE, backward, [RCCL gradient all-reduce], AdamW + cosine LR) on the
HIP engine, captured as a hipGraph on 1 GPU.  The sampler leg times a 50-step
FlowMatchEuler sampling of 8 images (one UNet forward + Euler update per step).

Multi-GPU: ``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N``;
each rank trains on its own batch of 8 (weak scaling) with a real gradient
all-reduce; the timed region is bracketed by barrier + synchronize and the max
over ranks is reported.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "flow-matching-and-diffusion-models_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# model.unet block of the reference's configs/flow_matching/ldct_flow_matching.json
LDCT_FM_UNET = {
    "sample_size": 256, "in_channels": 1, "out_channels": 1, "layers_per_block": 2,
    "block_out_channels": [128, 128, 256, 256, 512, 512],
    "down_block_types": ["DownBlock2D", "DownBlock2D", "DownBlock2D", "DownBlock2D", "AttnDownBlock2D", "DownBlock2D"],
    "up_block_types": ["UpBlock2D", "AttnUpBlock2D", "UpBlock2D", "UpBlock2D", "UpBlock2D", "UpBlock2D"],
    "attention_resolutions": [], "cross_attention_resolutions": [], "emb_activation_before_proj": False,
}
FWD_GFLOP_PER_IMAGE = 493.15          # SURVEY.md 8(a) a6 / Appendix A (torch.utils.flop_counter on the reference)
TRAIN_GFLOP_PER_IMAGE = 3 * FWD_GFLOP_PER_IMAGE
PEAK_BF16_TFLOPS = 2500.0            # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def conv_roofline(dev, iters=20, prob="fwd"):
    """Time the dominant kernels live with HIP events at the 256^2 level (128 -> 128 channels, batch 8),
    the problem that carries 8+3 of the 96 convs and ~55% of the UNet's FLOPs:
    ``fwd``   fused GN+SiLU -> 3x3 conv (conv3x3_halo<false,2>, statistics epilogue) -- the roofline line;
    ``dgrad`` its data gradient (conv3x3_halo<false,0>, flipped taps, SiLU' + GN-backward-sums epilogue);
    ``wgrad`` its weight gradient (wgrad_halo_kernel<2>, GN+SiLU recomputed; + the split-K reduce)."""
    from fmdiff.runtime import ops
    N, H, W, C, K = 8, 256, 256, 128, 128
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(N, H, W, C, device=dev, generator=g).to(torch.bfloat16)
    wf = torch.randn(K, C, 3, 3, device=dev, generator=g) * 0.03
    a = torch.rand(N, C, device=dev) + 0.5
    b = torch.randn(N, C, device=dev) * 0.1
    bias = torch.zeros(K, device=dev)
    out = torch.empty(N, H, W, K, device=dev, dtype=torch.bfloat16)
    if prob == "fwd":
        w = ops.prep_weights(wf, 0)
        wt = ops.tile_weights(w)

        def fn():
            ops.conv(x, K, w, pro=(a, b, True), bias=bias, out=out, want_stats=True, wgt_tiled=wt)
        kernel = "conv3x3_halo9b<false, 2, 0, 16> (GN+SiLU prologue, 3x3, 8x256x256x128->128, fused stats)"
        kid = ["conv3x3_halo9b<false, 2, 0, 16>"]
    elif prob == "dgrad":
        w = ops.prep_weights(wf, 3)
        wt = ops.tile_weights(w)
        dy = torch.randn(N, H, W, K, device=dev, generator=g).to(torch.bfloat16)

        def fn():
            ops.conv(dy, C, w, out=out, want_stats=True, ep=(x, None, a, b), wgt_tiled=wt)
        kernel = ("conv3x3_halo9b<false, 0, 0, 16> data gradient (flipped taps, SiLU' + GN-backward-sums epilogue, "
                  "8x256x256x128->128)")
        kid = ["conv3x3_halo9b<false, 0, 0, 16>"]
    else:
        dy = torch.randn(N, H, W, K, device=dev, generator=g).to(torch.bfloat16)
        dw = torch.zeros(K, C, 3, 3, device=dev)
        db = torch.zeros(K, device=dev)

        def fn():
            ops.wgrad(x, dy, dw, pro=(a, b, True), db=db)
        kernel = "wgrad_halo_kernel<2, false> + wgrad_reduce2 (GN+SiLU recomputed, 8x256x256x128->128x3x3, fp32 dW)"
        kid = ["wgrad_halo_kernel<2, false>", "wgrad_reduce2"]
    for _ in range(3):
        fn()
    # In the train step the 134 MB input arrives cold (written by an earlier kernel, evicted by the ones
    # in between); a back-to-back loop would serve it from the 256 MB Infinity Cache.  So every timed
    # launch follows a 512 MB write that evicts it, and only the conv itself is inside the events.
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    torch.cuda.synchronize()
    for e0, e1 in evs:
        flush.fill_(1)
        e0.record()
        fn()
        e1.record()
    torch.cuda.synchronize()
    ms = sum(e0.elapsed_time(e1) for e0, e1 in evs) / iters
    del flush
    flops = 2.0 * N * H * W * K * C * 9
    return dict(kernel=kernel, kernel_id=kid, ms=ms, tflops=flops / ms / 1e9, flops_per_launch=flops)


def pmc_traffic(kernel_ids):
    """HBM bytes per launch of the timed kernel(s) from the newest committed rocprofv3 PMC summary whose
    ``kernel_id`` names exactly these kernels (profiles/r*_traffic.json: FETCH_SIZE x2 + WRITE_SIZE, separate --pmc
    passes over the same problem, tools/gpu_pmc.sh + tools/pmc_traffic.py); None when no summary of THESE kernels is
    committed (a summary of another kernel is never reported)."""
    import glob
    import re
    want = sorted([kernel_ids] if isinstance(kernel_ids, str) else kernel_ids)
    best = None
    for fn in glob.glob(os.path.join(REPO, "profiles", "r*_traffic.json")):
        with open(fn) as f:
            j = json.load(f)
        kid = j.get("kernel_id")
        if kid is None or sorted([kid] if isinstance(kid, str) else kid) != want:
            continue
        rnd = int(re.match(r"r(\d+)_", os.path.basename(fn)).group(1))
        if best is None or rnd > best[0]:
            best = (rnd, fn, float(j["traffic_bytes_per_launch"]))
    return None if best is None else dict(bytes=best[2], file=os.path.relpath(best[1], REPO))


CONFIG_E_FWD_GFLOP = 32854.2   # forward GFLOP per 128^3 sample (torch flop counter on the reference)


def config_e_leg(dev, size=128, steps=5, warmup=2):
    """BASELINE.json configs[4] on one GPU: EfficientUNetND with spatial_dims=3 from the same ldct_flow_matching.json
    model block (308,246,913 parameters), one graph-captured FM train step on a synthetic (1,1,128,128,128) volume
    (+ its concatenated LDCT volume), batch 1 (the per-rank batch of the 8-GPU DDP config).  Returns ms/step,
    samples/s and the step's fraction of the dense bf16 MFMA peak at 3 x forward FLOPs."""
    from fmdiff.models.generators import DiffusionUNetFactory
    from fmdiff.pipelines.train.fused import FusedTrainStep
    torch.manual_seed(0)
    model = DiffusionUNetFactory().build(dict(LDCT_FM_UNET, spatial_dims=3, sample_size=size), "concatenate", 1).to(dev)
    nparam = sum(p.numel() for p in model.parameters())
    g = torch.Generator(device=dev).manual_seed(7)
    clean = torch.rand(1, 1, size, size, size, device=dev, generator=g)
    ldct = (clean + 0.05 * torch.randn(1, 1, size, size, size, device=dev, generator=g)).clamp(0, 1)
    tr = FusedTrainStep(model, lr=1e-4, warmup=500, total_steps=100000, num_train_timesteps=1000)
    tr.capture(clean, ldct, warmup_iters=2)
    for _ in range(warmup):
        tr.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = tr.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    gflop = 3 * CONFIG_E_FWD_GFLOP * (size / 128) ** 3
    out = dict(workload=f"config E: EfficientUNetND spatial_dims=3, {size}^3, batch 1, graph-captured FM train step",
               params=nparam, ms_per_step=dt * 1e3, samples_per_sec=1.0 / dt, tflops=gflop / dt / 1e3,
               mfma_frac=gflop / dt / 1e3 / PEAK_BF16_TFLOPS, loss=float(loss), steps=steps)
    del tr, model
    torch.cuda.empty_cache()
    return out


LDCT_VAE = dict(in_channels=1, out_channels=1, resolution=256, base_ch=128, down_channels=[128, 256, 512, 512],
                num_res_blocks=2, attn_resolutions=[], z_channels=4, embed_dim=4, dropout=0.0, use_attention=True,
                spatial_dims=2, emb_channels=None, use_scale_shift_norm=False, double_z=True, attn_heads=4,
                attn_dim_head=64)   # model block of the reference's configs/LDCT/LDCT_autoencoder_kl.json
CONFIG_D_GF = (269.2, 618.7, 7.748)   # encode, decode, one latent UNet step, GFLOP per image


def config_d_leg(dev, batch=8, steps=50, reps=3):
    """BASELINE.json configs[3] on one GPU: AutoencoderKL of LDCT_autoencoder_kl.json (82,599,141 parameters) + the
    latent FM UNet (the LDCT FM UNet block with 4 latent channels, concatenate conditioning on the encoded latent),
    random init; encode_vae_batch -> 50-step FlowMatchEuler sampler (graph-replayed) -> decode_vae_batch on
    synthetic 256x256 images, batch 8 (reference vae_utils.py:54-85, pipelines/utils.py:163-220).  Median of
    ``reps`` timed passes after one warm-up pass."""
    import warnings
    from fmdiff.models.generators import DiffusionUNetFactory
    from fmdiff.models.vae import AutoencoderKL
    from fmdiff.pipelines.latent import decode_vae_batch, encode_vae_batch
    from fmdiff.pipelines.train.fused import FusedFlowSampler
    torch.manual_seed(0)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        vae = AutoencoderKL(**LDCT_VAE).to(dev).eval()
    unet = DiffusionUNetFactory().build(dict(LDCT_FM_UNET, in_channels=4, out_channels=4, sample_size=32),
                                        "concatenate", 4).to(dev)
    sampler = FusedFlowSampler(unet, steps)
    g = torch.Generator(device=dev).manual_seed(3)
    img = torch.rand(batch, 1, 256, 256, device=dev, generator=g)
    times = []
    with torch.no_grad():
        for r in range(reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            cond = encode_vae_batch(vae, img).contiguous()
            lat = sampler.sample(torch.randn(cond.shape, device=dev, generator=g), cond, use_graph=True)
            out = decode_vae_batch(vae, lat)
            torch.cuda.synchronize()
            if r:
                times.append(time.perf_counter() - t0)
    dt = sorted(times)[len(times) // 2]
    gf = batch * (CONFIG_D_GF[0] + CONFIG_D_GF[1] + steps * CONFIG_D_GF[2])
    res = dict(workload=f"config D: AutoencoderKL encode -> {steps}-step latent FM-Euler -> decode, batch {batch}, "
                        f"256x256 -> 4x32x32", images_per_sec=batch / dt, ms=dt * 1e3, tflops=gf / dt / 1e3,
               mfma_frac=gf / dt / 1e3 / PEAK_BF16_TFLOPS, out_mean=float(out.mean()))
    del vae, unet, sampler
    torch.cuda.empty_cache()
    return res


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(iters=3, batch=2, sampler_steps=3):
    """The oracle (fp32 PyTorch-CPU restatement of the reference, proven bit-exact in
    tests/test_oracle_golden.py) timed on this host, per BASELINE.md section 3: one FM train step
    (fwd+bwd+AdamW) at batch ``batch`` on the config-B model, median of ``iters`` after one warm-up; and a
    bounded sample of the 50-step FlowMatchEuler sampler (the last ``sampler_steps`` steps of the 50-step
    schedule at the same batch, one UNet forward + Euler update each, timed after one warm-up step)."""
    from oracle import schedulers as OS
    from oracle import spec as S
    from oracle import train_step as OT
    from oracle import unet as U
    # the GPU box gives one GPU a 16-CPU share (os.cpu_count() reports the whole host)
    threads = min(os.cpu_count() or 1, int(os.environ.get("FMD_CPU_THREADS", "16")))
    torch.set_num_threads(threads)
    spec = S.derive_spec(LDCT_FM_UNET, "concatenate", 1)
    sd = {k: v.requires_grad_() for k, v in U.seeded_state_dict(spec, 0).items()}
    g = torch.Generator().manual_seed(0)
    B = batch
    clean = torch.rand(B, 1, 256, 256, generator=g)
    ldct = (clean + 0.05 * torch.randn(B, 1, 256, 256, generator=g)).clamp(0, 1)
    state = {}
    times = []
    for i in range(iters + 1):
        noise = torch.randn(B, 1, 256, 256, generator=g)
        t = torch.rand(B, generator=g)
        t0 = time.perf_counter()
        for p in sd.values():
            p.grad = None
        _, sc = OT.fm_loss(sd, spec, clean, ldct, noise, t, 1000)
        sc.backward()
        OT.adamw_step(sd, 1e-4, i + 1, state)
        dt = time.perf_counter() - t0
        log(f"[bench] cpu baseline train iter {i}: {dt:.2f} s ({threads} threads)")
        if i:
            times.append(dt)
    times.sort()
    med = times[len(times) // 2]
    # sampler: warm-up step, then the timed last `sampler_steps` steps of the 50-step schedule
    sched = OS.FlowMatchEuler(1000, 1.0)
    init = torch.randn(B, 1, 256, 256, generator=g)
    sdd = {k: v.detach() for k, v in sd.items()}
    OT.sample(sdd, spec, sched, 50, init, ldct, last_n_steps=1)
    t0 = time.perf_counter()
    OT.sample(sdd, spec, sched, 50, init, ldct, last_n_steps=sampler_steps)
    ds = (time.perf_counter() - t0) / sampler_steps
    log(f"[bench] cpu baseline sampler: {ds:.2f} s per step at batch {B}")
    return dict(value=B / med, unit="train images/s", cores=threads, kind="port", cpu_model=_cpu_model(),
                sampler_steps_per_sec=1.0 / ds, sampler_images_per_sec=B / (50 * ds),
                sample=f"oracle FM train step (fwd+bwd+AdamW), batch {B}, 256x256, config-B EfficientUNetND fp32, "
                       f"median of {iters} after 1 warm-up ({med:.2f} s/step); sampler: last {sampler_steps} of 50 "
                       f"FlowMatchEuler steps at batch {B} after 1 warm-up ({ds:.2f} s/step, images/s extrapolated "
                       f"to the 50-step loop)")


def _launch_ranks(n: int) -> int:
    """Run this script under ``python -m torch.distributed.run --nproc-per-node n`` (rendezvous on 127.0.0.1, a
    free port) as a child process; returns its exit code.  Called before any GPU work in this process."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    log(f"[bench] launching {n} ranks: {' '.join(cmd)}")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--img", type=int, default=256)
    ap.add_argument("--sampler-steps", type=int, default=50)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sampler", action="store_true")
    ap.add_argument("--no-roofline", action="store_true", help="skip the per-kernel roofline legs")
    ap.add_argument("--no-config-e", action="store_true", help="skip the config E (3-D 128^3) leg")
    ap.add_argument("--no-config-d", action="store_true", help="skip the config D (latent diffusion) leg")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `bench.py --gpus N` outside a launcher: start N rank processes (torch.distributed.run, the reference's
        # torchrun launch, README.md:56-59) BEFORE this process touches the GPU, and exit with their status;
        # rank 0 prints the JSON line
        sys.exit(_launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        log(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: reporting the launcher's world size")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; FMD_DIST_BACKEND=gloo + more ranks than GPUs rehearses the N-rank path (split graph
    # captures, overlapped bucket all-reduces, 1/world AdamW) on a one-GPU box (ranks share the device)
    dev_idx = local % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(dev_idx)
        dist.init_process_group(os.environ.get("FMD_DIST_BACKEND", "nccl"))
    dev = torch.device("cuda", dev_idx)
    torch.cuda.set_device(dev)
    # all work on a created stream: collectives after graph replays on the legacy null stream were measured to
    # corrupt gradient buckets on this stack (fused.py _own_stream)
    torch.cuda.set_stream(torch.cuda.Stream(dev))

    from fmdiff.models.generators import DiffusionUNetFactory
    from fmdiff.pipelines.train.fused import FusedFlowSampler, FusedSampler, FusedTrainStep

    torch.manual_seed(1234 + rank)
    model = DiffusionUNetFactory().build(LDCT_FM_UNET, "concatenate", 1).to(dev)
    if world > 1:   # identical initial replicas
        for p in model.parameters():
            dist.broadcast(p.data, 0)
    B, HW = args.batch, args.img
    g = torch.Generator(device=dev).manual_seed(99 + rank)
    clean = torch.rand(B, 1, HW, HW, device=dev, generator=g)
    ldct = (clean + 0.05 * torch.randn(B, 1, HW, HW, device=dev, generator=g)).clamp(0, 1)

    trainer = FusedTrainStep(model, lr=1e-4, warmup=500, total_steps=100 * 1000, num_train_timesteps=1000)
    use_graph = not args.no_graph   # N > 1: forward + backward replayed, all-reduce + AdamW issued eagerly
    if use_graph:
        try:
            trainer.capture(clean, ldct, warmup_iters=2)
        except RuntimeError as e:   # keep the N-rank run alive if this stack refuses the capture
            log(f"[bench] hipGraph capture failed ({e}); running the step eagerly")
            use_graph = False
    if use_graph:
        run = trainer.replay
    else:
        def run():
            return trainer.step(clean, ldct)
    for _ in range(args.warmup):
        loss = run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    tt = torch.tensor([dt], device=dev)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    dt = float(tt.item())
    loss_v = float(loss.item())
    ms_step = dt / args.steps * 1e3
    train_ips = world * B * args.steps / dt
    log(f"[bench] train: {ms_step:.2f} ms/step, {train_ips:.2f} img/s (world {world}), loss {loss_v:.4f}")

    samp = {}
    if not args.no_sampler:
        from fmdiff.pipelines.schedulers import DDPMScheduler
        from fmdiff.pipelines.utils import model_throughput

        def time_sampler(sampler, noise=None):
            """One untimed call (capture + warm-up), then one call timed between barriers (max over ranks)."""
            init = torch.randn(B, 1, HW, HW, device=dev, generator=g)
            sampler.sample(init, ldct, use_graph=use_graph, generator=g)
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            timing = {}
            t0 = time.perf_counter()
            sampler.sample(init, ldct, use_graph=use_graph, generator=g, timing=timing)
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            ds = torch.tensor([time.perf_counter() - t0], device=dev)
            if world > 1:
                dist.all_reduce(ds, op=dist.ReduceOp.MAX)
            return float(ds.item()), timing

        # config B: the 50-step FlowMatchEuler sampler (the metric's "sampler steps/sec")
        ds, timing = time_sampler(FusedFlowSampler(model, args.sampler_steps))
        samp = dict(sampler_images_per_sec=world * B / ds, sampler_steps_per_sec=args.sampler_steps / ds,
                    sampler_ms_per_step=ds / args.sampler_steps * 1e3, sampler_steps=args.sampler_steps,
                    sampler_mfma_frac=(world * B / ds) * args.sampler_steps * FWD_GFLOP_PER_IMAGE
                    / (world * PEAK_BF16_TFLOPS * 1e3),
                    # the reference's evaluate-side fields (diffusion_like.py:287-313), this rank's loop
                    sampler_model_throughput=model_throughput(timing, B))
        log(f"[bench] sampler: {samp['sampler_images_per_sec']:.2f} img/s, {samp['sampler_ms_per_step']:.2f} ms/step")
        # config C: DDPM sampling of the same 113 M EfficientUNetND (configs/diffusion/ldct_ddpm.json betas),
        # 50 leading-spaced steps (the graph-replayed FusedSampler; variance noise drawn up front)
        ddpm = FusedSampler(model, DDPMScheduler(1000, beta_start=0.00085, beta_end=0.012), args.sampler_steps)
        dd, _ = time_sampler(ddpm)
        samp.update(ddpm_sampler_images_per_sec=world * B / dd, ddpm_sampler_ms_per_step=dd / args.sampler_steps * 1e3,
                    ddpm_sampler_steps=args.sampler_steps)
        log(f"[bench] ddpm sampler: {samp['ddpm_sampler_images_per_sec']:.2f} img/s, "
            f"{samp['ddpm_sampler_ms_per_step']:.2f} ms/step")

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    roofline = back = None
    if not args.no_roofline:
        roof = conv_roofline(dev)
        log(f"[bench] dominant conv: {roof['ms']:.3f} ms, {roof['tflops']:.1f} TFLOP/s")
        tr = pmc_traffic(roof["kernel_id"])
        roofline = {"bound": "mfma", "achieved": roof["tflops"], "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                    "frac": roof["tflops"] / PEAK_BF16_TFLOPS, "traffic": tr and tr["bytes"], "kernel": roof["kernel"],
                    "kernel_ms": roof["ms"], "flops_per_launch": roof["flops_per_launch"],
                    "traffic_source": tr and tr["file"]}
        # the same problem's backward kernels (the step's next two largest buckets), same protocol
        back = {"peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s"}
        for prob in ("dgrad", "wgrad"):
            r = conv_roofline(dev, prob=prob)
            tr = pmc_traffic(r["kernel_id"])
            back[prob] = {"achieved": r["tflops"], "frac": r["tflops"] / PEAK_BF16_TFLOPS, "kernel": r["kernel"],
                          "kernel_ms": r["ms"], "flops_per_launch": r["flops_per_launch"],
                          "traffic": tr and tr["bytes"], "traffic_source": tr and tr["file"]}
            log(f"[bench] {prob}: {r['ms']:.3f} ms, {r['tflops']:.1f} TFLOP/s")
    cfg_e = None
    if world == 1 and not args.no_config_e:
        try:
            cfg_e = config_e_leg(dev)
            log(f"[bench] config E: {cfg_e['ms_per_step']:.1f} ms/step, {cfg_e['mfma_frac']:.3f} of peak")
        except Exception as e:  # pragma: no cover
            cfg_e = dict(error=str(e))
    cfg_d = None
    if world == 1 and not args.no_config_d:
        try:
            cfg_d = config_d_leg(dev)
            log(f"[bench] config D: {cfg_d['images_per_sec']:.1f} images/s ({cfg_d['ms']:.1f} ms per batch)")
        except Exception as e:  # pragma: no cover
            cfg_d = dict(error=str(e))
    step_tflops = train_ips / world * TRAIN_GFLOP_PER_IMAGE / 1e3
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline()
        except Exception as e:  # pragma: no cover
            cpu = dict(value=None, error=str(e))
    res = {
        "metric": "train images/sec + sampler steps/sec, LDCT 256x256 UNet at 1/2/4/8 MI355X",
        "value": train_ips,
        "unit": "train images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic LDCT-shaped tensors (clean U[0,1], ldct = clamp(clean + 0.05 N(0,1))), random init",
        "config": {"workload": "LDCT 2D 256x256 flow-matching train step (configs/flow_matching/ldct_flow_matching.json,"
                               " EfficientUNetND 113M, concatenate conditioning) + 50-step FlowMatchEuler sampler",
                   "global_batch": world * B, "per_gpu_batch": B, "img": HW, "parallelism": f"dp{world}",
                   "hipgraph": use_graph},
        "train_loss": loss_v,
        "train_mfma_frac": step_tflops / PEAK_BF16_TFLOPS,
        **samp,
        "roofline": roofline,
        "roofline_backward": back,
        "config_e_ms_per_step": cfg_e.get("ms_per_step") if cfg_e else None,
        "config_e": cfg_e,
        "config_d": cfg_d,
        "cpu_baseline": cpu,
    }
    print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
