"""Golden fixture for config D end to end at its own architecture (BASELINE.json configs[3]).

Run in the build container only (the reference never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_d_latent.py

The reference composes config D across ``encode_vae_batch`` -> ``sample_with_scheduler`` -> ``decode_vae_batch``
(``src/utils/model_utils/vae_utils.py:54-85``, ``src/pipelines/utils.py:163-220``).  This script builds:

* the VAE of ``configs/LDCT/LDCT_autoencoder_kl.json`` with the reference's own ``VAEFactory.build_from_json``
  (82,599,141 parameters), filled by ``seeded_params.fill_module`` (seed 3131, as make_vae_golden_d.py);
* the latent UNet: the ``model.unet`` block of ``configs/flow_matching/ldct_flow_matching.json`` with 4 latent
  channels in and out and concatenate conditioning on the encoded latent (8 input channels), built by the
  reference's ``DiffusionUNetFactory``, parameters ``oracle.unet.seeded_state_dict`` (seed 7171);

and runs, at 256x256 (latents 4x32x32), batch 2: ``encode_vae_batch`` (reference) of the conditioning images, five
FlowMatchEuler steps of the reference's sampling loop (``sample_with_scheduler``'s body restated here verbatim in
structure: ``cat([current, cond])`` -> model -> ``scheduler.step``; the reference module imports diffusers, which is
absent, so the scheduler is ``oracle.schedulers.FlowMatchEuler``, the KAT-pinned restatement of diffusers'
FlowMatchEulerDiscreteScheduler, shift 1) from an injected initial latent, and ``decode_vae_batch`` (reference).
Records the images, the initial latent, the encoded conditioning latent, the sampled latent and the decoded images.
Output: ``tests/golden/golden_d_latent.pt`` (tensors only; ``weights_only=True``).
"""
from __future__ import annotations

import json
import os
import sys
import warnings

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REF, "src"))
sys.path.insert(0, HERE)

from models.generators import DiffusionUNetFactory  # noqa: E402  (reference)
from models.generators.vaefactory import VAEFactory  # noqa: E402  (reference)

def _load_vae_utils():
    """The reference's ``src/utils/model_utils/vae_utils.py`` loaded as a file: its package ``__init__`` imports
    ``diffusion_utils`` -> ``pipelines.utils`` -> diffusers (absent); the module itself needs only VAEFactory."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("ref_vae_utils", os.path.join(REF, "src/utils/model_utils/vae_utils.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


_VU = _load_vae_utils()
encode_vae_batch, decode_vae_batch = _VU.encode_vae_batch, _VU.decode_vae_batch  # (reference)

import seeded_params as SP  # noqa: E402
from oracle import schedulers as OS  # noqa: E402
from oracle import spec as S  # noqa: E402
from oracle import unet as U  # noqa: E402

VAE_CFG = "configs/LDCT/LDCT_autoencoder_kl.json"
FM_CFG = "configs/flow_matching/ldct_flow_matching.json"
IMG, B, STEPS = 256, 2, 5
VAE_SEED, UNET_SEED, DATA_SEED = 3131, 7171, 2727


def main():
    torch.set_num_threads(8)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        vae = VAEFactory().build_from_json(os.path.join(REF, VAE_CFG)).eval()
    SP.fill_module(vae, VAE_SEED)
    E = int(json.load(open(os.path.join(REF, VAE_CFG)))["model"]["embed_dim"])
    ucfg = dict(json.load(open(os.path.join(REF, FM_CFG)))["model"]["unet"], in_channels=E, out_channels=E,
                sample_size=IMG // 8)
    unet = DiffusionUNetFactory().build(ucfg, "concatenate", E).eval()
    unet.load_state_dict(U.seeded_state_dict(S.derive_spec(ucfg, "concatenate", E), UNET_SEED))
    g = torch.Generator().manual_seed(DATA_SEED)
    imgs = torch.rand(B, 1, IMG, IMG, generator=g)
    init = torch.randn(B, E, IMG // 8, IMG // 8, generator=g)
    sched = OS.FlowMatchEuler(1000, 1.0)
    with torch.no_grad():
        cond = encode_vae_batch(vae, imgs)
        sched.set_timesteps(STEPS)
        current = init.clone()
        for t in sched.timesteps:   # sample_with_scheduler body (pipelines/utils.py:200-219), concatenate mode
            model_input = torch.cat([current, cond], dim=1)
            pred = unet(model_input, t.expand(current.size(0)))
            current = sched.step(pred, t, current).prev_sample
        out = decode_vae_batch(vae, current)
    res = {"imgs": imgs, "init": init, "cond": cond, "latent": current, "out": out,
           "timesteps": sched.timesteps.clone(),
           "meta": torch.tensor(list(json.dumps(dict(ucfg=ucfg, E=E, steps=STEPS, vae_seed=VAE_SEED,
                                                     unet_seed=UNET_SEED)).encode()), dtype=torch.uint8)}
    torch.save(res, os.path.join(HERE, "golden_d_latent.pt"))
    print({k: tuple(v.shape) for k, v in res.items()}, float(out.mean()), float(current.abs().mean()))


if __name__ == "__main__":
    main()
