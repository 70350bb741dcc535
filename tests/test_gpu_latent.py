"""Config D composition on the GPU: ``latent_flow_sample`` (AutoencoderKL encode -> latent FM-Euler sampler ->
decode; the reference's encode_vae_batch + sample_with_scheduler + decode_vae_batch,
src/utils/model_utils/vae_utils.py:54-85, src/pipelines/utils.py:163-220) against the oracle composition:
oracle/vae.py (pinned to the reference's own AutoencoderKL by tests/golden/vae_golden.pt) + the oracle UNet +
the oracle FM-Euler loop.  Tolerance: relative L2 < 3e-2 on the decoded images (bf16 through an encoder, five
latent UNet evaluations and a decoder; each stage alone is ~1e-2)."""
import json
import os
import sys
import warnings

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "flow-matching-and-diffusion-models_amd")]

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / max(b.norm(), 1e-30))


@pytest.mark.parametrize("use_graph,small_conv", [(True, False), (False, False), (True, True)])
def test_latent_flow_sample_vs_oracle_composition(use_graph, small_conv, monkeypatch):
    """small_conv: the sampler's no-tape UNet evaluations through fmd_conv_small where the plan takes the level
    (runtime/ops.py SMALL_CONV), against the same oracle composition."""
    from fmdiff.models.generators import DiffusionUNetFactory
    from fmdiff.models.vae import AutoencoderKL
    from fmdiff.pipelines.latent import latent_flow_sample
    from fmdiff.pipelines.train.fused import FusedFlowSampler
    from oracle import schedulers as OS
    from oracle import spec as S
    from oracle import train_step as OT
    from oracle import unet as U
    from oracle import vae as V
    from fmdiff.runtime import ops
    monkeypatch.setattr(ops, "SMALL_CONV", small_conv)
    G = torch.load(os.path.join(REPO, "tests", "golden", "vae_golden.pt"), weights_only=True)
    vcfg = json.loads(bytes(G["cfg_json"].tolist()).decode())
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        vae = AutoencoderKL(**vcfg)
    vae.load_state_dict(G["state"])
    vae = vae.to(DEV).eval()
    E = vcfg["embed_dim"]
    ucfg = dict(in_channels=E, out_channels=E, layers_per_block=1, block_out_channels=[32, 64],
                attention_resolutions=[], sample_size=8)
    unet = DiffusionUNetFactory().build(ucfg, "concatenate", E).to(DEV)
    spec = S.derive_spec(ucfg, "concatenate", E)
    sd = U.seeded_state_dict(spec, 31)
    unet.load_state_dict(sd)
    steps = 5
    g = torch.Generator().manual_seed(17)
    imgs = torch.rand(2, 1, 32, 32, generator=g)
    noise = torch.randn(2, E, 8, 8, generator=g)
    got = latent_flow_sample(vae, FusedFlowSampler(unet, steps), imgs.to(DEV), noise.to(DEV), use_graph=use_graph)
    # oracle composition
    with torch.no_grad():
        mode = V.encode_moments(G["state"], vcfg, imgs * 2.0 - 1.0)[:, :E]
        lat = OT.sample(sd, spec, OS.FlowMatchEuler(1000, 1.0), steps, noise, cond=mode)
        ref = (V.decode(G["state"], vcfg, lat).clamp(-1.0, 1.0) + 1.0) * 0.5
    err = _rel(got, ref)
    print(f"latent_flow_sample graph={use_graph} small_conv={small_conv}: decoded rel L2 {err:.3e}")
    assert got.shape == ref.shape
    assert err < 3e-2
