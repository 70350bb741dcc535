"""Config D's latent UNet at its own architecture (the LDCT flow-matching UNet of bench.py with 4 latent + 4 condition
channels at 32x32, batch 8, random weights): the forward-only small-level paths of round 6 -- fmd_conv_small at 16^2
and below (runtime/ops.py SMALL_CONV) and the GroupNorm fold inside the 32^2 halo convs (HALO_FOLD) -- against the
round-5 launches (both off) on the same inputs, one no-grad UNet evaluation each (the sampler's step,
src/pipelines/utils.py:163-220 -> EfficientUNetND.forward, src/models/unet/unet.py).  Each path rounds to bf16 in its
own order, so the check is a relative L2 bound across ~60 convs, not equality."""
import os
import sys

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "flow-matching-and-diffusion-models_amd")]

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / max(b.norm(), 1e-30))


def test_latent_unet_small_level_paths_agree(monkeypatch):
    from bench import LDCT_FM_UNET
    from fmdiff.models.generators import DiffusionUNetFactory
    from fmdiff.runtime import ops
    from oracle import spec as S
    from oracle import unet as U
    ucfg = dict(LDCT_FM_UNET, in_channels=4, out_channels=4, sample_size=32)
    unet = DiffusionUNetFactory().build(ucfg, "concatenate", 4)
    # seeded weights with a non-zero output conv and non-trivial GroupNorm affines (the test's own tensors)
    unet.load_state_dict(U.seeded_state_dict(S.derive_spec(ucfg, "concatenate", 4), 31))
    unet = unet.to(DEV).eval()
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn(8, 4, 32, 32, device=DEV, generator=g)
    cond = torch.randn(8, 4, 32, 32, device=DEV, generator=g)
    t = torch.rand(8, device=DEV, generator=g) * 999.0
    outs = {}
    for small, fold in ((False, False), (True, False), (False, True), (True, True)):
        monkeypatch.setattr(ops, "SMALL_CONV", small)
        monkeypatch.setattr(ops, "HALO_FOLD", fold)
        with torch.no_grad():
            outs[(small, fold)] = unet(x, t, context=cond).float()
        torch.cuda.synchronize()
    base = outs[(False, False)]
    assert torch.isfinite(base).all()
    for k, v in outs.items():
        err = _rel(v, base)
        print(f"[latent paths] small_conv={k[0]} halo_fold={k[1]}: rel L2 vs round-5 path {err:.2e}")
        assert err < 2e-2, (k, err)
