import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "flow-matching-and-diffusion-models_amd")
for p in (REPO, PKG_ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built HIP library")


def _gpu_ok():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_ok():
        return
    skip = pytest.mark.skip(reason="no ROCm GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def golden():
    import json

    import torch
    d = os.path.join(REPO, "tests", "golden")
    tensors = torch.load(os.path.join(d, "golden.pt"), weights_only=True)
    meta = json.load(open(os.path.join(d, "golden.json")))
    return tensors, meta


@pytest.fixture(scope="session")
def golden_b256():
    """Config B at its bench resolution (256x256, batch 2): tests/golden/make_golden_b256.py."""
    import json

    import torch
    d = os.path.join(REPO, "tests", "golden")
    tensors = torch.load(os.path.join(d, "golden_b256.pt"), weights_only=True)
    meta = json.load(open(os.path.join(d, "golden_b256.json")))
    return tensors, meta


@pytest.fixture(scope="session")
def golden_attn():
    """Reference SpatialCrossAttention / DiffusersAttentionND(context_dim) fixtures: make_golden_attn.py."""
    import json

    import torch
    d = os.path.join(REPO, "tests", "golden")
    tensors = torch.load(os.path.join(d, "golden_attn.pt"), weights_only=True)
    meta = json.load(open(os.path.join(d, "golden_attn.json")))
    return tensors, meta


@pytest.fixture(scope="session")
def golden_ddpm():
    """Reference DDPM train steps on configs C (256^2) and A (MNIST diffusers): make_golden_ddpm.py."""
    import json

    import torch
    d = os.path.join(REPO, "tests", "golden")
    tensors = torch.load(os.path.join(d, "golden_ddpm.pt"), weights_only=True)
    meta = json.load(open(os.path.join(d, "golden_ddpm.json")))
    return tensors, meta


@pytest.fixture(scope="session")
def golden_e():
    """Config E at its own architecture (308 M 3-D EfficientUNetND; 64^3 forward, 32^3 FM step): make_golden_e.py."""
    import json

    import torch
    d = os.path.join(REPO, "tests", "golden")
    tensors = torch.load(os.path.join(d, "golden_e.pt"), weights_only=True)
    meta = json.load(open(os.path.join(d, "golden_e.json")))
    return tensors, meta
