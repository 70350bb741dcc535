"""The trainer entry points end to end on one GPU (world 1), with the real FusedTrainStep.

``flow_matching_lib.train`` / ``diffusion_lib.train`` on a synthetic ``{"target", "image"}`` dataset
(reference ``flow_matching_lib.py:33-248``, ``diffusion_lib.py:34-250``): hipGraph-replayed full batches
plus an eager ragged last batch, device-side epoch loss, checkpoints in torch AdamW / LambdaLR format
(loadable by ``torch.optim.AdamW``), visual grids through ``decode_diffusion_batch``, resume; and the
pinned-host -> side-stream ``DevicePrefetcher``.
"""
import json
import math
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

UNET = {"sample_size": 32, "in_channels": 1, "out_channels": 1, "layers_per_block": 1, "block_out_channels": [32, 64],
        "attention_resolutions": []}


def _dataset(n, seed=0):
    from fmdiff.data import TensorPairDataset
    g = torch.Generator().manual_seed(seed)
    clean = torch.rand(n, 1, 32, 32, generator=g)
    ldct = (clean + 0.05 * torch.randn(n, 1, 32, 32, generator=g)).clamp(0, 1)
    return TensorPairDataset(clean, ldct)


def _cfg(tmp, model_type, epochs, sched):
    cfg = {"training": {"batch_size": 2, "num_epochs": epochs, "learning_rate": 1e-3, "lr_warmup_steps": 2,
                        "conditioning": "concatenate", "channels": 1, "num_workers": 0, "seed": 3,
                        "save_images": True, "save_images_every": 2, "visual_samples": 4, "num_inference_steps": 4,
                        "save_model_epochs": 1, "output_dir": os.path.join(tmp, "runs", model_type)},
           "model": {"unet": UNET, "scheduler": sched, "model_type": model_type}}
    p = os.path.join(tmp, f"{model_type}.json")
    with open(p, "w") as f:
        json.dump(cfg, f)
    return p


@pytest.mark.parametrize("kind", ["flow_matching", "diffusion"])
def test_train_entry_point_world1(tmp_path, kind):
    from fmdiff.models.generators import DiffusionUNetFactory
    from fmdiff.pipelines.train import diffusion_lib, flow_matching_lib
    sched = ({"name": "flow_match_euler", "num_train_timesteps": 1000, "num_inference_steps": 4}
             if kind == "flow_matching" else
             {"name": "ddpm", "num_train_timesteps": 1000, "num_inference_steps": 4,
              "params": {"beta_start": 0.00085, "beta_end": 0.012}})
    lib, prefix = (flow_matching_lib, "flow") if kind == "flow_matching" else (diffusion_lib, "diff")
    ds = _dataset(7)
    cfg = _cfg(str(tmp_path), kind, 2, sched)
    lib.train(ds, cfg)
    out = os.path.join(str(tmp_path), "runs", f"{kind}_run1")
    rows = open(os.path.join(out, "metrics.csv")).read().strip().splitlines()
    losses = [float(r.split(",")[1]) for r in rows[1:]]
    print(kind, "epoch losses", losses)
    assert len(losses) == 2 and all(math.isfinite(v) and v > 0 for v in losses)
    for f in (f"{prefix}_last.pt", f"{prefix}_best.pt", "epochs/epoch0002/epoch.pt", "visuals/epoch0002_output.png"):
        assert os.path.exists(os.path.join(out, f)), f
    ck = torch.load(os.path.join(out, f"{prefix}_last.pt"), weights_only=True)
    steps = 2 * math.ceil(7 / 2)
    assert ck["lr_scheduler"]["last_epoch"] == steps
    # drop-in: the reference's torch AdamW accepts the optimizer state (keys, per-parameter moments, step count)
    m = DiffusionUNetFactory().build(UNET, "concatenate", 1)
    m.load_state_dict(ck["model"])
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3)
    opt.load_state_dict(ck["optimizer"])
    st = opt.state_dict()["state"]
    assert len(st) == len(list(m.parameters())) and all(int(v["step"]) == steps for v in st.values())
    assert all(torch.isfinite(v["exp_avg"]).all() and (v["exp_avg_sq"] >= 0).all() for v in st.values())
    # resume for one more epoch: starts at epoch 3 with the saved moments and step count
    with open(cfg) as f:
        c = json.load(f)
    c["training"]["num_epochs"] = 3
    c["training"]["output_dir"] = out
    c["training"]["save_images"] = False
    with open(cfg, "w") as f:
        json.dump(c, f)
    lib.train(ds, cfg, resume=os.path.join(out, f"{prefix}_last.pt"))
    ck3 = torch.load(os.path.join(out, f"{prefix}_last.pt"), weights_only=True)
    assert ck3["epoch"] == 3 and ck3["lr_scheduler"]["last_epoch"] == steps + math.ceil(7 / 2)
    assert len(open(os.path.join(out, "metrics.csv")).read().strip().splitlines()) == 4


def test_device_prefetcher_delivers_every_batch_in_order():
    """Pinned staging + side-stream copies: every batch arrives intact, in order, on the device, also when
    the consumer overwrites nothing and a batch's buffers are reused two batches later."""
    from torch.utils.data import DataLoader
    from fmdiff.data import DevicePrefetcher
    ds = _dataset(9, seed=5)
    loader = DataLoader(ds, batch_size=2, shuffle=False)
    got = []
    for b in DevicePrefetcher(loader, "cuda"):
        assert b["target"].is_cuda and b["image"].is_cuda
        x = b["target"] * 2.0 + b["image"]        # consume on the compute stream
        got.append(x.cpu())
    ref = [ds.target[i:i + 2] * 2.0 + ds.image[i:i + 2] for i in range(0, 9, 2)]
    assert len(got) == len(ref)
    for a, b in zip(got, ref):
        assert torch.equal(a, b)
