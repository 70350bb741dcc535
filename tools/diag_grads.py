"""Per-parameter gradient check of a small UNet config vs the oracle (GPU box diagnostic).

usage: python tools/diag_grads.py   (edit CFG)"""
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "flow-matching-and-diffusion-models_amd")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

CFG = dict(in_channels=1, out_channels=1, layers_per_block=1, block_out_channels=[32, 64, 64, 64],
           attention_resolutions=[], sample_size=8)


def main():
    from fmdiff.models.generators import DiffusionUNetFactory
    from oracle import spec as S
    from oracle import train_step as OT
    from oracle import unet as U
    cfg = dict(CFG)
    if len(sys.argv) > 1:
        cfg["sample_size"] = int(sys.argv[1])
    if len(sys.argv) > 2:
        cfg["block_out_channels"] = [int(v) for v in sys.argv[2].split(",")]
    model = DiffusionUNetFactory().build(cfg, "concatenate", 1).to("cuda")
    spec = S.derive_spec(cfg, "concatenate", 1)
    sd = U.seeded_state_dict(spec, 11)
    model.load_state_dict(sd)
    g = torch.Generator().manual_seed(5)
    s = cfg["sample_size"]
    clean, ldct, noise = (torch.randn(2, 1, s, s, generator=g) for _ in range(3))
    t = torch.rand(2, generator=g)
    sdg = {k: v.clone().requires_grad_() for k, v in sd.items()}
    _, scaled = OT.fm_loss(sdg, spec, clean, ldct, noise, t, 1000)
    scaled.backward()
    cd, ld, nd, td = clean.cuda(), ldct.cuda(), noise.cuda(), t.cuda()
    tb = td.view(-1, 1, 1, 1)
    pred = model((1.0 - tb) * cd + tb * nd, (td * 999).long(), context=ld)
    F.mse_loss(pred, nd - cd).backward()
    for k, p in model.named_parameters():
        gk = p.grad.double().cpu()
        r = sdg[k].grad.double()
        cos = float((gk * r).sum() / (gk.norm() * r.norm() + 1e-30))
        rel = float((gk - r).norm() / (r.norm() + 1e-30))
        flag = "  <<<" if cos < 0.99 else ""
        print(f"{k:48s} cos {cos:+.4f} rel {rel:.3e} |ref| {float(r.norm()):.3e}{flag}")


if __name__ == "__main__":
    main()
