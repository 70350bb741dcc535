"""Micro-benchmark of the softmax attention cores (GPU box; also run under rocprofv3 --kernel-trace --stats).

usage: python tools/attn_micro.py [--iters 20] 
Problems (batch 8):
  vae_mid   : SpatialSelfAttention of the VAE mid block, 32x32 latent grid -> T=1024, 4 heads x 64 (raw split)
  unet_mid  : EfficientUNetND config-B mid block, 8x8 -> T=64, 4 heads x 64 (raw split)
  diff_t256 : DiffusersAttentionND at the 16x16 level, T=256, 16 heads x 8 (view/transpose split)
  cross     : SpatialCrossAttention, Tq=256 (16x16) over Tk=1024 context tokens, 4 heads x 64
TF/s counts the two T x T x dh products of the forward (4 T^2 dh flops per head) and the five of the backward.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "flow-matching-and-diffusion-models_amd")]

import torch  # noqa: E402

from fmdiff.runtime import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--impl", default="mfma")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    B = 8
    probs = {"vae_mid": (1024, 1024, 4, 64, 1, 0), "unet_mid": (64, 64, 4, 64, 1, 0),
             "diff_t256": (256, 256, 16, 8, 0, 0), "cross": (256, 1024, 4, 64, 1, 1)}
    for name, (Tq, Tk, heads, dh, raw, cross) in probs.items():
        if a.only and name not in a.only.split(","):
            continue
        inner = heads * dh
        if cross:
            q = (torch.randn(B, Tq, inner, device=dev, generator=g) * 0.5).to(torch.bfloat16)
            kv = (torch.randn(B, Tk, 2 * inner, device=dev, generator=g) * 0.5).to(torch.bfloat16)
            fwd = lambda: ops.cross_attention_fwd(q, kv, Tq, Tk, heads, dh, None, raw)  # noqa: E731
        else:
            qkv = (torch.randn(B, Tq, 3 * inner, device=dev, generator=g) * 0.5).to(torch.bfloat16)
            fwd = lambda: ops.attention_fwd(qkv, Tq, heads, dh, raw)  # noqa: E731
        dout = (torch.randn(B, Tq, inner, device=dev, generator=g) * 0.5).to(torch.bfloat16)
        for impl in a.impl.split(","):
            assert impl == "mfma", "the VALU softmax kernels were removed in round 3"
            o, lse = fwd()
            if cross:
                bwd = lambda: ops.cross_attention_bwd(q, kv, o, dout, lse, Tq, Tk, heads, dh, None, raw)  # noqa: E731
            else:
                bwd = lambda: ops.attention_bwd(qkv, o, dout, lse, Tq, heads, dh, raw)  # noqa: E731
            for label, fn, nprod in (("fwd", fwd, 2), ("bwd", bwd, 5)):
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / a.iters
                flops = 2.0 * nprod * B * heads * Tq * Tk * dh
                print(f"{name:9s} {impl:4s} {label} {ms * 1e3:9.1f} us/call {flops / ms / 1e9:7.2f} TFLOP/s", flush=True)



if __name__ == "__main__":
    main()
