"""Micro-benchmark of the fused AdamW + cosine-schedule launch on config B's flat parameter buffer (GPU box).

usage: [FMD_LIB=...] python tools/adamw_micro.py [--n 113008257] [--iters 20]
Prints us/launch and the achieved HBM rate at the algorithmic 28 B/param (read p, g, m, v; write p, m, v).
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
    ap.add_argument("--n", type=int, default=113008257)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    p, g, m, v = (torch.randn(a.n, device=dev) * 0.01 for _ in range(4))
    v.abs_()
    ctr = torch.zeros(1, dtype=torch.int32, device=dev)
    for _ in range(5):
        ops.adamw_sched(p, g, m, v, ctr, 1e-4, 500, 100000)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        ops.adamw_sched(p, g, m, v, ctr, 1e-4, 500, 100000)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / a.iters * 1e3
    print(f"adamw_sched n={a.n}: {us:.1f} us/launch, {28 * a.n / us / 1e3:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
