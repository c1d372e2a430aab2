#!/usr/bin/env python3
"""Time pg_directgcn_head_f32 at the bench shape (N = 160000, F = 128 -> 64 -> 20), HIP events, min of rounds.
usage: python tools/head_probe.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
M, F, H, C = 160000, 128, 64, 20
h = torch.randn(M, F, generator=g).to(dev)
W1, b1 = (torch.randn(H, F, generator=g) * 0.1).to(dev), (torch.randn(H, generator=g) * 0.1).to(dev)
W2, b2 = (torch.randn(C, H, generator=g) * 0.1).to(dev), (torch.randn(C, generator=g) * 0.1).to(dev)
z = torch.relu(h @ W1.t() + b1)
lp_ref = torch.log_softmax(z @ W2.t() + b2, -1)
lp, emb = ops.head(h, W1, b1, W2, b2, 1e-12)
print("max |lp - torch|", float((lp - lp_ref).abs().max()))
ts = []
for _ in range(5):
    for _ in range(3):
        ops.head(h, W1, b1, W2, b2, 1e-12)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.head(h, W1, b1, W2, b2, 1e-12)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / 20)
print("head ms", " ".join(f"{t:.4f}" for t in ts), "min", f"{min(ts):.4f}")
