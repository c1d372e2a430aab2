#!/usr/bin/env python3
"""Time train.Adam's step (one pg_adam_f32 launch) over config 5's parameter volume: three per-node constants
[160,000, 256] (bf16 gradients, as train_step files them) plus 40 small fp32 tensors, with the library named by
PG_DIRECTGCN_LIB; HIP events over 20 steps after 3 warm-ups, and a checksum of the parameters after them."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops, train  # noqa: E402

dev = torch.device("cuda", 0)
gen = torch.Generator().manual_seed(0)
big = [torch.nn.Parameter((torch.randn(160_000, 256, generator=gen) * 0.1).to(dev)) for _ in range(3)]
small = [torch.nn.Parameter(torch.randn(256, 256, generator=gen).to(dev)) for _ in range(40)]
gbig = [(torch.randn(160_000, 256, generator=gen) * 1e-3).to(dev).to(torch.bfloat16) for _ in range(3)]
for p in small:
    p.grad = torch.randn(p.shape, generator=gen).to(dev) * 1e-3
opt = train.Adam(big + small, lr=1e-3)


def step():
    for p, g in zip(big, gbig):
        ops._DEFERRED_GRADS[p.data_ptr()] = g
    try:
        opt.step()
    finally:
        ops._DEFERRED_GRADS.clear()


for _ in range(3):
    step()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    step()
e1.record()
torch.cuda.synchronize()
cs = sum(float(p.detach().double().sum()) for p in big + small)
print(json.dumps({"lib": os.environ.get("PG_DIRECTGCN_LIB", "default").split("/")[-1],
                  "adam_step_ms": round(e0.elapsed_time(e1) / 20, 4), "checksum": cs}), flush=True)
