#!/usr/bin/env python3
"""Time ops.head_train_bf16 alone (config 5's head: M = 160,000, bf16 h [M, 256], hidden 128, 20 classes, dropout
0.5) with the library named by PG_DIRECTGCN_LIB: HIP events over 20 calls after 3 warm-ups; one JSON line."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
M, Fd, C = 160000, 256, 20
torch.manual_seed(0)
model = pkg.ProtGramDirectGCN([128, 256, 256, 256], M, C, 4, 0, 512, 0.5, True).to(dev).train()
W1, b1, W2, b2, p_drop = model.head_train_args()
h = torch.randn(M, Fd, device=dev).to(torch.bfloat16)
y = torch.randint(0, C, (M,), device=dev)
seed = torch.randint(0, 2 ** 62, (1,), device=dev, dtype=torch.int64)
call = lambda: ops.head_train_bf16(h, W1, b1, W2, b2, y, 1.0 / M, p_drop, seed, None)  # noqa: E731
for _ in range(3):
    call()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    call()
e1.record()
torch.cuda.synchronize()
print(json.dumps({"lib": os.environ.get("PG_DIRECTGCN_LIB", "default").split("/")[-1],
                  "head_ms": round(e0.elapsed_time(e1) / 20, 4)}), flush=True)
