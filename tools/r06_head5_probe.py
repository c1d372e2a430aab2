#!/usr/bin/env python3
"""Round 6: config 5's prediction head training step at B(20,4) (M = 160,000 rows, bf16 h [M, 256], hidden 128,
20 classes, dropout 0.5): ops.head_train_bf16 (one kernel + its partial reduction) against the framework ops it
replaces in train_step (h.float(), decoder Linear / ReLU / Dropout / Linear via ops.row_linear, log_softmax, nll,
autograd backward to the bf16 h). HIP events over `reps` calls, min / median of interleaved rounds.
usage: python tools/r06_head5_probe.py [rounds=7] [reps=10]  -> one JSON line"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
dev = torch.device("cuda:0")
M, Fd, H, C = 160000, 256, 128, 20
torch.manual_seed(0)
model = pkg.ProtGramDirectGCN([128, 256, 256, 256], M, C, 4, 0, 512, 0.5, True).to(dev).train()
dec = model.decoder_fc
h0 = torch.randn(M, Fd, device=dev).to(torch.bfloat16)
y = torch.randint(0, C, (M,), device=dev)
seed = torch.randint(0, 2 ** 62, (1,), device=dev, dtype=torch.int64)


def kernel():
    h = h0.detach().requires_grad_(True)
    loss, dh, grads = ops.head_train_bf16(h, dec[0].weight, dec[0].bias, dec[3].weight, dec[3].bias, y, 1.0, 0.5, seed)
    torch.autograd.backward(h, grad_tensors=dh)
    return loss


def framework():
    h = h0.detach().requires_grad_(True)
    lp, _ = model.head(h.float(), need_emb=False)
    loss = -lp.float().gather(1, y.view(-1, 1)).mean()
    loss.backward()
    return loss


def timeit(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


cases = {"kernel": kernel, "framework": framework}
for fn in cases.values():
    for _ in range(3):
        fn()
torch.cuda.synchronize()
ts = {k: [] for k in cases}
for _ in range(rounds):
    for k, fn in cases.items():
        ts[k].append(timeit(fn))
out = {"M": M, "F": Fd, "H": H, "C": C, "rounds": rounds, "reps": reps}
for k, v in ts.items():
    v.sort()
    out[f"{k}_ms_min"] = round(v[0], 4)
    out[f"{k}_ms_med"] = round(v[len(v) // 2], 4)
print(json.dumps(out))
