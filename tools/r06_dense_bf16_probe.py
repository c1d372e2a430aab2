#!/usr/bin/env python3
"""Time the bf16 dense forward (pg_directgcn_dense_bf16 through ops.layer_dense) at config 5's shapes, M = 160,000:
F_in = F_out = 256 with the identity residual and the per-node constant, and F_in = 128 -> F_out = 256 with the
projected residual; HIP events over 20 calls after 5 warm-ups, with an output checksum (to compare library builds
named by PG_DIRECTGCN_LIB bit for bit). One JSON line."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
M = 160_000
res = {"lib": os.environ.get("PG_DIRECTGCN_LIB", "default").split("/")[-1]}
seed = torch.tensor([12345], dtype=torch.int64, device=dev)
for Fi, Fo, drop in ((256, 256, None), (128, 256, None), (256, 256, (0.5, seed))):
    gen = torch.Generator().manual_seed(3)
    torch.manual_seed(0)
    conv = pkg.DirectGCNLayer(Fi, Fo, M, True).to(dev)
    with torch.no_grad():
        for n_, p_ in conv.named_parameters():
            if n_.startswith("C_"):
                p_.copy_(torch.rand(p_.shape, generator=gen) + 0.5)
            elif n_ == "constant":
                p_.copy_(torch.randn(p_.shape, generator=gen) * 0.1)
    prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in conv._dense_params())))
    Z = torch.randn(M, 3 * Fi, generator=gen).to(dev).to(torch.bfloat16)
    X = torch.randn(M, Fi, generator=gen).to(dev).to(torch.bfloat16)
    const = conv.constant.detach()
    if Fi == Fo:
        call = lambda: ops.layer_dense(Z, prm, 0, constant=const, res_x=X, act=True, drop=drop)  # noqa: E731
    else:
        torch.manual_seed(1)
        lin = torch.nn.Linear(Fi, Fo).to(dev)
        W, b = lin.weight.detach(), lin.bias.detach()
        call = lambda: ops.layer_dense(Z, prm, 0, constant=const, res_x=X, W_res=W, b_res=b, act=True,  # noqa: E731
                                       drop=drop)
    for _ in range(5):
        Y = call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        Y = call()
    e1.record()
    torch.cuda.synchronize()
    v = Y.view(torch.int16).to(torch.int64)
    w = torch.arange(v.numel(), device=dev, dtype=torch.int64).view_as(v) % 1000003
    tag = f"F{Fi}_{Fo}" + ("_drop" if drop else "")
    res[tag + "_ms"] = round(e0.elapsed_time(e1) / 20, 4)
    res[tag + "_sum"] = int((v * w).sum())
print(json.dumps(res), flush=True)
