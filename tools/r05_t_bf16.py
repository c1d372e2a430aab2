#!/usr/bin/env python3
"""Transposed propagation on bf16 G at B(20,4): the 4x4-block kernel (default) against the transposed middle-tile
kernel (PG_FLAG_MID_TRANSPOSED), F = 128 and 256; HIP events over 20 calls after 5 warm-ups; one JSON line."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda", 0)
N, s, d, c = pkg.synth.de_bruijn_edges(4)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
res = {}
for F in (128, 256):
    G = torch.randn(N, 3 * F, generator=torch.Generator().manual_seed(F)).to(dev).to(torch.bfloat16)
    for name, fl in (("block4", ops.default_flags()), ("mid", ops.default_flags() | _lib.PG_FLAG_MID_TRANSPOSED)):
        for _ in range(5):
            ops.spmm3_t(g, G, flags=fl)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            out = ops.spmm3_t(g, G, flags=fl)
        e1.record()
        torch.cuda.synchronize()
        res[f"{name}_F{F}_ms"] = round(e0.elapsed_time(e1) / 20, 4)
    a = ops.spmm3_t(g, G, flags=ops.default_flags()).float()
    b = ops.spmm3_t(g, G, flags=ops.default_flags() | _lib.PG_FLAG_MID_TRANSPOSED).float()
    res[f"maxdiff_F{F}"] = float((a - b).abs().max())
print(json.dumps(res), flush=True)
