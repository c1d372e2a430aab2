#!/usr/bin/env python3
"""Time the bf16 dense backward of one config-5 layer (F_in = F_out = 256, M = 160,000, leaky-relu, the constant's
fp32 gradient, dZ) with the library named by PG_DIRECTGCN_LIB (a diagnostics build of tools/r06_dgrad_exp_build.sh):
HIP events over 20 calls after 5 warm-ups; one JSON line."""
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
M, F = int(os.environ.get("PROBE_M", 160_000)), 256
gen = torch.Generator().manual_seed(3)
conv = pkg.DirectGCNLayer(F, F, M, True).to(dev)
prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in conv._dense_params())))
Z = torch.randn(M, 3 * F, generator=gen).to(dev).to(torch.bfloat16)
Y = torch.randn(M, F, generator=gen).to(dev).to(torch.bfloat16)
dY = torch.randn(M, F, generator=gen).to(dev).to(torch.bfloat16)
packs = list(ops.pack_weights_bf16(prm))
call = lambda: ops.layer_dense_backward(dY, Z, Y, prm, 0, act=True, packs=packs, dpre_f32=True)  # noqa: E731
for _ in range(5):
    call()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    call()
e1.record()
torch.cuda.synchronize()
print(json.dumps({"lib": os.environ.get("PG_DIRECTGCN_LIB", "default").split("/")[-1],
                  "bwd_ms": round(e0.elapsed_time(e1) / 20, 4)}), flush=True)
