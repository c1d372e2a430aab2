#!/usr/bin/env python3
"""Time the bf16 dense backward (pg_directgcn_dense_bwd_bf16) at B(20,4) rows, F = 128 and 256 (the library named by
PG_DIRECTGCN_LIB): HIP events over 20 calls after 5 warm-ups; prints one JSON line."""
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
for F in (128, 256):
    gen = torch.Generator().manual_seed(3)
    conv = pkg.DirectGCNLayer(F, F, M, True).to(dev)
    prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in conv._dense_params())))
    Z = torch.randn(M, 3 * F, generator=gen).to(dev).to(torch.bfloat16)
    Y = torch.randn(M, F, generator=gen).to(dev).to(torch.bfloat16)
    dY = torch.randn(M, F, generator=gen).to(dev).to(torch.bfloat16)
    packs = list(ops.pack_weights_bf16(prm))
    Zf, Yf, dYf = Z.float(), Y.float(), dY.float()

    def timed(call):
        for _ in range(5):
            call()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            call()
        e1.record()
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) / 20, 4)

    res[f"bwd_bf16_F{F}_ms"] = timed(lambda: ops.layer_dense_backward(dY, Z, Y, prm, 0, act=True, packs=packs))
    from protgram_directgcn_amd import _lib
    res[f"bwd_bf16_dgradtiled_F{F}_ms"] = timed(lambda: ops.layer_dense_backward(
        dY, Z, Y, prm, 0, act=True, packs=packs, flags=ops.default_flags() | _lib.PG_FLAG_DGRAD_BF16_TILED))
    res[f"bwd_f32_F{F}_ms"] = timed(lambda: ops.layer_dense_backward(dYf, Zf, Yf, prm, 0, act=True))
    res[f"bwd_f32_wgradf32mfma_F{F}_ms"] = timed(lambda: ops.layer_dense_backward(
        dYf, Zf, Yf, prm, 0, act=True, flags=ops.default_flags() | _lib.PG_FLAG_WGRAD_F32MFMA))
    res[f"bwd_f32_dgradf32mfma_F{F}_ms"] = timed(lambda: ops.layer_dense_backward(
        dYf, Zf, Yf, prm, 0, act=True, flags=ops.default_flags() | _lib.PG_FLAG_DGRAD_F32MFMA))
print(json.dumps(res), flush=True)
