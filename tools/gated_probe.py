#!/usr/bin/env python3
"""pg_spmm3_gated_f32 vs pg_spmm3_f32 (interleaved timing) and the forward step with / without the pre-gated
inference path. usage: python tools/gated_probe.py [ngram]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
F = 128
dev = torch.device("cuda:0")
N, s, d, c = pkg.synth.de_bruijn_edges(n)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
x = torch.randn(N, F, generator=torch.Generator().manual_seed(1234)).to(dev)
torch.manual_seed(0)
model = pkg.ProtGramDirectGCN([F, F, F], N, 20, n, 0, 512, 0.5, True).to(dev).eval()
layer = model.convs[0]
prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in layer._dense_params())))
data = pkg.Data(x=x, graph=g)


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def fwd(pre):
    ops.PREGATED_INFERENCE = pre
    with torch.no_grad():
        model(data)


variants = {"spmm3": lambda: ops.spmm3(g, x), "spmm3_gated": lambda: ops.spmm3_gated(g, x, prm, 0),
            "fwd_ungated": lambda: fwd(False), "fwd_pregated": lambda: fwd(True)}
res = {k: [] for k in variants}
for _ in range(4):
    for k, fn in variants.items():
        res[k].append(timeit(fn))
for k, v in res.items():
    print(f"{k:14s} " + " ".join(f"{t:.4f}" for t in v) + f"   min {min(v):.4f}")
