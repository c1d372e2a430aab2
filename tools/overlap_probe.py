#!/usr/bin/env python3
"""Can the TD-bound spmm3 and the MFMA-bound dense kernel share the chip? Times each alone, both back to back on
one stream, and both on two streams (independent buffers). usage: python tools/overlap_probe.py [ngram] [F]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
F = int(sys.argv[2]) if len(sys.argv) > 2 else 128
dev = torch.device("cuda:0")
N, s, d, c = pkg.synth.de_bruijn_edges(n)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
x = torch.randn(N, F, device=dev)
torch.manual_seed(0)
layer = pkg.DirectGCNLayer(F, F, N).to(dev)
prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in layer._dense_params())))
Z1 = ops.spmm3(g, x)
Z2 = Z1.clone()
const = layer.constant.detach()
Y = torch.empty(N, F, device=dev)
sA = torch.cuda.Stream()
sB = torch.cuda.Stream()


def spmm():
    ops.spmm3(g, x, out=Z1)


def dense():
    ops.layer_dense(Z2, prm, 0, constant=const, res_x=x, act=True, out=Y)


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


def serial():
    spmm()
    dense()


def two_streams():
    cur = torch.cuda.current_stream()
    sA.wait_stream(cur)
    sB.wait_stream(cur)
    with torch.cuda.stream(sA):
        spmm()
    with torch.cuda.stream(sB):
        dense()
    cur.wait_stream(sA)
    cur.wait_stream(sB)


res = {k: [] for k in ("spmm", "dense", "serial", "two_streams")}
for _ in range(4):
    for k, fn in (("spmm", spmm), ("dense", dense), ("serial", serial), ("two_streams", two_streams)):
        res[k].append(timeit(fn))
for k, v in res.items():
    print(f"{k:12s} " + " ".join(f"{t:.4f}" for t in v) + f"   min {min(v):.4f}")
