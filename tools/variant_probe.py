#!/usr/bin/env python3
"""Interleaved timing of SpMM variants (several rounds, one process) to separate kernel differences from
run-to-run drift. usage: python tools/variant_probe.py [ngram] [F]"""
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
x32 = torch.randn(N, F, device=dev)
x16 = x32.to(torch.bfloat16)
G16 = torch.randn(N, 3 * F, device=dev).to(torch.bfloat16)
G32 = G16.float()


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


from protgram_directgcn_amd._lib import PG_FLAG_NO_NGRAM as CSR  # noqa: E402

variants = {
    "f32": lambda: ops.spmm3(g, x32, flags=0),            # n-gram tile kernel on B(20,n)
    "f32_csr": lambda: ops.spmm3(g, x32, flags=CSR),
    "f32_csr_u8": lambda: ops.spmm3(g, x32, flags=CSR | 4),
    "f32t": lambda: ops.spmm3_t(g, G32, flags=0),
    "f32t_csr": lambda: ops.spmm3_t(g, G32, flags=CSR),
    "bf16_u4": lambda: ops.spmm3(g, x16, flags=0),
    "bf16_u8": lambda: ops.spmm3(g, x16, flags=4),
    "bf16t_u4": lambda: ops.spmm3_t(g, G16, flags=0),
    "bf16t_u8": lambda: ops.spmm3_t(g, G16, flags=4),
}
res = {k: [] for k in variants}
for _ in range(4):
    for k, fn in variants.items():
        res[k].append(timeit(fn))
for k, v in res.items():
    print(f"{k:10s} " + " ".join(f"{t:.4f}" for t in v) + f"   min {min(v):.4f}")

# dense backward (fp32 and bf16) at this F, identity residual, vector gates
torch.manual_seed(0)
layer = pkg.DirectGCNLayer(F, F, N).to(dev)
prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in layer._dense_params())))
Z32 = ops.spmm3(g, x32)
Z16 = ops.spmm3(g, x16)
Y32 = ops.layer_dense(Z32, prm, 0, constant=layer.constant.detach(), res_x=x32, act=True)
Y16 = ops.layer_dense(Z16, prm, 0, constant=layer.constant.detach(), res_x=x16, act=True)
dY32 = torch.randn(N, F, device=dev)
dY16 = dY32.to(torch.bfloat16)
bw = {
    "dense_f32": lambda: ops.layer_dense(Z32, prm, 0, constant=layer.constant.detach(), res_x=x32, act=True),
    "dense_bf16": lambda: ops.layer_dense(Z16, prm, 0, constant=layer.constant.detach(), res_x=x16, act=True),
    "dbwd_f32": lambda: ops.layer_dense_backward(dY32, Z32, Y32, prm, 0, res_x=x32, act=True),
    "dbwd_bf16": lambda: ops.layer_dense_backward(dY16, Z16, Y16, prm, 0, res_x=x16, act=True),
}
res = {k: [] for k in bw}
for _ in range(3):
    for k, fn in bw.items():
        res[k].append(timeit(fn, reps=10))
for k, v in res.items():
    print(f"{k:10s} " + " ".join(f"{t:.4f}" for t in v) + f"   min {min(v):.4f}")
