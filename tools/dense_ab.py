#!/usr/bin/env python3
"""A/B timing of the dense layer kernels in the in-tree library on the bench's layer-1 shape (B(20,n), F = 128,
vector gates, constant, identity residual): the default (dense_x3p_kernel<.., IL>: interleaved LDS-DMA issue) against
PG_FLAG_DENSE_NO_IL (all pieces at the top of the iteration), interleaved rounds (min and median per launch, HIP events), and a bit-equality check.
usage: python tools/dense_ab.py [n=4] [rounds=20] [reps=20]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops  # noqa: E402
from protgram_directgcn_amd._lib import PG_FLAG_DENSE_NO_IL  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
n = int(args[0]) if args else 4
rounds = int(args[1]) if len(args) > 1 else 20
reps = int(args[2]) if len(args) > 2 else 20
dev = torch.device("cuda:0")
N, s, d, c = pkg.synth.de_bruijn_edges(n)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
import bench  # noqa: E402

model = bench.bench_model(pkg, N, 128, 2, n).to(dev).eval()
layer = model.convs[0]
x = torch.randn(N, 128, generator=torch.Generator().manual_seed(1234)).to(dev)
prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in layer._dense_params())))
Z = ops.spmm3(g, x)
Y = torch.empty(N, 128, device=dev)
base = ops.default_flags()
variants = {"x3p_il": base, "x3p_no_il": base | PG_FLAG_DENSE_NO_IL}


def run(fl):
    return ops.layer_dense(Z, prm, 0, constant=layer.constant.detach(), res_x=x, act=True, flags=fl, out=Y)


with torch.no_grad():
    outs = {k: run(fl).clone() for k, fl in variants.items()}
    same = all(torch.equal(outs["x3p_il"], v) for v in outs.values())
    times = {k: [] for k in variants}
    for _ in range(rounds):
        for k, fl in variants.items():
            for _ in range(3):
                run(fl)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                run(fl)
            e1.record()
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / reps * 1e3)
res = {k: {"min_us": round(min(v), 2), "median_us": round(sorted(v)[len(v) // 2], 2)} for k, v in times.items()}
res["bit_identical"] = same
res["shape"] = f"B(20,{n}) M={N} F=128, vector gates, constant, identity residual (layer_dense calls incl. host)"
print(json.dumps(res))
