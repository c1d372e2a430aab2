#!/usr/bin/env python3
"""Per-rank cost of the node-range + all-gather partition (shard.sharded_forward, the exchange path) measured on
one GPU at P ranks: every timed rank runs exactly its local work -- layer 1 over its row block reading the
replicated input, layer 2 over its row block reading the all-gathered layer-1 output (here the single-GPU
layer-1 output, which is what the all-gather assembles: shards of `per` rows, rank-major), dense + head -- with
HIP events; the all-gather itself is stated by volume (bytes every rank receives per forward) and modelled at an
assumed per-rank receive bandwidth, since one GPU cannot run it. Rows are compared with the single-GPU forward (the
row-mapped dense kernel of a row block rounds differently from the single-GPU split-bf16 kernel: max |d| reported).
usage: python tools/exchange_probe.py [ngram=5] [F=128] [P=8] [reps=20] [recv_GBs=300]"""
import dataclasses
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import shard  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
F = int(sys.argv[2]) if len(sys.argv) > 2 else 128
P = int(sys.argv[3]) if len(sys.argv) > 3 else 8
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
recv_gbs = float(sys.argv[5]) if len(sys.argv) > 5 else 300.0
dev = torch.device("cuda:0")
N, s, d, c = pkg.synth.de_bruijn_edges(n)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
del s, d, c
assert N % P == 0, "the probe reads the gathered buffer with global row ids: N must be a multiple of P"
torch.manual_seed(0)
model = pkg.ProtGramDirectGCN([F, F, F], N, 20, n, 0, 512, 0.5, True).to(dev).eval()
x = torch.randn(N, F, generator=torch.Generator().manual_seed(1234)).to(dev)
gc = dataclasses.replace(g, ngram=None)  # a rank's row block has no n-gram tile plan: CSR kernels throughout


def timeit(fn):
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


with torch.no_grad():
    c1, c2 = model.convs
    h1 = c1.fused_forward(x, gc, None, res_x=x, act=True)  # what the all-gather assembles on every rank
    lp_ref, emb_ref = model(pkg.Data(x=x, graph=gc))
    single_ms = timeit(lambda: model(pkg.Data(x=x, graph=g)))
    out = {"ngram": n, "N": N, "F": F, "P": P, "single_gpu_forward_ms": round(single_ms, 4), "ranks": {}}
    for rank in sorted({0, P // 2, P - 1}):
        part = shard.partition(gc, rank, P)
        plan = shard.gather_plan(part, 1)  # chunks = 1: buffer column ids = global ids when N % P == 0

        def local():
            Z = shard.ops.spmm3(part.local, x)
            hl = shard._dense_local(c1, part, Z, model.res_projs[0], x[part.r0:part.r1], 0, part.n_local)
            Z2 = shard.ops.spmm3(plan.remap, h1)
            h2 = shard._dense_local(c2, part, Z2, model.res_projs[1], hl, 0, part.n_local)
            return model.head(h2)

        lp, emb = local()
        dmax = max(float((lp - lp_ref[part.r0:part.r1]).abs().max()), float((emb - emb_ref[part.r0:part.r1]).abs().max()))
        ms = timeit(local)
        out["ranks"][rank] = {"rows": part.n_local, "local_ms": round(ms, 4), "max_abs_diff_vs_single_gpu": dmax}
    recv = (P - 1) * (N // P) * F * 4  # bytes every rank receives per forward (one layer boundary)
    out["allgather_bytes_received_per_rank"] = recv
    out["allgather_ms_modelled"] = round(recv / (recv_gbs * 1e6), 4)
    out["allgather_model"] = f"{recv_gbs:.0f} GB/s receive per rank (assumption; xGMI: 7 links per MI355X)"
    worst = max(v["local_ms"] for v in out["ranks"].values())
    out["step_ms_modelled_no_overlap"] = round(worst + out["allgather_ms_modelled"], 4)
    out["speedup_modelled_no_overlap"] = round(single_ms / out["step_ms_modelled_no_overlap"], 2)
    out["speedup_compute_only"] = round(single_ms / worst, 2)
print(json.dumps(out, indent=1))
