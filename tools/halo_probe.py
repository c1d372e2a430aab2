#!/usr/bin/env python3
"""Per-rank cost of the halo-recompute partition, measured on one GPU: for P in 1,2,3,4,8 every rank's forward
(shard.halo_forward, exactly the work that rank does on its own GPU: the path has no collective) is timed
in turn with HIP events; the max over ranks is the P-GPU step time up to launch skew.
usage: python tools/halo_probe.py [ngram] [F] [reps]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import shard  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
F = int(sys.argv[2]) if len(sys.argv) > 2 else 128
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 50
dev = torch.device("cuda:0")
N, s, d, c = pkg.synth.de_bruijn_edges(n)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
torch.manual_seed(0)
model = pkg.ProtGramDirectGCN([F, F, F], N, 20, n, 0, 512, 0.5, True).to(dev).eval()
x = torch.randn(N, F, generator=torch.Generator().manual_seed(1234)).to(dev)
data = pkg.Data(x=x, graph=g)


def timeit(fn):
    with torch.no_grad():
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


t1 = timeit(lambda: model(data))
print(f"single GPU: {t1:.4f} ms/step")
for P in (2, 3, 4, 8):
    ts, rows = [], []
    for r in range(P):
        hp = shard.halo_partition(g, r, P, 2)
        inp = shard.halo_inputs(model, hp, x)
        ts.append(timeit(lambda: shard.halo_forward(model, hp, inp)))
        rows.append(hp.layer_rows)
    m = max(ts)
    print(f"P={P}: per-rank ms {' '.join(f'{t:.4f}' for t in ts)}  max {m:.4f}  speedup {t1 / m:.2f}x  "
          f"rows/layer (max) {max(r[0] for r in rows)}/{max(r[1] for r in rows)}")
