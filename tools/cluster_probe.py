#!/usr/bin/env python3
"""Cluster-GCN training epoch on the 4-gram graph: the reference's _train_model_clustered loop
(protgram_directgcn_trainer.py:125-141: per subgraph zero_grad -> autocast forward -> weighted nll + L2 ->
GradScaler backward/step) over subgraphs from cluster.build_subgraphs (320 clusters of ~500 nodes, the
reference's default for N > 10k). Prints the subgraph build time and ms per subgraph step.
usage: python tools/cluster_probe.py [ngram] [dims=128,128,128]"""
import os
import random
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import cluster  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
dims = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [128, 128, 128]
dev = torch.device("cuda:0")
N, s, d, c = pkg.synth.de_bruijn_edges(n)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
# the reference matrices as COO (what the trainer slices): the shared pattern with the three weights
rows = torch.repeat_interleave(torch.arange(N, device=dev), g.rowptr[1:] - g.rowptr[:-1])
ei = torch.stack([g.edges3[:, 0].long(), rows])
w = [g.edges3[:, k].contiguous().view(torch.float32) for k in (1, 2, 3)]
x = torch.randn(N, dims[0], generator=torch.Generator().manual_seed(1234)).to(dev)
y = (torch.arange(N, device=dev) // (20 ** (n - 1)))
torch.cuda.synchronize()
t0 = time.perf_counter()
parts = cluster.range_clusters(N, cluster.cluster_count(N), order=g.row_order.long())
subs = cluster.build_subgraphs(N, parts, ei, w[0], ei, w[1], ei, w[2], x, y)
torch.cuda.synchronize()
t_build = time.perf_counter() - t0
kept = sum(dd.graph.nnz for dd in subs)
print(f"{len(subs)} subgraphs built in {t_build:.3f}s; intra-cluster entries {kept} of {g.nnz} "
      f"({100.0 * kept / g.nnz:.1f}%)")

torch.manual_seed(0)
model = pkg.ProtGramDirectGCN(dims, N, int(y.max()) + 1, n, 0, 512, 0.5, True).to(dev).train()
opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=0.0)
scaler = torch.amp.GradScaler("cuda", enabled=True)


def epoch():
    random.shuffle(subs)
    tot = 0.0
    for bd in subs:
        opt.zero_grad()
        with torch.amp.autocast("cuda", enabled=True):
            out, _ = model(data=bd)
            loss = F.nll_loss(out, bd.y) * (bd.num_nodes / N)
            loss = loss + 1e-7 * sum(p.norm(2).pow(2) for p in model.parameters() if p.requires_grad)
        scaler.scale(loss).backward()
        scaler.step(opt)
        scaler.update()
        tot += loss.item()  # the reference's per-step host sync (trainer :140)
    return tot / len(subs)


random.seed(0)
epoch()
torch.cuda.synchronize()
t0 = time.perf_counter()
avg = epoch()
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print(f"epoch {dt:.3f}s = {1e3 * dt / len(subs):.3f} ms per subgraph step (avg loss {avg:.4f})")
