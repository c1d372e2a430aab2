#!/usr/bin/env python3
"""One rank's forward of the middle partition (shard.MiddleRunner, graphs replayed), its ghost-row exchange filled
locally from a precomputed layer-1 output: the target for `rocprofv3 --kernel-trace --stats` to see where a rank's
time goes. usage: python tools/middle_rank_run.py [ngram=4] [P=8] [rank=0] [reps=50] [chunks=1]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops, shard  # noqa: E402
from protgram_directgcn_amd.graph import take  # noqa: E402
import bench  # noqa: E402

a = [int(v) for v in sys.argv[1:]]
n, P, rank, reps, chunks = (a + [4, 8, 0, 50, 1][len(a):])[:5]
dev = torch.device("cuda:0")
N, s, d, c = pkg.synth.de_bruijn_edges(n)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
model = bench.bench_model(pkg, N, 128, 2, n).to(dev).eval()
x = torch.randn(N, 128, generator=torch.Generator().manual_seed(1234)).to(dev)
with torch.no_grad():
    conv = model.convs[0]
    prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in conv._dense_params())))
    h0 = model._apply_pe(x)
    h1 = ops.layer_dense(ops.spmm3(g, h0), prm, 0, constant=conv.constant.detach(), res_x=h0, act=True)


def fill(self, i, c):
    r0, r1 = self.recv_slices[c]
    self.recv[i][r0:r1] = take(h1, self.mp.recv_ids[r0:r1])


shard.MiddleRunner._exchange = fill
mp = shard.middle_partition(g, rank, P, chunks=chunks)
run = shard.MiddleRunner(model, mp, x)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    run()
e1.record()
torch.cuda.synchronize()
print(f"B(20,{n}) P={P} rank {rank} chunks {chunks}: {e0.elapsed_time(e1) / reps:.4f} ms per forward "
      f"(exchange fill included: {int(mp.recv_ids.numel())} rows per boundary)")
