#!/usr/bin/env python3
"""PG_FLAG_SPMM_CU_CHUNKS (persistent, CU-chunked schedule) against the default window SpMM: bit-exactness and
interleaved timing (HIP events, min of rounds), plain and gated. usage: python tools/cu_chunk_probe.py [ngram]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops  # noqa: E402
from protgram_directgcn_amd._lib import PG_FLAG_SPMM_CU_CHUNKS as CU, PG_FLAG_SPMM_SC1 as SC1  # noqa: E402
from protgram_directgcn_amd._lib import PG_FLAG_SPMM_OCC6 as OCC6, PG_FLAG_SPMM_OCC8 as OCC8  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
F = 128
dev = torch.device("cuda:0")
N, s, d, c = pkg.synth.de_bruijn_edges(n)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
x = torch.randn(N, F, generator=torch.Generator().manual_seed(1234)).to(dev)
torch.manual_seed(0)
layer = pkg.DirectGCNLayer(F, F, N).to(dev)
with torch.no_grad():
    for name, q in layer.named_parameters():
        if name.startswith("C_"):
            q.uniform_(0.5, 1.5)
prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in layer._dense_params())))
v = {"plain": lambda: ops.spmm3(g, x, flags=0), "plain_cu": lambda: ops.spmm3(g, x, flags=CU),
     "gated": lambda: ops.spmm3_gated(g, x, prm, 0, flags=0), "gated_cu": lambda: ops.spmm3_gated(g, x, prm, 0, flags=CU),
     "plain_sc1": lambda: ops.spmm3(g, x, flags=SC1), "gated_sc1": lambda: ops.spmm3_gated(g, x, prm, 0, flags=SC1),
     "gated_occ6": lambda: ops.spmm3_gated(g, x, prm, 0, flags=OCC6),
     "gated_occ8": lambda: ops.spmm3_gated(g, x, prm, 0, flags=OCC8)}
print("plain bit-exact:", torch.equal(v["plain"](), v["plain_cu"]()), " gated bit-exact:",
      torch.equal(v["gated"](), v["gated_cu"]()), " sc1 bit-exact:", torch.equal(v["plain"](), v["plain_sc1"]()),
      torch.equal(v["gated"](), v["gated_sc1"]()), " occ bit-exact:", torch.equal(v["gated"](), v["gated_occ6"]()),
      torch.equal(v["gated"](), v["gated_occ8"]()))


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


res = {k: [] for k in v}
for _ in range(5):
    for k, fn in v.items():
        res[k].append(timeit(fn))
for k, t in res.items():
    print(f"{k:9s} " + " ".join(f"{a:.4f}" for a in t) + f"   min {min(t):.4f} ms")
