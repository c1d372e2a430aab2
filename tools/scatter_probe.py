#!/usr/bin/env python3
"""Timing of the middle partition's backward propagation at config 5's rank shapes (4-gram, P = 8, rank 0, F = 256,
bf16 dZ): the scatter kernel (pg_spmm3t_ngram_scatter_bf16) per chunks-per-workgroup setting (0: the library's choice), the two gather-sums
that follow it, and the transposed CSR kernel over the rank's column block it replaces. HIP events, median of reps.
  python tools/scatter_probe.py [--F 256] [--world 8] [--rank 0] [--fp32]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops, shard  # noqa: E402
from protgram_directgcn_amd._lib import PG_FLAG_SCATTER_CPW_SHIFT  # noqa: E402


def timed(fn, reps=None):
    reps = reps or a.reps
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return round(ts[len(ts) // 2] * 1000, 2)  # us


ap = argparse.ArgumentParser()
ap.add_argument("--F", type=int, default=256)
ap.add_argument("--world", type=int, default=8)
ap.add_argument("--rank", type=int, default=0)
ap.add_argument("--n", type=int, default=4)
ap.add_argument("--fp32", action="store_true")
ap.add_argument("--cpw", type=int, nargs="*", default=[0, 2, 4, 8, 16])
ap.add_argument("--reps", type=int, default=30)
ap.add_argument("--no-csr", action="store_true")
a = ap.parse_args()
dev = torch.device("cuda", 0)
N, s, d, c = pkg.synth.de_bruijn_edges(a.n)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
mp_ = shard.middle_partition(g, a.rank, a.world)
sc = shard.middle_scatter(mp_)
mt = shard.middle_transpose(mp_)
G = torch.randn(mp_.n_own, 3 * a.F, generator=torch.Generator().manual_seed(1)).to(dev)
if not a.fp32:
    G = G.to(torch.bfloat16)
out = {"n": a.n, "world": a.world, "rank": a.rank, "F": a.F, "dtype": "f32" if a.fp32 else "bf16",
       "n_mid": mp_.m1 - mp_.m0, "n_own": mp_.n_own, "ghost_rows": int(mp_.recv_ids.numel())}
base = ops.default_flags()
ref = ops.spmm3t_scatter(sc.splan, G)
for cpw in a.cpw:
    fl = base | (cpw << PG_FLAG_SCATTER_CPW_SHIFT)
    assert torch.equal(ops.spmm3t_scatter(sc.splan, G, flags=fl), ref)
    out[f"scatter_us_cpw{cpw or 'auto'}"] = timed(lambda: ops.spmm3t_scatter(sc.splan, G, flags=fl))
T = ref
hd = G.dtype
out["gather_sum_send_us"] = timed(lambda: ops.rows_gather_sum(T, sc.send_ptr, sc.send_idx, int(mp_.recv_ids.numel()),
                                                              a.F, out_dtype=hd))
recv = torch.zeros(int(mp_.send_pos.numel()), a.F, device=dev, dtype=hd)
out["gather_sum_own_us"] = timed(lambda: ops.rows_gather_sum(T, sc.own_ptr, sc.own_idx, mp_.n_own, a.F, B=recv,
                                                             out_dtype=hd))
if not a.no_csr:
    out["csr_spmm3t_rows_us"] = timed(lambda: ops.spmm3t_rows(mt.rowptr, mt.edges3, mt.rows, G, mp_.n))
# algorithmic bytes of the scatter kernel: G read once per direction, T written once, the plan read once per group
es = G.element_size()
out["scatter_bytes_G_T"] = 2 * mp_.n_own * 3 * a.F * es + 3 * mp_.n_own * a.F * 4
print(json.dumps(out))
