#!/usr/bin/env python3
"""Time the propagation kernels at B(20,n), F: n-gram tile forward (default / LDS-weight variant), the CSR window
kernel, and the transposed kernels (min of interleaved rounds, HIP events), plus a max-|d| check vs the CSR result.
Transposed: the 4x4-block kernel (default), the off-diagonal middle-tile kernel (alone, accumulating, and with the
diagonal term on the host under PG_FLAG_MID_TRANSPOSED) and the CSR kernel.
usage: python tools/ngram_probe_k.py [n=4] [F=128] [reps=20]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops  # noqa: E402
from protgram_directgcn_amd._lib import (PG_FLAG_MID_LOADER_SYNC, PG_FLAG_MID_TRANSPOSED,  # noqa: E402
                                         PG_FLAG_NGRAM_BLOCK4, PG_FLAG_NO_NGRAM)

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
F = int(sys.argv[2]) if len(sys.argv) > 2 else 128
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
dev = torch.device("cuda:0")
N, s, d, c = pkg.synth.de_bruijn_edges(n)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
assert g.ngram is not None
x = torch.randn(N, F, device=dev)
G = torch.randn(N, 3 * F, device=dev)
dXa = torch.zeros(N, F, device=dev)
Gb = G.to(torch.bfloat16)


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


prm = {k: torch.rand(N, 1, device=dev) + 0.5 for k in ("C_in", "C_out", "C_directed", "C_undirected", "C_all")}
prm["W_main_in"] = torch.zeros(F, F, device=dev)
ALT = [int(a, 0) for a in os.environ.get("PG_PROBE_ALT", "").split(",") if a]
cases = {"fwd_ngram": lambda: ops.spmm3(g, x), "gated_ngram": lambda: ops.spmm3_gated(g, x, prm, 0),
         "fwd_block4": lambda: ops.spmm3(g, x, flags=PG_FLAG_NGRAM_BLOCK4),
         "gated_block4": lambda: ops.spmm3_gated(g, x, prm, 0, flags=PG_FLAG_NGRAM_BLOCK4),
         "fwd_csr": lambda: ops.spmm3(g, x, flags=PG_FLAG_NO_NGRAM),
         "fwd_sync": lambda: ops.spmm3(g, x, flags=ops.default_flags() | PG_FLAG_MID_LOADER_SYNC),
         "bwd_ngram": lambda: ops.spmm3_t(g, G),
         "bwd_mid": lambda: ops.spmm3_t(g, G, flags=ops.default_flags() | PG_FLAG_MID_TRANSPOSED),
         "bwd_offdiag": lambda: ops.spmm3t_offdiag(g, G),
         "bwd_offdiag_acc": lambda: ops.spmm3t_offdiag(g, G, out=dXa),
         "bwd_csr": lambda: ops.spmm3_t(g, G, flags=PG_FLAG_NO_NGRAM),
         "bwd_bf16_mid": lambda: ops.spmm3_t(g, Gb, flags=ops.default_flags() | PG_FLAG_MID_TRANSPOSED),
         "bwd_bf16_block4": lambda: ops.spmm3_t(g, Gb)}
for a in ALT:
    cases[f"fwd_alt{a:#x}"] = (lambda a: lambda: ops.spmm3(g, x, flags=a))(a)
    cases[f"gated_alt{a:#x}"] = (lambda a: lambda: ops.spmm3_gated(g, x, prm, 0, flags=a))(a)
cases = {k: fn for k, fn in cases.items() if fn() is not None}
best = {k: 1e9 for k in cases}
for _ in range(4):
    for k, fn in cases.items():
        best[k] = min(best[k], timeit(fn))
ref = ops.spmm3(g, x, flags=PG_FLAG_NO_NGRAM)
for k in [c for c in ["fwd_ngram", "fwd_block4"] + [f"fwd_alt{a:#x}" for a in ALT] if c in cases]:
    z = cases[k]()
    print(f"{k}: max |d| vs csr {float((z - ref).abs().max()):.3e}")
refb = ops.spmm3_t(g, G, flags=PG_FLAG_NO_NGRAM)
for k in ("bwd_ngram", "bwd_mid"):
    print(f"{k}: max |d| vs csr {float((cases[k]() - refb).abs().max()):.3e} (max |ref| {float(refb.abs().max()):.3e})")
refg = ops.spmm3_gated(g, x, prm, 0, flags=PG_FLAG_NO_NGRAM)
for k in [c for c in ("gated_ngram", "gated_block4") if c in cases]:
    z = cases[k]()
    if z is None:
        print(f"{k}: no gated kernel for this graph (the dense kernel gates)")
        continue
    print(f"{k}: max |d| vs csr {float((z - refg).abs().max()):.3e} (max |ref| {float(refg.abs().max()):.3e})")
comp = g.compulsory_bytes(F)
print(" ".join(f"{k}={v:.4f}ms" for k, v in best.items()), f"compulsory_fwd={comp / 1e6:.1f}MB "
      f"-> {comp / best['fwd_ngram'] / 1e6:.0f} GB/s")
if "bwd_bf16_mid" in best:  # bf16 full product: G read three times (out, in, own rows), dX written, the plan once
    bb = 3 * N * 3 * F * 2 + N * F * 2 + g.ngram.mplan.numel() * 4
    print(f"bf16 mid bytes {bb / 1e6:.1f}MB -> {bb / best['bwd_bf16_mid'] / 1e6:.0f} GB/s")
if "bwd_offdiag" in best:  # its algorithmic bytes: G read twice (out- and in-sources), dX written, the plan once
    ob = 2 * N * 3 * F * 4 + N * F * 4 + g.ngram.mplan.numel() * 4
    print(f"offdiag bytes {ob / 1e6:.1f}MB -> {ob / best['bwd_offdiag'] / 1e6:.0f} GB/s; "
          f"with accumulate +{N * F * 4 / 1e6:.1f}MB")
