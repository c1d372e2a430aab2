#!/usr/bin/env python3
"""A/B timing of the mapped middle-tile kernel (pg_spmm3_ngram_mid_map_f32) against the plain one.

  1. B(20,4), F = 128: the plain kernel (g.ngram) and the mapped kernel with the IDENTITY row map (every n-gram a
     node at its own grid row; no residual) on the same graph and input: the cost of the row map alone;
  2. the builder-produced 4-gram level of bench.py --graph fasta: the mapped kernel alone, the residual pass alone,
     and the whole propagation (ops.spmm3).
HIP events around each launch, median of --reps after warm-up. Prints one JSON line.
"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import graph as gr, ops  # noqa: E402


def timed(fn, reps):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return round(ts[len(ts) // 2] * 1e3, 2)  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--fasta-seqs", type=int, default=8000)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    lib = ops.load_library()
    fl = ops.default_flags()
    out = {}
    N, s, d, c = pkg.synth.de_bruijn_edges(4)
    g = pkg.build_propagation_csr(N, s, d, c, device=dev)
    x = torch.randn(N, 128, generator=torch.Generator().manual_seed(1234)).to(dev)
    Z = torch.empty(N, 384, device=dev)
    ng = g.ngram
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    out["plain_us"] = timed(lambda: lib.pg_spmm3_ngram_mid_f32(ng.K, ng.n, N, ops._p(ng.mplan), ops._p(x), 128, 128,
                                                                None, ops._p(Z), 384, fl, st), args.reps)
    keys = torch.arange(N, dtype=torch.int64, device=dev)
    m = gr.build_ngram_map(g, keys, gr.GRID_LETTERS, 4)
    Zm = torch.empty(N, 384, device=dev)
    out["identity_map_us"] = timed(lambda: lib.pg_spmm3_ngram_mid_map_f32(m.K, m.n, ops._p(m.mplan), ops._p(m.gmap),
                                                                          ops._p(x), 128, 128, ops._p(Zm), 384, fl, st),
                                   args.reps)
    torch.cuda.synchronize()
    out["identity_map_max_abs_diff"] = float((Zm - Z).abs().max())
    # the fasta level
    seqs = pkg.synth.protein_sequences(args.fasta_seqs, 350, seed=1)
    tr = pkg.ngram.ngram_transitions(seqs, 4, device=dev)
    gf = pkg.build_propagation_csr(tr.num_nodes, tr.src.cpu().numpy(), tr.dst.cpu().numpy(), tr.cnt.cpu().numpy(),
                                   device=dev, transitions=tr)
    mf = gf.ngram_map
    Nf = tr.num_nodes
    xf = torch.randn(Nf, 128, generator=torch.Generator().manual_seed(1234)).to(dev)
    Zf = torch.empty(Nf, 384, device=dev)
    out["fasta"] = {"nodes": Nf, "grid_nodes": mf.n_grid, "off_grid_rows": mf.n_off, "grid_rows_with_residual":
                    mf.n_acc, "residual_entries": mf.nnz_res}
    out["fasta"]["mapped_us"] = timed(lambda: lib.pg_spmm3_ngram_mid_map_f32(
        mf.K, mf.n, ops._p(mf.mplan), ops._p(mf.gmap), ops._p(xf), 128, 128, ops._p(Zf), 384, fl, st), args.reps)
    out["fasta"]["residual_us"] = timed(lambda: lib.pg_spmm3_resid_f32(
        mf.res_rows.numel(), ops._p(mf.res_rowptr), ops._p(mf.res_rows), ops._p(mf.res_edges), ops._p(xf), 128, 128,
        ops._p(Zf), 384, fl, st), args.reps)
    out["fasta"]["propagation_us"] = timed(lambda: ops.spmm3(gf, xf, out=Zf), args.reps)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
