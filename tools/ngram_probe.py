#!/usr/bin/env python3
"""n-gram producer at scale: GPU keys + sorts (ngram.ngram_transitions) for levels n = 1..5 on random protein
sequences, then build_propagation_csr; the Python restatement of the reference builder timed on a sample.
usage: python tools/ngram_probe.py [num_seqs] [length]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ngram  # noqa: E402

nseq = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
L = int(sys.argv[2]) if len(sys.argv) > 2 else 500
seqs = pkg.synth.random_sequences(nseq, L, seed=3)
dev = torch.device("cuda:0")
ngram.ngram_transitions(seqs[:10], 2, device=dev)  # warm
for n in range(1, 6):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr = ngram.ngram_transitions(seqs, n, device=dev)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    g = pkg.build_propagation_csr(tr.num_nodes, tr.src.cpu().numpy(), tr.dst.cpu().numpy(), tr.cnt.cpu().numpy(),
                                  device=dev)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"n={n}: {nseq}x{L} residues -> N={tr.num_nodes} E={tr.src.numel()} in {1e3 * (t1 - t0):.1f} ms; "
          f"CSR (nnz/adj {g.nnz}) in {1e3 * (t2 - t1):.1f} ms")
sample = seqs[:2000]
t0 = time.perf_counter()
pkg.synth.fasta_edges(4, ngram.preprocess(sample))
dt = time.perf_counter() - t0
print(f"python restatement n=4 on {len(sample)} sequences: {dt:.2f}s ({1e6 * dt / (len(sample) * L):.2f} us/residue)")
