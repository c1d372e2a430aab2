#!/usr/bin/env python3
"""Runs each transposed propagation kernel at B(20,4), F = 128 (fp32) `reps` times, untimed: the program the
rocprofv3 --pmc passes behind profiles/r04_transposed_traffic.json trace (per-kernel FETCH_SIZE / WRITE_SIZE averages,
tools/pmc_traffic.py) and its --kernel-trace --stats run. Kernels: the 4x4-block kernel (pg_spmm3t_ngram_f32, the
default), the off-diagonal middle-tile kernel (pg_spmm3t_ngram_mid_offdiag_f32) writing dX and accumulating into it.
usage: python tools/tprobe.py [reps=10] [F=128]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
F = int(sys.argv[2]) if len(sys.argv) > 2 else 128
dev = torch.device("cuda:0")
N, s, d, c = pkg.synth.de_bruijn_edges(4)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
G = torch.randn(N, 3 * F, device=dev)
acc = torch.zeros(N, F, device=dev)
for _ in range(reps):
    ops.spmm3_t(g, G)
    ops.spmm3t_offdiag(g, G)
    ops.spmm3t_offdiag(g, G, out=acc)
torch.cuda.synchronize()
print("ok", reps, F)
