#!/usr/bin/env python3
"""Run the default hot-path kernels on the 4-gram workload a few times (target for rocprofv3 --pmc passes).
usage: python tools/kprobe.py [reps]"""
import dataclasses
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda:0")
N, s, d, c = pkg.synth.de_bruijn_edges(4)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
kin, kout = pkg.graph.class_keys(N, torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev))
gt = dataclasses.replace(g, tiles=pkg.graph.build_row_tiles(g, kin, kout, 128))
x = torch.randn(N, 128, device=dev)
torch.manual_seed(0)
layer = pkg.DirectGCNLayer(128, 128, N).to(dev)
prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in layer._dense_params())))
W1, b1 = torch.randn(64, 128, device=dev) * 0.1, torch.zeros(64, device=dev)
W2, b2 = torch.randn(20, 64, device=dev) * 0.1, torch.zeros(20, device=dev)
dY = torch.randn(N, 128, device=dev)
for _ in range(reps):
    Zg = ops.spmm3_gated(g, x, prm, 0)  # spmm_win_kernel<32,1,4,0,256,true>: the inference (bench) propagation
    ops.layer_dense(Zg, prm, 0, constant=layer.constant.detach(), res_x=x, act=True, pregated=True)  # dense_ws
    Z = ops.spmm3(g, x)                 # spmm_win_kernel<32,1,4,0>: the training propagation
    ops.spmm3(gt, x)                    # spmm3_tiled_full_kernel (opt-in row tiles)
    ops.spmm3_t(g, Z)                   # spmm_win_kernel<..,2>: transposed propagation (backward)
    Y = ops.layer_dense(Z, prm, 0, constant=layer.constant.detach(), res_x=x, act=True)
    ops.layer_dense_backward(dY, Z, Y, prm, 0, res_x=x, act=True)  # dgrad / wgrad / reduce
    ops.head(Y, W1, b1, W2, b2, 1e-12)
torch.cuda.synchronize()
print("ok")
