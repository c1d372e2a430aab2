#!/usr/bin/env python3
"""Phase stamps (s_memtime, wave 0 of every block) of the pipelined split-bf16 dense kernel under timing-probe
variants that drop one piece of work each: which phase each piece costs. usage: python tools/x3p_stamps.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops  # noqa: E402

N, F = 160000, 128
dev = torch.device("cuda:0")
torch.manual_seed(0)
layer = pkg.DirectGCNLayer(F, F, N).to(dev)
prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in layer._dense_params())))
const = layer.constant.detach()
Z = torch.randn(N, 3 * F, device=dev)
x = torch.randn(N, F, device=dev)
Y = torch.empty(N, F, device=dev)
names = ["top wait+B1", "Es + DMA issue", "MFMA(i)", "split(i+1)", "CR wait+B2", "epilogue(i-1)"]
variants = {"full": 0, "no A DMA": 2, "no MFMA": 4, "no split": 8, "no G": 16, "no CR": 32, "no epi": 64 | 1,
            "no Y store": 1, "no DMA at all": 2 | 16 | 32}
print(f"{'variant':14s} " + " ".join(f"{n[:12]:>12s}" for n in names) + "       total   (cycles/block, mean)")
for k, dbg in variants.items():
    fl = (1 << 14) | ((128 | dbg) << 20)
    for _ in range(3):
        ops.layer_dense(Z, prm, 0, constant=const, res_x=x, act=True, flags=fl, out=Y, pregated=True)
    torch.cuda.synchronize()
    st = Y[:256, :6].double().mean(0)
    print(f"{k:14s} " + " ".join(f"{v:12.0f}" for v in st.tolist()) + f"  {float(st.sum()):10.0f}")
