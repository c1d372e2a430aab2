#!/usr/bin/env python3
"""Diagnose per-row gate gradients of pg_directgcn_dense_bwd_f32 at B(20,4), F=128: dgate from the kernel vs
float64 math on the same inputs (Z, dY, Y, parameters), repeated runs for determinism; prints the worst rows.
usage: python tools/dgate_probe.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops  # noqa: E402
from test_gpu_configs import _model  # noqa: E402

dev = torch.device("cuda:0")
n = 4
N, s, d, c = pkg.synth.de_bruijn_edges(n)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
m = _model(pkg, [128, 128, 128], N, n).to(dev).eval()
x = torch.randn(N, 128, generator=torch.Generator().manual_seed(1234)).to(dev)
conv = m.convs[0]
prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in conv._dense_params())))
Z = ops.spmm3(g, x)
Y = ops.layer_dense(Z, prm, 0, constant=conv.constant.detach(), res_x=x, act=True)
dY = torch.randn(N, 128, generator=torch.Generator().manual_seed(9)).to(dev) * 1e-5
outs = [ops.layer_dense_backward(dY, Z, Y, prm, 0, res_x=x, act=True) for _ in range(3)]
for k in ("dgate", "dZ", "dpre", "dB"):
    same = all(torch.equal(outs[0][k], o[k]) for o in outs[1:])
    print(f"{k}: deterministic over 3 runs: {same}")
# float64 reference of dgate
Zd, dYd, Yd = Z.double(), dY.double(), Y.double()
dpre = dYd * torch.where(Yd > 0, 1.0, 0.01)
P = {k: v.double() for k, v in prm.items()}
W = [P["W_main_in"] + P["W_shared"], P["W_main_out"] + P["W_shared"], P["W_undirected"] + P["W_shared"]]
b = [P["b_main_in"] + P["b_dir_shared_in"], P["b_main_out"] + P["b_dir_shared_out"],
     P["b_undirected"] + P["b_undirected_shared"]]
ds = torch.stack([((dpre @ W[q]) * Zd[:, q * 128:(q + 1) * 128]).sum(1) + dpre @ b[q] for q in range(3)])
ci, co, cd, cu, ca = (P[k].reshape(-1) for k in ("C_in", "C_out", "C_directed", "C_undirected", "C_all"))
ref = torch.stack([ds[0] * ca * cd, ds[1] * ca * cd, ca * (ds[0] * ci + ds[1] * co), ds[2] * ca,
                   cd * (ds[0] * ci + ds[1] * co) + ds[2] * cu])
got = outs[0]["dgate"].double()
err = (got - ref).abs()
scale = ref.abs().amax(1, keepdim=True)
rel = err / scale
worst = rel.amax(0)
top = torch.topk(worst, 8)
print("dgate max rel err (per gate):", rel.amax(1).tolist())
for v, r in zip(top.values.tolist(), top.indices.tolist()):
    print(f"row {r}: rel {v:.3e} got {got[:, r].tolist()} ref {ref[:, r].tolist()}")
dpre_err = (outs[0]["dpre"].double() - dpre).abs().max().item()
print("dpre max abs err", dpre_err)
gerr = ((outs[0]["dZ"].double() - torch.cat([((dpre @ W[q]) * torch.stack([ca * cd * ci, ca * cd * co, ca * cu])[q]
                                              .unsqueeze(1)) for q in range(3)], 1)).abs().max().item())
print("dZ max abs err", gerr)
