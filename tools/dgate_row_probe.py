#!/usr/bin/env python3
"""Config-3 training backward at B(20,4): for every layer_dense_backward call, the kernel's per-row gate
gradients at the rows that disagree most with float64 math on the SAME inputs (dY, Z, Y, parameters).
usage: python tools/dgate_row_probe.py [row]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402
import torch.nn.functional as Fn  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops  # noqa: E402
from test_gpu_configs import _labels, _model  # noqa: E402

row = int(sys.argv[1]) if len(sys.argv) > 1 else 52642
dev = torch.device("cuda:0")
n, dims, LAM = 4, [128, 128, 128], 1e-7
N, s, d, c = pkg.synth.de_bruijn_edges(n)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
x = torch.randn(N, 128, generator=torch.Generator().manual_seed(1234))
y = _labels(N, n).to(dev)
orig = ops.layer_dense_backward
calls = []


def rec(dY, Z, Y, prm, gate_mode, **kw):
    out = orig(dY, Z, Y, prm, gate_mode, **kw)
    torch.cuda.synchronize()
    F = Z.size(1) // 3
    P = {k: v.detach().double() for k, v in prm.items()}
    dpre = dY.double() * torch.where(Y.double() > 0, 1.0, 0.01)
    W = [P["W_main_in"] + P["W_shared"], P["W_main_out"] + P["W_shared"], P["W_undirected"] + P["W_shared"]]
    b = [P["b_main_in"] + P["b_dir_shared_in"], P["b_main_out"] + P["b_dir_shared_out"],
         P["b_undirected"] + P["b_undirected_shared"]]
    Zd = Z.double()
    ds = torch.stack([((dpre @ W[q]) * Zd[:, q * F:(q + 1) * F]).sum(1) + dpre @ b[q] for q in range(3)])
    err = (out["dpre"].double() - dpre).abs().max().item()
    # the kernel's ds, recovered from dgate: d0 = dgate_in / (ca cd)
    ci, co, cd, cu, ca = (P[k].reshape(-1) for k in ("C_in", "C_out", "C_directed", "C_undirected", "C_all"))
    dg = out["dgate"].double()
    ds_k = torch.stack([dg[0] / (ca * cd), dg[1] / (ca * cd), dg[3] / ca])
    rel = ((ds_k - ds).abs() / (ds.abs().amax(1, keepdim=True) + 1e-30)).amax(0)
    top = torch.topk(rel, 4)
    calls.append(f"call {len(calls)}: dpre max|d| {err:.2e}; ds rel err top rows {top.indices.tolist()} "
                 f"{[f'{v:.2e}' for v in top.values.tolist()]}; row {row}: kernel ds {ds_k[:, row].tolist()} "
                 f"f64 ds {ds[:, row].tolist()}")
    return out


ops.layer_dense_backward = rec
m = _model(pkg, dims, N, n).to(dev).eval()
xd = x.to(dev).requires_grad_(True)
h = xd
for conv in m.convs:
    h = conv.fused_forward(h, g, None, res_x=h, act=True)
lp, _ = m.head(h)
(Fn.nll_loss(lp, y) + LAM * sum(p.norm(2).pow(2) for p in m.parameters())).backward()
torch.cuda.synchronize()
for ln in calls:
    print(ln, flush=True)
print(f"C_in_vec grad layer0 at {row}: {float(m.convs[0].C_in_vec.grad.flatten()[row]):.6e}")
