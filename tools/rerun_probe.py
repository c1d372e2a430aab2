#!/usr/bin/env python3
"""Run the config-3 GPU backward (tests/test_gpu_configs.py::test_config3...) several times in one process and
compare every layer_dense_backward call's inputs and outputs between runs, bit for bit (nondeterminism hunt).
usage: python tools/rerun_probe.py [runs]"""
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

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
dev = torch.device("cuda:0")
n, dims, LAM = 4, [128, 128, 128], 1e-7
N, s, d, c = pkg.synth.de_bruijn_edges(n)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
m = _model(pkg, dims, N, n).to(dev).eval()
x = torch.randn(N, 128, generator=torch.Generator().manual_seed(1234))
y = _labels(N, n).to(dev)

calls = []
orig = ops.layer_dense_backward


def rec(dY, Z, Y, prm, *a, **k):
    out = orig(dY, Z, Y, prm, *a, **k)
    torch.cuda.synchronize()
    calls.append({"dY": dY.detach().clone(), "Z": Z.detach().clone(), "Y": Y.detach().clone(),
                  **{kk: v.detach().clone() for kk, v in out.items() if v is not None}})
    return out


ops.layer_dense_backward = rec
results = []
for r in range(runs):
    calls.clear()
    m.zero_grad(set_to_none=True)
    xd = x.to(dev).requires_grad_(True)
    h = xd
    for conv in m.convs:
        h = conv.fused_forward(h, g, None, res_x=h, act=True)
    lp, _ = m.head(h)
    (Fn.nll_loss(lp, y) + LAM * sum(p.norm(2).pow(2) for p in m.parameters())).backward()
    torch.cuda.synchronize()
    grads = {k: p.grad.detach().clone() for k, p in m.named_parameters()}
    grads["x"] = xd.grad.detach().clone()
    results.append((list(calls), grads))
    with torch.no_grad():
        m(pkg.Data(x=xd, graph=g))
base_calls, base_grads = results[0]
for r in range(1, runs):
    cs, gs = results[r]
    for i, (a, b) in enumerate(zip(base_calls, cs)):
        for k in a:
            if not torch.equal(a[k], b[k]):
                diff = (a[k].double() - b[k].double()).abs()
                idx = diff.flatten().nonzero().flatten()
                print(f"run {r} call {i} {k}: {idx.numel()} elements differ, first flat {idx[:6].tolist()} "
                      f"max |d| {float(diff.max()):.3e} (shape {tuple(a[k].shape)})")
    for k in base_grads:
        if not torch.equal(base_grads[k], gs[k]):
            diff = (base_grads[k].double() - gs[k].double()).abs()
            idx = diff.flatten().nonzero().flatten()
            print(f"run {r} grad {k}: {idx.numel()} differ, first {idx[:6].tolist()} max {float(diff.max()):.3e}")
print("done", runs, "runs")
