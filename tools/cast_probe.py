#!/usr/bin/env python3
"""Does a GPU fp32 -> fp64 cast of the model's gradient tensors agree with the host cast? (config-3 model,
B(20,4), after the trainer-loss backward). Prints every tensor whose two casts differ.
usage: python tools/cast_probe.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402
import torch.nn.functional as Fn  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from test_gpu_configs import _labels, _model  # noqa: E402

dev = torch.device("cuda:0")
n, dims, LAM = 4, [128, 128, 128], 1e-7
N, s, d, c = pkg.synth.de_bruijn_edges(n)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
m = _model(pkg, dims, N, n).to(dev).eval()
x = torch.randn(N, 128, generator=torch.Generator().manual_seed(1234))
xd = x.to(dev).requires_grad_(True)
lp, _ = m(pkg.Data(x=xd, graph=g))
(Fn.nll_loss(lp, _labels(N, n).to(dev)) + LAM * sum(p.norm(2).pow(2) for p in m.parameters())).backward()
torch.cuda.synchronize()
for k, p in list(m.named_parameters()) + [("x", xd)]:
    gr = p.grad
    a = gr.detach().double().cpu()
    b = gr.detach().cpu().double()
    info = f"{k}: shape {tuple(gr.shape)} stride {gr.stride()} offset {gr.storage_offset()} contiguous {gr.is_contiguous()}"
    if not torch.equal(a, b):
        bad = (a != b).flatten().nonzero().flatten()
        print(f"DIFFER {info}: {bad.numel()} elements, first {bad[:5].tolist()} gpu-cast {a.flatten()[bad[:3]].tolist()} "
              f"host-cast {b.flatten()[bad[:3]].tolist()}", flush=True)
    else:
        print(f"same   {info}", flush=True)
