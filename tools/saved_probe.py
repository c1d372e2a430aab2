#!/usr/bin/env python3
"""Are the tensors autograd saved for the dense backward still what the forward produced? Config-3 model at B(20,4)
(x requires grad, trainer loss), retain_graph backward, then every LayerDense node's saved Z / Y compared with a
recomputation. Repeated `reps` times in one process.
usage: python tools/saved_probe.py [reps]"""
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

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
dev = torch.device("cuda:0")
n, dims, LAM = 4, [128, 128, 128], 1e-7
N, s, d, c = pkg.synth.de_bruijn_edges(n)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
x = torch.randn(N, 128, generator=torch.Generator().manual_seed(1234))
y = _labels(N, n).to(dev)
for rep in range(reps):
    m = _model(pkg, dims, N, n).to(dev).eval()
    xd = x.to(dev).requires_grad_(True)
    h, hs = xd, [xd]
    for conv in m.convs:
        h = conv.fused_forward(h, g, None, res_x=h, act=True)
        hs.append(h)
    lp, _ = m.head(h)
    loss = Fn.nll_loss(lp, y) + LAM * sum(p.norm(2).pow(2) for p in m.parameters())
    # snapshot the saved tensors right after the forward
    nodes, seen, stack = [], set(), [loss.grad_fn]
    while stack:
        f = stack.pop()
        if f is None or id(f) in seen:
            continue
        seen.add(id(f))
        if type(f).__name__ == "LayerDenseBackward":
            nodes.append(f)
        stack.extend(nf for nf, _ in f.next_functions)
    before = [[t.detach().clone() for t in nd.saved_tensors[:6]] for nd in nodes]
    loss.backward(retain_graph=True)
    torch.cuda.synchronize()
    for k, nd in enumerate(nodes):
        after = nd.saved_tensors[:6]
        for j, name in enumerate(("Z", "res_x", "constant", "W_res", "rows", "Y")):
            if after[j].numel() and not torch.equal(before[k][j], after[j]):
                bad = (before[k][j] != after[j]).reshape(after[j].size(0), -1).any(1).nonzero().flatten()
                print(f"rep {rep} node {k}: saved {name} CHANGED during backward at rows {bad[:8].tolist()}", flush=True)
    # Z vs a recomputation from the layer input
    for k, nd in enumerate(nodes):
        Z = nd.saved_tensors[0]
        ok = any(torch.equal(Z, ops.spmm3(g, hh.detach())) for hh in hs)
        print(f"rep {rep} node {k}: saved Z equals spmm3 of a layer input: {ok}", flush=True)
    gC = m.convs[0].C_in_vec.grad.flatten()
    print(f"rep {rep}: C_in_vec grad at 52642 = {float(gC[52642]):.6e}", flush=True)
    del loss, lp, h, hs, nodes, before
