#!/usr/bin/env python3
"""foreach torch.optim.Adam vs train.Adam on the real model (3-gram, eval mode: no dropout), same start:
max parameter difference per step, plus gradient-aliasing check (two parameters sharing a .grad tensor)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
dev = torch.device("cuda:0")
N, s, d, c = pkg.synth.de_bruijn_edges(3)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
x = torch.randn(N, 64, generator=torch.Generator().manual_seed(1234)).to(dev)
y = (torch.arange(N, device=dev) // 400) % 20
data = pkg.Data(x=x, graph=g)


def make():
    torch.manual_seed(0)
    return pkg.ProtGramDirectGCN([64, 64, 64], N, 20, 3, 0, 512, 0.5, True).to(dev).eval()


m1, m2 = make(), make()
o1 = torch.optim.Adam(m1.parameters(), lr=1e-3)
o2 = pkg.train.Adam(m2.parameters(), lr=1e-3)
for step in range(6):
    for m, o in ((m1, o1), (m2, o2)):
        o.zero_grad()
        lp, _ = m(data)
        loss = F.nll_loss(lp, y) + 1e-7 * sum(p.norm(2).pow(2) for p in m.parameters())
        loss.backward()
        if step == 0 and m is m1:
            ptrs = {}
            for name, p in m.named_parameters():
                ptrs.setdefault(p.grad.data_ptr(), []).append(name)
            shared = [v for v in ptrs.values() if len(v) > 1]
            print("grad tensors shared between parameters:", shared)
        o.step()
    diff = max((a - b).abs().max().item() for a, b in zip(m1.parameters(), m2.parameters()))
    worst = max(((a - b).abs().max().item(), n) for (n, a), b in zip(m1.named_parameters(), m2.parameters()))
    print(f"step {step}: max |p_foreach - p_ours| = {diff:.3e} ({worst[1]})")
