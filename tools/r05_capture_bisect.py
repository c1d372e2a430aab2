#!/usr/bin/env python3
"""Which part of train.train_step breaks when replayed from a HIP graph: captures stage 1 (forward + loss),
2 (+ backward), 3 (+ train.Adam, the whole step via GraphedTrainStep) or 4 (stage 3 with torch.optim.SGD) on the
graphed test's model (3-gram, dims [64, 64, 64], eval mode) and replays it, synchronising after every replay.
  tools/r05_capture_bisect.py <stage>"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import train  # noqa: E402

stage = int(sys.argv[1])
dims = [64, 64, 64]
for a in sys.argv[2:]:
    if a.startswith("--dims="):
        dims = [int(v) for v in a.split("=", 1)[1].split(",")]
dev = torch.device("cuda", 0)
N, s, d, c = pkg.synth.de_bruijn_edges(3)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
x = torch.randn(N, dims[0], generator=torch.Generator().manual_seed(1234)).to(dev)
y = (torch.arange(N, device=dev) // 400) % 20
data = pkg.Data(x=x, graph=g)
torch.manual_seed(0)
m = pkg.ProtGramDirectGCN(dims, N, 20, 3, 0, 512, 0.5, True).to(dev).eval()
opt = torch.optim.SGD(m.parameters(), lr=1e-3) if stage == 4 else train.Adam(m.parameters(), lr=1e-3)


def body():
    if stage >= 3:
        return train.train_step(m, data, y, opt, l2_lambda=1e-3)
    opt.zero_grad(set_to_none=True)
    lp, _ = m(data=data)
    loss = train.nll_mean(lp, y)
    if stage == 2:
        loss.backward()
    return loss


for _ in range(3):
    body()
torch.cuda.synchronize()
print(f"stage {stage}: eager ok", flush=True)
train.prepare_capture(dev)
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr, capture_error_mode="thread_local"):
    out = body()
keep = list(getattr(opt, "_tl_cache", {}).values()) + train.flush_deferred()
print(f"stage {stage}: captured, {len(keep)} kept objects", flush=True)
train.check_deferred(keep)
print(f"stage {stage}: descriptor tables checked", flush=True)
if "--no-replay" in sys.argv:
    sys.exit(0)
for i in range(3):
    gr.replay()
    torch.cuda.synchronize()
    print(f"stage {stage}: replay {i} ok, loss {float(out):.6f}", flush=True)
