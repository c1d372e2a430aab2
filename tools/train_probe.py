#!/usr/bin/env python3
"""Config 3 / 5 training step (4-gram, dims [128,128,128] or --dims=128,256,256,256, C=20): reference loop of
protgram_directgcn_trainer.py:91-100 (nll + 1e-7 * sum ||p||^2, Adam lr 1e-3). Prints ms/step."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
amp = "--amp" in sys.argv
bf16 = "--bf16" in sys.argv
fused = "--fused" in sys.argv          # train.train_step instead of the reference loop body
adam_fused = "--adam-fused" in sys.argv
our_adam = "--our-adam" in sys.argv     # train.Adam (one HIP launch per step)
graphed = "--graph" in sys.argv         # train.GraphedTrainStep (implies --fused)
NO_OPTS = [a for a in sys.argv[2:] if a.startswith("--no")]
if "--no-span" in sys.argv:             # the 4x4-block transposed kernel instead of ops.PropagateDense
    from protgram_directgcn_amd import ops as _ops
    _ops.SPAN_BACKWARD = False
if "--no-fdrop" in sys.argv:            # F.dropout after each layer instead of the dropout fused into the dense epilogue
    from protgram_directgcn_amd import ops as _ops
    _ops.FUSED_DROPOUT = False
if "--no-head" in sys.argv:             # the framework ops for the prediction head instead of ops.head_train
    pkg.train.HEAD_FUSED = False
dims = [128, 128, 128]
for a in sys.argv:
    if a.startswith("--dims="):
        dims = [int(v) for v in a.split("=", 1)[1].split(",")]
dev = torch.device("cuda:0")
n = 4
N, s, d, c = pkg.synth.de_bruijn_edges(n)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
torch.manual_seed(0)
model = pkg.ProtGramDirectGCN(dims, N, 20, n, 0, 512, 0.5, True).to(dev)
x = torch.randn(N, dims[0], generator=torch.Generator().manual_seed(1234)).to(dev)
y = torch.arange(N, device=dev) // (20 ** (n - 1))
if bf16:
    model.compute_dtype = torch.bfloat16
data = pkg.Data(x=x, graph=g)
if our_adam:
    opt = pkg.train.Adam(model.parameters(), lr=1e-3, weight_decay=0.0)
else:
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=0.0, fused=True if adam_fused else None)
model.train()


scaler = torch.amp.GradScaler("cuda", enabled=amp)
gstep = pkg.train.GraphedTrainStep(model, data, y, opt, l2_lambda=1e-7, scaler=scaler) if graphed else None


def step():
    if gstep is not None:
        return gstep()
    if fused:
        return pkg.train.train_step(model, data, y, opt, l2_lambda=1e-7, scaler=scaler)
    opt.zero_grad()
    with torch.amp.autocast("cuda", enabled=amp):
        out, _ = model(data=data)
        loss = F.nll_loss(out, y) + 1e-7 * sum(p.norm(2).pow(2) for p in model.parameters() if p.requires_grad)
    scaler.scale(loss).backward()
    scaler.step(opt)
    scaler.update()
    return loss


for _ in range(5 if graphed else 3):
    step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    loss = step()
torch.cuda.synchronize()
print(f"train step dims={dims} (amp={amp}, bf16={bf16}, fused={fused}, adam_fused={adam_fused}, our_adam={our_adam}, graph={graphed}, opts={NO_OPTS}) {1e3 * (time.perf_counter() - t0) / steps:.3f} ms  loss {loss.item():.4f}")
