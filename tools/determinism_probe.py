#!/usr/bin/env python3
"""Bitwise reproducibility of a training step: ShardedTrainer (world 1, no collectives) on B(20,3), dims
[128,128,128], fp32 and bf16, repeated from the same start; reports which gradients / parameters differ between
repetitions (tests/test_gpu_rccl.py compares two such runs through different collective paths).
  python tools/determinism_probe.py [reps=6]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import shard  # noqa: E402
from test_gpu_rccl import _model  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
dev = torch.device("cuda", 0)
N, s, d, c = pkg.synth.de_bruijn_edges(3)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
x = torch.randn(N, 128, generator=torch.Generator().manual_seed(1234)).to(dev)
y = (torch.arange(N, device=dev) // 400) % 20
part = shard.partition(g, 0, 1, transpose=True)
out = {}
for dt in (torch.float32, torch.bfloat16):
    runs = []
    for r in range(reps):
        m = _model(pkg, N, [128, 128, 128], dev, 3)
        m.compute_dtype = dt
        tr = shard.ShardedTrainer(m, part, lr=1e-3, l2_lambda=1e-3)
        rec = {}
        loss1 = tr.step(x, y).clone()
        for name, p in list(m.named_parameters()):
            gg = p.grad
            if gg is None and shard._is_node_param(name, p, N):
                leaf = tr.own[int(name.split(".")[1])].get(name.split(".")[-1])
                gg = leaf.grad if leaf is not None else None
            if gg is not None:
                rec["grad1 " + name] = gg.detach().clone()
        loss2 = tr.step(x, y).clone()
        tr.gather()
        rec["loss"] = torch.stack([loss1, loss2])
        for k, v in m.state_dict().items():
            rec["param " + k] = v.detach().clone()
        runs.append(rec)
    torch.cuda.synchronize()
    diffs = {}
    for r in range(1, reps):
        for k, v in runs[0].items():
            w = runs[r][k]
            if not torch.equal(v, w):
                diffs.setdefault(k, []).append((r, float((v.float() - w.float()).abs().max()),
                                                int((v != w).sum())))
    out[str(dt)] = {"reps": reps, "differing": {k: v for k, v in list(diffs.items())[:20]},
                    "n_differing": len(diffs)}
print(json.dumps(out))
