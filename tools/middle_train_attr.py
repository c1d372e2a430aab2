#!/usr/bin/env python3
"""Attribute the GPU time of one config-5 MiddleTrainer rank step (bf16, rank 0 of P = 8, no-op collectives, eager)
to the host call sites that launched it: torch.profiler with stacks; per (kernel, aten op, first package frame),
device µs per step. Used to find framework glue (copies, fills, casts) worth removing from the step.
  python tools/middle_train_attr.py [--steps 5] [--rank 0]"""
import argparse
import collections
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tools")]
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import shard  # noqa: E402
from test_gpu_configs import _labels, _model  # noqa: E402
from middle_train_probe import SoloComm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--rank", type=int, default=0)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    n, dims, lam = 4, [128, 256, 256, 256], 1e-7
    N, s, d, c = pkg.synth.de_bruijn_edges(n)
    g = pkg.build_propagation_csr(N, s, d, c, device=dev)
    x = torch.randn(N, dims[0], generator=torch.Generator().manual_seed(1234)).to(dev)
    y = _labels(N, n).to(dev)
    mp_ = shard.middle_partition(g, args.rank, 8)
    m = _model(pkg, dims, N, n).to(dev).eval()
    m.compute_dtype = torch.bfloat16
    tr = shard.MiddleTrainer(m, mp_, l2_lambda=lam, comm=SoloComm())
    yo = y[mp_.own]
    for _ in range(3):
        tr.step(x, yo)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for _ in range(args.steps):
            tr.step(x, yo)
        torch.cuda.synchronize()
    agg = collections.defaultdict(lambda: [0.0, 0])
    for e in prof.events():
        if not e.kernels:
            continue
        chain, par = [], e.cpu_parent
        while par is not None and len(chain) < 5:
            chain.append(par.name[:28])
            par = par.cpu_parent
        frame = " < ".join(chain) or "-"
        for k in e.kernels:
            key = (k.name[:60], e.name[:40], frame[:150])
            agg[key][0] += k.duration / args.steps
            agg[key][1] += 1
    tot = sum(v[0] for v in agg.values())
    print(f"device time attributed per step: {tot:.1f} us")
    for (kn, op, fr), (us, cnt) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:60]:
        print(f"{us:8.1f} us {cnt / args.steps:5.1f}x  {kn:60s} | {op:40s} | {fr}")


if __name__ == "__main__":
    main()
