#!/usr/bin/env python3
"""Targets for rocprofv3 --pmc passes (one counter group per run).

  python tools/kprobe.py [reps]                 every hot-path kernel on the 4-gram workload (forward,
                                                training forward, backward, head), `reps` times
  python tools/kprobe.py --forward [reps] ...   exactly bench.py's step (the eval forward of its model on its
                                                workload), `reps` times: bench.py's live roofline.traffic
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("reps", nargs="?", type=int, default=5)
ap.add_argument("--forward", action="store_true")
ap.add_argument("--ngram", type=int, default=4)
ap.add_argument("--feat", type=int, default=128)
ap.add_argument("--layers", type=int, default=2)
ap.add_argument("--bf16", action="store_true")
ap.add_argument("--fused-norm", action="store_true")
ap.add_argument("--entry", choices=("coo", "graph"), default="coo")
ap.add_argument("--graph", choices=("debruijn", "fasta"), default="debruijn")
ap.add_argument("--fasta-seqs", type=int, default=8000)
args = ap.parse_args()
reps = args.reps
dev = torch.device("cuda:0")
import bench  # noqa: E402
wl = bench.build_workload(pkg, args, dev, keep_raw=args.fused_norm or not args.forward)
N, g, tr = wl["N"], wl["graph"], wl["transitions"]

if args.forward:
    model = bench.bench_model(pkg, N, args.feat, args.layers, args.ngram).to(dev).eval()
    model.fused_norm = args.fused_norm
    x = torch.randn(N, args.feat, generator=torch.Generator().manual_seed(1234)).to(dev)
    if args.bf16:
        model.compute_dtype = torch.bfloat16
        x = x.to(torch.bfloat16)
    if args.entry == "coo" and not args.fused_norm:  # bench.py's default: the trainer's COO wiring
        data = pkg.synth.trainer_data(g, x)
        del g
        if tr is not None:  # as bench.py: the level's node map attached to the graph the COO wiring yields
            with torch.no_grad():
                pkg.attach_ngram_map(model.graph_of(data), tr)
    else:
        data = pkg.Data(x=x, graph=g)
    with torch.no_grad():
        for _ in range(reps):
            model(data)
    torch.cuda.synchronize()
    print("ok")
    sys.exit(0)

x = torch.randn(N, 128, device=dev)
torch.manual_seed(0)
layer = pkg.DirectGCNLayer(128, 128, N).to(dev)
prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in layer._dense_params())))
W1, b1 = torch.randn(64, 128, device=dev) * 0.1, torch.zeros(64, device=dev)
W2, b2 = torch.randn(20, 64, device=dev) * 0.1, torch.zeros(20, device=dev)
dY = torch.randn(N, 128, device=dev)
for _ in range(reps):
    Zg = ops.spmm3_gated(g, x, prm, 0)  # the 4x4-block kernel's gated store (None: the middle-tile default gates later)
    if Zg is not None:
        ops.layer_dense(Zg, prm, 0, constant=layer.constant.detach(), res_x=x, act=True, pregated=True)
    Z = ops.spmm3(g, x)                 # the propagation (inference and training: middle-tile kernel)
    ops.spmm3_t(g, Z)                   # transposed propagation (backward)
    Y = ops.layer_dense(Z, prm, 0, constant=layer.constant.detach(), res_x=x, act=True)
    ops.layer_dense_backward(dY, Z, Y, prm, 0, res_x=x, act=True)  # dgrad / wgrad / reduce
    ops.head(Y, W1, b1, W2, b2, 1e-12)
torch.cuda.synchronize()
print("ok")
