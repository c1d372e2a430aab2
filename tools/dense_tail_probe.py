#!/usr/bin/env python3
"""Dense kernel time vs row count around multiples of the block-slot count (tail effect check)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
F = 128
Mmax = 200000
torch.manual_seed(0)
layer = pkg.DirectGCNLayer(F, F, Mmax).to(dev)
prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in layer._dense_params())))
Z = torch.randn(Mmax, 3 * F, device=dev)
x = torch.randn(Mmax, F, device=dev)


def timeit(fn, reps=30):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for fl, name in ((0, "bm128w8"), (8, "bm64w8")):
    for tiles in (512, 768, 1024, 1152, 1250, 1280, 1536):
        M = tiles * 128
        if M > Mmax:
            continue
        t = timeit(lambda: ops.layer_dense(Z[:M], prm, 0, constant=layer.constant.detach(), res_x=x[:M], act=True,
                                           flags=fl))
        print(f"{name} M={M:7d} ({tiles} x128 tiles) {t:.4f} ms  {1e6 * t / M:.3f} ns/row")
