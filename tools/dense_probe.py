#!/usr/bin/env python3
"""Interleaved timing of pg_directgcn_dense_f32 variants (flags) at the bench shape, plus a value check of
each against the default. usage: python tools/dense_probe.py [ngram] [F]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
F = int(sys.argv[2]) if len(sys.argv) > 2 else 128
dev = torch.device("cuda:0")
N = 20 ** n
torch.manual_seed(0)
layer = pkg.DirectGCNLayer(F, F, N).to(dev)
with torch.no_grad():  # non-trivial gates and biases
    for name, q in layer.named_parameters():
        if name.startswith("C_"):
            q.uniform_(0.5, 1.5)
        elif "bias" in name:
            q.uniform_(-0.1, 0.1)
prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in layer._dense_params())))
const = layer.constant.detach()
Z = torch.randn(N, 3 * F, device=dev)
x = torch.randn(N, F, device=dev)
Y = torch.empty(N, F, device=dev)

variants = {"default": 0, "pre": 1 << 14, "x3_32": 1 << 17, "x3_32_pre": (1 << 17) | (1 << 14)}
for a in sys.argv[3:]:
    k, v = a.split("=")
    variants[k] = int(v, 0)


# pre-gated operand (what pg_spmm3_gated_f32 produces): s_q * Z_q
ca, cd = prm["C_all"].view(-1, 1), prm["C_directed"].view(-1, 1)
Zg = torch.cat([Z[:, :F] * (ca * cd * prm["C_in"].view(-1, 1)), Z[:, F:2 * F] * (ca * cd * prm["C_out"].view(-1, 1)),
                Z[:, 2 * F:] * (ca * prm["C_undirected"].view(-1, 1))], 1).contiguous()
PRE = 1 << 14


def run(fl):
    if fl & PRE:
        return ops.layer_dense(Zg, prm, 0, constant=const, res_x=x, act=True, flags=fl & ~PRE, out=Y, pregated=True)
    return ops.layer_dense(Z, prm, 0, constant=const, res_x=x, act=True, flags=fl, out=Y)


ref = run(0).clone()
# float64 reference on the first R rows: error of every variant against the exact formula
R = 8192
s64 = {k: prm[k][:R].double().view(-1, 1) for k in ("C_in", "C_out", "C_directed", "C_undirected", "C_all")}
sg = [s64["C_all"] * s64["C_directed"] * s64["C_in"], s64["C_all"] * s64["C_directed"] * s64["C_out"],
      s64["C_all"] * s64["C_undirected"]]
Wd = [(prm[a] + prm["W_shared"]).double() for a in ("W_main_in", "W_main_out", "W_undirected")]
bd = [(prm[a] + prm[b]).double() for a, b in (("b_main_in", "b_dir_shared_in"), ("b_main_out", "b_dir_shared_out"),
                                              ("b_undirected", "b_undirected_shared"))]
Zd = Z[:R].double()
y64 = sum(sg[q] * (Zd[:, q * F:(q + 1) * F] @ Wd[q].t() + bd[q]) for q in range(3)) + const[:R].double() + x[:R].double()
y64 = torch.nn.functional.leaky_relu(y64, 0.01)
for k, fl in variants.items():
    out = run(fl)
    d = (out - ref).abs().max().item()
    e = (out[:R].double() - y64).abs()
    print(f"{k:10s} max|d| vs default {d:.3e}   vs float64: max abs {e.max().item():.3e}, "
          f"max abs/(1+|y|) {(e / (1 + y64.abs())).max().item():.3e}, mean abs {e.mean().item():.3e}")


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


res = {k: [] for k in variants}
for _ in range(4):
    for k, fl in variants.items():
        res[k].append(timeit(lambda: run(fl)))
for k, v in res.items():
    print(f"{k:10s} " + " ".join(f"{t:.4f}" for t in v) + f"   min {min(v):.4f}")

# phase stamps of the pipelined split-bf16 kernel (flags bit 27 = dbg 128): per-block wave-0 cycle sums in Y rows
for pre in (False, True):
    fl = (1 << 27) | (PRE if pre else 0)
    run(fl)
    torch.cuda.synchronize()
    st = Y[:256, :6].double()
    names = ["top wait+B1", "Es + DMA issue", "MFMA(i)", "split(i+1)", "CR wait+B2", "epilogue(i-1)"]
    tot = st.sum(1)
    print(f"stamps ({'pre-gated' if pre else 'ungated'}): cycles per block, mean over blocks (total {tot.mean():.0f}, "
          f"max {tot.max():.0f})")
    for i, nm in enumerate(names):
        print(f"   {nm:28s} {st[:, i].mean():10.0f}  ({100 * st[:, i].mean() / tot.mean():5.1f} %)")
