#!/usr/bin/env python3
"""Where the pipelined split-bf16 dense kernel's time goes (dense_x3p_kernel, pg_dense.hip): builds a diagnostics copy
with -DPG_DENSE_EXP (flag bits 24..28 skip phases: 1 MFMAs, 2 split, 4 Y stores, 8 A DMA, 16 constant / residual DMA;
results are garbage in those runs), and times the bench's layer-1 dense launch at B(20,n), F=128 with each set of
phases skipped (min of interleaved rounds, HIP events).
usage: python tools/dense_exp.py --build (in the container), then python tools/dense_exp.py [n=4] [reps=20]"""
import ctypes
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(REPO, "tools", "libdense_exp.so")
if "--build" in sys.argv:
    src = os.path.join(REPO, "protgram-directgcn_amd", "csrc")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                           "-DPG_DENSE_EXP", f"-I{REPO}/include", f"-I{src}", os.path.join(src, "pg_dense.hip"),
                           os.path.join(src, "pg_abi.cpp"), "-o", SO])
    print("built", SO)
    sys.exit(0)

sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import _lib, ops  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
n = int(args[0]) if args else 4
reps = int(args[1]) if len(args) > 1 else 20
dev = torch.device("cuda:0")
N, s, d, c = pkg.synth.de_bruijn_edges(n)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
import bench  # noqa: E402

model = bench.bench_model(pkg, N, 128, 2, n).to(dev).eval()
layer = model.convs[0]
x = torch.randn(N, 128, device=dev)
prm = dict(zip(ops._DENSE_KEYS, layer._dense_params()))
Z = ops.spmm3_gated(g, x, prm, 0)
pregated = Z is not None
if Z is None:
    Z = ops.spmm3(g, x)
Y = torch.empty(N, 128, device=dev)
lib = ctypes.CDLL(SO)
fn = lib.pg_directgcn_dense_f32
fn.restype, fn.argtypes = _lib.SIGNATURES["pg_directgcn_dense_f32"]
a, keep = ops._layer_args(Z, prm, 0, None, layer.constant, x, None, True, ops.LEAKY_SLOPE)
a.Y, a.ldy = ops._p(Y), Y.stride(0)
raw = [ops._f32c(prm[k].detach()) for k in ops._PACK_KEYS]
(a.W_main_in, a.W_main_out, a.W_undirected, a.W_shared, a.b_main_in, a.b_dir_shared_in, a.b_main_out,
 a.b_dir_shared_out, a.b_undirected, a.b_undirected_shared) = [ops._p(t) for t in raw]
base = (_lib.PG_FLAG_DENSE_PREGATED if pregated else 0) | (_lib.PG_FLAG_DENSE_NO_IL if "--no-il" in sys.argv else 0)
st = ops._stream(Z)


def run(exp):
    rc = fn(ctypes.byref(a), None, base | (exp << 24), st)
    assert rc == 0, lib.pg_last_error()


def timeit(exp):
    for _ in range(3):
        run(exp)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run(exp)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


if "--stamps" in sys.argv:  # per-iteration cycle breakdown of waves 0 (MFMA first) and 4 (split first)
    import numpy as np
    NB, NIT, NPT = 64, 48, 8
    buf = torch.zeros(NB * 2 * NIT * NPT, dtype=torch.int64, device=dev)
    lib.pg_dense_set_stamps.argtypes = [ctypes.c_void_p]
    for _ in range(20):
        run(0)
    torch.cuda.synchronize()
    assert lib.pg_dense_set_stamps(ctypes.c_void_p(buf.data_ptr())) == 0
    run(0)
    torch.cuda.synchronize()
    lib.pg_dense_set_stamps(None)
    t = buf.view(NB, 2, NIT, NPT).cpu().numpy().astype(np.float64)
    names = ["wait_A+B1", "issue_dma", "first_phase", "second_phase", "wait_CR", "B2", "epilogue", "to_next_top"]
    res = {}
    for w, wn in ((0, "wave0_mfma_first"), (1, "wave4_split_first")):
        seg = {}
        v = t[:, w]
        its = slice(2, 36)
        for k in range(NPT - 1):
            d = v[:, its, k + 1] - v[:, its, k]
            seg[names[k + 1 if k else 0]] = float(np.median(d))
        seg["wait_A+B1"] = float(np.median(v[:, its, 1] - v[:, its, 0]))
        seg["issue_dma"] = float(np.median(v[:, its, 2] - v[:, its, 1]))
        seg["first_phase"] = float(np.median(v[:, its, 3] - v[:, its, 2]))
        seg["second_phase"] = float(np.median(v[:, its, 4] - v[:, its, 3]))
        seg["wait_CR"] = float(np.median(v[:, its, 5] - v[:, its, 4]))
        seg["B2"] = float(np.median(v[:, its, 6] - v[:, its, 5]))
        seg["epilogue"] = float(np.median(v[:, its, 7] - v[:, its, 6]))
        seg["iteration"] = float(np.median(v[:, 3:37, 0] - v[:, 2:36, 0]))
        res[wn] = {k: round(x, 1) for k, x in seg.items()}
    print("stamps (median cycles per iteration, s_memtime ticks, iterations 2..35 of blocks 0..63):",
          json.dumps(res) if "json" in globals() else res)
    sys.exit(0)

run(0)
ref = ops.layer_dense(Z, prm, 0, constant=layer.constant, res_x=x, act=True, pregated=pregated)
torch.cuda.synchronize()
print(f"exp=0 vs product kernel: max |d| {float((Y - ref).abs().max()):.3e}")
cases = {"all": 0, "no_mfma": 1, "no_split": 2, "no_mfma_split": 3, "no_store": 4, "no_A_dma": 8, "no_CR_dma": 16,
         "no_dma": 24, "no_dma_store": 28, "skeleton": 31, "mfma_only": 30, "split_only": 29}
best = {k: 1e9 for k in cases}
for _ in range(4):
    for k, e in cases.items():
        best[k] = min(best[k], timeit(e))
print(" ".join(f"{k}={v * 1e3:.1f}us" for k, v in best.items()))
