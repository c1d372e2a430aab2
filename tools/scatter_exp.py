#!/usr/bin/env python3
"""Where the scatter kernel's time goes (ngram_scatter_kernel, pg_ngram_scatter.hip): a diagnostics copy built with
-DPG_SCATTER_EXP reads flag bits 24..28 as phase skips (1 MFMAs + their LDS reads, 2 stores, 4 the D rows, 8 the
LDS-DMA; results garbage in those runs) at 8 chunks per workgroup; timed at config 5's rank-0 shapes (4-gram, P = 8,
F = 256, bf16), median of HIP-event reps.
usage: python tools/scatter_exp.py --build (in the container), then python tools/scatter_exp.py [--fp32]"""
import ctypes
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(REPO, "tools", "libscatter_exp.so")
if "--build" in sys.argv:
    src = os.path.join(REPO, "protgram-directgcn_amd", "csrc")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                           "-DPG_SCATTER_EXP", f"-I{REPO}/include", f"-I{src}", os.path.join(src, "pg_ngram_scatter.hip"),
                           os.path.join(src, "pg_abi.cpp"), "-o", SO])
    print("built", SO)
    sys.exit(0)

sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops, shard  # noqa: E402

fp32 = "--fp32" in sys.argv
dev = torch.device("cuda", 0)
N, s, d, c = pkg.synth.de_bruijn_edges(4)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
mp_ = shard.middle_partition(g, 0, 8)
sc = shard.middle_scatter(mp_)
F = 256
G = torch.randn(mp_.n_own, 3 * F, generator=torch.Generator().manual_seed(1)).to(dev)
if not fp32:
    G = G.to(torch.bfloat16)
T = torch.empty(3 * mp_.n_own, F, device=dev)
lib = ctypes.CDLL(SO)
fn = lib.pg_spmm3t_ngram_scatter_f32 if fp32 else lib.pg_spmm3t_ngram_scatter_bf16
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
               ctypes.c_int64, ctypes.c_uint32, ctypes.c_void_p]
stream = torch.cuda.current_stream().cuda_stream


def run(exp):
    rc = fn(sc.splan.data_ptr(), sc.splan.size(0), G.data_ptr(), G.stride(0), F, T.data_ptr(), T.stride(0),
            (exp << 24), stream)
    assert rc == 0


ref = ops.spmm3t_scatter(sc.splan, G)
run(0)
torch.cuda.synchronize()
assert torch.equal(T, ref), "diagnostics build at exp 0 differs from the library"
res = {"dtype": "f32" if fp32 else "bf16", "cpw": 8}
sets = {"all": 0, "no_mfma": 1, "no_stores": 2, "no_diag": 4, "no_dma": 8, "no_mfma_stores": 3, "dma_only": 7,
        "mfma_only": 14, "nothing": 15}
for name, e in sets.items():
    ts = []
    for _ in range(3):
        run(e)
    for _ in range(25):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        run(e)
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1000)
    ts.sort()
    res[name] = round(ts[len(ts) // 2], 2)
print(json.dumps(res))
