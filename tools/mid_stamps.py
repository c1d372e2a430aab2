#!/usr/bin/env python3
"""Where the middle-tile kernel's time goes: builds a diagnostics copy of pg_ngram_mid.hip with -DPG_MID_STAMPS
(s_memtime at each phase boundary of every chunk, compute wave 0 and loader wave 0 of every block), runs it at
B(20,n), and prints per-phase cycle statistics. usage: python tools/mid_stamps.py [n=4] [F=128] [flags=0]
(the library is built beforehand in the container: tools/mid_stamps.py --build)"""
import ctypes
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(REPO, "tools", "libmid_stamps.so")  # travels with the tree (protgram-directgcn_amd/build does not)
if "--build" in sys.argv:
    src = os.path.join(REPO, "protgram-directgcn_amd", "csrc")
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                           "-fno-slp-vectorize", "-DPG_MID_STAMPS", f"-I{REPO}/include", f"-I{src}",
                           os.path.join(src, "pg_ngram_mid.hip"), os.path.join(src, "pg_abi.cpp"), "-o", SO])
    print("built", SO)
    sys.exit(0)

sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
args = [a for a in sys.argv[1:] if not a.startswith("--")]
n = int(args[0]) if args else 4
F = int(args[1]) if len(args) > 1 else 128
flags = int(args[2], 0) if len(args) > 2 else 0
dev = torch.device("cuda:0")
N, s, d, c = pkg.synth.de_bruijn_edges(n)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
x = torch.randn(N, F, device=dev)
Z = torch.empty(N, 3 * F, device=dev)
lib = ctypes.CDLL(SO)
f = lib.pg_mid_stamped
vp, i64 = ctypes.c_void_p, ctypes.c_int64
f.argtypes = [ctypes.c_int, ctypes.c_int, i64, vp, vp, i64, i64, vp, i64, ctypes.c_uint32, vp, vp]
CH, PT = 32, 8
st = torch.zeros(256 * 2 * CH * PT, dtype=torch.int64, device=dev)
stream = vp(torch.cuda.current_stream().cuda_stream)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for rep in range(3):
    st.zero_()
    e0.record()
    rc = f(20, n, N, vp(g.ngram.mplan.data_ptr()), vp(x.data_ptr()), F, F, vp(Z.data_ptr()), 3 * F, flags,
           vp(st.data_ptr()), stream)
    assert rc == 0, rc
    e1.record()
    torch.cuda.synchronize()
ms = e0.elapsed_time(e1)
ref = pkg.ops.spmm3(g, x, flags=pkg._lib.PG_FLAG_NO_NGRAM)
print("max |d| vs csr", float((Z - ref).abs().max()))
a = st.view(256, 2, CH, PT).cpu().numpy().astype(np.int64)
names_c = ["start->outdone", "outdone->M", "M->indone", "indone->S", "S->stored+W"]
names_l = ["(chunk)->M", "M->dmaout_done", "dmaout_done->S", "S->dmain_done"]
for role, names in ((0, names_c), (1, names_l)):
    r = a[:, role]
    valid = r[:, :, 0] > 0
    for k, nm in enumerate(names):
        if role == 0:
            dlt = r[:, :, k + 1] - r[:, :, k]
        else:
            dlt = (r[:, :, k + 1] - r[:, :, k]) if k < 4 else None
        v = dlt[valid & (r[:, :, k + 1] > 0)]
        if v.size:
            print(f"{'compute' if role == 0 else 'loader '} {nm:18s} median {np.median(v):8.0f} mean {v.mean():8.0f} "
                  f"p90 {np.percentile(v, 90):8.0f} cycles (n={v.size})")
# whole-chunk cycle
r = a[:, 0]
tot = r[:, 1:, 0] - r[:, :-1, 0]
v = tot[(r[:, 1:, 0] > 0) & (r[:, :-1, 0] > 0)]
print(f"compute chunk-to-chunk median {np.median(v):.0f} cycles; blocks x chunks = {int((r[:, :, 0] > 0).sum())}")
# whole-kernel timeline (slot CH-1, pt 5: entry, 6: after the first chunk's operands are in, 7: exit), compute wave 0
c0 = a[:, 0, CH - 1]
t0 = a[:, :, CH - 1, 5][a[:, :, CH - 1, 5] > 0].min()
ent, rdy, ext = c0[:, 5] - t0, c0[:, 6] - t0, c0[:, 7] - t0
span = max(a[:, :, CH - 1, 7].max() - t0, 1)
print(f"kernel {ms * 1e3:.1f} us (events, incl. launch); stamp span {span} cycles -> {span / (ms * 1e3):.0f} cycles/us")
for nm, v in (("entry", ent), ("first operands in", rdy), ("exit", ext), ("busy (exit - entry)", ext - ent)):
    print(f"  {nm:20s} min {v.min():8d} median {int(np.median(v)):8d} max {v.max():8d} cycles")
nchunks = (a[:, 0, :CH - 1, 0] > 0).sum(1)
busy = ext - ent
for k in sorted(set(nchunks.tolist())):
    sel = nchunks == k
    print(f"  blocks with {k:2d} chunks: {int(sel.sum()):3d}, busy median {int(np.median(busy[sel]))} max {busy[sel].max()}")
xcd = np.arange(a.shape[0]) % 8
print("  busy median by XCD (blockIdx % 8):", [int(np.median(busy[xcd == i])) for i in range(8)])
print("  first operands in by XCD:", [int(np.median(rdy[xcd == i] - ent[xcd == i])) for i in range(8)])
per_chunk = np.diff(a[:, 0, :, 0], axis=1)
ok = (a[:, 0, 1:, 0] > 0) & (a[:, 0, :-1, 0] > 0)
print("  chunk median by XCD:", [int(np.median(per_chunk[(xcd == i)[:, None] & ok])) for i in range(8)])
