#!/usr/bin/env python3
"""A/B timing of the middle-tile kernel: the in-tree library's pg_spmm3_ngram_mid_f32 against a reference build of
pg_ngram_mid.hip from another revision (tools/libmid_ab.so, built beforehand in the container:
`python tools/mid_ab.py --build <git-rev>`), interleaved rounds on the same inputs (box-to-box clock differences
cancel); prints min / median per-launch ms of each and checks that both give the same bits.
usage: python tools/mid_ab.py [n=4] [F=128] [rounds=30]"""
import ctypes
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(REPO, "tools", "libmid_ab.so")
if "--build" in sys.argv:
    rev = sys.argv[sys.argv.index("--build") + 1]
    src = os.path.join(REPO, "protgram-directgcn_amd", "csrc")
    tmp = "/tmp/pg_ngram_mid_ab.hip"
    with open(tmp, "w") as f:
        f.write(subprocess.check_output(["git", "-C", REPO, "show", f"{rev}:protgram-directgcn_amd/csrc/pg_ngram_mid.hip"],
                                        text=True))
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                           f"-I{REPO}/include", f"-I{src}", tmp, os.path.join(src, "pg_abi.cpp"), "-o", SO])
    print("built", SO, "from", rev)
    sys.exit(0)

sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
n = int(args[0]) if args else 4
F = int(args[1]) if len(args) > 1 else 128
rounds = int(args[2]) if len(args) > 2 else 30
dev = torch.device("cuda:0")
N, s, d, c = pkg.synth.de_bruijn_edges(n)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
x = torch.randn(N, F, generator=torch.Generator().manual_seed(3)).to(dev)
Za, Zb = torch.empty(N, 3 * F, device=dev), torch.empty(N, 3 * F, device=dev)
vp, i64 = ctypes.c_void_p, ctypes.c_int64
sig = [ctypes.c_int, ctypes.c_int, i64, vp, vp, i64, i64, vp, vp, i64, ctypes.c_uint32, vp]
new = ops.load_library().pg_spmm3_ngram_mid_f32
old = ctypes.CDLL(SO).pg_spmm3_ngram_mid_f32
old.argtypes, old.restype = sig, ctypes.c_int
stream = vp(torch.cuda.current_stream().cuda_stream)
fl = ops.default_flags()


def launch(fn, Z):
    rc = fn(20, n, N, vp(g.ngram.mplan.data_ptr()), vp(x.data_ptr()), F, F, None, vp(Z.data_ptr()), 3 * F, fl, stream)
    assert rc == 0, rc


def timed(fn, Z, k=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(k):
        launch(fn, Z)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / k


for _ in range(20):  # clock ramp
    launch(new, Za)
    launch(old, Zb)
torch.cuda.synchronize()
ta, tb = [], []
for _ in range(rounds):
    ta.append(timed(new, Za))
    tb.append(timed(old, Zb))
ta.sort()
tb.sort()
print(f"B(20,{n}) F={F}: in-tree {ta[0]:.4f} min / {ta[len(ta) // 2]:.4f} median ms; reference build "
      f"{tb[0]:.4f} / {tb[len(tb) // 2]:.4f}; same bits: {bool(torch.equal(Za, Zb))}")
