#!/usr/bin/env python3
"""Diagnostics (round 5): stage dumps of the bf16 dgrad kernel's lead tiles (libpgdgcn_dbg.so, -DPG_DGRAD_DBG) over
repeated calls on the same inputs with cold caches: which stage (accumulator tile, A image, bias partials, epilogue
parts, final gate partials) first differs between runs."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PG_DIRECTGCN_LIB", os.path.join(REPO, "protgram-directgcn_amd", "libpgdgcn_dbg.so"))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops  # noqa: E402
import test_gpu_parity as T  # noqa: E402

dev = torch.device("cuda", 0)
lib = ops.load_library()
lib.pg_dgrad_debug_buffer.restype = ctypes.c_int
lib.pg_dgrad_debug_buffer.argtypes = [ctypes.c_void_p]
Z, xres, prm, const, r, W_res, b_res, dY = T._dense_case(20000, 128, 128, False, True, False, 3)
dv = {k: v.to(dev) for k, v in prm.items()}
Zg, dYg, xg = Z.to(dev).to(torch.bfloat16), dY.to(dev).to(torch.bfloat16), xres.to(dev).to(torch.bfloat16)
packs = []
Y = ops.layer_dense(Zg, dv, 0, res_x=xg, act=True, packs=packs)
BM, TLD, LDKB = 128, 132, 72
stride = 2 * BM * TLD + 2 * BM * LDKB + 12 * BM
nblk = (20000 + BM - 1) // BM
dbg = torch.full((nblk * stride,), float("nan"), device=dev)
assert lib.pg_dgrad_debug_buffer(ctypes.c_void_p(dbg.data_ptr())) == 0
flush = torch.empty(1 << 29, device=dev)
runs = []
for rep in range(10):
    flush.fill_(float(rep))
    dbg.fill_(float("nan"))
    torch.cuda.synchronize()
    out = ops.layer_dense_backward(dYg, Zg, Y, dv, 0, res_x=xg, act=True, packs=packs)
    torch.cuda.synchronize()
    runs.append((dbg.clone().view(nblk, stride), out["dgate"].clone()))
names = [("acc", 0, BM * TLD), ("parts", BM * TLD, BM * TLD), ("A", 2 * BM * TLD, 2 * BM * LDKB),
         ("Pd", 2 * BM * TLD + 2 * BM * LDKB, 12 * BM)]
rep = []
for k in range(1, len(runs)):
    d, g = runs[k]
    d0, g0 = runs[0]
    ent = {"run": k, "dgate_rows": sorted({int(c) for c in (g != g0).nonzero()[:, 1].tolist()})[:20]}
    for nm, o, n in names:
        a, b = d0[:, o:o + n], d[:, o:o + n]
        diff = (a != b) & ~(torch.isnan(a) & torch.isnan(b))
        if nm in ("acc", "parts"):  # padding columns 128..131 of T are never written nor read
            diff = diff & (torch.arange(n, device=dev) % TLD < 128)
        if nm == "A":  # padding columns 64..71 of the A images
            diff = diff & (torch.arange(n, device=dev) % LDKB < 64)
        idx = diff.nonzero()
        ent[nm] = {"n": int(idx.size(0)), "first": idx[:6].tolist()}
        if nm in ("acc", "parts") and idx.size(0):
            ent[nm]["rows_cols"] = [(int(bk), int(e) // TLD, int(e) % TLD) for bk, e in idx[:8].tolist()]
            ent[nm]["rows"] = sorted({(int(bk), int(e) // TLD) for bk, e in idx.tolist()})[:16]
            ent[nm]["vals"] = [(float(a[bk, e]), float(b[bk, e])) for bk, e in idx[:4].tolist()]
    rep.append(ent)
print(json.dumps(rep))
# the differing bias partials against the dumped A images and the packed bias sums (float64)
bsum = packs[0][128 * 384:128 * 384 + 3 * 128].view(3, 128).double()
detail = []
blk_rows = set()
for k in range(1, len(runs)):
    d, _ = runs[k]
    d0, _ = runs[0]
    o = 2 * BM * TLD + 2 * BM * LDKB
    diff = (d[:, o:o + 12 * BM] != d0[:, o:o + 12 * BM]).nonzero().tolist()
    for bk, e in diff:
        blk_rows.add((bk, e))
for bk, e in sorted(blk_rows)[:6]:
    qt, rem = divmod(e, 3 * BM)
    row, sg = divmod(rem, 3)
    A = runs[0][0][bk, 2 * BM * TLD:2 * BM * TLD + 2 * BM * LDKB].view(2, BM, LDKB).double()
    ks = [t * 64 + 16 * qt + 8 * c + x for t in range(2) for c in range(2) for x in range(8)]
    dr = torch.stack([A[k_ // 64, row, k_ % 64] for k_ in ks])
    # A holds the raw bf16 bit patterns as floats: rebuild the values
    bits = dr.to(torch.int64).to(torch.int32) << 16
    vals = bits.view(torch.float32).double()
    ref = float((vals * bsum[sg, ks]).sum())
    detail.append({"block": bk, "row": row, "sg": sg, "qt": qt, "ref": ref,
                   "runs": [float(r_[0][bk, 2 * BM * TLD + 2 * BM * LDKB + e]) for r_ in runs]})
print(json.dumps(detail))
# which inputs reproduce a wrong partial: every (sg', set of k) alternative, and per-chunk substitutions
alts = []
for ent in detail[:4]:
    bk, row, sg, qt = ent["block"], ent["row"], ent["sg"], ent["qt"]
    A = runs[0][0][bk, 2 * BM * TLD:2 * BM * TLD + 2 * BM * LDKB].view(2, BM, LDKB)
    Av = (A.to(torch.int64).to(torch.int32) << 16).view(torch.float32).double()
    wrong = [v for v in ent["runs"] if v != ent["runs"][0]] or [v for v in ent["runs"]]
    target = wrong[0] if wrong[0] != ent["runs"][0] else None
    chunks = [(t, c) for t in range(2) for c in range(2)]
    parts = {}
    for t, c in chunks:
        ks = [t * 64 + 16 * qt + 8 * c + x for x in range(8)]
        drc = torch.stack([Av[t, row, (k_ % 64)] for k_ in ks])
        for s2 in range(3):
            for kofs in range(0, 128, 8):
                kk = [(k_ + kofs) % 128 for k_ in ks]
                parts[(t, c, s2, kofs)] = float((drc * bsum[s2, kk]).sum())
    good = sum(parts[(t, c, sg, 0)] for t, c in chunks)
    best = []
    for (t, c) in chunks:
        for s2 in range(3):
            for kofs in range(0, 128, 8):
                v = good - parts[(t, c, sg, 0)] + parts[(t, c, s2, kofs)]
                if target is not None:
                    best.append((abs(v - target), t, c, s2, kofs))
    best.sort()
    alts.append({"row": row, "good": good, "target": target, "best": best[:3]})
print(json.dumps(alts))
