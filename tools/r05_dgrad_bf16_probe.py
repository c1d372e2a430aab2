#!/usr/bin/env python3
"""Round-5 probe of the bf16 dense backward's run-to-run differences (tools/r05_bf16det.py phase 2: only dgate
varies, in row pairs 8b+6, 8b+7 of the first 32 rows of a 128-row block). Calls pg_directgcn_dense_bwd_bf16 with its
workspace in hand and compares the per-n-tile gate partials dsp [ntn, 3, M] across repetitions, against a float64
reference of the same partials (from the kernel's own bf16 dpre, the packed bf16 weights and Z).
  python tools/r05_dgrad_bf16_probe.py [reps=30]"""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import _lib, ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
dev = torch.device("cuda", 0)
M, F = 8000, 128
K = 3 * F


from protgram_directgcn_amd import shard  # noqa: E402

sys.path.insert(0, os.path.join(REPO, "tests"))
from test_gpu_rccl import _model  # noqa: E402

rec = []
real_bwd = ops.layer_dense_backward


def rec_bwd(dY, Z, Y, prm, gate_mode, **kw):
    rec.append((dY.detach().clone(), Z.detach().clone(), Y.detach().clone(),
                {k: v.detach().clone() for k, v in prm.items()}, [t.clone() for t in (kw.get("packs") or [])]))
    return real_bwd(dY, Z, Y, prm, gate_mode, **kw)


ops.layer_dense_backward = rec_bwd
Ng, sg, dg, cg = pkg.synth.de_bruijn_edges(3)
gph = pkg.build_propagation_csr(Ng, sg, dg, cg, device=dev)
xg = torch.randn(Ng, 128, generator=torch.Generator().manual_seed(1234)).to(dev)
yg = (torch.arange(Ng, device=dev) // 400) % 20
mdl = _model(pkg, Ng, [128, 128, 128], dev, 3)
mdl.compute_dtype = torch.bfloat16
shard.ShardedTrainer(mdl, shard.partition(gph, 0, 1, transpose=True), lr=1e-3, l2_lambda=1e-3).step(xg, yg)
torch.cuda.synchronize()
ops.layer_dense_backward = real_bwd
dY, Z, Y, prm, packs = rec[0]  # the last layer's backward (autograd runs it first)
packed, p16 = packs
lib = ops.load_library()


POISON = {"mode": None}


def poison():
    keep = []
    for k in range(8, 25):
        for _ in range(2):
            t = torch.empty(1 << k, device=dev)
            t.view(torch.int32).random_() if POISON["mode"] == "random" else t.fill_(1e30)
            keep.append(t)
    del keep


def run(flags):
    if POISON["mode"] in ("random", "big"):
        poison()
    shift = torch.empty(int(torch.randint(1, 4096, (1,))), device=dev) if POISON["mode"] == "shift" else None
    a, keep = ops._layer_args(Z, prm, 0, None, None, None, None, True, ops.LEAKY_SLOPE, Y=Y)
    dpre = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    dZ = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    dgate = torch.empty(5, M, device=dev)
    gates = torch.empty(M, 4, device=dev)
    dW = torch.empty(F * K + 4 * F, device=dev)
    nwork = lib.pg_directgcn_dense_bwd_workspace(ctypes.byref(a))
    work = torch.full((int(nwork),), float("nan"), device=dev)
    g = _lib.LayerGradArgs()
    g.dY, g.lddy = ops._p(dY), dY.stride(0)
    g.dpre, g.ldp = ops._p(dpre), dpre.stride(0)
    g.dZ, g.lddz = ops._p(dZ), dZ.stride(0)
    g.dgate, g.gates, g.dW = ops._p(dgate), ops._p(gates), ops._p(dW)
    g.work, g.work_floats = ops._p(work), work.numel()
    _lib.check(lib.pg_directgcn_dense_bwd_bf16(ctypes.byref(a), ops._p(packed), ops._p(p16), ctypes.byref(g), flags,
                                              ops._stream(Z)), "bwd_bf16")
    torch.cuda.synchronize()
    off_dsp = K * F  # plan_of: up4(K * F_out) floats of (bf16) BT first
    ntn = K // 128
    dsp = work[off_dsp:off_dsp + ntn * 3 * M].view(ntn, 3, M).clone()
    del keep, shift
    return {"dsp": dsp, "dgate": dgate, "dZ": dZ, "dpre": dpre, "dW": dW}


out = {}
MODES = (("plain", ops.default_flags(), None), ("poison_random", ops.default_flags(), "random"),
         ("poison_big", ops.default_flags(), "big"), ("shift", ops.default_flags(), "shift"),
         ("no_remap_random", ops.default_flags() | _lib.PG_FLAG_NO_XCD_REMAP, "random"))
if os.environ.get("PROBE_MODES"):
    MODES = tuple(m for m in MODES if m[0] in os.environ["PROBE_MODES"].split(","))
for fname, fl, mode in MODES:
    POISON["mode"] = mode
    ref = run(fl)
    var = {}
    for r in range(reps):
        o = run(fl)
        for k in ref:
            d = (o[k] != ref[k]) & ~(torch.isnan(o[k].float()) & torch.isnan(ref[k].float()))
            if bool(d.any()):
                ent = var.setdefault(k, {"reps": 0, "where": set()})
                ent["reps"] += 1
                for w in d.nonzero()[:64].tolist():
                    ent["where"].add(tuple(w))
    # float64 reference of the partials of the differing (nt, q, m)
    dp = ref["dpre"].double()
    BT = p16.view(F, K).double()  # packed bf16 [F_out, K]
    G = dp @ BT  # [M, K]
    part = (G * Z.double()).view(M, 3, F).sum(-1)  # <G_q, Z_q>
    bsum = packed[F * K:F * K + 3 * F].view(3, F).double()
    bd = dp @ bsum.t()  # [M, 3]
    det = {}
    for k, v in var.items():
        det[k] = {"reps": v["reps"], "n_where": len(v["where"]), "where": sorted(v["where"])[:24]}
    if "dsp" in var:
        samp = []
        for (nt, q, m) in sorted(var["dsp"]["where"])[:8]:
            vals = sorted({float(run(fl)["dsp"][nt, q, m]) for _ in range(6)})
            samp.append({"nt": nt, "q": q, "m": m, "values": vals, "ref_part": float(part[m, q]),
                         "ref_bd": float(bd[m, q]), "ref_sum": float(part[m, q] + bd[m, q]) if nt == 0 else None})
        det["dsp_samples"] = samp
    out[fname] = det
    print(json.dumps({"lib": os.environ.get("PG_DIRECTGCN_LIB", "default"), fname: {
        k: (v if k == "dsp_samples" else {"reps": v["reps"], "n_where": v["n_where"]}) for k, v in det.items()}},
        default=str), flush=True)
