#!/usr/bin/env python3
"""Column-piece A/B of the 4x4-block transposed n-gram kernels (pg_spmm3t_ngram_bf16 / _f32) at B(20,4):
F = 256 at 4 features per lane (PG_FLAG_NGRAMT_WIDE), 2 (two 128-feature halves of a plan block on two waves of a
workgroup, PG_FLAG_NGRAMT_HALVES) or 1 (four 64-feature quarters, PG_FLAG_NGRAMT_NARROW); F = 128 at 2 or 1. Each variant's output is
compared bit for bit with the wide one; times are HIP-event averages over `reps` launches, interleaved rounds.
usage: python tools/r06_tsplit_probe.py [reps=20] > profiles/r06_tsplit_probe.json"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import _lib, ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda:0")
N, s, d, c = pkg.synth.de_bruijn_edges(4)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
ng = g.ngram
lib = _lib.load_library()
base = ops.default_flags()
out = {"graph": "B(20,4)", "n_rows": int(N), "reps": reps, "kernels": {}}
torch.manual_seed(0)
for dt in ("bf16", "f32"):
    for F in (256, 128):
        G = torch.randn(N, 3 * F, device=dev)
        G = G.to(torch.bfloat16) if dt == "bf16" else G
        fn = lib.pg_spmm3t_ngram_bf16 if dt == "bf16" else lib.pg_spmm3t_ngram_f32
        variants = {"wide": _lib.PG_FLAG_NGRAMT_WIDE, "narrow": _lib.PG_FLAG_NGRAMT_NARROW,
                    "default": 0}
        if F == 256:
            variants["halves"] = _lib.PG_FLAG_NGRAMT_HALVES
        variants["default_acc"] = -1  # the default variant accumulating into dX
        outs, times = {}, {k: [] for k in variants}
        for name, fl in variants.items():
            dX = torch.empty(N, F, device=dev, dtype=G.dtype)
            outs[name] = dX
        for rnd in range(3):
            for name, fl in variants.items():
                dX = outs[name]
                acc = 1 if fl < 0 else 0
                call = lambda: fn(ng.K, ng.n, N, ops._p(ng.plan), ops._p(G), G.stride(0), F, ops._p(dX),
                                  dX.stride(0), acc, base | max(fl, 0), ops._stream(G))
                assert call() == 0, name
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    call()
                e1.record()
                torch.cuda.synchronize()
                times[name].append(e0.elapsed_time(e1) / reps * 1e3)
        key = f"{dt}_F{F}"
        out["kernels"][key] = {
            name: {"us_min": round(min(t), 1), "us_all": [round(x, 1) for x in t],
                   "bit_identical_to_wide": name == "default_acc" or bool(torch.equal(outs[name].view(torch.int16 if dt == "bf16" else torch.int32),
                                                             outs["wide"].view(torch.int16 if dt == "bf16" else torch.int32)))}
            for name, t in times.items()}
        print(key, {k: v["us_min"] for k, v in out["kernels"][key].items()}, file=sys.stderr, flush=True)
print(json.dumps(out, indent=1))
