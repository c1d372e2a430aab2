#!/usr/bin/env python3
"""Round-5 bisection of the bf16 training step's last-bit non-reproducibility (profiles/r04_determinism_probe.json).

Phase 1: the bf16 ShardedTrainer step (world 1, B(20,3), dims [128,128,128], as tools/determinism_probe.py) repeated
R times from the same start; every ops.layer_dense_backward call records its inputs (dY, Z, Y, the packed weights)
and outputs (dpre, dZ, dgate, dB, dbsum). Before runs 2.. the caching allocator is "poisoned": blocks of many sizes
filled with NaN / 1e30 / random bits are allocated and freed, so a kernel that reads memory it did not write sees
different values in different runs. Report: per call, which recorded tensors differ from run 0.
Phase 2: the bf16 dense backward alone on fixed inputs, 40 repetitions with poisoned workspaces: do its outputs vary?
  python tools/r05_bf16det.py [reps=5]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops, shard  # noqa: E402
from test_gpu_rccl import _model  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda", 0)


def poison(kind: int):
    """Allocate and free blocks of many sizes filled with a pattern (the allocator hands them out again)."""
    keep = []
    sizes = [1 << k for k in range(8, 27)]  # 256 .. 64M elements (fp32)
    for s in sizes:
        for _ in range(3):
            t = torch.empty(s, device=dev, dtype=torch.float32)
            if kind == 0:
                t.fill_(float("nan"))
            elif kind == 1:
                t.fill_(1e30)
            else:
                t.view(torch.int32).random_()
            keep.append(t)
    torch.cuda.synchronize()
    del keep


def snap(v):
    if torch.is_tensor(v):
        return v.detach().clone()
    if isinstance(v, dict):
        return {k: snap(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [snap(x) for x in v]
    return v


calls = []
replay = []
real_bwd = ops.layer_dense_backward


def rec_bwd(dY, Z, Y, prm, gate_mode, **kw):
    out = real_bwd(dY, Z, Y, prm, gate_mode, **kw)
    packs = kw.get("packs")
    calls.append({"in.dY": snap(dY), "in.Z": snap(Z), "in.Y": snap(Y),
                  "in.packed": snap(packs[0]) if packs else None, "in.p16": snap(packs[1]) if packs else None,
                  "in.gates": [snap(prm[k]) for k in ("C_in", "C_out", "C_directed", "C_undirected", "C_all")],
                  **({"out." + k: snap(v) for k, v in out.items()} if out is not None else {})})
    replay.append((snap(dY), snap(Z), snap(Y), {k: snap(v) for k, v in prm.items()}, gate_mode,
                   {k: snap(v) for k, v in kw.items()}))
    return out


ops.layer_dense_backward = rec_bwd

N, s, d, c = pkg.synth.de_bruijn_edges(3)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
x = torch.randn(N, 128, generator=torch.Generator().manual_seed(1234)).to(dev)
y = (torch.arange(N, device=dev) // 400) % 20
part = shard.partition(g, 0, 1, transpose=True)
runs = []
for r in range(reps):
    if r >= 1:
        poison(r % 3)
    calls.clear()
    if r == 0:
        replay.clear()
    else:
        keep_replay = list(replay)
    m = _model(pkg, N, [128, 128, 128], dev, 3)
    m.compute_dtype = torch.bfloat16
    tr = shard.ShardedTrainer(m, part, lr=1e-3, l2_lambda=1e-3)
    loss = tr.step(x, y).clone()
    grads = {}
    for name, p in m.named_parameters():
        gg = p.grad
        if gg is None and shard._is_node_param(name, p, N):
            leaf = tr.own[int(name.split(".")[1])].get(name.split(".")[-1])
            gg = leaf.grad if leaf is not None else None
        if gg is not None:
            grads[name] = gg.detach().clone()
    torch.cuda.synchronize()
    print(f"[bf16det] run {r} done", file=sys.stderr, flush=True)
    if r > 0:
        replay[:] = keep_replay
    runs.append({"loss": loss, "grads": grads, "calls": [dict(cl) for cl in calls]})


def cmp(a, b):
    if a is None or b is None:
        return None if a is b else "none-mismatch"
    if isinstance(a, list):
        r = [cmp(u, v) for u, v in zip(a, b)]
        r = [z for z in r if z]
        return r or None
    if not torch.equal(a, b):
        da = (a.float() - b.float())
        nan = int(torch.isnan(a.float()).sum()) + int(torch.isnan(b.float()).sum())
        return {"n": int((a != b).sum()), "max": float(da.abs().nan_to_num(0).max()), "nan": nan,
                "where": [list(map(int, w)) for w in (a != b).nonzero()[:4].tolist()]}
    return None


report = {"phase1": []}
for r in range(1, reps):
    ent = {"run": r, "loss_equal": bool(torch.equal(runs[r]["loss"], runs[0]["loss"])), "grads": {}, "calls": []}
    for k, v in runs[0]["grads"].items():
        dd = cmp(v, runs[r]["grads"][k])
        if dd:
            ent["grads"][k] = dd
    for i, (c0, c1) in enumerate(zip(runs[0]["calls"], runs[r]["calls"])):
        diffs = {k: cmp(c0[k], c1[k]) for k in c0}
        diffs = {k: v for k, v in diffs.items() if v}
        if diffs:
            ent["calls"].append({"call": i, "diffs": diffs})
    report["phase1"].append(ent)
print(json.dumps(report), flush=True)

# phase 2: the bf16 dense backward alone on the recorded inputs of run 0's calls
ops.layer_dense_backward = real_bwd
ph2 = []
for i, (dY, Z, Y, prm, gm, kw) in enumerate(replay):
    ref = None
    nd = []
    for rep in range(40):
        poison(rep % 3)
        out = real_bwd(dY, Z, Y, prm, gm, **kw)
        out = {k: snap(v) for k, v in out.items() if v is not None}
        if ref is None:
            ref = out
            continue
        dd = {k: cmp(ref[k], out[k]) for k in ref}
        dd = {k: v for k, v in dd.items() if v}
        if dd:
            nd.append({"rep": rep, "diffs": dd})
    print(f"[bf16det] phase 2 call {i} done", file=sys.stderr, flush=True)
    ph2.append({"call": i, "n_differing_reps": len(nd), "first": nd[:3]})
print(json.dumps({"phase2": ph2}), flush=True)
