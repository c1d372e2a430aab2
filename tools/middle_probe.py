#!/usr/bin/env python3
"""Per-rank cost of the middle partition (shard.middle_partition / middle_forward), measured on one GPU: for P in
2, 4, 8 every rank's forward is timed in turn with HIP events -- as the bench runs it (shard.MiddleRunner: per-segment
HIP graphs) and eagerly (shard.middle_forward) -- its ghost-row all_to_all replaced by the local part of the exchange
(the received rows are taken from a precomputed layer-1 output, once: the timed runner forward is the rank's local
work only). The exchange itself is priced from the measured byte counts: per rank pair one xGMI link, so the
all_to_all takes max over (sender, receiver) pairs of bytes / link rate; it is printed for the stated link rates,
without and with overlap (max(compute, exchange) vs compute + exchange). The replicate mode (layers before the last
over all rows, no exchange) is timed as is: its per-rank time is the step's.
usage: python tools/middle_probe.py [ngram] [F] [reps] [--out FILE]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops, shard  # noqa: E402
from protgram_directgcn_amd.graph import take  # noqa: E402
import bench  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
if out in args:
    args.remove(out)
n = int(args[0]) if args else 4
F = int(args[1]) if len(args) > 1 else 128
reps = int(args[2]) if len(args) > 2 else 30
CHUNKS = 4  # bench.py --chunks default: layer 1 in 4 middle sub-ranges, each exchanged as soon as it is computed
LINK_GBS = (50.0, 100.0)  # assumed achieved all_to_all rate per xGMI peer link and direction (GB/s)
dev = torch.device("cuda:0")
N, s, d, c = pkg.synth.de_bruijn_edges(n)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
del s, d, c
model = bench.bench_model(pkg, N, F, 2, n).to(dev).eval()
x = torch.randn(N, F, generator=torch.Generator().manual_seed(1234)).to(dev)
data = pkg.Data(x=x, graph=g)


def timeit(fn):
    with torch.no_grad():
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


t1 = timeit(lambda: model(data))
with torch.no_grad():
    conv = model.convs[0]
    prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in conv._dense_params())))
    h0 = model._apply_pe(x)
    h1 = ops.layer_dense(ops.spmm3(g, h0), prm, 0 if conv.use_vector_coeffs else 1,
                         constant=conv.constant.detach() if conv.use_vector_coeffs else None, res_x=h0, act=True)
print(f"B(20,{n}) F={F}: single GPU {t1:.4f} ms/step", flush=True)


def fill_once(self, i, c):  # layer-1 rows stand in for every boundary's received rows (timing only)
    done = self.__dict__.setdefault("_filled", set())
    if (i, c) not in done:
        r0, r1 = self.recv_slices[c]
        self.recv[i][r0:r1] = take(h1, self.mp.recv_ids[r0:r1])
        done.add((i, c))


report = {"ngram": n, "F": F, "N": N, "single_gpu_ms": round(t1, 4), "link_gbs_assumed": LINK_GBS, "P": {}}
for P in (2, 3, 4, 8):
    ts, tc, te, tr, ghosts, link = [], [], [], [], [], 0
    for r in range(P):
        mp = shard.middle_partition(g, r, P)
        inp = shard.middle_inputs(model, mp)
        buf = h1.clone()

        def local_exchange(mp_, h_own, group=None, buf=buf):
            buf.index_copy_(0, mp_.own, h_own)
            return buf

        shard_exchange = shard._exchange_rows
        shard._exchange_rows = local_exchange
        try:
            te.append(timeit(lambda: shard.middle_forward(model, mp, x, inp)))
        finally:
            shard._exchange_rows = shard_exchange
        # the bench's path: MiddleRunner (per-segment HIP graphs), the exchange's receive side filled locally; one
        # exchange after layer 1, and layer 1 in CHUNKS sub-ranges (each exchanged as soon as it is computed)
        runner_exchange = shard.MiddleRunner._exchange
        shard.MiddleRunner._exchange = fill_once
        try:
            run = shard.MiddleRunner(model, mp, x, inp)
            ts.append(timeit(run))
            del run
            mpc = shard.middle_partition(g, r, P, chunks=CHUNKS)
            run = shard.MiddleRunner(model, mpc, x, inp)
            tc.append(timeit(run))
            del run, mpc
            run = shard.MiddleRunner(model, mp, x, inp, replicate=True)  # no exchange: its time is the step's
            tr.append(timeit(run))
            del run
        finally:
            shard.MiddleRunner._exchange = runner_exchange
        ghosts.append(int(mp.recv_ids.numel()))
        link = max(link, max(mp.recv_counts))
        del mp, inp, buf
    m, mc = max(ts), max(tc)
    row_b = F * 4
    xch = {f"{gb:g}": round(link * row_b / (gb * 1e9) * 1e3, 4) for gb in LINK_GBS}  # ms per layer boundary
    # serial: one exchange after layer 1 (chunks = 1); overlapped bound: layer 1 in sub-ranges, the exchange hidden
    # behind the compute as far as it goes (max of the two)
    est = {k: {"serial_ms": round(m + v, 4), "overlapped_bound_ms": round(max(mc, v), 4),
               "speedup_serial": round(t1 / (m + v), 2), "speedup_overlapped_bound": round(t1 / max(mc, v), 2)}
           for k, v in xch.items()}
    report["P"][P] = {"rank_ms_graphs": [round(t, 4) for t in ts], "max_rank_ms": round(m, 4),
                      f"rank_ms_graphs_chunks{CHUNKS}": [round(t, 4) for t in tc], "max_rank_ms_chunked": round(mc, 4),
                      "eager_rank_ms": [round(t, 4) for t in te], "eager_max_rank_ms": round(max(te), 4),
                      "replicate_rank_ms": [round(t, 4) for t in tr], "replicate_max_rank_ms": round(max(tr), 4),
                      "replicate_speedup": round(t1 / max(tr), 2),
                      "compute_speedup": round(t1 / m, 2), "ghost_rows_max": max(ghosts),
                      "ghost_MB_max": round(max(ghosts) * row_b / 1e6, 2), "max_rows_per_link": link,
                      "exchange_ms_per_link_rate": xch, "estimate": est}
    print(f"P={P}: replicate-first-layers {max(tr):.4f} ms = {t1 / max(tr):.2f}x (no exchange); "
          f"max per-rank ms: graphs {m:.4f}, graphs + {CHUNKS} sub-ranges {mc:.4f}, eager {max(te):.4f}; "
          f"compute speedup {t1 / m:.2f}x; ghost rows/rank <= {max(ghosts)} ({max(ghosts) * row_b / 1e6:.1f} MB), "
          f"busiest link {link} rows; "
          + "; ".join(f"@{k} GB/s/link: exchange {v:.4f} ms -> {t1 / (m + v):.2f}x serial, "
                      f"<= {t1 / max(mc, v):.2f}x overlapped" for k, v in xch.items()), flush=True)
if out:
    with open(out, "w") as f:
        json.dump(report, f, indent=1)
