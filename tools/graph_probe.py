#!/usr/bin/env python3
"""Eager vs HIP-graph replay of the 4-gram forward (torch.cuda.CUDAGraph drives hipGraph on ROCm): the
library's launches go to the caller's stream, so they capture. usage: python tools/graph_probe.py [ngram]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
dev = torch.device("cuda:0")
N, s, d, c = pkg.synth.de_bruijn_edges(n)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
torch.manual_seed(0)
model = pkg.ProtGramDirectGCN([128, 128, 128], N, 20, n, 0, 512, 0.5, True).to(dev).eval()
x = torch.randn(N, 128, generator=torch.Generator().manual_seed(1234)).to(dev)
data = pkg.Data(x=x, graph=g)


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


with torch.no_grad():
    ref = model(data)
    eager = timeit(lambda: model(data))
    s_ = torch.cuda.Stream()
    s_.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s_):
        for _ in range(3):
            model(data)
    torch.cuda.current_stream().wait_stream(s_)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        out = model(data)
    gr.replay()
    torch.cuda.synchronize()
    same = torch.equal(out[0], ref[0]) and torch.equal(out[1], ref[1])
    graphed = timeit(gr.replay)
    # can timing events be captured too?
    ev_ok = True
    try:
        g2 = torch.cuda.CUDAGraph()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.graph(g2):
            e0.record()
            model(data)
            e1.record()
        g2.replay()
        torch.cuda.synchronize()
        ev_ms = e0.elapsed_time(e1)
    except Exception as ex:  # noqa: BLE001
        ev_ok, ev_ms = False, repr(ex)[:120]
print(f"eager {eager:.4f} ms  graph {graphed:.4f} ms  identical={same}  captured-events {ev_ok} {ev_ms}")

# host-side cost of one forward (launch path), and with the bench's per-launch timing hooks
import time  # noqa: E402

from protgram_directgcn_amd import ops  # noqa: E402

with torch.no_grad():
    for hooks in (False, True):
        ops.SPMM_EVENTS = [] if hooks else None
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(50):
            model(data)
        t_cpu = (time.perf_counter() - t0) / 50 * 1e3
        torch.cuda.synchronize()
        t_all = (time.perf_counter() - t0) / 50 * 1e3
        print(f"hooks={hooks}: host {t_cpu:.4f} ms/forward, wall {t_all:.4f} ms/forward")
    ops.SPMM_EVENTS = None
