#!/usr/bin/env python3
"""Golden-vector generator: runs the REFERENCE's own hot-path code in this build container.

Container-only. Refuses to run when ``/root/reference`` is absent (the GPU box has no copy).
It imports ``src/models/protgram_directgcn.py`` (DirectGCNLayer / ProtGramDirectGCN) and
``src/utils/graph_utils.py`` (DirectedNgramGraph) unchanged, with the PyG boundary supplied by
``pyg_boundary.py`` (restated semantics, see that file), and writes small ``.npz`` fixtures
into ``tests/golden/``. No reference source or bytecode is written anywhere
(``sys.dont_write_bytecode``); only inputs and outputs are stored.

Cases (plus F6):
  f1_fasta2      2-gram graph from random FASTA: matrices, 1-layer + 2-layer model fwd, grads,
                 two reference training steps (eval-mode: dropout masks are RNG-stream specific)
  f1_debruijn2   complete B(20,2) synthetic graph (bench generator): matrices + 1-layer fwd/grads
  f2_edge        hand-made edge cases: raw self-loop, source-only / sink-only / isolated ids
  f2_empty       graph with an edge file of zero rows (A_in/A_out empty, A_u = self-loops only)
  f3_bench       benchmarker wiring (gnn_benchmarker.py:297-305): edge_weight None, non-symmetric,
                 distinct in/out/undirected patterns
  f4_cluster     clustered subgraph with original_indices (vector coeffs) + scalar-coefficient mode
  f5_fasta3      3-gram random-FASTA graph, F=64 (full)
  f5_debruijn3   complete B(20,3): matrix checksums + sampled entries; F=64 output samples + column stats
  f6_pe1         1-gram graph with the positional-embedding path (_apply_pe, protgram_directgcn.py:182-193)

Usage:  python tools/golden/make_golden.py
"""
import contextlib
import importlib.util
import io
import os
import sys
import tempfile

sys.dont_write_bytecode = True
REF = "/root/reference"
if not os.path.isdir(os.path.join(REF, "src")):
    sys.exit("make_golden.py: /root/reference is absent; fixtures can only be generated in the build container")

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(REPO, "tests", "golden")

sys.path.insert(0, HERE)
import pyg_boundary  # noqa: E402

pyg_boundary.install()
sys.path.insert(0, REF)

import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from src.models.protgram_directgcn import DirectGCNLayer, ProtGramDirectGCN  # noqa: E402
from src.utils.graph_utils import DirectedNgramGraph  # noqa: E402

_spec = importlib.util.spec_from_file_location("pg_synth", os.path.join(REPO, "protgram-directgcn_amd", "synth.py"))
synth = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(synth)

torch.set_num_threads(8)


def quiet(fn, *a, **kw):
    with contextlib.redirect_stdout(io.StringIO()):
        return fn(*a, **kw)


def ref_graph(N, src, dst, cnt, n, with_file=True):
    nodes = {i: f"g{i}" for i in range(N)}
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "edges.parquet")
        if with_file:
            pd.DataFrame({"source": np.asarray(src, np.int64), "target": np.asarray(dst, np.int64),
                          "weight": np.asarray(cnt, np.float32)}).to_parquet(path)
        g = quiet(DirectedNgramGraph, nodes=nodes, edge_file_path=path, epsilon_propagation=1e-9, n_value=n)
    return g


def mats(g, prefix=""):
    out = {}
    for tag, m in (("in", g.mathcal_A_in), ("out", g.mathcal_A_out), ("und", g.A_undirected_norm_sparse)):
        m = m.coalesce()
        out[f"{prefix}{tag}_idx"] = m.indices().numpy().astype(np.int64)
        out[f"{prefix}{tag}_val"] = m.values().numpy().astype(np.float32)
    return out


def randomize(module, seed):
    gen = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in module.named_parameters():
            leaf = name.split(".")[-1]
            if leaf.startswith("C_"):
                p.copy_(torch.rand(p.shape, generator=gen) + 0.5)
            elif "bias" in leaf:
                p.copy_(torch.rand(p.shape, generator=gen) * 0.2 - 0.1)


def sd(module, prefix):
    return {f"{prefix}{k}": v.detach().numpy().copy() for k, v in module.state_dict().items()}


def grads(module, prefix):
    return {f"{prefix}{k}": (p.grad.numpy().copy() if p.grad is not None else np.zeros(p.shape, np.float32))
            for k, p in module.named_parameters()}


def layer_case(fx, ei, ew, fin, fout, num_nodes, vec=True, orig=None, x=None, seed=11, tag="L", with_grads=True):
    """ei/ew: dict in/out/und -> tensors (ew may be None)."""
    N = int(num_nodes) if x is None else x.shape[0]
    torch.manual_seed(0)
    layer = DirectGCNLayer(fin, fout, num_nodes, vec)
    randomize(layer, seed)
    if x is None:
        x = torch.randn(N, fin, generator=torch.Generator().manual_seed(1234))
    x = x.clone().requires_grad_(True)
    y = layer(x, ei["in"], ew["in"], ei["out"], ew["out"], ei["und"], ew["und"], orig)
    fx[f"{tag}_x"] = x.detach().numpy()
    fx[f"{tag}_y"] = y.detach().numpy()
    fx.update(sd(layer, f"{tag}_p:"))
    if with_grads:
        R = torch.randn(y.shape, generator=torch.Generator().manual_seed(99))
        (y * R).sum().backward()
        fx[f"{tag}_R"] = R.numpy()
        fx[f"{tag}_gx"] = x.grad.numpy()
        fx.update(grads(layer, f"{tag}_g:"))
    fx[f"{tag}_cfg"] = np.array([fin, fout, num_nodes, int(vec)], np.int64)
    if orig is not None:
        fx[f"{tag}_orig"] = orig.numpy()


class _D:
    pass


def model_case(fx, ei, ew, dims, N, C, n, x, seed=21, tag="M", train_steps=2, one_gram_dim=0):
    torch.manual_seed(0)
    model = ProtGramDirectGCN(layer_dims=dims, num_graph_nodes=N, task_num_output_classes=C, n_gram_len=n,
                              one_gram_dim=one_gram_dim, max_pe_len=512, dropout=0.5, use_vector_coeffs=True)
    randomize(model, seed)
    init = sd(model, f"{tag}_p:")
    data = pyg_boundary.Data(x=x.clone().requires_grad_(True), edge_index_in=ei["in"], edge_weight_in=ew["in"],
                             edge_index_out=ei["out"], edge_weight_out=ew["out"],
                             edge_index_undirected_norm=ei["und"], edge_weight_undirected_norm=ew["und"])
    model.eval()
    lp, emb = model(data)
    R1 = torch.randn(lp.shape, generator=torch.Generator().manual_seed(7))
    R2 = torch.randn(emb.shape, generator=torch.Generator().manual_seed(8))
    ((lp * R1).sum() + (emb * R2).sum()).backward()
    fx.update(init)
    fx[f"{tag}_x"] = x.numpy()
    fx[f"{tag}_logp"] = lp.detach().numpy()
    fx[f"{tag}_emb"] = emb.detach().numpy()
    fx[f"{tag}_R1"], fx[f"{tag}_R2"] = R1.numpy(), R2.numpy()
    fx[f"{tag}_gx"] = data.x.grad.numpy()
    fx.update(grads(model, f"{tag}_g:"))
    fx[f"{tag}_cfg"] = np.array(list(dims) + [N, C, n, one_gram_dim], np.int64)
    if train_steps:
        # protgram_directgcn_trainer.py:91-100 on CPU (autocast/GradScaler disabled there), L2 over
        # ALL params (config.py:74 lambda=1e-7 -> Adam weight_decay 0, trainer :354). eval() keeps
        # the dropout masks out of the fixture.
        y = torch.randint(0, C, (N,), generator=torch.Generator().manual_seed(5))
        opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=0.0)
        model.zero_grad(set_to_none=True)
        data.x = x.clone()
        losses = []
        for _ in range(train_steps):
            opt.zero_grad()
            out, _ = model(data=data)
            primary = F.nll_loss(out, y)
            l2 = sum(p.norm(2).pow(2) for p in model.parameters() if p.requires_grad)
            loss = primary + 1e-7 * l2
            loss.backward()
            opt.step()
            losses.append(loss.item())
        fx[f"{tag}_train_y"] = y.numpy()
        fx[f"{tag}_train_loss"] = np.array(losses, np.float64)
        fx.update(sd(model, f"{tag}_train_p:"))


def graph_tensors(g):
    ei = {"in": g.mathcal_A_in.coalesce().indices(), "out": g.mathcal_A_out.coalesce().indices(),
          "und": g.A_undirected_norm_sparse.coalesce().indices()}
    ew = {"in": g.mathcal_A_in.coalesce().values(), "out": g.mathcal_A_out.coalesce().values(),
          "und": g.A_undirected_norm_sparse.coalesce().values()}
    return ei, ew


def save(name, fx):
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, **fx)
    print(f"  wrote {os.path.relpath(path, REPO)} ({os.path.getsize(path) / 1024:.0f} KiB)")


def raw(fx, N, src, dst, cnt, n):
    fx["N"] = np.array([N], np.int64)
    fx["n"] = np.array([n], np.int64)
    fx["src"], fx["dst"], fx["cnt"] = np.asarray(src, np.int64), np.asarray(dst, np.int64), np.asarray(cnt, np.float32)


def case_f1_fasta2():
    seqs = synth.random_sequences(64, 400, seed=0)
    N, s, d, c, _ = synth.fasta_edges(2, seqs)
    g = ref_graph(N, s, d, c, 2)
    fx = {}
    raw(fx, N, s, d, c, 2)
    fx.update(mats(g))
    ei, ew = graph_tensors(g)
    layer_case(fx, ei, ew, 32, 32, N)
    x = torch.randn(N, 32, generator=torch.Generator().manual_seed(1234))
    model_case(fx, ei, ew, [32, 32, 16], N, 5, 2, x)
    save("f1_fasta2", fx)


def case_f1_debruijn2():
    N, s, d, c = synth.de_bruijn_edges(2)
    g = ref_graph(N, s, d, c, 2)
    fx = {}
    raw(fx, N, s, d, c, 2)
    fx.update(mats(g))
    ei, ew = graph_tensors(g)
    layer_case(fx, ei, ew, 32, 32, N)
    save("f1_debruijn2", fx)


def case_f2_edge():
    # ids 0..11; node 9 source-only, 10 sink-only, 11 isolated (N > max edge id), 2->2 raw self-loop,
    # 4<->5 mutual pair, 6 only a self-loop.
    N = 12
    e = [(0, 1, 3), (1, 2, 1), (2, 2, 5), (2, 0, 2), (3, 4, 1), (4, 5, 7), (5, 4, 2), (6, 6, 4),
         (9, 0, 2), (9, 3, 1), (1, 10, 6), (5, 10, 1), (7, 8, 1), (8, 7, 1), (0, 3, 9)]
    e.sort()
    s, d, c = (np.array([t[i] for t in e]) for i in range(3))
    g = ref_graph(N, s, d, c, 2)
    fx = {}
    raw(fx, N, s, d, c, 2)
    fx.update(mats(g))
    ei, ew = graph_tensors(g)
    layer_case(fx, ei, ew, 8, 8, N)
    layer_case(fx, ei, ew, 8, 12, N, tag="L2")  # F_in != F_out
    save("f2_edge", fx)


def case_f2_empty():
    N = 6
    g = ref_graph(N, np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, np.float32), 2)
    fx = {}
    raw(fx, N, [], [], [], 2)
    fx.update(mats(g))
    ei, ew = graph_tensors(g)
    layer_case(fx, ei, ew, 8, 8, N)
    save("f2_empty", fx)


def case_f3_bench():
    # gnn_benchmarker.py:297-305 wiring: out = edge_index, in = edge_index[[1,0]], edge_attr None.
    # The undirected input is a GCN-normalised symmetric matrix built here (the benchmarker's own
    # _get_undirected_normalized_edges is broken); it is only an input.
    rng = np.random.default_rng(3)
    N, E = 50, 220
    pairs = set()
    while len(pairs) < E:
        a, b = (int(v) for v in rng.integers(0, N, 2))
        pairs.add((a, b))
    ei_out = torch.tensor(sorted(pairs), dtype=torch.long).t().contiguous()
    ei_in = ei_out[[1, 0]]
    und = torch.cat([ei_out, ei_out[[1, 0]]], 1)
    und = torch.unique(und, dim=1)
    und = torch.cat([und, torch.arange(N).repeat(2, 1)], 1)
    deg = torch.zeros(N).scatter_add_(0, und[1], torch.ones(und.size(1)))
    dis = deg.pow(-0.5)
    w_und = dis[und[0]] * dis[und[1]]
    ei = {"in": ei_in, "out": ei_out, "und": und}
    ew = {"in": None, "out": None, "und": w_und}
    fx = {"N": np.array([N], np.int64), "in_idx": ei_in.numpy(), "out_idx": ei_out.numpy(),
          "und_idx": und.numpy(), "und_val": w_und.numpy()}
    layer_case(fx, ei, ew, 16, 16, N)
    x = torch.randn(N, 16, generator=torch.Generator().manual_seed(1234))
    model_case(fx, ei, ew, [16, 16, 8], N, 3, 1, x, train_steps=1)
    save("f3_bench", fx)


def case_f4_cluster():
    seqs = synth.random_sequences(64, 400, seed=0)
    N, s, d, c, _ = synth.fasta_edges(2, seqs)
    g = ref_graph(N, s, d, c, 2)
    ei_full, ew_full = graph_tensors(g)
    rng = np.random.default_rng(4)
    subset = torch.tensor(np.sort(rng.choice(N, size=120, replace=False)), dtype=torch.long)
    # torch_geometric.utils.subgraph(subset, ei, ew, relabel_nodes=True): keep edges with both ends in
    # subset, relabel node v -> position of v in subset (trainer :183-196)
    pos = torch.full((N,), -1, dtype=torch.long)
    pos[subset] = torch.arange(subset.numel())
    ei, ew = {}, {}
    for k in ("in", "out", "und"):
        keep = (pos[ei_full[k][0]] >= 0) & (pos[ei_full[k][1]] >= 0)
        ei[k] = pos[ei_full[k][:, keep]]
        ew[k] = ew_full[k][keep]
    fx = {"N": np.array([N], np.int64), "subset": subset.numpy()}
    for k in ("in", "out", "und"):
        fx[f"{k}_idx"], fx[f"{k}_val"] = ei[k].numpy(), ew[k].numpy()
    x_full = torch.randn(N, 32, generator=torch.Generator().manual_seed(1234))
    layer_case(fx, ei, ew, 32, 32, N, orig=subset, x=x_full[subset], tag="L")
    layer_case(fx, ei, ew, 32, 24, 0, vec=True, x=x_full[subset], tag="S")  # num_nodes=0: scalar C_*, no constant
    layer_case(fx, ei, ew, 32, 32, N, vec=False, x=x_full[subset], tag="V")  # vector coeffs off, constant kept
    save("f4_cluster", fx)


def case_f5_fasta3():
    seqs = synth.random_sequences(40, 300, seed=1)
    N, s, d, c, _ = synth.fasta_edges(3, seqs)
    g = ref_graph(N, s, d, c, 3)
    fx = {}
    raw(fx, N, s, d, c, 3)
    fx.update(mats(g))
    ei, ew = graph_tensors(g)
    layer_case(fx, ei, ew, 64, 64, N, with_grads=False)
    save("f5_fasta3", fx)


def case_f5_debruijn3():
    N, s, d, c = synth.de_bruijn_edges(3)
    g = ref_graph(N, s, d, c, 3)
    ei, ew = graph_tensors(g)
    fx = {"N": np.array([N], np.int64), "n": np.array([3], np.int64)}
    rng = np.random.default_rng(5)
    for k in ("in", "out", "und"):
        idx, val = ei[k].numpy(), ew[k].numpy()
        pick = np.sort(rng.choice(val.size, size=4096, replace=False))
        fx[f"{k}_nnz"] = np.array([val.size], np.int64)
        fx[f"{k}_sum"] = np.array([val.astype(np.float64).sum(), (val.astype(np.float64) ** 2).sum()])
        fx[f"{k}_pick_idx"] = idx[:, pick]
        fx[f"{k}_pick_val"] = val[pick]
    torch.manual_seed(0)
    layer = DirectGCNLayer(64, 64, N, True)
    randomize(layer, 11)
    x = torch.randn(N, 64, generator=torch.Generator().manual_seed(1234))
    with torch.no_grad():
        y = layer(x, ei["in"], ew["in"], ei["out"], ew["out"], ei["und"], ew["und"])
    rows = np.sort(rng.choice(N, size=512, replace=False))
    fx["L_rows"] = rows
    fx["L_y_rows"] = y[rows].numpy()
    y64 = y.double()
    fx["L_colsum"] = y64.sum(0).numpy()
    fx["L_colsq"] = (y64 ** 2).sum(0).numpy()
    fx["L_xsum"] = np.array([x.double().sum().item(), (x.double() ** 2).sum().item()])
    fx.update(sd(layer, "L_p:"))
    save("f5_debruijn3", fx)


def case_f6_pe1():
    seqs = synth.random_sequences(8, 200, seed=2)
    N, s, d, c, _ = synth.fasta_edges(1, seqs)
    g = ref_graph(N, s, d, c, 1)
    fx = {}
    raw(fx, N, s, d, c, 1)
    fx.update(mats(g))
    ei, ew = graph_tensors(g)
    x = torch.randn(N, 16, generator=torch.Generator().manual_seed(1234))
    # The reference's in-place PE add (protgram_directgcn.py:191) raises under autograd when x does
    # not require grad (so the reference cannot TRAIN at n=1 with PE); inference and x-with-grad work.
    model_case(fx, ei, ew, [16, 16, 8], N, N, 1, x, train_steps=0, one_gram_dim=16)
    save("f6_pe1", fx)


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    for fn in (case_f1_fasta2, case_f1_debruijn2, case_f2_edge, case_f2_empty, case_f3_bench,
               case_f4_cluster, case_f5_fasta3, case_f5_debruijn3, case_f6_pe1):
        print(fn.__name__)
        fn()
