"""Builder-produced graphs on the middle-tile kernel (graph.build_ngram_map / pg_spmm3_ngram_mid_map_f32 + the residual
pass pg_spmm3_resid_f32).

run_graph_builder.py pads every sequence (data_builder.py:29-35) and numbers the n-grams PRESENT by sorted-string rank
(:164-173), so a real level-n graph is not the complete 20^n grid: the mapped plan runs its grid part on the tile
kernel at node rows and everything else (rows of n-grams with ' ' / X / U / B / Z, entries without a grid slot) on the
CSR kernel. Tolerances as tests/test_gpu_parity.py: propagation within |d| <= 1e-5 + 1e-5|ref| of the oracle's
propagate() (the tile kernel sums in another order), layer outputs the same against the reference's golden vectors.
"""
import numpy as np
import pytest
import torch

from golden_util import load, params, t
from oracle import directgcn_cpu as oc
from test_gpu_parity import assert_close

pytestmark = pytest.mark.gpu


def _csr_flags():
    from protgram_directgcn_amd import _lib, ops
    return ops.default_flags() | _lib.PG_FLAG_NO_NGRAM


def _oracle_mats(g):
    """(edge_index, [w_in, w_out, w_und]) of the graph's GPU-built weights, in the reference's flow."""
    N = g.n_rows
    e = g.edges3.cpu().numpy()
    rows = torch.from_numpy(np.repeat(np.arange(N), np.diff(g.rowptr.cpu().numpy())))
    ei = torch.stack([torch.from_numpy(e[:, 0].astype(np.int64)), rows])
    return ei, [torch.from_numpy(e[:, 1 + j].copy().view(np.float32)) for j in range(3)]


def _count(monkeypatch, lib, name):
    hits = []
    real = getattr(lib, name)
    monkeypatch.setattr(lib, name, lambda *a: hits.append(1) or real(*a))
    return hits


def test_fasta3_golden_layer_on_mapped_plan(pkg, cuda, monkeypatch):
    """f5_fasta3 (6,201 of the 8,000 3-grams, the reference's sorted-string ids): the node strings are regenerated
    from the fixture's seeded sequences (tools/golden/make_golden.py case_f5_fasta3), the graph gets the mapped plan,
    and the layer output matches the reference's own L_y."""
    from protgram_directgcn_amd import ngram, ops
    fx = load("f5_fasta3")
    N = int(fx["N"][0])
    seqs = pkg.synth.random_sequences(40, 300, seed=1)
    N2, s, d, c, strings = pkg.synth.fasta_edges(3, seqs)
    assert N2 == N and np.array_equal(s, fx["src"]) and np.array_equal(d, fx["dst"])
    tr = ngram.transitions_from_table(3, s, d, c, strings, alphabet=pkg.synth.ALPHABET, device=cuda)
    g = pkg.build_propagation_csr(N, fx["src"], fx["dst"], fx["cnt"], device=cuda, transitions=tr)
    assert g.ngram is None and g.ngram_map is not None
    m = g.ngram_map
    assert m.n_grid == N and m.n_off == 0 and m.nnz_res == 0  # all on the grid, all in grid slots
    lib = ops.load_library()
    hits = _count(monkeypatch, lib, "pg_spmm3_ngram_mid_map_f32")
    layer = pkg.DirectGCNLayer(*(int(v) for v in fx["L_cfg"][:3]), bool(fx["L_cfg"][3]))
    layer.load_state_dict(params(fx, "L_p"))
    layer = layer.to(cuda)
    with torch.no_grad():
        y = layer.fused_forward(t(fx["L_x"]).to(cuda), g)
    assert hits, "the mapped middle-tile kernel did not run"
    assert_close(y, fx["L_y"], "f5_fasta3 layer on the mapped plan vs the reference")
    x = t(fx["L_x"]).to(cuda)
    Z = ops.spmm3(g, x)
    Zc = ops.spmm3(g, x, flags=_csr_flags())
    assert_close(Z, Zc, "mapped vs CSR propagation")


@pytest.mark.parametrize("n,nseq,rare,F", [(2, 6, 0.05, 16), (3, 60, 0.01, 32), (3, 200, 0.003, 48),
                                            (3, 60, 0.01, 144), (2, 6, 0.05, 256)])
def test_padded_builder_graph_small(pkg, cuda, monkeypatch, n, nseq, rare, F):
    """Padded (' ') builder graphs with non-standard letters, built by ngram.ngram_transitions: off-grid rows,
    grid rows with residual entries, and grid slots all present; min_fill=0 forces the mapped plan on sparse grids.
    Each adjacency against the oracle's propagate() on the same GPU-built weights; the CSR kernel bit-exact. The
    widths cover the residual pass's lane layouts (16 lanes per row up to F = 64, 32 at 128, 64 above)."""
    from protgram_directgcn_amd import graph as gr, ngram, ops
    seqs = pkg.synth.protein_sequences(nseq, 120, seed=n * 100 + nseq, rare=rare, composition="uniform")
    tr = ngram.ngram_transitions(seqs, n, device=cuda)
    g = pkg.build_propagation_csr(tr.num_nodes, tr.src.cpu().numpy(), tr.dst.cpu().numpy(), tr.cnt.cpu().numpy(),
                                  device=cuda)
    assert g.ngram is None
    g.ngram_map = gr.build_ngram_map(g, tr.node_keys, tr.alphabet, n, min_fill=0.0)
    m = g.ngram_map
    assert m is not None and m.n_off > 0 and m.n_acc > 0 and m.nnz_res > 0
    # every node string on the grid maps to its base-20 number; the others are off
    strings = tr.node_strings()
    ginv = m.ginv.cpu().numpy()
    for i in range(0, len(strings), max(1, len(strings) // 300)):
        sgl = strings[i]
        if all(ch in gr.GRID_LETTERS for ch in sgl):
            want = 0
            for ch in sgl:
                want = want * 20 + gr.GRID_LETTERS.index(ch)
            assert ginv[i] == want, (sgl, ginv[i], want)
        else:
            assert ginv[i] == -1, sgl
    x = torch.randn(tr.num_nodes, F, generator=torch.Generator().manual_seed(3)).to(cuda)
    lib = ops.load_library()
    hits = _count(monkeypatch, lib, "pg_spmm3_ngram_mid_map_f32")
    res = _count(monkeypatch, lib, "pg_spmm3_resid_f32")
    Z = ops.spmm3(g, x).cpu()
    assert hits and len(res) == 1
    Zc = ops.spmm3(g, x, flags=_csr_flags()).cpu()
    ei, w = _oracle_mats(g)
    for j in range(3):
        ref = oc.propagate(ei, x.cpu(), w[j])
        assert torch.equal(Zc[:, j * F:(j + 1) * F], ref), j
        assert_close(Z[:, j * F:(j + 1) * F], ref, f"mapped propagation {j} (n={n})")
    assert int(m.res_rowptr[-1]) == m.nnz_res and m.res_rows.numel() == m.n_off + m.n_acc


def test_padded_fasta_4gram_at_size(pkg, cuda, monkeypatch):
    """a padded FASTA-built 4-gram graph with >= 150k nodes (ngram.py on protein-like sequences
    with the Swiss-Prot composition and rare X/U/B/Z) takes the mapped middle-tile kernel (launch counted), and the
    full layer forward matches the oracle within 1e-5; each adjacency of the propagation too."""
    from protgram_directgcn_amd import ngram, ops
    seqs = pkg.synth.protein_sequences(8000, 350, seed=1)
    tr = ngram.ngram_transitions(seqs, 4, device=cuda)
    N = tr.num_nodes
    assert N >= 150_000, N
    g = pkg.build_propagation_csr(N, tr.src.cpu().numpy(), tr.dst.cpu().numpy(), tr.cnt.cpu().numpy(), device=cuda,
                                  transitions=tr)
    assert g.ngram is None and g.ngram_map is not None
    m = g.ngram_map
    assert m.n_grid > 0.9 * N and m.n_off > 0
    F = 128
    torch.manual_seed(0)
    layer = pkg.DirectGCNLayer(F, F, N, True)
    with torch.no_grad():
        for name, p in layer.named_parameters():
            if name.startswith("C_"):
                p.uniform_(0.5, 1.5)
            elif "bias" in name:
                p.uniform_(-0.1, 0.1)
    layer = layer.to(cuda)
    x = torch.randn(N, F, generator=torch.Generator().manual_seed(1234))
    xd = x.to(cuda)
    lib = ops.load_library()
    hits = _count(monkeypatch, lib, "pg_spmm3_ngram_mid_map_f32")
    with torch.no_grad():
        y = layer.fused_forward(xd, g)
        Z = ops.spmm3(g, xd).cpu()
    assert len(hits) == 2, "the mapped middle-tile kernel did not run"
    ei, w = _oracle_mats(g)
    p = {k: v.detach().cpu() for k, v in layer.state_dict().items()}
    with torch.no_grad():
        y_ref = oc.layer_forward(p, x, ei, w[0], ei, w[1], ei, w[2])
    assert_close(y, y_ref, "padded 4-gram layer")
    for j in range(3):
        assert_close(Z[:, j * F:(j + 1) * F], oc.propagate(ei, x, w[j]), f"padded 4-gram propagation {j}")


def test_mapped_through_model_and_backward(pkg, cuda):
    """A 2-layer model forward + backward on a mapped graph (the forward's propagation on the mapped kernel, the
    backward's transposed propagation on the CSR kernel) against the same model on the CSR kernels only."""
    from protgram_directgcn_amd import ngram, ops
    seqs = pkg.synth.protein_sequences(200, 200, seed=5, rare=0.005, composition="uniform")
    tr = ngram.ngram_transitions(seqs, 3, device=cuda)
    g = pkg.build_propagation_csr(tr.num_nodes, tr.src.cpu().numpy(), tr.dst.cpu().numpy(), tr.cnt.cpu().numpy(),
                                  device=cuda, transitions=tr)
    assert g.ngram_map is not None
    N = tr.num_nodes
    torch.manual_seed(1)
    m = pkg.ProtGramDirectGCN([32, 64, 32], N, 7, 3, 0, 0, 0.0, True).to(cuda).eval()  # no decoder dropout
    x = torch.randn(N, 32, device=cuda, requires_grad=True)
    y = torch.randint(0, 7, (N,), device=cuda)
    outs = []
    for csr in (False, True):
        with pytest.MonkeyPatch.context() as mp:
            if csr:
                fl = _csr_flags()
                mp.setattr(ops, "default_flags", lambda: fl)
            m.zero_grad()
            x.grad = None
            lp, emb = m(pkg.Data(x=x, graph=g))
            torch.nn.functional.nll_loss(lp, y).backward()
            outs.append((lp.detach().clone(), x.grad.clone(),
                         {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None}))
    (a, ga, pa), (b, gb, pb) = outs
    assert_close(a, b, "log-probs mapped vs CSR", rtol=1e-4, atol=1e-5)
    assert_close(ga, gb, "dx mapped vs CSR", rtol=1e-3, atol=1e-6)
    for k in pa:
        scale = float(pb[k].abs().max()) + 1e-12
        assert float((pa[k] - pb[k]).abs().max()) <= 1e-3 * scale + 1e-7, k
