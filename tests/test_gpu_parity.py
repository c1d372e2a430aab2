"""GPU parity: the HIP path (through the C-ABI library) against the oracle and the reference's golden
vectors. Tolerances:
  * propagation kernels (pg_spmm3/pg_spmm1/fused-norm): BIT-EXACT vs the oracle's propagate(), which
    is the reference's index_select -> mul -> scatter_add_ (same operation order, see pg_spmm.hip)
  * GPU-built weights (pg_edges_normalize_f32): bit-exact vs the IEEE closed form; <= 1 ulp vs the
    reference matrices (torch CPU sqrt is MKL's, not correctly rounded; tests/test_host.py)
  * layer / model OUTPUTS (reassociated A(xW) = (Ax)W + MFMA accumulation order):
    |d| <= 1e-5 + 1e-5*|ref| elementwise (BASELINE.json north_star: fp32 within 1e-5)
  * GRADIENTS are long reductions (over all N rows for weights) whose elements can cancel to values far
    below the summed magnitude; they are checked against the tensor's scale:
    |d| <= 2e-5*max|ref| + 1e-4*|ref|  (observed errors ~1e-7 of the summed magnitude)
"""
import functools

import numpy as np
import pytest
import torch

from golden_util import graph, load, params, t
from oracle import directgcn_cpu as oc
from oracle import graph_cpu as og

pytestmark = pytest.mark.gpu
RTOL = ATOL = 1e-5

FLAG_VARIANTS = [0, 1, 2, 4, 6, 128, 132]  # C window (default), no XCD remap, B LDS staging, C u8, B u4, A, A u4


def assert_close(got, ref, what, rtol=RTOL, atol=ATOL):
    got = got.detach().float().cpu()
    ref = torch.as_tensor(ref).float().cpu()
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    err = (got - ref).abs()
    bad = err > atol + rtol * ref.abs()
    assert not bool(bad.any()), f"{what}: {int(bad.sum())} elements out of tolerance, max |d| {err.max().item():.3e}"


def assert_grad_close(got, ref, what):
    ref = torch.as_tensor(ref).float().cpu()
    scale = float(ref.abs().max()) if ref.numel() else 0.0
    assert_close(got, ref, what, rtol=1e-4, atol=2e-5 * scale + 1e-7)


def dev_graph(ei, ew, dev):
    return ({k: v.to(dev) for k, v in ei.items()}, {k: (v.to(dev) if v is not None else None) for k, v in ew.items()})


# ---------------------------------------------------------------------------------------------
# propagation kernels
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("name,F", [("f1_fasta2", 32), ("f1_debruijn2", 128), ("f2_edge", 16), ("f5_fasta3", 64),
                                    ("f5_fasta3", 256), ("f3_bench", 48), ("f2_empty", 8), ("f4_cluster", 20)])
def test_spmm3_bitexact(pkg, cuda, name, F):
    from protgram_directgcn_amd import ops
    fx = load(name)
    ei, ew = graph(fx)
    N = int(fx["N"][0]) if name != "f4_cluster" else int(fx["subset"].size)
    x = torch.randn(N, F, generator=torch.Generator().manual_seed(3))
    ref = [oc.propagate(ei[k], x, ew[k]) for k in ("in", "out", "und")]
    dei, dew = dev_graph(ei, ew, cuda)
    g = pkg.graph.csr_from_coo(N, dei["in"], dew["in"], dei["out"], dew["out"], dei["und"], dew["und"])
    for fl in FLAG_VARIANTS:  # the CSR kernels (PG_FLAG_NO_NGRAM): bit-exact to the reference's propagate()
        Z = ops.spmm3(g, x.to(cuda), flags=fl | _lib_csr()).cpu()
        for k in range(3):
            assert torch.equal(Z[:, k * F:(k + 1) * F], ref[k]), (name, F, fl, k)
    if g.ngram is not None:  # all 20^n n-grams present (f1_*): through the COO boundary the tile kernel by default
        assert N == 400
        Z = ops.spmm3(g, x.to(cuda)).cpu()
        for k in range(3):
            assert_close(Z[:, k * F:(k + 1) * F], ref[k], f"{name} tile kernel slice {k}")


@pytest.mark.parametrize("name", ["f1_fasta2", "f1_debruijn2", "f2_edge", "f5_fasta3", "f6_pe1"])
def test_gpu_weights_and_fusednorm(pkg, cuda, name):
    """GPU-built propagation weights and the fused-normalisation SpMM."""
    from protgram_directgcn_amd import ops
    fx = load(name)
    N = int(fx["N"][0])
    g = pkg.build_propagation_csr(N, fx["src"], fx["dst"], fx["cnt"], device=cuda)
    e = g.edges3.cpu().numpy()
    rows = np.repeat(np.arange(N), np.diff(g.rowptr.cpu().numpy()))
    key = e[:, 0].astype(np.int64) * N + rows
    order = np.argsort(key)
    for j, k in enumerate(("in", "out", "und")):
        idx = fx[f"{k}_idx"]
        np.testing.assert_array_equal(key[order], idx[0] * N + idx[1])
        ulp = np.abs(e[order, 1 + j].astype(np.int64) - fx[f"{k}_val"].view(np.int32).astype(np.int64))
        assert ulp.max() <= (0 if k == "und" else 1), (k, ulp.max())
    # ... and bit-exact against the IEEE closed form (correctly rounded sqrt: pg::sqrt_rn)
    from test_host import _closed_form
    _, _, wcf = _closed_form(g.raw.cpu().numpy(), g.node_norm.cpu().numpy(), g.rowptr.cpu().numpy())
    for j, k in enumerate(("in", "out", "und")):
        assert np.array_equal(e[:, 1 + j], wcf[k].view(np.int32)), k
    # fused-norm SpMM == SpMM over the materialised weights, bit for bit; == oracle on those weights
    F = 32
    x = torch.randn(N, F, generator=torch.Generator().manual_seed(4)).to(cuda)
    for fl in FLAG_VARIANTS:
        Z0 = ops.spmm3(g, x, flags=fl | _lib_csr())
        Z1 = ops.spmm3(g, x, fused=True, flags=fl)
        assert torch.equal(Z0, Z1), fl
    src_idx = torch.from_numpy(e[:, 0].astype(np.int64))
    ei = torch.stack([src_idx, torch.from_numpy(rows)])
    for j in range(3):
        w = torch.from_numpy(e[:, 1 + j].copy().view(np.float32))
        ref = oc.propagate(ei, x.cpu(), w)
        assert torch.equal(Z0[:, j * F:(j + 1) * F].cpu(), ref)


@pytest.mark.parametrize("name,F", [("f1_fasta2", 32), ("f3_bench", 16), ("f5_fasta3", 64)])
def test_spmm3_transpose_matches_autograd(pkg, cuda, name, F):
    from protgram_directgcn_amd import ops
    fx = load(name)
    ei, ew = graph(fx)
    N = int(fx["N"][0])
    x = torch.randn(N, F, generator=torch.Generator().manual_seed(5), requires_grad=True)
    Gs = torch.randn(N, 3 * F, generator=torch.Generator().manual_seed(6))
    Z = torch.cat([oc.propagate(ei[k], x, ew[k]) for k in ("in", "out", "und")], 1)
    (Z * Gs).sum().backward()
    dei, dew = dev_graph(ei, ew, cuda)
    g = pkg.graph.csr_from_coo(N, dei["in"], dew["in"], dei["out"], dew["out"], dei["und"], dew["und"])
    for fl in FLAG_VARIANTS:
        dX = ops.spmm3_t(g, Gs.to(cuda), flags=fl)
        assert_grad_close(dX, x.grad, f"{name} dX flags={fl}")


def test_schedule_does_not_change_results(pkg, cuda):
    """The CSR kernels' locality schedule changes no bit (n-gram plan off: it has no schedule)."""
    import dataclasses
    from protgram_directgcn_amd import ops
    N, s, d, c = pkg.synth.de_bruijn_edges(3)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda, ngram_alphabet=None)
    assert g.row_order is not None and g.ngram is None
    g0 = dataclasses.replace(g, row_order=None)
    x = torch.randn(N, 64, device=cuda)
    for fl in FLAG_VARIANTS:
        assert torch.equal(ops.spmm3(g, x, flags=fl), ops.spmm3(g0, x, flags=fl))
        assert torch.equal(ops.spmm3(g, x, fused=True, flags=fl), ops.spmm3(g0, x, flags=fl))
    G = torch.randn(N, 192, device=cuda)
    assert torch.equal(ops.spmm3_t(g, G), ops.spmm3_t(g0, G))


def test_spmm_deterministic(pkg, cuda):
    from protgram_directgcn_amd import ops
    N, s, d, c = pkg.synth.de_bruijn_edges(3)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    x = torch.randn(N, 64, device=cuda)
    Z0 = ops.spmm3(g, x)
    for _ in range(3):
        assert torch.equal(ops.spmm3(g, x), Z0)
    G = torch.randn(N, 192, device=cuda)
    assert torch.equal(ops.spmm3_t(g, G), ops.spmm3_t(g, G))


# ---------------------------------------------------------------------------------------------
# layer and model vs the reference's golden vectors
# ---------------------------------------------------------------------------------------------
def _layer_from_fixture(pkg, fx, tag, dev):
    fin, fout, nn_, vec = (int(v) for v in fx[f"{tag}_cfg"])
    layer = pkg.DirectGCNLayer(fin, fout, nn_, bool(vec))
    layer.load_state_dict(params(fx, f"{tag}_p"))
    return layer.to(dev)


@pytest.mark.parametrize("name,tag", [("f1_fasta2", "L"), ("f1_debruijn2", "L"), ("f2_edge", "L"), ("f2_edge", "L2"),
                                      ("f2_empty", "L"), ("f3_bench", "L"), ("f4_cluster", "L"), ("f4_cluster", "S"),
                                      ("f4_cluster", "V"), ("f5_fasta3", "L")])
def test_layer_forward_backward_vs_reference(pkg, cuda, name, tag):
    fx = load(name)
    ei, ew = graph(fx)
    dei, dew = dev_graph(ei, ew, cuda)
    layer = _layer_from_fixture(pkg, fx, tag, cuda)
    x = t(fx[f"{tag}_x"]).to(cuda).requires_grad_(True)
    orig = t(fx[f"{tag}_orig"]).to(cuda) if f"{tag}_orig" in fx else None
    y = layer(x, dei["in"], dew["in"], dei["out"], dew["out"], dei["und"], dew["und"], orig)
    assert_close(y, fx[f"{tag}_y"], f"{name}/{tag} y")
    if f"{tag}_R" in fx:
        (y * t(fx[f"{tag}_R"]).to(cuda)).sum().backward()
        assert_grad_close(x.grad, fx[f"{tag}_gx"], f"{name}/{tag} grad x")
        for k, p in layer.named_parameters():
            g = p.grad if p.grad is not None else torch.zeros_like(p)
            assert_grad_close(g, fx[f"{tag}_g:{k}"], f"{name}/{tag} grad {k}")


def _model_from_fixture(pkg, fx, dev, prefix="M_p"):
    cfg = fx["M_cfg"]
    dims, (N, C, n, ogd) = [int(v) for v in cfg[:-4]], [int(v) for v in cfg[-4:]]
    m = pkg.ProtGramDirectGCN(dims, N, C, n, ogd, 512, 0.5, True)
    m.load_state_dict(params(fx, prefix))
    return m.to(dev), dims, N, n, ogd


@pytest.mark.parametrize("name", ["f1_fasta2", "f3_bench", "f6_pe1"])
def test_model_forward_backward_vs_reference(pkg, cuda, name):
    fx = load(name)
    ei, ew = graph(fx)
    dei, dew = dev_graph(ei, ew, cuda)
    m, dims, N, n, ogd = _model_from_fixture(pkg, fx, cuda)
    m.eval()
    x = t(fx["M_x"]).to(cuda).requires_grad_(True)
    data = pkg.Data(x=x, edge_index_in=dei["in"], edge_weight_in=dew["in"], edge_index_out=dei["out"],
                    edge_weight_out=dew["out"], edge_index_undirected_norm=dei["und"],
                    edge_weight_undirected_norm=dew["und"])
    lp, emb = m(data)
    assert_close(lp, fx["M_logp"], f"{name} log_probs")
    assert_close(emb, fx["M_emb"], f"{name} embeddings")
    ((lp * t(fx["M_R1"]).to(cuda)).sum() + (emb * t(fx["M_R2"]).to(cuda)).sum()).backward()
    assert_grad_close(x.grad, fx["M_gx"], f"{name} grad x")
    for k, p in m.named_parameters():
        g = p.grad if p.grad is not None else torch.zeros_like(p)
        assert_grad_close(g, fx[f"M_g:{k}"], f"{name} grad {k}")


def test_training_steps_vs_reference(pkg, cuda):
    """Two steps of the reference's full-batch loop (trainer :91-100; eval-mode dropout, see fixture)."""
    import torch.nn.functional as F
    fx = load("f1_fasta2")
    ei, ew = graph(fx)
    dei, dew = dev_graph(ei, ew, cuda)
    m, dims, N, n, ogd = _model_from_fixture(pkg, fx, cuda)
    m.eval()
    data = pkg.Data(x=t(fx["M_x"]).to(cuda), edge_index_in=dei["in"], edge_weight_in=dew["in"],
                    edge_index_out=dei["out"], edge_weight_out=dew["out"], edge_index_undirected_norm=dei["und"],
                    edge_weight_undirected_norm=dew["und"])
    y = t(fx["M_train_y"]).to(cuda)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=0.0)
    losses = []
    for _ in range(len(fx["M_train_loss"])):
        opt.zero_grad()
        out, _ = m(data=data)
        loss = F.nll_loss(out, y) + 1e-7 * sum(p.norm(2).pow(2) for p in m.parameters() if p.requires_grad)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    np.testing.assert_allclose(losses, fx["M_train_loss"], rtol=1e-5)
    ref = params(fx, "M_train_p")
    for k, v in m.state_dict().items():
        assert_grad_close(v, ref[k], f"param after 2 steps {k}")


def test_debruijn3_layer_samples(pkg, cuda):
    fx = load("f5_debruijn3")
    N, s, d, c = pkg.synth.de_bruijn_edges(3)
    layer = pkg.DirectGCNLayer(64, 64, N, True)
    layer.load_state_dict(params(fx, "L_p"))
    layer = layer.to(cuda)
    x = torch.randn(N, 64, generator=torch.Generator().manual_seed(1234)).to(cuda)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    with torch.no_grad():
        y = layer.fused_forward(x, g)  # n-gram tile propagation (g.ngram)
        y_f = layer.fused_forward(x, g, fused_norm=True)  # CSR kernel with in-kernel weights
    assert g.ngram is not None
    assert_close(y, y_f, "n-gram tile vs fused-norm CSR layer")
    assert_close(y[t(fx["L_rows"]).to(cuda)], fx["L_y_rows"], "3-gram sampled rows")
    np.testing.assert_allclose(y.double().sum(0).cpu().numpy(), fx["L_colsum"], rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("n,F", [(4, 128)])
def test_full_size_4gram_layer_vs_oracle(pkg, cuda, n, F):
    """BASELINE config size (4-gram, F=128): full forward vs the oracle on the same inputs, plus
    size-independent properties (linearity of the propagation, CSR-vs-fused identity)."""
    from protgram_directgcn_amd import ops
    N, s, d, c = pkg.synth.de_bruijn_edges(n)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
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
    with torch.no_grad():
        y = layer.fused_forward(xd, g)
        a, b = torch.randn(2).tolist()
        x2 = torch.randn(N, F, device=cuda)
        Z1, Z2 = ops.spmm3(g, xd), ops.spmm3(g, x2)
        Z12 = ops.spmm3(g, a * xd + b * x2)
        assert_close(Z12, a * Z1 + b * Z2, "linearity", rtol=1e-4, atol=1e-4)
    # oracle on the reference-order matrices rebuilt from our (GPU) weights: equal up to sqrt ulps
    e = g.edges3.cpu().numpy()
    rows = torch.from_numpy(np.repeat(np.arange(N), np.diff(g.rowptr.cpu().numpy())))
    ei = torch.stack([torch.from_numpy(e[:, 0].astype(np.int64)), rows])
    w = [torch.from_numpy(e[:, 1 + j].copy().view(np.float32)) for j in range(3)]
    p = {k: v.detach().cpu() for k, v in layer.state_dict().items()}
    with torch.no_grad():
        y_ref = oc.layer_forward(p, x, ei, w[0], ei, w[1], ei, w[2])
    assert_close(y, y_ref, "4-gram layer")
    Z = ops.spmm3(g, xd, flags=_lib_csr())  # the CSR kernel: bit-exact
    Zn = ops.spmm3(g, xd)  # the n-gram tile kernel (g.ngram): within fp32 summation-order rounding
    assert g.ngram is not None
    for j in range(3):
        ref = oc.propagate(ei, x, w[j])
        assert torch.equal(Z[:, j * F:(j + 1) * F].cpu(), ref), j
        assert_close(Zn[:, j * F:(j + 1) * F], ref, f"n-gram tile propagation {j}")


@pytest.mark.parametrize("n,F,drop", [(2, 16, 0.0), (2, 48, 0.3), (3, 64, 0.0), (3, 128, 0.5), (3, 256, 0.2),
                                      (4, 32, 0.1)])
def test_ngram_mid_kernel_vs_csr(pkg, cuda, monkeypatch, n, F, drop):
    """The middle-tile forward (pg_spmm3_ngram_mid_f32, the default n-gram kernel for F % 16 == 0) against the
    bit-exact CSR kernel, on complete de Bruijn graphs and on graphs with a random share of the transitions dropped
    (zero plan slots), at F not served by the 4x4-block kernel; also called through the C-ABI with padded rows
    (ldx > F, ldz > 3F) that must stay untouched."""
    from protgram_directgcn_amd import _lib, ops
    N, s, d, c = pkg.synth.de_bruijn_edges(n)
    if drop:
        keep = np.random.default_rng(n * 1000 + F).random(s.size) >= drop
        s, d, c = s[keep], d[keep], c[keep]
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    assert g.ngram is not None and g.ngram.mplan is not None
    x = torch.randn(N, F, generator=torch.Generator().manual_seed(7)).to(cuda)
    lib = ops.load_library()
    hits = []
    real = lib.pg_spmm3_ngram_mid_f32
    monkeypatch.setattr(lib, "pg_spmm3_ngram_mid_f32", lambda *a: hits.append(1) or real(*a))
    Z = ops.spmm3(g, x)
    assert hits, "the middle-tile kernel did not run"
    Zc = ops.spmm3(g, x, flags=_lib_csr())
    assert_close(Z, Zc, f"mid kernel n={n} F={F} drop={drop}")
    if F in (64, 128, 256):
        Zb = ops.spmm3(g, x, flags=ops.default_flags() | _lib.PG_FLAG_NGRAM_BLOCK4)
        assert_close(Zb, Zc, f"4x4-block kernel n={n} F={F}")
    # raw C-ABI call on padded rows
    xp = torch.randn(N, F + 16, generator=torch.Generator().manual_seed(8)).to(cuda)
    xp[:, :F] = x
    Zp = torch.full((N, 3 * F + 32), 7.0, device=cuda)
    ng = g.ngram
    torch.cuda.synchronize()
    rc = real(ng.K, ng.n, N, ops._p(ng.mplan), ops._p(xp), xp.stride(0), F, None, ops._p(Zp), Zp.stride(0),
              ops.default_flags(), ops._stream(xp))
    assert rc == 0, rc
    torch.cuda.synchronize()
    assert torch.equal(Zp[:, :3 * F], Z)  # same kernel, same order: the same bits
    assert bool((Zp[:, 3 * F:] == 7.0).all())
    # shapes it does not take answer PG_ERR_UNSUPPORTED (the caller falls back), never launch
    assert real(ng.K, ng.n, N, ops._p(ng.mplan), ops._p(xp), xp.stride(0), F + 8, None, ops._p(Zp), Zp.stride(0),
                ops.default_flags(), ops._stream(xp)) == _lib.PG_ERR_UNSUPPORTED


@pytest.mark.parametrize("n,F,drop", [(2, 16, 0.0), (3, 64, 0.3), (3, 128, 0.0), (4, 32, 0.1), (4, 128, 0.0)])
def test_ngram_mid_kernel_bf16(pkg, cuda, monkeypatch, n, F, drop):
    """The bf16 middle-tile kernel (pg_spmm3_ngram_mid_bf16, bf16 mode's default on complete n-gram graphs) computes
    the fp32 kernel's sums on the exactly widened bf16 rows and rounds each once: it equals bf16(fp32 middle-tile
    kernel on x.float()) bit for bit, and the bf16 CSR kernel within one bf16 rounding; the middle-range variant
    (pg_spmm3_ngram_mid_rows_bf16) gives the same rows in middle-major order; padded rows stay untouched."""
    from protgram_directgcn_amd import ops
    N, s, d, c = pkg.synth.de_bruijn_edges(n)
    if drop:
        keep = np.random.default_rng(n * 1000 + F).random(s.size) >= drop
        s, d, c = s[keep], d[keep], c[keep]
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    xb = torch.randn(N, F, generator=torch.Generator().manual_seed(9)).to(torch.bfloat16).to(cuda)
    lib = ops.load_library()
    hits = []
    real = lib.pg_spmm3_ngram_mid_bf16
    monkeypatch.setattr(lib, "pg_spmm3_ngram_mid_bf16", lambda *a: hits.append(1) or real(*a))
    Zb = ops.spmm3(g, xb)
    assert hits and Zb.dtype == torch.bfloat16, "the bf16 middle-tile kernel did not run"
    Zf = ops.spmm3(g, xb.float())
    assert torch.equal(Zb, Zf.to(torch.bfloat16))
    Zc = ops.spmm3(g, xb, flags=_lib_csr())  # bf16 CSR kernel: fp32 sums in CSR order, one rounding
    diff = (Zb.float() - Zc.float()).abs()
    assert bool((diff <= 2.0 ** -7 * Zc.float().abs() + 1e-6).all()), float(diff.max())
    ng = g.ngram
    nm = N // (ng.K * ng.K)
    m0, m1 = nm // 3, nm // 3 + max(1, nm // 4)
    Zr = ops.spmm3_middles(g, xb, m0, m1)
    M_ = torch.arange(m0, m1).view(-1, 1, 1)
    a_ = torch.arange(ng.K).view(1, -1, 1)
    b_ = torch.arange(ng.K).view(1, 1, -1)
    rows = (a_ * (N // ng.K) + M_ * ng.K + b_).reshape(-1).to(cuda)
    assert torch.equal(Zr, Zb[rows])
    xp = torch.zeros(N, F + 8, dtype=torch.bfloat16, device=cuda)
    xp[:, :F] = xb
    Zp = torch.full((N, 3 * F + 4), 7.0, dtype=torch.bfloat16, device=cuda)
    torch.cuda.synchronize()
    rc = real(ng.K, ng.n, N, ops._p(ng.mplan), ops._p(xp), xp.stride(0), F, ops._p(Zp), Zp.stride(0),
              ops.default_flags(), ops._stream(xp))
    assert rc == 0, rc
    torch.cuda.synchronize()
    assert torch.equal(Zp[:, :3 * F], Zb) and bool((Zp[:, 3 * F:] == 7.0).all())


@pytest.mark.parametrize("F,H,C", [(128, 64, 20), (128, 64, 32), (128, 64, 1), (32, 16, 5), (256, 128, 50), (16, 8, 400),
                                   (34, 17, 3), (12, 6, 1)])
def test_head_kernel_vs_torch(pkg, cuda, F, H, C):
    import torch.nn.functional as Fn
    from protgram_directgcn_amd import ops
    g = torch.Generator().manual_seed(F * 1000 + C)
    M = 1000
    h = torch.randn(M, F, generator=g)
    h[5] = 0.0  # zero row: emb = 0 / (0 + eps)
    W1, b1 = torch.randn(H, F, generator=g) * 0.2, torch.randn(H, generator=g) * 0.1
    W2, b2 = torch.randn(C, H, generator=g) * 0.2, torch.randn(C, generator=g) * 0.1
    z = Fn.relu(h @ W1.t() + b1)
    lp_ref = Fn.log_softmax(z @ W2.t() + b2, dim=-1)
    emb_ref = h / (torch.norm(h, p=2, dim=1, keepdim=True) + 1e-12)
    lp, emb = ops.head(h.to(cuda), W1.to(cuda), b1.to(cuda), W2.to(cuda), b2.to(cuda), 1e-12)
    assert_close(lp, lp_ref, "log_probs")
    assert_close(emb, emb_ref, "emb")


@pytest.mark.parametrize("name", ["f1_fasta2", "f3_bench", "f6_pe1"])
def test_model_inference_path_vs_reference(pkg, cuda, name):
    """eval + no_grad: the extract_gcn_node_embeddings path (models_utils.py:265-273), fused head kernel."""
    fx = load(name)
    ei, ew = graph(fx)
    dei, dew = dev_graph(ei, ew, cuda)
    m, dims, N, n, ogd = _model_from_fixture(pkg, fx, cuda)
    m.eval()
    data = pkg.Data(x=t(fx["M_x"]).to(cuda), edge_index_in=dei["in"], edge_weight_in=dew["in"],
                    edge_index_out=dei["out"], edge_weight_out=dew["out"], edge_index_undirected_norm=dei["und"],
                    edge_weight_undirected_norm=dew["und"])
    with torch.no_grad():
        lp, emb = m(data)
    assert_close(lp, fx["M_logp"], f"{name} log_probs (no_grad)")
    assert_close(emb, fx["M_emb"], f"{name} embeddings (no_grad)")


@pytest.mark.parametrize("M,Fin,Fout,proj,vec,rows", [(1000, 128, 128, False, True, False), (777, 64, 128, True, True, True),
                                                      (300, 32, 16, False, False, False), (513, 20, 12, True, True, False),
                                                      (129, 16, 40, True, True, True), (64, 128, 96, False, True, True),
                                                      (31, 128, 128, False, True, False), (4097, 64, 128, False, True, False),
                                                      (2050, 128, 128, False, False, False), (700, 128, 128, True, True, False),
                                                      (1500, 64, 128, True, True, False), (17, 128, 128, False, True, False), (1, 128, 128, False, True, False),
                                                      (5, 128, 128, False, False, False),
                                                      (8200, 128, 128, False, True, False), (4111, 128, 128, True, True, False)])
def test_dense_kernel_variants_vs_float64(pkg, cuda, M, Fin, Fout, proj, vec, rows):
    """pg_directgcn_dense_f32 (the split-bf16 W-stationary kernels where their shape applies -- flags 0 -- and the
    tiled fp32 kernel, PG_FLAG_DENSE_TILED; pre-gated operands) against the same formula in float64. Pre-gated: the
    operand is s_q * Z_q (what pg_spmm3_gated_f32 stores) with PG_FLAG_DENSE_PREGATED."""
    from protgram_directgcn_amd import ops
    from protgram_directgcn_amd._lib import PG_FLAG_DENSE_A_CACHED, PG_FLAG_DENSE_TILED, PG_FLAG_NO_XCD_REMAP
    g = torch.Generator().manual_seed(M + Fin + Fout)
    Ntot = M + 37
    Z = torch.randn(M, 3 * Fin, generator=g)
    xres = torch.randn(M, Fin, generator=g)
    prm = {k: torch.randn(Fout, Fin, generator=g) * 0.1 for k in ("W_main_in", "W_main_out", "W_undirected", "W_shared")}
    for k in ("b_main_in", "b_dir_shared_in", "b_main_out", "b_dir_shared_out", "b_undirected", "b_undirected_shared"):
        prm[k] = torch.randn(Fout, generator=g) * 0.1
    gate = 0 if vec else 1
    for k in ("C_in", "C_out", "C_directed", "C_undirected", "C_all"):
        prm[k] = torch.rand((Ntot, 1) if vec else (1,), generator=g) + 0.5
    const = torch.randn(Ntot, Fout, generator=g) if vec else None
    r = torch.randperm(Ntot, generator=g)[:M] if rows else None
    W_res = torch.randn(Fout, Fin, generator=g) * 0.1 if proj else None
    b_res = torch.randn(Fout, generator=g) * 0.1 if proj else None
    if not proj and Fin != Fout:
        xres = None
    # float64 reference
    d = {k: v.double() for k, v in prm.items()}
    idx = r if r is not None else torch.arange(M)
    gv = (lambda k: d[k][idx]) if vec else (lambda k: d[k].expand(M, 1))
    s = [gv("C_all") * gv("C_directed") * gv("C_in"), gv("C_all") * gv("C_directed") * gv("C_out"),
         gv("C_all") * gv("C_undirected")]
    Wk = [d["W_main_in"] + d["W_shared"], d["W_main_out"] + d["W_shared"], d["W_undirected"] + d["W_shared"]]
    bk = [d["b_main_in"] + d["b_dir_shared_in"], d["b_main_out"] + d["b_dir_shared_out"],
          d["b_undirected"] + d["b_undirected_shared"]]
    Zd = Z.double()
    y = sum(s[k] * (Zd[:, k * Fin:(k + 1) * Fin] @ Wk[k].t() + bk[k]) for k in range(3))
    if const is not None:
        y = y + const.double()[idx]
    if xres is not None:
        y = y + (xres.double() @ W_res.double().t() + b_res.double() if proj else xres.double())
    y = torch.nn.functional.leaky_relu(y, 0.01)
    dv = {k: v.to(cuda) for k, v in prm.items()}
    for fl in (0, PG_FLAG_DENSE_A_CACHED, PG_FLAG_DENSE_TILED, PG_FLAG_NO_XCD_REMAP | PG_FLAG_DENSE_TILED,
               PG_FLAG_NO_XCD_REMAP):
        out = ops.layer_dense(Z.to(cuda), dv, gate, rows=None if r is None else r.to(cuda),
                              constant=None if const is None else const.to(cuda),
                              res_x=None if xres is None else xres.to(cuda),
                              W_res=None if W_res is None else W_res.to(cuda),
                              b_res=None if b_res is None else b_res.to(cuda), act=True, flags=fl)
        assert_close(out, y.float(), f"dense flags={fl}", rtol=2e-5, atol=2e-5)
    sf = [v.float() for v in s]  # fp32 gates -> the pre-gated operand
    Zg = torch.cat([Z[:, k * Fin:(k + 1) * Fin] * sf[k] for k in range(3)], 1)
    for fl, pre in ((0, True), (PG_FLAG_DENSE_TILED, True), (0, False), (PG_FLAG_DENSE_TILED, False)):
        out = ops.layer_dense((Zg if pre else Z).to(cuda), dv, gate, rows=None if r is None else r.to(cuda),
                              constant=None if const is None else const.to(cuda),
                              res_x=None if xres is None else xres.to(cuda),
                              W_res=None if W_res is None else W_res.to(cuda),
                              b_res=None if b_res is None else b_res.to(cuda), act=True, flags=fl, pregated=pre)
        assert_close(out, y.float(), f"dense flags={fl} pregated={pre}", rtol=2e-5, atol=2e-5)


@pytest.mark.parametrize("M,vec", [(1, True), (5, True), (17, False), (700, True), (2050, True), (8200, False),
                                   (40_000, True)])
def test_dense_dma_interleave_bitexact(pkg, cuda, M, vec):
    """The default dense_x3p_kernel<.., IL = true> (the next-but-one tile's LDS-DMA pieces issued between the MFMA
    k-steps) against PG_FLAG_DENSE_NO_IL (all at the top of the iteration) moves only instruction issue: the same bits, for full and partial tiles, vector and scalar gates,
    pre-gated operands, the identity residual and none, and the n-gram row map (pg_directgcn_dense_ngram_rows_f32)."""
    from protgram_directgcn_amd import ops
    from protgram_directgcn_amd._lib import PG_FLAG_DENSE_NO_IL
    Z, xres, prm, const, _, _, _, _ = _dense_case(M, 128, 128, False, vec, False, 1000 + M)
    dv = {k: v.to(cuda) for k, v in prm.items()}
    gate = 0 if vec else 1
    c = None if const is None else const.to(cuda)
    base = ops.default_flags()
    for pre in (False, True):
        for res in (xres.to(cuda), None):
            a = ops.layer_dense(Z.to(cuda), dv, gate, constant=c, res_x=res, act=True, flags=base, pregated=pre)
            b = ops.layer_dense(Z.to(cuda), dv, gate, constant=c, res_x=res, act=True, flags=base | PG_FLAG_DENSE_NO_IL,
                                pregated=pre)
            assert torch.equal(a, b), (M, vec, pre, res is None)
    if vec and M % 400 == 0 or M == 40_000:
        Kn1 = 20 ** 3  # 4-gram rows of middles 0 .. M/400 - 1, residual read and output written at the global rows
        N = 20 ** 4
        X = torch.randn(N, 128, generator=torch.Generator().manual_seed(3)).to(cuda)
        Zm = Z.to(cuda)
        cm = torch.randn(M, 128, generator=torch.Generator().manual_seed(4)).to(cuda)
        pm = {k: (v[:M] if v.dim() and v.size(0) >= M and k.startswith("C_") else v) for k, v in dv.items()}
        outs = []
        for fl in (base, base | PG_FLAG_DENSE_NO_IL):
            Y = torch.full((N, 128), 7.0, device=cuda)
            ops.layer_dense_ngram_rows(Zm, pm, 0, Kn1, 0, constant=cm, res_x=X, map_res=True, out=Y, map_out=True,
                                       act=True, flags=fl)
            outs.append(Y)
        assert torch.equal(outs[0], outs[1])


def _dense_case(M, Fin, Fout, proj, vec, rows, seed):
    g = torch.Generator().manual_seed(seed)
    Ntot = M + 37
    Z = torch.randn(M, 3 * Fin, generator=g)
    xres = torch.randn(M, Fin, generator=g)
    prm = {k: torch.randn(Fout, Fin, generator=g) * 0.1 for k in ("W_main_in", "W_main_out", "W_undirected", "W_shared")}
    for k in ("b_main_in", "b_dir_shared_in", "b_main_out", "b_dir_shared_out", "b_undirected", "b_undirected_shared"):
        prm[k] = torch.randn(Fout, generator=g) * 0.1
    for k in ("C_in", "C_out", "C_directed", "C_undirected", "C_all"):
        prm[k] = torch.rand((Ntot, 1) if vec else (1,), generator=g) + 0.5
    const = torch.randn(Ntot, Fout, generator=g) if vec else None
    r = torch.randperm(Ntot, generator=g)[:M] if rows else None
    W_res = torch.randn(Fout, Fin, generator=g) * 0.1 if proj else None
    b_res = torch.randn(Fout, generator=g) * 0.1 if proj else None
    if not proj and Fin != Fout:
        xres = None
    dY = torch.randn(M, Fout, generator=g)
    return Z, xres, prm, const, r, W_res, b_res, dY


@pytest.mark.parametrize("M,Fin,Fout,proj,vec,rows", [(1000, 128, 128, False, True, False), (777, 64, 128, True, True, True),
                                                      (300, 32, 16, False, False, False), (513, 20, 12, True, True, False),
                                                      (129, 16, 40, True, True, True), (64, 128, 96, False, True, True),
                                                      (5000, 32, 32, False, True, False), (300, 18, 10, True, True, False),
                                                      (257, 7, 5, True, True, False), (100, 13, 30, False, True, True),
                                                      (64, 6, 9, True, False, False), (2000, 256, 256, False, True, False),
                                                      (1500, 128, 256, False, True, True), (20, 128, 128, False, True, False)])
def test_dense_backward_vs_float64(pkg, cuda, M, Fin, Fout, proj, vec, rows):
    """Autograd of the fused dense layer (pg_directgcn_dense_bwd_f32: the MFMA kernels, or its any-shape kernels
    when F_in / F_out are not multiples of 4) against float64 autograd of protgram_directgcn.py:100-133 + residual
    + leaky_relu."""
    _dense_backward_check(pkg, cuda, M, Fin, Fout, proj, vec, rows)


def _layer_drop_keep(seed: int, M: int, F: int, p: float):
    """The fused layer dropout's draw restated on the host (pg_common.h, drop_hash): element e = m F + j is kept
    when the top 24 bits of murmur3's 32-bit finalizer of (e * 0x9E3779B1 + seed_lo) ^ seed_hi reach p 2^24."""
    e = np.arange(M * F, dtype=np.uint64)
    x = ((e * np.uint64(0x9E3779B1) + np.uint64(seed & 0xFFFFFFFF)) & np.uint64(0xFFFFFFFF)) ^ np.uint64(seed >> 32)
    for sh, mul in ((16, 0x85EBCA6B), (13, 0xC2B2AE35), (16, None)):
        x ^= x >> np.uint64(sh)
        if mul is not None:
            x = (x * np.uint64(mul)) & np.uint64(0xFFFFFFFF)
    thr = int(p * 16777216.0 + 0.5)
    return torch.from_numpy((x >> np.uint64(8)) >= np.uint64(thr)).view(M, F)


@pytest.mark.parametrize("M,Fin,Fout,proj,vec,rows", [(1000, 128, 128, False, True, False), (777, 64, 128, True, True, True),
                                                      (64, 128, 96, False, True, True), (300, 18, 10, True, True, False),
                                                      (2000, 256, 256, False, True, False)])
def test_dense_fused_dropout_vs_float64(pkg, cuda, M, Fin, Fout, proj, vec, rows):
    """The layer dropout fused into the dense epilogue (drop = (p, seed), every forward kernel: the pipelined and
    32-row split-bf16 kernels and the tiled one) and its gradient read off the stored output (pg::act_grad, every
    dgrad kernel incl. the any-shape one): the same float64 autograd check with the kernel's mask restated on the
    host, forward included (dropped elements exactly 0)."""
    _dense_backward_check(pkg, cuda, M, Fin, Fout, proj, vec, rows, drop=0.5 if M % 2 else 0.3)


def _dense_backward_check(pkg, cuda, M, Fin, Fout, proj, vec, rows, drop=0.0):
    from protgram_directgcn_amd import ops
    Z, xres, prm, const, r, W_res, b_res, dY = _dense_case(M, Fin, Fout, proj, vec, rows, 7 * M + Fin)
    seed = 0x0123_4567_89AB_CDEF + M
    gate = 0 if vec else 1
    # float64 reference through autograd
    d = {k: v.double().requires_grad_(True) for k, v in prm.items()}
    Zd = Z.double().requires_grad_(True)
    xd = xres.double().requires_grad_(True) if xres is not None else None
    cd = const.double().requires_grad_(True) if const is not None else None
    Wrd = W_res.double().requires_grad_(True) if proj else None
    brd = b_res.double().requires_grad_(True) if proj else None
    idx = r if r is not None else torch.arange(M)
    gv = (lambda k: d[k][idx]) if vec else (lambda k: d[k].expand(M, 1))
    s = [gv("C_all") * gv("C_directed") * gv("C_in"), gv("C_all") * gv("C_directed") * gv("C_out"),
         gv("C_all") * gv("C_undirected")]
    Wk = [d["W_main_in"] + d["W_shared"], d["W_main_out"] + d["W_shared"], d["W_undirected"] + d["W_shared"]]
    bk = [d["b_main_in"] + d["b_dir_shared_in"], d["b_main_out"] + d["b_dir_shared_out"],
          d["b_undirected"] + d["b_undirected_shared"]]
    y = sum(s[k] * (Zd[:, k * Fin:(k + 1) * Fin] @ Wk[k].t() + bk[k]) for k in range(3))
    if cd is not None:
        y = y + cd[idx]
    if xd is not None:
        y = y + (xd @ Wrd.t() + brd if proj else xd)
    y = torch.nn.functional.leaky_relu(y, 0.01)
    if drop > 0:
        keep = _layer_drop_keep(seed, M, Fout, drop)
        y = y * keep.double() / (1.0 - drop)
    (y * dY.double()).sum().backward()
    # device path
    dv = {k: v.to(cuda).requires_grad_(True) for k, v in prm.items()}
    Zg = Z.to(cuda).requires_grad_(True)
    xg = xres.to(cuda).requires_grad_(True) if xres is not None else None
    cg = const.to(cuda).requires_grad_(True) if const is not None else None
    Wrg = W_res.to(cuda).requires_grad_(True) if proj else None
    brg = b_res.to(cuda).requires_grad_(True) if proj else None
    dr = (drop, torch.tensor([seed], dtype=torch.int64, device=cuda)) if drop > 0 else None
    out = ops.LayerDense.apply(Zg, xg, cg, Wrg, brg, None if r is None else r.to(cuda), gate, True, 0.01, dr,
                               *[dv[k] for k in ops._DENSE_KEYS])
    assert_close(out, y.detach().float(), "forward", rtol=2e-5, atol=2e-5)
    if drop > 0:
        assert torch.equal(out.detach().cpu() == 0, ~keep), "dropped elements"
    out.backward(dY.to(cuda))
    assert_grad_close(Zg.grad, Zd.grad, "dZ")
    for k in ops._DENSE_KEYS:
        assert_grad_close(dv[k].grad, d[k].grad, f"d{k}")
    if xg is not None:
        assert_grad_close(xg.grad, xd.grad, "dres_x")
    if cg is not None:
        assert_grad_close(cg.grad, cd.grad, "dconstant")
    if proj:
        assert_grad_close(Wrg.grad, Wrd.grad, "dW_res")
        assert_grad_close(brg.grad, brd.grad, "db_res")


@pytest.mark.parametrize("M,rows", [(1000, False), (3001, True)])
def test_dense_backward_f32mfma_wgrad_vs_float64(pkg, cuda, monkeypatch, M, rows):
    """The fp32-MFMA weight gradient (PG_FLAG_WGRAD_F32MFMA: wgrad_kernel instead of the default split-bf16
    wgrad_x3_kernel at these shapes) through the same float64 autograd check."""
    from protgram_directgcn_amd._lib import PG_FLAG_WGRAD_F32MFMA
    monkeypatch.setenv("PG_SPMM_FLAGS", hex(PG_FLAG_WGRAD_F32MFMA))
    test_dense_backward_vs_float64(pkg, cuda, M, 128, 128, False, True, rows)


def test_dense_backward_deterministic(pkg, cuda):
    from protgram_directgcn_amd import ops
    Z, xres, prm, const, r, W_res, b_res, dY = _dense_case(20000, 128, 128, False, True, False, 3)
    dv = {k: v.to(cuda) for k, v in prm.items()}
    Zg, dYg = Z.to(cuda), dY.to(cuda)
    Y = ops.layer_dense(Zg, dv, 0, res_x=xres.to(cuda), act=True)
    a = ops.layer_dense_backward(dYg, Zg, Y, dv, 0, res_x=xres.to(cuda), act=True)
    b = ops.layer_dense_backward(dYg, Zg, Y, dv, 0, res_x=xres.to(cuda), act=True)
    c = ops.layer_dense_backward(dYg, Zg, Y, dv, 0, res_x=xres.to(cuda), act=True, need_dZ=False)
    assert a is not None and c["dZ"] is None
    for k in ("dpre", "dZ", "dgate", "dB", "dbsum"):
        assert torch.equal(a[k], b[k]), k
        if k != "dZ":
            assert torch.equal(a[k], c[k]), k


_FLUSH = []


def _poison_allocator(dev, seed):
    """Allocate and free blocks of many sizes filled with random bits: the caching allocator hands them out again,
    and the caches go cold (the condition under which the round-4 bf16 dense backward's gate gradients varied)."""
    import os
    if os.environ.get("PG_POISON_MODE") == "flush":  # diagnostics: cold caches only, no reused blocks
        if not _FLUSH:
            _FLUSH.append(torch.empty(1 << 29, device=dev))
        _FLUSH[0].fill_(float(seed))
        torch.cuda.synchronize()
        return
    g = torch.Generator(device=dev).manual_seed(seed)
    keep = []
    for k in range(8, 25):
        for _ in range(2):
            t_ = torch.empty(1 << k, device=dev)
            t_.view(torch.int32).random_(generator=g)
            keep.append(t_)
    torch.cuda.synchronize()
    del keep


def test_dense_backward_bf16_deterministic(pkg, cuda):
    """bf16 twin of test_dense_backward_deterministic, with the allocator's blocks poisoned and the caches cold before
    each call: every output bit-identical over 12 calls (round 4: the lead n-tile's segment-0 gate partials of two
    rows in eight differed in the last bit in about half of such runs, while the kernel spilled registers to scratch;
    tools/r05_dgrad_bf16_probe.py)."""
    from protgram_directgcn_amd import ops
    Z, xres, prm, const, r, W_res, b_res, dY = _dense_case(20000, 128, 128, False, True, False, 3)
    dv = {k: v.to(cuda) for k, v in prm.items()}
    Zg, dYg, xg = Z.to(cuda).to(torch.bfloat16), dY.to(cuda).to(torch.bfloat16), xres.to(cuda).to(torch.bfloat16)
    packs = []
    Y = ops.layer_dense(Zg, dv, 0, res_x=xg, act=True, packs=packs)
    assert Y.dtype == torch.bfloat16 and len(packs) == 2
    ref = None
    for rep in range(12):
        _poison_allocator(cuda, rep)
        out = ops.layer_dense_backward(dYg, Zg, Y, dv, 0, res_x=xg, act=True, packs=packs)
        assert out is not None
        out = {k: v.clone() for k, v in out.items() if v is not None}
        if ref is None:
            ref = out
            continue
        for k in ("dpre", "dZ", "dgate", "dB", "dbsum"):
            assert torch.equal(out[k], ref[k]), (rep, k, int((out[k] != ref[k]).sum()))


@pytest.mark.parametrize("M,P,N", [(160000, 20, 64), (160000, 64, 128), (1000, 128, 384), (33, 4, 8), (0, 8, 8),
                                   (70001, 256, 132)])
def test_gemm_at_b_vs_float64(pkg, cuda, M, P, N):
    from protgram_directgcn_amd import ops
    g = torch.Generator().manual_seed(M + P + N)
    A, B = torch.randn(M, P, generator=g), torch.randn(M, N, generator=g)
    C, cs = ops.gemm_at_b(A.to(cuda), B.to(cuda))
    assert_grad_close(C, A.double().t() @ B.double(), "A^T B")
    assert_grad_close(cs, A.double().sum(0), "colsum")
    C2, cs2 = ops.gemm_at_b(A.to(cuda), B.to(cuda))
    assert torch.equal(C, C2) and torch.equal(cs, cs2)


def test_training_steps_under_autocast_and_gradscaler(pkg, cuda):
    """The reference trainer's exact loop (protgram_directgcn_trainer.py:91-100: autocast + GradScaler +
    L2 term + Adam): the model's Functions compute in fp32 inside autocast, so the steps match the fp32
    fixture (the GradScaler factor is a power of two: exact)."""
    import torch.nn.functional as F
    fx = load("f1_fasta2")
    ei, ew = graph(fx)
    dei, dew = dev_graph(ei, ew, cuda)
    m, dims, N, n, ogd = _model_from_fixture(pkg, fx, cuda)
    m.eval()
    data = pkg.Data(x=t(fx["M_x"]).to(cuda), edge_index_in=dei["in"], edge_weight_in=dew["in"],
                    edge_index_out=dei["out"], edge_weight_out=dew["out"], edge_index_undirected_norm=dei["und"],
                    edge_weight_undirected_norm=dew["und"])
    y = t(fx["M_train_y"]).to(cuda)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=0.0)
    scaler = torch.amp.GradScaler("cuda", enabled=True)
    losses = []
    for _ in range(len(fx["M_train_loss"])):
        opt.zero_grad()
        with torch.amp.autocast("cuda", enabled=True):
            out, emb = m(data=data)
            assert out.dtype == torch.float32 and emb.dtype == torch.float32
            loss = F.nll_loss(out, y) + 1e-7 * sum(p.norm(2).pow(2) for p in m.parameters() if p.requires_grad)
        scaler.scale(loss).backward()
        scaler.step(opt)
        scaler.update()
        losses.append(loss.item())
    np.testing.assert_allclose(losses, fx["M_train_loss"], rtol=1e-5)
    ref = params(fx, "M_train_p")
    for k, v in m.state_dict().items():
        assert_grad_close(v, ref[k], f"param after 2 autocast steps {k}")


# ------------------------------------------------------------------------------------------------
# bf16 mode (config 5): bf16 storage, fp32 accumulation
# ------------------------------------------------------------------------------------------------
def _bf16_graphs(pkg, cuda):
    fx = load("f5_fasta3")
    ei, ew = graph(fx)
    dei, dew = dev_graph(ei, ew, cuda)
    g1 = pkg.graph.csr_from_coo(int(fx["N"].item()), dei["in"], dew["in"], dei["out"], dew["out"], dei["und"], dew["und"],
                                cache=False)
    N, s, d, c = pkg.synth.de_bruijn_edges(3)
    g2 = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    return [("fasta3", g1, ei, ew), ("debruijn3", g2, None, None)]


@pytest.mark.parametrize("F", [16, 64, 128, 256])
def test_spmm3_bf16_exact(pkg, cuda, F):
    """pg_spmm3_bf16 / pg_spmm3t_bf16 against bf16(fp32 propagation of the same bf16 inputs) -- the fp32
    kernels, bit-exact to the reference's propagate, on the widened input: equal up to one bf16 rounding
    step (the bf16 kernels accumulate with FMA)."""
    from protgram_directgcn_amd import ops
    for name, g, _, _ in _bf16_graphs(pkg, cuda):
        x = torch.randn(g.n_rows, F, generator=torch.Generator().manual_seed(F)).to(cuda).to(torch.bfloat16)
        Z = ops.spmm3(g, x)
        assert Z.dtype == torch.bfloat16
        ref32 = ops.spmm3(g, x.float(), flags=_lib_csr())
        _assert_bf16_round(Z, ref32, (name, F))
        G = torch.randn(g.n_rows, 3 * F, generator=torch.Generator().manual_seed(F + 1)).to(cuda).to(torch.bfloat16)
        dX = ops.spmm3_t(g, G)
        assert dX.dtype == torch.bfloat16
        _assert_bf16_round(dX, ops.spmm3_t(g, G.float()), (name, F, "T"))


def _assert_bf16_round(got, ref32, what):
    """got (bf16) within one bf16 ulp of the fp32 reference (plus fp32-level slack near zero), and equal to
    its RNE rounding on the vast majority of entries."""
    g, r = got.float(), ref32.float()
    ulp = torch.where(r != 0, 2.0 ** (torch.floor(torch.log2(r.abs())) - 7), torch.zeros_like(r))
    scale = float(r.abs().max())
    bad = (g - r).abs() > ulp + 1e-6 * scale
    assert not bool(bad.any()), (what, int(bad.sum()))
    same = float((got == ref32.to(torch.bfloat16)).float().mean())
    assert same > 0.99, (what, same)


def _lib_csr():
    from protgram_directgcn_amd._lib import PG_FLAG_NO_NGRAM
    return PG_FLAG_NO_NGRAM


@pytest.mark.parametrize("M,Fin,Fout,proj,vec,rows", [(1000, 128, 128, False, True, False), (777, 64, 128, True, True, True),
                                                      (300, 32, 16, False, False, False), (5000, 256, 256, False, True, False),
                                                      (129, 16, 40, True, True, True), (64, 128, 96, False, True, True)])
def test_dense_bf16_vs_float64(pkg, cuda, M, Fin, Fout, proj, vec, rows):
    """pg_directgcn_dense_bf16 against float64 math on the same bf16 operands (bf16(s*Z), bf16 weights):
    what remains is fp32 accumulation and the final bf16 rounding."""
    from protgram_directgcn_amd import ops
    Z, xres, prm, const, r, W_res, b_res, _ = _dense_case(M, Fin, Fout, proj, vec, rows, 11 * M + Fin)
    Zb = Z.to(torch.bfloat16)
    xb = xres.to(torch.bfloat16) if xres is not None else None
    gate = 0 if vec else 1
    dv = {k: v.to(cuda) for k, v in prm.items()}
    out = ops.layer_dense(Zb.to(cuda), dv, gate, rows=None if r is None else r.to(cuda),
                          constant=None if const is None else const.to(cuda), res_x=None if xb is None else xb.to(cuda),
                          W_res=None if W_res is None else W_res.to(cuda), b_res=None if b_res is None else b_res.to(cuda),
                          act=True)
    assert out.dtype == torch.bfloat16
    bf = lambda t: t.to(torch.bfloat16).double()  # noqa: E731
    idx = r if r is not None else torch.arange(M)
    gv = (lambda k: prm[k][idx]) if vec else (lambda k: prm[k].expand(M, 1))
    s = [gv("C_all") * gv("C_directed") * gv("C_in"), gv("C_all") * gv("C_directed") * gv("C_out"),
         gv("C_all") * gv("C_undirected")]
    Wk = [prm["W_main_in"] + prm["W_shared"], prm["W_main_out"] + prm["W_shared"], prm["W_undirected"] + prm["W_shared"]]
    bk = [prm["b_main_in"] + prm["b_dir_shared_in"], prm["b_main_out"] + prm["b_dir_shared_out"],
          prm["b_undirected"] + prm["b_undirected_shared"]]
    Zf = Zb.float()
    y = sum(bf(s[k] * Zf[:, k * Fin:(k + 1) * Fin]) @ bf(Wk[k]).t() + s[k].double() * bk[k].double() for k in range(3))
    if const is not None:
        y = y + const.double()[idx]
    if xb is not None:
        y = y + (xb.double() @ bf(W_res).t() + b_res.double() if proj else xb.double())
    y = torch.nn.functional.leaky_relu(y, 0.01)
    got = out.double().cpu()
    err = (got - y).abs()
    tol = 2.0 ** -8 * y.abs() + 1e-5 * float(y.abs().max())
    assert not bool((err > tol).any()), f"max |d| {float(err.max()):.3e}"


def test_model_bf16_forward_close_to_fp32(pkg, cuda):
    """bf16 mode end to end (3-gram, dims [64,64,64]): log-probs and embeddings stay within bf16-level error
    of the fp32 model."""
    N, s, d, c = pkg.synth.de_bruijn_edges(3)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    torch.manual_seed(0)
    m = pkg.ProtGramDirectGCN([64, 64, 64], N, 20, 3, 0, 512, 0.5, True).to(cuda).eval()
    x = torch.randn(N, 64, generator=torch.Generator().manual_seed(1234)).to(cuda)
    data = pkg.Data(x=x, graph=g)
    with torch.no_grad():
        lp32, e32 = m(data)
        m.compute_dtype = torch.bfloat16
        lp16, e16 = m(data)
    assert lp16.dtype == torch.float32 and e16.dtype == torch.float32
    assert float((lp16 - lp32).abs().max()) < 0.05 * float(lp32.abs().max())
    assert float((e16 - e32).abs().max()) < 0.02


@pytest.mark.parametrize("F,H,C", [(128, 64, 20), (256, 128, 20), (64, 32, 5)])
def test_head_bf16_input_equals_widened(pkg, cuda, F, H, C):
    from protgram_directgcn_amd import ops
    g = torch.Generator().manual_seed(F + C)
    h = torch.randn(3001, F, generator=g).to(torch.bfloat16).to(cuda)
    W1, b1 = (torch.randn(H, F, generator=g) * 0.1).to(cuda), (torch.randn(H, generator=g) * 0.1).to(cuda)
    W2, b2 = (torch.randn(C, H, generator=g) * 0.1).to(cuda), (torch.randn(C, generator=g) * 0.1).to(cuda)
    lp, emb = ops.head(h, W1, b1, W2, b2, 1e-12)
    lp32, emb32 = ops.head(h.float(), W1, b1, W2, b2, 1e-12)
    assert torch.equal(lp, lp32) and torch.equal(emb, emb32)


@pytest.mark.parametrize("M,Fin,Fout,proj,vec,rows", [(1000, 128, 128, False, True, False), (777, 64, 128, True, True, True),
                                                      (300, 32, 16, False, False, False), (5000, 256, 256, False, True, False),
                                                      (129, 16, 40, True, True, True), (300, 20, 12, True, True, False)])
def test_dense_backward_bf16_vs_float64(pkg, cuda, M, Fin, Fout, proj, vec, rows, drop=0.0):
    """bf16-mode autograd of the dense layer (pg_directgcn_dense_bwd_bf16; the last case, F not a multiple of 8,
    runs the fp32 backward kernels on widened copies) against float64 autograd on the same bf16-valued activations, with the leaky_relu
    mask taken from the device's own (bf16) forward output -- near y = 0 a float64 forward can pick the
    other slope. Tolerance: bf16 rounding of dpre, s*Z and the stored gradients, 2% of each gradient's max."""
    from protgram_directgcn_amd import ops
    Z, xres, prm, const, r, W_res, b_res, dY = _dense_case(M, Fin, Fout, proj, vec, rows, 13 * M + Fin)
    Zb, dYb = Z.to(torch.bfloat16), dY.to(torch.bfloat16)
    xb = xres.to(torch.bfloat16) if xres is not None else None
    gate = 0 if vec else 1
    d = {k: v.double().requires_grad_(True) for k, v in prm.items()}
    Zd = Zb.double().requires_grad_(True)
    xd = xb.double().requires_grad_(True) if xb is not None else None
    cd = const.double().requires_grad_(True) if const is not None else None
    Wrd = W_res.double().requires_grad_(True) if proj else None
    brd = b_res.double().requires_grad_(True) if proj else None
    idx = r if r is not None else torch.arange(M)
    gv = (lambda k: d[k][idx]) if vec else (lambda k: d[k].expand(M, 1))
    s = [gv("C_all") * gv("C_directed") * gv("C_in"), gv("C_all") * gv("C_directed") * gv("C_out"),
         gv("C_all") * gv("C_undirected")]
    Wk = [d["W_main_in"] + d["W_shared"], d["W_main_out"] + d["W_shared"], d["W_undirected"] + d["W_shared"]]
    bk = [d["b_main_in"] + d["b_dir_shared_in"], d["b_main_out"] + d["b_dir_shared_out"],
          d["b_undirected"] + d["b_undirected_shared"]]
    y = sum(s[k] * (Zd[:, k * Fin:(k + 1) * Fin] @ Wk[k].t() + bk[k]) for k in range(3))
    if cd is not None:
        y = y + cd[idx]
    if xd is not None:
        y = y + (xd @ Wrd.t() + brd if proj else xd)
    dv = {k: v.to(cuda).requires_grad_(True) for k, v in prm.items()}
    Zg = Zb.to(cuda).requires_grad_(True)
    xg = xb.to(cuda).requires_grad_(True) if xb is not None else None
    cg = const.to(cuda).requires_grad_(True) if const is not None else None
    Wrg = W_res.to(cuda).requires_grad_(True) if proj else None
    brg = b_res.to(cuda).requires_grad_(True) if proj else None
    seed = 0x7EDC_BA98_7654_3210 + M
    dr = (drop, torch.tensor([seed], dtype=torch.int64, device=cuda)) if drop > 0 else None
    out = ops.LayerDense.apply(Zg, xg, cg, Wrg, brg, None if r is None else r.to(cuda), gate, True, 0.01, dr,
                               *[dv[k] for k in ops._DENSE_KEYS])
    assert out.dtype == torch.bfloat16
    o64 = out.detach().cpu().double()
    mask = torch.where(o64 > 0, 1.0, 0.01)
    if drop > 0:  # kept elements scaled, dropped ones exactly 0 (the device's mask against the host restatement)
        keep = _layer_drop_keep(seed, M, Fout, drop)
        assert not bool((o64[~keep] != 0).any()), "dropped elements"
        mask = mask * keep.double() / (1.0 - drop)
    (y * mask * dYb.double()).sum().backward()  # leaky_relu' from the device's forward output
    out.backward(dYb.to(cuda))
    assert Zg.grad.dtype == torch.bfloat16

    def close(got, ref, what):
        got, ref = got.detach().double().cpu(), ref.detach().double()
        err = (got - ref).abs()
        tol = 2e-2 * float(ref.abs().max()) + 2e-2 * ref.abs() + 1e-6
        assert not bool((err > tol).any()), f"{what}: max |d| {float(err.max()):.3e} vs max|ref| {float(ref.abs().max()):.3e}"

    close(Zg.grad, Zd.grad, "dZ")
    for k in ops._DENSE_KEYS:
        close(dv[k].grad, d[k].grad, f"d{k}")
    if xg is not None:
        close(xg.grad, xd.grad, "dres_x")
    if cg is not None:
        close(cg.grad, cd.grad, "dconstant")
    if proj:
        close(Wrg.grad, Wrd.grad, "dW_res")
        close(brg.grad, brd.grad, "db_res")


@pytest.mark.parametrize("M,Fin,Fout,proj,vec,rows", [(5000, 256, 256, False, True, False), (1000, 128, 256, True, True, True),
                                                      (300, 20, 12, True, True, False)])
def test_dense_fused_dropout_bf16_vs_float64(pkg, cuda, M, Fin, Fout, proj, vec, rows):
    """bf16 mode with the fused layer dropout (dense_bf16_kernel's epilogue; the bf16 dgrad kernel, or the fp32 ones on
    widened copies for F % 8 != 0), through the bf16 float64 autograd check."""
    test_dense_backward_bf16_vs_float64(pkg, cuda, M, Fin, Fout, proj, vec, rows, drop=0.5)


def test_model_bf16_training_step_close_to_fp32(pkg, cuda):
    """One bf16-mode training step (autocast + GradScaler loop of the trainer) vs the fp32 model: the loss
    agrees to bf16 precision and every parameter gradient points the same way (cosine > 0.99)."""
    import torch.nn.functional as F
    N, s, d, c = pkg.synth.de_bruijn_edges(3)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    x = torch.randn(N, 64, generator=torch.Generator().manual_seed(1234)).to(cuda)
    y = (torch.arange(N, device=cuda) // 400) % 20
    data = pkg.Data(x=x, graph=g)
    grads, losses = [], []
    for dt in (torch.float32, torch.bfloat16):
        torch.manual_seed(0)
        m = pkg.ProtGramDirectGCN([64, 128, 128, 128], N, 20, 3, 0, 512, 0.5, True).to(cuda).eval()
        m.compute_dtype = dt
        with torch.amp.autocast("cuda", enabled=True):
            lp, _ = m(data)
            loss = F.nll_loss(lp, y) + 1e-7 * sum(p.norm(2).pow(2) for p in m.parameters())
        loss.backward()
        losses.append(float(loss))
        grads.append({k: p.grad.detach().float().clone() for k, p in m.named_parameters()})
    assert abs(losses[0] - losses[1]) < 2e-2 * abs(losses[0])
    for k, g32 in grads[0].items():
        g16 = grads[1][k]
        cos = float((g32 * g16).sum() / (g32.norm() * g16.norm() + 1e-30))
        assert cos > 0.99, (k, cos)


def test_clustered_subgraphs_on_gpu(pkg, cuda):
    """Cluster-GCN path: the model on each built subgraph (prebuilt CSR in data.graph) equals the model on the
    same subgraph's COO fields, and the oracle with original_indices; one clustered_forward over the
    block-diagonal union equals the per-cluster forwards bit for bit."""
    from protgram_directgcn_amd import cluster
    N, s, d, c = pkg.synth.de_bruijn_edges(3)
    mats = og.build_matrices(N, s, d, c)
    ei = {k: v[0].to(cuda) for k, v in mats.items()}
    ew = {k: v[1].to(cuda) for k, v in mats.items()}
    order = pkg.graph.locality_schedule(N, torch.from_numpy(s).to(cuda), torch.from_numpy(d).to(cuda)).long()
    parts = cluster.range_clusters(N, cluster.cluster_count(N), order=order)
    x = torch.randn(N, 32, generator=torch.Generator().manual_seed(1234)).to(cuda)
    subs = cluster.build_subgraphs(N, parts, ei["in"], ew["in"], ei["out"], ew["out"], ei["und"], ew["und"], x)
    assert len(subs) == 16
    torch.manual_seed(0)
    m = pkg.ProtGramDirectGCN([32, 32, 16], N, 7, 3, 0, 512, 0.5, True).to(cuda).eval()
    with torch.no_grad():
        for p_ in m.parameters():
            if p_.dim() == 2 and p_.size(1) == 1:
                p_.uniform_(0.5, 1.5)
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    outs = []
    with torch.no_grad():
        for dd in subs[:5] + subs[-2:]:
            lp, emb = m(dd)
            coo = pkg.Data(x=dd.x, edge_index_in=dd.edge_index_in, edge_weight_in=dd.edge_weight_in,
                           edge_index_out=dd.edge_index_out, edge_weight_out=dd.edge_weight_out,
                           edge_index_undirected_norm=dd.edge_index_undirected_norm,
                           edge_weight_undirected_norm=dd.edge_weight_undirected_norm,
                           original_indices=dd.original_indices)
            lp2, emb2 = m(coo)
            assert torch.equal(lp, lp2) and torch.equal(emb, emb2)
            lpr, embr = oc.model_forward(sd, [32, 32, 16], dd.x.cpu(), dd.edge_index_in.cpu(), dd.edge_weight_in.cpu(),
                                         dd.edge_index_out.cpu(), dd.edge_weight_out.cpu(),
                                         dd.edge_index_undirected_norm.cpu(), dd.edge_weight_undirected_norm.cpu(),
                                         original_indices=dd.original_indices.cpu(), n_gram_len=3)
            assert_close(lp, lpr, "cluster log_probs")
            assert_close(emb, embr, "cluster emb")
        lp_all, emb_all = cluster.clustered_forward(m, subs)
        for dd in subs:
            lp, emb = m(dd)
            assert torch.equal(lp_all[dd.original_indices], lp) and torch.equal(emb_all[dd.original_indices], emb)


@pytest.mark.parametrize("amp", [False, True])
def test_train_step_matches_reference_loop(pkg, cuda, amp):
    """train.train_step (fused L2 value/gradient, gather nll, no host sync) against the reference trainer's
    loop (protgram_directgcn_trainer.py:91-100: nll_loss + l2_lambda * sum p.norm(2).pow(2), backward, step),
    3 steps, with and without autocast + GradScaler. SGD: parameter updates are linear in the gradients."""
    import torch.nn.functional as F
    from protgram_directgcn_amd import train
    N, s, d, c = pkg.synth.de_bruijn_edges(3)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    x = torch.randn(N, 64, generator=torch.Generator().manual_seed(1234)).to(cuda)
    y = (torch.arange(N, device=cuda) // 400) % 20
    data = pkg.Data(x=x, graph=g)
    lam = 1e-3
    runs = []
    for fused in (False, True):
        torch.manual_seed(0)
        m = pkg.ProtGramDirectGCN([64, 64, 64], N, 20, 3, 0, 512, 0.5, True).to(cuda).eval()
        opt = torch.optim.SGD(m.parameters(), lr=0.05)
        scaler = torch.amp.GradScaler("cuda", enabled=amp)
        losses = []
        for _ in range(3):
            if fused:
                losses.append(float(train.train_step(m, data, y, opt, l2_lambda=lam, scaler=scaler)))
            else:
                opt.zero_grad()
                with torch.amp.autocast("cuda", enabled=amp):
                    out, _ = m(data=data)
                    loss = F.nll_loss(out, y) + lam * sum(p.norm(2).pow(2) for p in m.parameters() if p.requires_grad)
                scaler.scale(loss).backward()
                scaler.step(opt)
                scaler.update()
                losses.append(float(loss))
        runs.append((losses, {k: v.detach().clone() for k, v in m.state_dict().items()}))
    np.testing.assert_allclose(runs[1][0], runs[0][0], rtol=2e-6)
    for k, v in runs[0][1].items():
        assert_grad_close(runs[1][1][k], v.cpu(), f"param {k}")


@pytest.mark.parametrize("amp,adam", [(False, True), (True, True), (False, False)])
def test_graphed_train_step_matches_eager(pkg, cuda, amp, adam):
    """train.GraphedTrainStep (the whole train_step captured as a HIP graph after its warm-up steps, then replayed):
    eight steps from the same start give the same losses and parameters, bit for bit, as eight eager train_step calls
    (dropout off, so both runs draw nothing): train.Adam with the folded L2 term, with and without GradScaler, and
    torch SGD with the L2 gradient added by pg_multi_axpy_f32 (its descriptor table built inside the capture, in the
    arena of train.prepare_capture; checked by train.check_deferred before the first replay)."""
    from protgram_directgcn_amd import train
    N, s, d, c = pkg.synth.de_bruijn_edges(3)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    x = torch.randn(N, 64, generator=torch.Generator().manual_seed(1234)).to(cuda)
    y = (torch.arange(N, device=cuda) // 400) % 20
    data = pkg.Data(x=x, graph=g)
    runs = []
    for graphed in (False, True):
        torch.manual_seed(0)
        m = pkg.ProtGramDirectGCN([64, 64, 64], N, 20, 3, 0, 512, 0.5, True).to(cuda).eval()
        opt = train.Adam(m.parameters(), lr=1e-3) if adam else torch.optim.SGD(m.parameters(), lr=1e-2)
        scaler = torch.amp.GradScaler("cuda", enabled=amp)
        if graphed:
            st = train.GraphedTrainStep(m, data, y, opt, l2_lambda=1e-3, scaler=scaler)
            st.CHECK = True
            losses = [float(st()) for _ in range(8)]
            assert st._graph is not None and st.failed is None, st.failed
            st.close()
        else:
            losses = [float(train.train_step(m, data, y, opt, l2_lambda=1e-3, scaler=scaler)) for _ in range(8)]
        runs.append((losses, {k: v.detach().clone() for k, v in m.state_dict().items()}))
    assert runs[0][0] == runs[1][0], runs[0][0]
    for k, v in runs[0][1].items():
        assert torch.equal(runs[1][1][k], v), k


@pytest.mark.parametrize("amp,adam", [(False, True), (True, True), (False, False)])
def test_graphed_train_step_follows_lr_schedule(pkg, cuda, amp, adam):
    """the reference loop's ReduceLROnPlateau (protgram_directgcn_trainer.py:84, :102) through
    train.fit around a captured step. The scheduler is forced to halve the learning rate after every epoch (patience
    0, a 99 % relative threshold no loss meets), so eight epochs run at eight learning rates: the GraphedTrainStep
    (captured after its warm-up steps, train.Adam reading lr from its device scalars; torch SGD captured again at
    every change) gives the same losses, learning rates and parameters, bit for bit, as eager train_step calls."""
    from protgram_directgcn_amd import train
    N, s, d, c = pkg.synth.de_bruijn_edges(3)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    x = torch.randn(N, 64, generator=torch.Generator().manual_seed(1234)).to(cuda)
    y = (torch.arange(N, device=cuda) // 400) % 20
    data = pkg.Data(x=x, graph=g)
    runs = []
    for graphed in (False, True):
        torch.manual_seed(0)
        m = pkg.ProtGramDirectGCN([64, 64, 64], N, 20, 3, 0, 512, 0.5, True).to(cuda).eval()
        opt = train.Adam(m.parameters(), lr=1e-2) if adam else torch.optim.SGD(m.parameters(), lr=5e-2)
        scaler = torch.amp.GradScaler("cuda", enabled=amp)
        sched = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, "min", patience=0, factor=0.5, threshold=0.99)
        if graphed:
            st = train.GraphedTrainStep(m, data, y, opt, l2_lambda=1e-3, scaler=scaler)
        else:
            st = lambda: train.train_step(m, data, y, opt, l2_lambda=1e-3, scaler=scaler)  # noqa: E731
        hist = train.fit(st, opt, 8, scheduler=sched, use_early_stopping=False)
        if graphed:
            assert st._graph is not None and st.failed is None
            # train.Adam: one capture, the replays read the refreshed device lr; SGD: captured again per change
            assert st.captures == (1 if adam else 8 - train.GraphedTrainStep.WARM), st.captures
            st.close()
        runs.append((hist, {k: v.detach().clone() for k, v in m.state_dict().items()}))
    lrs = [h["lr"][0] for h in runs[0][0]]
    # the first epoch sets the best loss; from then on the schedule acts every epoch
    assert lrs == [lrs[0]] + [lrs[0] * 0.5 ** i for i in range(7)], lrs
    assert runs[0][0] == runs[1][0], (runs[0][0], runs[1][0])
    for k, v in runs[0][1].items():
        assert torch.equal(runs[1][1][k], v), k


def test_graphed_train_step_bf16_input_refresh(pkg, cuda):
    """bf16 mode converts a step-invariant input once (ProtGramDirectGCN.bf16_input, cached by tensor and version); a
    captured step reads that cached copy, so GraphedTrainStep refreshes it before each replay: after new values are
    copied into data.x between replays, the replayed steps equal eager steps on the same inputs, bit for bit."""
    from protgram_directgcn_amd import train
    N, s, d, c = pkg.synth.de_bruijn_edges(3)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    x0 = torch.randn(N, 64, generator=torch.Generator().manual_seed(1234)).to(cuda)
    x1 = torch.randn(N, 64, generator=torch.Generator().manual_seed(99)).to(cuda)
    y = (torch.arange(N, device=cuda) // 400) % 20
    runs = []
    for graphed in (False, True):
        torch.manual_seed(0)
        m = pkg.ProtGramDirectGCN([64, 64, 64], N, 20, 3, 0, 512, 0.5, True).to(cuda).eval()
        m.compute_dtype = torch.bfloat16
        data = pkg.Data(x=x0.clone(), graph=g)
        opt = train.Adam(m.parameters(), lr=1e-3)
        st = train.GraphedTrainStep(m, data, y, opt) if graphed else (
            lambda: train.train_step(m, data, y, opt))  # noqa: E731
        losses = []
        for i in range(8):
            if i == 6:
                data.x.copy_(x1)  # new input values in place (the captured graph's address)
            losses.append(float(st()))
        if graphed:
            assert st._graph is not None
            st.close()
        runs.append((losses, {k: v.detach().clone() for k, v in m.state_dict().items()}))
    assert runs[0][0] == runs[1][0], runs
    assert runs[0][0][6] != runs[0][0][5]
    for k, v in runs[0][1].items():
        assert torch.equal(runs[1][1][k], v), k


def test_graphed_train_step_capture_failure_raises(pkg, cuda):
    """a step that cannot be captured (here: a host sync inside it) raises instead of silently
    running eager steps; eager_fallback=True keeps the old behaviour, with the reason in `failed`."""
    from protgram_directgcn_amd import train
    N, s, d, c = pkg.synth.de_bruijn_edges(2)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    x = torch.randn(N, 32, generator=torch.Generator().manual_seed(3)).to(cuda)
    y = (torch.arange(N, device=cuda) // 20) % 20
    data = pkg.Data(x=x, graph=g)
    torch.manual_seed(0)
    m = pkg.ProtGramDirectGCN([32, 32], N, 20, 2, 0, 512, 0.5, True).to(cuda).eval()
    opt = train.Adam(m.parameters(), lr=1e-3)

    class SyncingOpt(torch.optim.SGD):  # a host sync in the step: not capturable
        def step(self, closure=None):
            float(self.param_groups[0]["params"][0].sum())
            return super().step(closure)

    opt = SyncingOpt(m.parameters(), lr=1e-3)
    st = train.GraphedTrainStep(m, data, y, opt)
    for _ in range(train.GraphedTrainStep.WARM):
        st()
    with pytest.raises(RuntimeError, match="capture failed"):
        st()
    torch.cuda.synchronize()
    st2 = train.GraphedTrainStep(m, data, y, opt, eager_fallback=True)
    for _ in range(train.GraphedTrainStep.WARM + 2):
        loss = st2()
    assert st2.failed is not None and st2._graph is None and torch.isfinite(loss)


@pytest.mark.parametrize("amp", [False, True])
def test_train_step_adam_folded_l2_matches_reference_loop(pkg, cuda, amp):
    """train.train_step with train.Adam, where the L2 gradient 2*lambda*p rides in the Adam launch as extra weight
    decay (no separate gradient pass), against the reference loop with torch.optim.Adam (L2 term in the loss,
    weight_decay 0): 3 steps, with and without autocast + GradScaler."""
    import torch.nn.functional as F
    from protgram_directgcn_amd import train
    N, s, d, c = pkg.synth.de_bruijn_edges(3)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    x = torch.randn(N, 64, generator=torch.Generator().manual_seed(1234)).to(cuda)
    y = (torch.arange(N, device=cuda) // 400) % 20
    data = pkg.Data(x=x, graph=g)
    lam = 1e-3
    runs = []
    for ours in (False, True):
        torch.manual_seed(0)
        m = pkg.ProtGramDirectGCN([64, 64, 64], N, 20, 3, 0, 512, 0.5, True).to(cuda).eval()
        opt = train.Adam(m.parameters(), lr=1e-3) if ours else torch.optim.Adam(m.parameters(), lr=1e-3)
        scaler = torch.amp.GradScaler("cuda", enabled=amp)
        losses = []
        for _ in range(3):
            if ours:
                losses.append(float(train.train_step(m, data, y, opt, l2_lambda=lam, scaler=scaler)))
                assert getattr(opt, "_l2_extra", 0.0) == 0.0  # the fold is per call
            else:
                opt.zero_grad()
                with torch.amp.autocast("cuda", enabled=amp):
                    out, _ = m(data=data)
                    loss = F.nll_loss(out, y) + lam * sum(p.norm(2).pow(2) for p in m.parameters() if p.requires_grad)
                scaler.scale(loss).backward()
                scaler.step(opt)
                scaler.update()
                losses.append(float(loss))
        runs.append((losses, {k: v.detach().clone() for k, v in m.state_dict().items()}))
    np.testing.assert_allclose(runs[1][0], runs[0][0], rtol=1e-5)
    for k, v in runs[0][1].items():
        # Adam normalises each step to ~lr * sign(g): compare on that scale. An element whose gradient is within fp32
        # noise of zero (the data term and 2*lambda*p cancelling) can step the other way in one of the two summation
        # orders, by at most 2 lr per step; such elements must be rare
        err = (runs[1][1][k] - v).abs()
        assert float(err.max()) <= 3 * 2 * 1e-3 + 1e-6, (k, float(err.max()))
        assert int((err > 5e-5).sum()) <= max(1, err.numel() // 10000), (k, int((err > 5e-5).sum()))


def test_multi_tensor_helpers(pkg, cuda):
    from protgram_directgcn_amd import train
    g = torch.Generator().manual_seed(0)
    ts = [torch.randn(n, generator=g).to(cuda) for n in (1, 7, 65536, 65537, 300000)]
    ref = sum(float((t.double() ** 2).sum()) for t in ts)
    got = float(train.l2_sqsum(ts))
    assert abs(got - ref) <= 1e-5 * ref
    assert float(train.l2_sqsum(ts)) == got  # deterministic
    ps = [t.clone().requires_grad_(True) for t in ts]
    for p in ps:
        p.grad = torch.ones_like(p)
    train.add_l2_grad(ps, 0.25, scale=torch.tensor(4.0, device=cuda))
    for p, t in zip(ps, ts):
        assert torch.allclose(p.grad, 1 + 2.0 * t)


def test_fused_adam_matches_torch_adam(pkg, cuda):
    """train.Adam (one pg_adam_f32 launch) against torch.optim.Adam on identical gradients: 5 steps, two
    parameter groups, weight decay in one; then a GradScaler step with an inf gradient is skipped entirely."""
    from protgram_directgcn_amd import train
    g = torch.Generator().manual_seed(0)
    shapes = [(128, 128), (128,), (160000, 1), (70001,)]
    init = [torch.randn(s, generator=g).to(cuda) for s in shapes]
    grads = [[torch.randn(s, generator=g).to(cuda) * (10.0 ** -k) for s in shapes] for k in range(5)]
    ps_ref = [t.clone().requires_grad_(True) for t in init]
    ps_ours = [t.clone().requires_grad_(True) for t in init]
    groups = lambda ps: [{"params": ps[:2]}, {"params": ps[2:], "weight_decay": 0.01, "lr": 3e-3}]  # noqa: E731
    o_ref = torch.optim.Adam(groups(ps_ref), lr=1e-3)
    o_ours = train.Adam(groups(ps_ours), lr=1e-3)
    for gs in grads:
        for p, gg in zip(ps_ref, gs):
            p.grad = gg.clone()
        for p, gg in zip(ps_ours, gs):
            p.grad = gg.clone()
        o_ref.step()
        o_ours.step()
    for a, b in zip(ps_ours, ps_ref):
        d = (a.detach() - b.detach()).abs().max().item()
        assert d <= 1e-6 * max(1.0, b.detach().abs().max().item()), d
    for p in ps_ours:
        st = o_ours.state[p]
        assert set(st) == {"step", "exp_avg", "exp_avg_sq"} and float(st["step"]) == 5.0
    # GradScaler: an inf gradient skips the update and the step count, with no host sync in step()
    scaler = torch.amp.GradScaler("cuda")
    before = [p.detach().clone() for p in ps_ours]
    loss = sum((p * 1.0).sum() for p in ps_ours)
    o_ours.zero_grad()
    scaler.scale(loss).backward()
    ps_ours[0].grad[0, 0] = float("inf")
    scaler.step(o_ours)
    scaler.update()
    for p, b in zip(ps_ours, before):
        assert torch.equal(p.detach(), b)
    assert float(o_ours.state[ps_ours[0]]["step"]) == 5.0


def test_adam_bf16_deferred_gradient_matches_widened(pkg, cuda):
    """pg_adam_desc_t.gtype = 1 (ABI 4): a bf16 gradient filed through ops._DEFERRED_GRADS gives, bit for bit, the update
    of the same values widened to an fp32 .grad -- on the 16-B path, on a shape whose length is not a multiple of 4
    (the scalar tail) and on a gradient view that is not 8-B aligned (the scalar path), with weight decay,
    in one launch together with an fp32-gradient parameter; 3 steps."""
    from protgram_directgcn_amd import ops, train
    g = torch.Generator().manual_seed(5)
    shapes = [(1000, 64), (1001,), (70003,), (33, 7)]
    init = [torch.randn(s, generator=g).to(cuda) for s in shapes]
    gb = [[(torch.randn(s, generator=g) * 1e-2).to(cuda).to(torch.bfloat16) for s in shapes] for _ in range(3)]
    store = torch.zeros(70003 + 4, dtype=torch.bfloat16, device=cuda)  # a 4-B-offset view for shapes[2]
    ps_w = [torch.nn.Parameter(t.clone()) for t in init]
    ps_d = [torch.nn.Parameter(t.clone()) for t in init]
    o_w = train.Adam([{"params": ps_w[:2]}, {"params": ps_w[2:], "weight_decay": 0.01}], lr=1e-3)
    o_d = train.Adam([{"params": ps_d[:2]}, {"params": ps_d[2:], "weight_decay": 0.01}], lr=1e-3)
    for step in gb:
        for p, gg in zip(ps_w, step):
            p.grad = gg.float()
        o_w.step()
        try:
            for i, (p, gg) in enumerate(zip(ps_d, step)):
                if i == 3:
                    p.grad = gg.float()  # an fp32 gradient in the same launch
                elif i == 2:
                    view = store[2:2 + gg.numel()]
                    view.copy_(gg)
                    assert view.data_ptr() % 8 == 4
                    ops._DEFERRED_GRADS[p.data_ptr()] = view
                else:
                    ops._DEFERRED_GRADS[p.data_ptr()] = gg.contiguous()
            o_d.step()
        finally:
            ops._DEFERRED_GRADS.clear()
    for a, b in zip(ps_d, ps_w):
        assert torch.equal(a.detach(), b.detach())
        assert torch.equal(o_d.state[a]["exp_avg"], o_w.state[b]["exp_avg"])
        assert torch.equal(o_d.state[a]["exp_avg_sq"], o_w.state[b]["exp_avg_sq"])


def test_adam_checkpoint_round_trip_and_skipped_params(pkg, cuda, tmp_path):
    """train.Adam against torch.optim.Adam across a checkpoint loaded with map_location='cpu' (the step
    counters come back as host tensors), with parameters whose gradient is None on some steps (torch counts
    steps per parameter: a skipped parameter's bias correction stays behind)."""
    from protgram_directgcn_amd import train
    g = torch.Generator().manual_seed(1)
    shapes = [(64, 32), (32,), (1000, 1), (7,)]
    init = [torch.randn(s, generator=g).to(cuda) for s in shapes]
    ref = [t.clone().requires_grad_(True) for t in init]
    ours = [t.clone().requires_grad_(True) for t in init]
    opts = [torch.optim.Adam(ref, lr=1e-2), train.Adam(ours, lr=1e-2)]

    def do_step(skip):
        gs = [torch.randn(s, generator=g).to(cuda) for s in shapes]
        for i, (a, b) in enumerate(zip(ref, ours)):
            a.grad = None if i in skip else gs[i].clone()
            b.grad = None if i in skip else gs[i].clone()
        for o in opts:
            o.step()

    for skip in ((), (1,), (), (1, 3)):
        do_step(skip)
    torch.save({"ref": opts[0].state_dict(), "ours": opts[1].state_dict()}, tmp_path / "opt.pt")
    ck = torch.load(tmp_path / "opt.pt", map_location="cpu", weights_only=True)
    opts = [torch.optim.Adam(ref, lr=1e-2), train.Adam(ours, lr=1e-2)]
    opts[0].load_state_dict(ck["ref"])
    opts[1].load_state_dict(ck["ours"])
    for skip in ((2,), (), (0,)):
        do_step(skip)
    for a, b in zip(ours, ref):
        d = (a.detach() - b.detach()).abs().max().item()
        assert d <= 2e-6 * max(1.0, b.detach().abs().max().item()), d
        assert float(opts[1].state[a]["step"]) == float(opts[0].state[b]["step"])
        assert opts[1].state[a]["step"].device == a.device


@pytest.mark.gpu
@pytest.mark.parametrize("writer", ["torch_fused_adam", "pg_adam", "no_version_bump"])
def test_forward_sees_in_place_parameter_writes(pkg, cuda, writer):
    """Regression: packed weights are rebuilt on every forward, so parameter writes that leave the version
    counter alone (torch's fused Adam, raw kernels, .data copies) reach the next forward."""
    from protgram_directgcn_amd import train
    N, s, d, c = pkg.synth.de_bruijn_edges(2)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    x = torch.randn(N, 32, generator=torch.Generator().manual_seed(3)).to(cuda)
    torch.manual_seed(0)
    m = pkg.ProtGramDirectGCN([32, 32, 32], N, 5, 2, 0, 16, 0.5, True).to(cuda).eval()
    data = pkg.Data(x=x, graph=g)
    m(data)  # first forward: anything cached would be cached now
    if writer == "no_version_bump":
        with torch.no_grad():
            for p in m.parameters():
                p.data.mul_(1.5)
    else:
        opt = (torch.optim.Adam(m.parameters(), lr=1e-2, fused=True) if writer == "torch_fused_adam"
               else train.Adam(m.parameters(), lr=1e-2))
        lp, _ = m(data)
        lp.sum().backward()
        opt.step()
    lp, emb = m(data)
    torch.manual_seed(0)
    fresh = pkg.ProtGramDirectGCN([32, 32, 32], N, 5, 2, 0, 16, 0.5, True).to(cuda).eval()
    fresh.load_state_dict(m.state_dict())
    lp2, emb2 = fresh(data)
    assert torch.equal(lp, lp2) and torch.equal(emb, emb2)


@pytest.mark.gpu
@pytest.mark.parametrize("name,F", [("f1_fasta2", 32), ("f1_debruijn2", 128), ("f5_fasta3", 64)])
@pytest.mark.parametrize("vec", [True, False])
def test_spmm3_gated_bitexact(pkg, cuda, name, F, vec):
    """pg_spmm3_gated_f32 == the gates applied to pg_spmm3_f32's output with the same fp32 products
    ((c_all*c_dir)*c_in etc., then one rounding of s*Z), bit for bit."""
    from protgram_directgcn_amd import ops
    fx = load(name)
    ei, ew = graph(fx)
    N = int(fx["N"][0])
    dei, dew = dev_graph(ei, ew, cuda)
    g = pkg.graph.csr_from_coo(N, dei["in"], dew["in"], dei["out"], dew["out"], dei["und"], dew["und"])
    if not g.shared:
        pytest.skip("non-shared pattern")
    gen = torch.Generator().manual_seed(F)
    x = torch.randn(N, F, generator=gen).to(cuda)
    shape = (N, 1) if vec else (1,)
    prm = {k: (torch.rand(shape, generator=gen) + 0.5).to(cuda) for k in ("C_in", "C_out", "C_directed", "C_undirected",
                                                                          "C_all")}
    prm["W_main_in"] = torch.zeros(F, F, device=cuda)  # shape only
    fl = None
    Zg = ops.spmm3_gated(g, x, prm, 0 if vec else 1)
    if Zg is None:  # the middle-tile kernel (default on complete n-gram graphs) leaves the gates to the dense kernel
        from protgram_directgcn_amd import _lib
        assert ops._mid_ok(g, x, ops.default_flags())
        fl = ops.default_flags() | _lib.PG_FLAG_NGRAM_BLOCK4  # the 4x4-block tile kernel's gated store
        Zg = ops.spmm3_gated(g, x, prm, 0 if vec else 1, flags=fl)
    Z = ops.spmm3(g, x, flags=fl)
    cad = prm["C_all"] * prm["C_directed"]
    s = [cad * prm["C_in"], cad * prm["C_out"], prm["C_all"] * prm["C_undirected"]]
    ref = torch.cat([Z[:, k * F:(k + 1) * F] * s[k].view(-1, 1) for k in range(3)], 1)
    assert torch.equal(Zg, ref)


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_take_large_wide_rows(pkg, cuda):
    """graph.take on a > 1 GiB result of 512-B rows (the halo inputs' take(x_full, perm) shape at 5-gram, F = 128)
    equals the host gather bit for bit: pieces are sized by bytes, so no piece reaches the size at which ROCm
    torch's index gather was seen to drop a result's tail (tools/gather_probe.py)."""
    rows = (1 << 30) // 512 + 300_000  # 1.15 GiB of result
    gen = torch.Generator().manual_seed(7)
    t = torch.randn(rows, 128, generator=gen)
    idx = torch.randperm(rows, generator=gen)
    got = pkg.graph.take(t.to(cuda), idx.to(cuda))
    assert got.shape == (rows, 128)
    assert torch.equal(got.cpu(), t[idx])


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,F", [(torch.float32, 128), (torch.bfloat16, 128), (torch.float32, 5), (torch.bfloat16, 6)])
def test_rows_gather_scatter(pkg, cuda, dtype, F):
    """pg_rows_gather / pg_rows_scatter (the middle partition's exchange data movement) == torch indexing, bit for
    bit, on 16-B-vector rows and on rows of 4-B words only, with a strided source."""
    from protgram_directgcn_amd import ops
    gen = torch.Generator().manual_seed(F)
    src = torch.randn(5000, F + 4, generator=gen).to(dtype).to(cuda)[:, :F]  # row stride != row width
    idx = torch.randperm(5000, generator=gen)[:3001].to(cuda)
    got = ops.rows_gather(src, idx)
    assert torch.equal(got, src[idx])
    dst = torch.zeros(5000, F, dtype=dtype, device=cuda)
    ops.rows_scatter(got, idx, dst)
    ref = torch.zeros_like(dst)
    ref[idx] = src[idx]
    assert torch.equal(dst, ref)
    assert ops.rows_gather(src, idx[:0]).shape == (0, F)
    # the public calls validate their indices: out of range / repeated scatter rows raise on the host
    with pytest.raises(IndexError):
        ops.rows_gather(src, torch.tensor([0, 5000], device=cuda))
    with pytest.raises(IndexError):
        ops.rows_gather(src, torch.tensor([-1], device=cuda))
    with pytest.raises(IndexError):
        ops.rows_scatter(got[:2], torch.tensor([0, 5000], device=cuda), dst)
    with pytest.raises(ValueError):
        ops.rows_scatter(got[:2], torch.tensor([7, 7], device=cuda), dst)


@pytest.mark.gpu
@pytest.mark.parametrize("n,m0,nm", [(4, 37, 13), (3, 0, 20)])
def test_dense_ngram_rows_map(pkg, cuda, n, m0, nm):
    """pg_directgcn_dense_ngram_rows_f32 (the middle partition's dense launch): over the middle-major rows of the
    middles [m0, m0 + nm), reading the residual and writing the output at the global n-gram rows a.M.b, it equals
    layer_dense on the gathered residual rows bit for bit, and writes no other row."""
    from protgram_directgcn_amd import ops
    K, F = 20, 128
    N, Kn1 = K ** n, K ** (n - 1)
    gen = torch.Generator().manual_seed(n)
    M_ = torch.arange(m0, m0 + nm).view(-1, 1, 1)
    a = torch.arange(K).view(1, -1, 1)
    b = torch.arange(K).view(1, 1, -1)
    rows = (a * Kn1 + M_ * K + b).reshape(-1).to(cuda)  # middle-major order
    R = rows.numel()
    Z = torch.randn(R, 3 * F, generator=gen).to(cuda)
    X = torch.randn(N, F, generator=gen).to(cuda)
    prm = {k: torch.randn(F, F, generator=gen).mul_(0.05).to(cuda)
           for k in ("W_main_in", "W_main_out", "W_undirected", "W_shared")}
    for k in ("b_main_in", "b_dir_shared_in", "b_main_out", "b_dir_shared_out", "b_undirected", "b_undirected_shared"):
        prm[k] = torch.randn(F, generator=gen).mul_(0.1).to(cuda)
    for k in ("C_in", "C_out", "C_directed", "C_undirected", "C_all"):
        prm[k] = (torch.rand(R, 1, generator=gen) + 0.5).to(cuda)
    const = torch.randn(R, F, generator=gen).to(cuda)
    ref = ops.layer_dense(Z, prm, 0, constant=const, res_x=X[rows], act=True)
    Y = torch.full((N, F), float("nan"), device=cuda)
    got = ops.layer_dense_ngram_rows(Z, prm, 0, Kn1, m0, constant=const, res_x=X, map_res=True, out=Y, map_out=True,
                                     act=True)
    torch.cuda.synchronize()
    assert got is Y
    assert torch.equal(Y[rows], ref)
    keep = torch.ones(N, dtype=torch.bool, device=cuda)
    keep[rows] = False
    assert bool(torch.isnan(Y[keep]).all())
    compact = ops.layer_dense_ngram_rows(Z, prm, 0, Kn1, m0, constant=const, res_x=X, map_res=True, act=True)
    assert torch.equal(compact, ref)  # residual mapped, output compact (the last layer)
    with pytest.raises(Exception):  # a partial middle is refused on the host
        ops.layer_dense_ngram_rows(Z[:399], prm, 0, Kn1, m0, res_x=X, map_res=True, act=True)


# ---------------------------------------------------------------------------------------------
# PropagateDense (round 5): the span dense backward + the off-diagonal transposed kernel
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("n,F,res", [(3, 64, True), (3, 128, True), (3, 128, False), (4, 128, True), (3, 256, True)])
def test_propagate_dense_span_backward(pkg, cuda, n, F, res):
    """A layer whose input needs its gradient trains through ops.PropagateDense: the input's gradient (off-diagonal
    transposed middle-tile kernel accumulated into E = diagonal term + identity residual) and every parameter gradient
    against the Propagate3 + LayerDense path (4x4-block transposed kernel, autograd's residual add), and at n = 3 the
    input gradient against float64 on the host; E itself against its definition."""
    from protgram_directgcn_amd import ops
    N, s, d, c = pkg.synth.de_bruijn_edges(n)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    torch.manual_seed(3)
    conv = pkg.DirectGCNLayer(F, F, N, True).to(cuda)
    with torch.no_grad():
        gen = torch.Generator().manual_seed(9)
        for name, p in conv.named_parameters():
            if name.startswith("C_"):
                p.copy_((torch.rand(p.shape, generator=gen) + 0.5).to(cuda))
            elif "bias" in name:
                p.copy_((torch.rand(p.shape, generator=gen) * 0.2 - 0.1).to(cuda))
    x0 = torch.randn(N, F, generator=torch.Generator().manual_seed(4)).to(cuda)
    w = torch.randn(N, F, generator=torch.Generator().manual_seed(5)).to(cuda)
    assert ops.PropagateDense.supports(g, x0, F, x0 if res else None, None, None, False)
    got = {}
    for span in (True, False):
        ops.SPAN_BACKWARD = span
        try:
            x = x0.clone().requires_grad_(True)
            for p in conv.parameters():
                p.grad = None
            y = conv.fused_forward(x, g, res_x=x if res else None, act=True)
            (y * w).sum().backward()
            got[span] = {"x": x.grad.clone(), **{k: p.grad.clone() for k, p in conv.named_parameters()}}
            if span:
                y_span = y.detach()
        finally:
            ops.SPAN_BACKWARD = True
    for k, v in got[False].items():
        assert_grad_close(got[True][k], v, f"span vs 4x4 path: {k}")
    if n == 3:  # the input's gradient in float64: A^T (s * (dpre W'))-style chain through the oracle's autograd
        p64 = {k: v.detach().double().cpu().requires_grad_(False) for k, v in conv.state_dict().items()}
        m = og.build_matrices(N, s, d, c)
        xr = x0.double().cpu().requires_grad_(True)
        ei = [m[k][0] for k in ("in", "out", "und")]
        ew = [m[k][1].double() for k in ("in", "out", "und")]
        yr = oc.layer_forward(p64, xr, ei[0], ew[0], ei[1], ew[1], ei[2], ew[2])
        # leaky_relu with the GPU forward's slopes: a pre-activation within rounding of 0 would otherwise take the
        # other slope in float64 and move a whole neighbourhood of input-gradient rows (one such entry at F = 128)
        slope = torch.where(y_span.cpu() > 0, 1.0, ops.LEAKY_SLOPE).double()
        yr = ((yr + xr) if res else yr) * slope
        (yr * w.double().cpu()).sum().backward()
        assert_grad_close(got[True]["x"], xr.grad, "span input gradient vs float64")
    # E against its definition on the same dZ / dpre
    Z = ops.spmm3(g, x0)
    prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in conv._dense_params())))
    Y = ops.layer_dense(Z, prm, 0, constant=conv.constant.detach(), res_x=x0 if res else None, act=True)
    out = ops.layer_dense_backward(w, Z, Y, prm, 0, act=True, span=(g.ngram.diag3(), res))
    ref = (out["dZ"].view(N, 3, F) * g.ngram.diag3().unsqueeze(2)).sum(1) + (out["dpre"] if res else 0.0)
    assert_grad_close(out["E"], ref, "E = sum_q Wdiag_q dZ_q (+ dpre)")


@pytest.mark.parametrize("n,F,res", [(3, 64, True), (3, 64, False), (4, 128, True), (3, 256, True)])
def test_propagate_dense_bf16_backward(pkg, cuda, n, F, res):
    """bf16 mode, a layer whose input needs its gradient (config 5's layers 2 and 3): ops.PropagateDense runs the
    bf16 dense backward, then the 4x4-block transposed kernel ACCUMULATING into the identity residual's dpre (one fp32
    sum, one rounding). Against the Propagate3 + LayerDense path (the same transposed kernel into a fresh buffer, then
    autograd's bf16 add): every parameter gradient bit-identical (the same dense backward); the input gradient within
    one bf16 rounding (unit roundoff 2^-8) of the float64 sum of its two terms (dpre + A^T dZ on the same dZ), and
    within the old path's two roundings of it."""
    from protgram_directgcn_amd import ops
    N, s, d, c = pkg.synth.de_bruijn_edges(n)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    torch.manual_seed(3)
    conv = pkg.DirectGCNLayer(F, F, N, True).to(cuda)
    with torch.no_grad():
        gen = torch.Generator().manual_seed(9)
        for name, p in conv.named_parameters():
            if name.startswith("C_"):
                p.copy_((torch.rand(p.shape, generator=gen) + 0.5).to(cuda))
            elif "bias" in name:
                p.copy_((torch.rand(p.shape, generator=gen) * 0.2 - 0.1).to(cuda))
    x0 = torch.randn(N, F, generator=torch.Generator().manual_seed(4)).to(cuda).to(torch.bfloat16)
    w = torch.randn(N, F, generator=torch.Generator().manual_seed(5)).to(cuda).to(torch.bfloat16)
    assert ops.PropagateDense.supports(g, x0, F, x0 if res else None, None, None, False)
    lib = ops.load_library()
    got = {}
    for span in (True, False):
        ops.SPAN_BACKWARD = span
        try:
            x = x0.clone().requires_grad_(True)
            for p in conv.parameters():
                p.grad = None
            y = conv.fused_forward(x, g, res_x=x if res else None, act=True)
            assert y.dtype == torch.bfloat16
            y.backward(w)
            got[span] = {"x": x.grad.clone(), **{k: p.grad.clone() for k, p in conv.named_parameters()}}
        finally:
            ops.SPAN_BACKWARD = True
    for k, v in got[False].items():
        if k != "x":
            assert torch.equal(got[True][k], v), k
    # the input gradient from its two bf16 terms, in float64
    Z = ops.spmm3(g, x0)
    prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in conv._dense_params())))
    Y = ops.layer_dense(Z, prm, 0, constant=conv.constant.detach(), res_x=x0 if res else None, act=True)
    out = ops.layer_dense_backward(w, Z, Y, prm, 0, act=True)
    t32 = ops.spmm3_t(g, out["dZ"].float()).double()  # the fp32 transposed kernel on the same (exact) dZ values
    dp = out["dpre"].double() if res else torch.zeros_like(t32)
    ref = t32 + dp
    gx, gx_old = got[True]["x"].double(), got[False]["x"].double()
    # one bf16 rounding (unit roundoff 2^-8) of the fp32 sum, whose own order differs from t32's by fp32 rounding
    noise = 1e-5 * (t32.abs() + dp.abs())
    assert bool(((gx - ref).abs() <= 2.0 ** -8 * ref.abs() + noise).all()), float((gx - ref).abs().max())
    # the autograd path rounds the propagation term, then the sum
    assert bool(((gx - gx_old).abs() <= 2.0 ** -8 * (2 * ref.abs() + t32.abs()) + 2 * noise).all())
    del lib


# ---------------------------------------------------------------------------------------------------------------
# ops.head_train (round 5): the prediction head's training step in one kernel
def _drop_keep(seed: int, M: int, H: int, p: float):
    """The kernel's dropout draw restated on the host (pg_head_train.hip, drop_hash): keep (m, j) when the mixed
    index's top 24 of 32 bits are >= ceil(p 2^24)."""
    m = np.arange(M, dtype=np.uint64)[:, None]
    j = np.arange(H, dtype=np.uint64)[None, :]
    with np.errstate(over="ignore"):
        x = np.uint64(seed) ^ (np.uint64(0x9E3779B97F4A7C15) * (m * np.uint64(H) + j + np.uint64(1)))
        x ^= x >> np.uint64(33)
        x *= np.uint64(0xff51afd7ed558ccd)
        x ^= x >> np.uint64(33)
        x *= np.uint64(0xc4ceb9fe1a85ec53)
        x ^= x >> np.uint64(33)
    u = (x & np.uint64(0xffffffff)) >> np.uint64(8)
    thr = min(16777215, int(np.ceil(p * 16777216.0)))
    return torch.from_numpy(u >= np.uint64(thr))


@pytest.mark.parametrize("M,drop,scaled,F", [(3001, 0.0, False, 128), (64, 0.0, False, 128), (1000, 0.5, False, 128),
                                             (777, 0.5, True, 128), (20000, 0.25, False, 128)])
def test_head_train_vs_float64(pkg, cuda, M, drop, scaled, F):
    """ops.head_train (F = 128, hidden 64) against torch autograd in float64 on the same inputs: loss (nll mean x weight of
    decoder Linear -> ReLU -> Dropout -> Linear -> log_softmax), dh and the four decoder gradients; with dropout the
    kernel's counter-based mask is restated on the host (_drop_keep); with a loss scale (GradScaler) every gradient
    carries it and the loss does not."""
    from protgram_directgcn_amd import ops
    H, C, weight = F // 2, 20, 0.75
    gen = torch.Generator().manual_seed(M)
    h = torch.randn(M, F, generator=gen)
    W1, b1 = torch.randn(H, F, generator=gen) * 0.1, torch.randn(H, generator=gen) * 0.1
    W2, b2 = torch.randn(C, H, generator=gen) * 0.2, torch.randn(C, generator=gen) * 0.1
    y = torch.randint(0, C, (M,), generator=gen)
    seed = 0x1234_5678_9abc_def0 + M
    seed_t = torch.tensor([seed], dtype=torch.int64, device=cuda)
    s = 1024.0 if scaled else 1.0
    scale_t = torch.tensor(s, device=cuda) if scaled else None
    r = ops.head_train(h.to(cuda), W1.to(cuda), b1.to(cuda), W2.to(cuda), b2.to(cuda), y.to(cuda), weight, drop,
                       seed_t if drop > 0 else None, scale_t)
    assert r is not None
    # F = 256 (config 5) is declined: the caller runs the framework ops
    z = functools.partial(torch.zeros, device=cuda)
    assert ops.head_train(z(4, 256), z(128, 256), z(128), z(C, 128), z(C), y[:4].to(cuda)) is None
    loss, dh, grads = r
    torch.cuda.synchronize()
    # float64 reference
    ps = [t.double().requires_grad_(True) for t in (h, W1, b1, W2, b2)]
    a = torch.relu(ps[0] @ ps[1].t() + ps[2])
    if drop > 0:
        a = a * _drop_keep(seed, M, H, drop).double() / (1.0 - drop)
    lp = torch.log_softmax(a @ ps[3].t() + ps[4], dim=1)
    loss_r = torch.nn.functional.nll_loss(lp, y) * weight
    (loss_r * s).backward()
    assert abs(float(loss) - float(loss_r)) <= 1e-5 * abs(float(loss_r)), (float(loss), float(loss_r))
    for got, ref, what in [(dh, ps[0].grad, "dh")] + [(g, q.grad, n) for g, q, n in
                                                       zip(grads, ps[1:], ("dW1", "db1", "dW2", "db2"))]:
        assert_grad_close(got.cpu(), ref.float(), f"head_train {what}")


@pytest.mark.parametrize("M,drop,scaled", [(3001, 0.0, False), (16, 0.0, False), (1000, 0.5, False), (777, 0.5, True),
                                           (20000, 0.25, False), (160000, 0.5, False)])
def test_head_train_bf16_vs_float64(pkg, cuda, M, drop, scaled):
    """ops.head_train_bf16 (config 5's head: bf16 h [M, 256], hidden 128, 20 classes) against float64 autograd on the
    same bf16 h: loss, dh (bf16) and the four decoder gradients, with the dropout mask restated on the host and, when
    scaled, a GradScaler-style loss scale on every gradient. Stated bounds: the kernel's products use
    two-term bf16 splits (each within ~3 2^-16 of the exact product, fp32 sums), so the fp32 outputs obey
    |d| <= 2^-12 (|ref| + max|ref|) and the loss 2^-12 relative; dh is rounded once to bf16:
    |d| <= 2^-8 |ref| + 2^-12 max|ref|."""
    from protgram_directgcn_amd import ops
    F, H, C, weight = 256, 128, 20, 0.75
    gen = torch.Generator().manual_seed(M)
    h = torch.randn(M, F, generator=gen).to(torch.bfloat16)
    W1, b1 = torch.randn(H, F, generator=gen) * 0.1, torch.randn(H, generator=gen) * 0.1
    W2, b2 = torch.randn(C, H, generator=gen) * 0.2, torch.randn(C, generator=gen) * 0.1
    y = torch.randint(0, C, (M,), generator=gen)
    seed = 0x1234_5678_9abc_def0 + M
    seed_t = torch.tensor([seed], dtype=torch.int64, device=cuda)
    s = 1024.0 if scaled else 1.0
    scale_t = torch.tensor(s, device=cuda) if scaled else None
    r = ops.head_train_bf16(h.to(cuda), W1.to(cuda), b1.to(cuda), W2.to(cuda), b2.to(cuda), y.to(cuda), weight, drop,
                            seed_t if drop > 0 else None, scale_t)
    assert r is not None
    z = functools.partial(torch.zeros, device=cuda)
    assert ops.head_train_bf16(z(4, 128, dtype=torch.bfloat16), z(64, 128), z(64), z(C, 64), z(C), y[:4].to(cuda)) is None
    loss, dh, grads = r
    assert dh.dtype == torch.bfloat16
    torch.cuda.synchronize()
    ps = [t.double().to(cuda).requires_grad_(True) for t in (h, W1, b1, W2, b2)]
    zr = ps[0] @ ps[1].t() + ps[2]
    zr.retain_grad()
    a = torch.relu(zr)
    keep = _drop_keep(seed, M, H, drop).double().to(cuda) / (1.0 - drop) if drop > 0 else torch.ones_like(zr)
    lp = torch.log_softmax((a * keep) @ ps[3].t() + ps[4], dim=1)
    loss_r = torch.nn.functional.nll_loss(lp, y.to(cuda)) * weight
    (loss_r * s).backward()
    assert abs(float(loss) - float(loss_r)) <= 2.0 ** -12 * abs(float(loss_r)), (float(loss), float(loss_r))
    # ReLU's kink: where the exact pre-activation is within the kernel's error of 0 (W1's two-term split leaves
    # <= 2^-16 |W1| per element: band 2^-14 of the sum of the terms' magnitudes), the kernel's z can fall on the other
    # side and switch that unit's whole term: dh, dW1 and db1 get the switched term's size as slack
    with torch.no_grad():
        hd = ps[0].detach()
        band = 2.0 ** -14 * (hd.abs() @ ps[1].detach().abs().t() + ps[2].detach().abs())
        amb = zr.detach().abs() <= band
        gz = ((torch.log_softmax((a * keep) @ ps[3].t() + ps[4], 1).exp() - torch.nn.functional.one_hot(
            y.to(cuda), C).double()) * (s * weight / M)) @ ps[3].detach() * keep  # d/da then through the dropout
        gz_amb = (gz * amb).abs()
        slack = {"dh": gz_amb @ ps[1].detach().abs(), "dW1": gz_amb.t() @ hd.abs(), "db1": gz_amb.sum(0)}
        amb_rows = amb.any(1)
    assert int(amb.sum()) <= max(8, 2e-3 * amb.numel()), int(amb.sum())
    worst = {}
    for got, ref, what in [(dh, ps[0].grad, "dh")] + [(g, q.grad, n) for g, q, n in
                                                       zip(grads, ps[1:], ("dW1", "db1", "dW2", "db2"))]:
        got, ref = got.double(), ref.detach()
        mx = float(ref.abs().max())
        bound = (2.0 ** -8 * ref.abs() + 2.0 ** -12 * mx) if what == "dh" else 2.0 ** -12 * (ref.abs() + mx)
        bound = bound + slack.get(what, 0.0)
        d = (got - ref).abs()
        worst[what] = round(float((d / (2.0 ** -12 * (ref.abs() + mx))).max()), 3)
        assert bool((d <= bound).all()), (what, float(d.max()), mx)
    print(f"head_train_bf16 M={M}: max |d| / 2^-12 (|ref| + max|ref|):", worst, "kink rows", int(amb_rows.sum()))


def test_train_step_bf16_fused_head_matches_framework_head(pkg, cuda):
    """bf16 mode with a 256-wide last layer (config 5's head shape): train.train_step runs the prediction head in
    pg_head_train_bf16 (bf16 h in, bf16 dh out) -- against the framework ops on h.float() (HEAD_FUSED = False): one SGD
    step in eval mode (no dropout draw) from the same start, the loss within 2^-12 and every parameter gradient
    within the bf16 model tolerance of test_gpu_configs (2^-8 (16 |ref| + 16 max|ref|)): the kernel's products are
    within ~2^-15 of fp32's, and dh is rounded to bf16 either way."""
    from protgram_directgcn_amd import ops, train
    N, s, d, c = pkg.synth.de_bruijn_edges(3)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    x = torch.randn(N, 64, generator=torch.Generator().manual_seed(1234)).to(cuda)
    y = (torch.arange(N, device=cuda) // 400) % 20
    data = pkg.Data(x=x, graph=g)
    lib = ops.load_library()
    calls = []
    real = lib.pg_head_train_bf16
    runs = []
    for fused in (False, True):
        train.HEAD_FUSED = fused
        try:
            torch.manual_seed(0)
            m = pkg.ProtGramDirectGCN([64, 256, 256], N, 20, 3, 0, 512, 0.5, True).to(cuda).eval()
            m.compute_dtype = torch.bfloat16
            opt = torch.optim.SGD(m.parameters(), lr=0.0)
            lib.pg_head_train_bf16 = lambda *a: (calls.append(1), real(*a))[1]
            loss = float(train.train_step(m, data, y, opt, l2_lambda=0.0))
            runs.append((loss, {k: p.grad.detach().double().clone() for k, p in m.named_parameters()
                                if p.grad is not None}))
        finally:
            train.HEAD_FUSED = True
            lib.pg_head_train_bf16 = real
    assert len(calls) == 1  # the fused run only
    assert abs(runs[1][0] - runs[0][0]) <= 2.0 ** -12 * abs(runs[0][0]), (runs[0][0], runs[1][0])
    assert set(runs[0][1]) == set(runs[1][1])
    for k, ref in runs[0][1].items():
        got = runs[1][1][k]
        bound = 2.0 ** -8 * (16 * ref.abs() + 16 * float(ref.abs().max()))
        assert bool(((got - ref).abs() <= bound).all()), (k, float((got - ref).abs().max()), float(ref.abs().max()))


def test_train_step_bf16_deferred_constant_grads_bit_identical(pkg, cuda):
    """bf16 mode + train.Adam, no GradScaler: the per-node constants' gradients stay the layers' bf16 dpre, read by
    pg_adam_f32 as bf16 (gtype 1) instead of an fp32 .grad copy (train.DEFER_CONST_GRAD). 3 training-mode steps with
    dropout and the L2 term: losses and every parameter and Adam moment bit-identical to the fp32-.grad run. Layer 1
    (projected residual) runs LayerDense, layer 2 (identity residual) PropagateDense, whose dX then comes from
    pg_spmm3t_ngram_add_bf16 (dpre kept intact); the constants' .grad stay None and the table is emptied."""
    from protgram_directgcn_amd import ops, train
    N, s, d, c = pkg.synth.de_bruijn_edges(3)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    x = torch.randn(N, 64, generator=torch.Generator().manual_seed(1234)).to(cuda)
    y = (torch.arange(N, device=cuda) // 400) % 20
    data = pkg.Data(x=x, graph=g)
    lib = ops.load_library()
    real = lib.pg_spmm3t_ngram_add_bf16
    calls = []
    runs = []
    for defer in (False, True):
        train.DEFER_CONST_GRAD = defer
        try:
            torch.manual_seed(0)
            m = pkg.ProtGramDirectGCN([64, 256, 256], N, 20, 3, 0, 512, 0.5, True).to(cuda).train()
            m.compute_dtype = torch.bfloat16
            opt = train.Adam(m.parameters(), lr=1e-3)
            lib.pg_spmm3t_ngram_add_bf16 = lambda *a: (calls.append(defer), real(*a))[1]
            losses = [float(train.train_step(m, data, y, opt, l2_lambda=1e-7)) for _ in range(3)]
            consts = [k for k, p in m.named_parameters() if "constant" in k]
            assert consts
            if defer:
                assert all(dict(m.named_parameters())[k].grad is None for k in consts)
                assert not ops._DEFERRED_GRADS and not ops._DEFER_CONST_GRAD
            st = {k: (p.detach().clone(), opt.state[p]["exp_avg"].clone(), opt.state[p]["exp_avg_sq"].clone())
                  for k, p in m.named_parameters()}
            runs.append((losses, st))
        finally:
            train.DEFER_CONST_GRAD = True
            lib.pg_spmm3t_ngram_add_bf16 = real
    assert calls and all(calls)  # the deferred run only
    assert runs[0][0] == runs[1][0], (runs[0][0], runs[1][0])
    for k, (p0, m0, v0) in runs[0][1].items():
        p1, m1, v1 = runs[1][1][k]
        assert torch.equal(p0, p1) and torch.equal(m0, m1) and torch.equal(v0, v1), k


def test_train_step_fused_head_matches_framework_head(pkg, cuda):
    """train.train_step with the head in one kernel (HEAD_FUSED, the default) against the framework ops
    (HEAD_FUSED = False): 3 SGD steps with the L2 gradient (parameter updates linear in the gradients), eval mode (no
    dropout draw), losses and parameters within fp32 rounding of each other."""
    from protgram_directgcn_amd import train
    N, s, d, c = pkg.synth.de_bruijn_edges(3)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    x = torch.randn(N, 64, generator=torch.Generator().manual_seed(1234)).to(cuda)
    y = (torch.arange(N, device=cuda) // 400) % 20
    data = pkg.Data(x=x, graph=g)
    runs = []
    for fused in (False, True):
        train.HEAD_FUSED = fused
        try:
            torch.manual_seed(0)
            m = pkg.ProtGramDirectGCN([64, 128, 128], N, 20, 3, 0, 512, 0.5, True).to(cuda).eval()
            opt = torch.optim.SGD(m.parameters(), lr=0.05)
            losses = [float(train.train_step(m, data, y, opt, l2_lambda=1e-3)) for _ in range(3)]
            runs.append((losses, {k: v.detach().clone() for k, v in m.state_dict().items()}))
        finally:
            train.HEAD_FUSED = True
    np.testing.assert_allclose(runs[1][0], runs[0][0], rtol=2e-6)
    for k, v in runs[0][1].items():
        assert_grad_close(runs[1][1][k].cpu(), v.cpu(), f"param {k}")


def test_model_fused_dropout_matches_masked_layers(pkg, cuda, monkeypatch):
    """model.body() in training mode with the layer dropout fused into the dense epilogue (ops.FUSED_DROPOUT) against
    the same layers run without dropout and multiplied by the host restatement of the kernel's mask
    (_layer_drop_keep, seeds recorded from the body's one draw): at p = 0.5 the outputs are bit-identical, and the
    gradients of every parameter and of x through both layers (projected-residual LayerDense, then PropagateDense with
    the span backward) agree within fp32 rounding."""
    from protgram_directgcn_amd import ops
    N, s, d, c = pkg.synth.de_bruijn_edges(3)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    gen = torch.Generator().manual_seed(99)
    x = torch.randn(N, 64, generator=gen).to(cuda)
    w = torch.randn(N, 128, generator=gen).to(cuda)
    data = pkg.Data(x=x, graph=g)
    torch.manual_seed(0)
    m = pkg.ProtGramDirectGCN([64, 128, 128], N, 20, 3, 0, 512, 0.5, True).to(cuda).train()
    drawn = []
    randint = torch.randint

    def rec(*a, **k):
        t = randint(*a, **k)
        drawn.append(t)
        return t
    monkeypatch.setattr(torch, "randint", rec)
    assert ops.FUSED_DROPOUT
    xg = x.clone().requires_grad_(True)
    data.x = xg
    h = m.body(data)
    monkeypatch.setattr(torch, "randint", randint)
    assert len(drawn) == 1 and drawn[0].numel() == 2
    seeds = [int(v) for v in drawn[0].cpu()]
    (h * w).sum().backward()
    got = {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None}
    got_x = xg.grad.clone()
    m.zero_grad()
    # reference: the same layers without dropout, then the restated mask
    xr = x.clone().requires_grad_(True)
    hr = xr
    for i, (conv, res) in enumerate(zip(m.convs, m.res_projs)):
        if isinstance(res, torch.nn.Linear):
            hr = conv.fused_forward(hr, g, res_x=hr, W_res=res.weight, b_res=res.bias, act=True)
        else:
            hr = conv.fused_forward(hr, g, res_x=hr, act=True)
        keep = _layer_drop_keep(seeds[i], N, 128, 0.5).to(cuda)
        hr = hr * keep.float() * 2.0
        if i == 0:
            frac = float(keep.float().mean())
            assert abs(frac - 0.5) < 0.01, frac
    assert torch.equal(h.detach(), hr.detach())
    (hr * w).sum().backward()
    assert_grad_close(got_x, xr.grad, "dx")
    for k, p in m.named_parameters():
        if k in got:
            assert_grad_close(got[k], p.grad, f"d{k}")


@pytest.mark.parametrize("M,Fin,Fout,proj,rows,drop", [(5000, 256, 256, False, False, 0.0), (1000, 128, 256, True, True, 0.0),
                                                       (3001, 256, 128, False, False, 0.5), (777, 64, 192, True, False, 0.3),
                                                       (70, 256, 256, False, True, 0.0)])
def test_dgrad_bf16_resident_matches_tiled(pkg, cuda, M, Fin, Fout, proj, rows, drop):
    """The resident-A bf16 input gradient (dgrad_bf16r_kernel: dpre of 64 rows computed once for all n-tiles, the
    default where F_out <= 256, F_out % 64 == 0 and M >= 256 rows per CU; forced here by PG_FLAG_DGRAD_BF16_RESIDENT)
    against the per-n-tile kernel (PG_FLAG_DGRAD_BF16_TILED): every output of the bf16 dense backward bit-identical,
    with and without the fused dropout."""
    from protgram_directgcn_amd import ops
    from protgram_directgcn_amd._lib import PG_FLAG_DGRAD_BF16_RESIDENT, PG_FLAG_DGRAD_BF16_TILED, default_flags
    Z, xres, prm, const, r, W_res, b_res, dY = _dense_case(M, Fin, Fout, proj, True, rows, 31 * M + Fout)
    dv = {k: v.to(cuda) for k, v in prm.items()}
    Zb, dYb = Z.to(torch.bfloat16).to(cuda), dY.to(torch.bfloat16).to(cuda)
    xb = xres.to(torch.bfloat16).to(cuda) if xres is not None else None
    rg = r.to(cuda) if r is not None else None
    Wr = W_res.to(cuda) if proj else None
    br = b_res.to(cuda) if proj else None
    dr = (drop, torch.tensor([1234567 + M], dtype=torch.int64, device=cuda)) if drop > 0 else None
    Y = ops.layer_dense(Zb, dv, 0, rows=rg, constant=const.to(cuda), res_x=xb, W_res=Wr, b_res=br, act=True, drop=dr)
    assert Y.dtype == torch.bfloat16
    outs = []
    for fl in (default_flags() | PG_FLAG_DGRAD_BF16_RESIDENT, default_flags() | PG_FLAG_DGRAD_BF16_TILED):
        o = ops.layer_dense_backward(dYb, Zb, Y, dv, 0, rows=rg, res_x=xb, W_res=Wr, b_res=br, act=True, flags=fl,
                                     drop_p=drop, dpre_f32=True)
        assert o is not None
        # the kernel's fp32 copy of dpre (the per-node constant's gradient): exactly the bf16 values widened
        assert o["dpre_f32"] is not None and torch.equal(o["dpre_f32"], o["dpre"].float())
        outs.append(o)
    for k in ("dpre", "dZ", "dres", "dgate", "dB", "dbsum", "dpre_f32"):
        if outs[0][k] is None:
            continue
        assert torch.equal(outs[0][k], outs[1][k]), k


@pytest.mark.parametrize("F_out,F_in,S", [(128, 128, 3), (256, 128, 4), (40, 16, 3), (12, 20, 4)])
def test_dense_grads_layout_matches_torch(pkg, cuda, F_out, F_in, S):
    """pg_dense_grads_layout_f32 (the dense backward's weight and bias gradients in the parameters' layout, one
    launch) against the torch ops it replaces, run on the same values on the CPU: bit-identical segments, W_shared's
    (seg0 + seg1) + seg2 and bias pairs."""
    from protgram_directgcn_amd import ops
    gen = torch.Generator().manual_seed(F_out * 7 + S)
    dW = torch.randn(F_out * S * F_in + 4 * F_out, generator=gen)
    dB, dbsum = dW[:F_out * S * F_in].view(F_out, S * F_in), dW[F_out * S * F_in:].view(4, F_out)
    ref = ops.dense_grads_layout(dB, dbsum, F_in)  # CPU tensors: the torch ops
    dWg = dW.to(cuda)
    got = ops.dense_grads_layout(dWg[:F_out * S * F_in].view(F_out, S * F_in), dWg[F_out * S * F_in:].view(4, F_out), F_in)
    for a, b, what in zip(got, ref, ("segments", "W_shared", "bias pairs")):
        assert a.shape == b.shape and torch.equal(a.cpu(), b), what
