"""The n-gram tile propagation kernels (pg_ngram_spmm.hip) against the CSR kernels, which are bit-exact to the
reference's propagate() (tests/test_gpu_parity.py), and against the oracle directly.

Tolerance: the tile kernels sum the same w*x terms in another order with FMAs, so aggregates agree within fp32
summation rounding: |d| <= 1e-5 + 1e-5 |ref| (BASELINE.json's fp32 bound).
"""
import numpy as np
import pytest
import torch

from oracle import directgcn_cpu as oc
from test_gpu_parity import assert_close

pytestmark = pytest.mark.gpu


def _csr_flag():
    from protgram_directgcn_amd._lib import PG_FLAG_NO_NGRAM
    return PG_FLAG_NO_NGRAM


def _graph(pkg, cuda, n, keep=1.0, seed=0):
    """B(20,n) with a `keep` fraction of its transitions (missing transitions = zero plan weights)."""
    N, s, d, c = pkg.synth.de_bruijn_edges(n)
    if keep < 1.0:
        m = np.random.default_rng(seed).random(s.size) < keep
        s, d, c = s[m], d[m], c[m]
    return pkg.build_propagation_csr(N, s, d, c, device=cuda)


def test_plan_only_for_ngram_graphs(pkg, cuda):
    from golden_util import load
    assert _graph(pkg, cuda, 2).ngram is not None
    assert _graph(pkg, cuda, 3, keep=0.3).ngram is not None
    fx = load("f5_fasta3")  # sorted-string ids of the n-grams present: not the full 20^3 id space
    g = pkg.build_propagation_csr(int(fx["N"][0]), fx["src"], fx["dst"], fx["cnt"], device=cuda)
    assert g.ngram is None
    # a K^n-sized graph with one entry that is no transition: the plan kernel counts it and no plan is attached
    N, s, d, c = pkg.synth.de_bruijn_edges(3)
    s2, d2 = np.append(s, 0), np.append(d, 4321)
    assert pkg.build_propagation_csr(N, s2, d2, np.append(c, 1.0).astype(np.float32), device=cuda).ngram is None
    assert pkg.build_propagation_csr(N, s, d, c, device=cuda, ngram_alphabet=None).ngram is None


@pytest.mark.parametrize("n,keep", [(2, 1.0), (3, 1.0), (3, 0.5), (4, 1.0)])
@pytest.mark.parametrize("F", [64, 128, 256])
def test_ngram_spmm3_vs_csr(pkg, cuda, n, keep, F):
    from protgram_directgcn_amd import ops
    g = _graph(pkg, cuda, n, keep)
    assert g.ngram is not None
    x = torch.randn(g.n_rows, F, generator=torch.Generator().manual_seed(n * 100 + F)).to(cuda)
    from protgram_directgcn_amd._lib import PG_FLAG_NGRAM_BLOCK4
    b4 = ops.default_flags() | PG_FLAG_NGRAM_BLOCK4
    Z = ops.spmm3(g, x)  # the middle-tile kernel (default)
    Zc = ops.spmm3(g, x, flags=_csr_flag())
    assert_close(Z, Zc, f"n={n} keep={keep} F={F}")
    assert torch.equal(ops.spmm3(g, x), Z)  # deterministic
    from protgram_directgcn_amd._lib import PG_FLAG_MID_LOADER_SYNC
    assert torch.equal(ops.spmm3(g, x, flags=ops.default_flags() | PG_FLAG_MID_LOADER_SYNC), Z)  # speed only
    Zb = ops.spmm3(g, x, flags=b4)  # the 4x4-block tile kernel
    assert_close(Zb, Zc, f"block4 n={n} keep={keep} F={F}")
    assert torch.equal(ops.spmm3(g, x, flags=b4), Zb)
    # gated store (inference path) == gates applied to the ungated CSR aggregates
    N = g.n_rows
    gen = torch.Generator().manual_seed(5)
    prm = {k: (torch.rand(N, 1, generator=gen) + 0.5).to(cuda) for k in ("C_in", "C_out", "C_directed",
                                                                          "C_undirected", "C_all")}
    prm["W_main_in"] = torch.zeros(F, F, device=cuda)  # only its shape is read (F_in for the gate block)
    assert ops.spmm3_gated(g, x, prm, 0) is None  # the middle-tile kernel leaves the gates to the dense kernel
    Zg = ops.spmm3_gated(g, x, prm, 0, flags=b4)  # the 4x4-block kernel's gated store
    cad = prm["C_all"] * prm["C_directed"]
    s = [cad * prm["C_in"], cad * prm["C_out"], prm["C_all"] * prm["C_undirected"]]
    ref = torch.cat([Zc[:, k * F:(k + 1) * F] * s[k] for k in range(3)], 1)
    assert_close(Zg, ref, f"gated n={n} F={F}")


@pytest.mark.parametrize("n,keep", [(2, 1.0), (3, 1.0), (3, 0.5), (4, 1.0)])
@pytest.mark.parametrize("F", [16, 48, 64, 128, 256])
def test_ngram_spmm3t_vs_csr(pkg, cuda, n, keep, F):
    """The off-diagonal transposed middle-tile kernel (F % 16 == 0; odd chunk counts run without workgroup pairs) plus
    the plan's diagonal term (PG_FLAG_MID_TRANSPOSED), and the 4x4-block transposed kernel (default), against the CSR
    kernel; the off-diagonal kernel alone against the CSR result minus the diagonal term, its accumulate mode on a
    strided G view, and determinism."""
    from protgram_directgcn_amd import ops
    from protgram_directgcn_amd._lib import PG_FLAG_MID_NO_PAIRS, PG_FLAG_MID_TRANSPOSED
    g = _graph(pkg, cuda, n, keep)
    assert g.ngram is not None and g.symmetric
    N = g.n_rows
    G = torch.randn(N, 3 * F, generator=torch.Generator().manual_seed(F)).to(cuda)
    ref = ops.spmm3_t(g, G, flags=_csr_flag())
    mid = ops.default_flags() | PG_FLAG_MID_TRANSPOSED
    got = ops.spmm3_t(g, G, flags=mid)
    assert_close(got, ref, f"transposed middle-tile n={n} F={F}")
    if F in (64, 128, 256):
        from protgram_directgcn_amd._lib import PG_FLAG_NGRAMT_HALVES, PG_FLAG_NGRAMT_NARROW, PG_FLAG_NGRAMT_WIDE
        b4 = ops.spmm3_t(g, G)
        assert_close(b4, ref, f"block4 (default) n={n} F={F}")
        for vf in (PG_FLAG_NGRAMT_WIDE, PG_FLAG_NGRAMT_HALVES, PG_FLAG_NGRAMT_NARROW):  # features per lane: same bits
            assert torch.equal(ops.spmm3_t(g, G, flags=ops.default_flags() | vf), b4), vf
    # the off-diagonal part alone: ref minus sum_k Diag_k G_k
    d3 = g.ngram.diag3()
    assert d3.shape == (N, 3)
    diag = (G.view(N, 3, F) * d3.unsqueeze(2)).sum(1)
    off = ops.spmm3t_offdiag(g, G)
    assert off is not None
    assert_close(off + diag, ref, f"off-diagonal + diagonal n={n} F={F}")
    assert torch.equal(ops.spmm3t_offdiag(g, G), off)  # deterministic
    assert torch.equal(ops.spmm3t_offdiag(g, G, flags=ops.default_flags() | PG_FLAG_MID_NO_PAIRS), off)  # schedule only
    # accumulate on a strided G view: out += offdiag
    Gw = torch.randn(N, 3 * F + 16, generator=torch.Generator().manual_seed(7)).to(cuda)
    Gw[:, :3 * F] = G
    dX = torch.randn(N, F, generator=torch.Generator().manual_seed(8)).to(cuda)
    want = dX + off
    assert ops.spmm3t_offdiag(g, Gw[:, :3 * F], out=dX) is dX
    assert_close(dX, want, f"accumulate n={n} F={F}")


def test_ngram_spmm3_vs_oracle_and_fallback_widths(pkg, cuda):
    """Directly against the oracle's propagate (the reference's index_select -> mul -> scatter_add_), and widths
    the tile kernels do not take (here F = 24: the middle-tile kernel needs F % 16 == 0, the 4x4-block one
    F in {64, 128, 256}) run the CSR kernel bit-exactly."""
    from protgram_directgcn_amd import ops
    g = _graph(pkg, cuda, 3, keep=0.7, seed=3)
    N = g.n_rows
    e = g.edges3.cpu().numpy()
    rows = torch.from_numpy(np.repeat(np.arange(N), np.diff(g.rowptr.cpu().numpy())))
    ei = torch.stack([torch.from_numpy(e[:, 0].astype(np.int64)), rows])
    for F in (128, 24):
        x = torch.randn(N, F, generator=torch.Generator().manual_seed(F))
        Z = ops.spmm3(g, x.to(cuda)).cpu()
        for j in range(3):
            ref = oc.propagate(ei, x, torch.from_numpy(e[:, 1 + j].copy().view(np.float32)))
            if F == 24:
                assert torch.equal(Z[:, j * F:(j + 1) * F], ref), j
            else:
                assert_close(Z[:, j * F:(j + 1) * F], ref, f"oracle {j}")


@pytest.mark.parametrize("n,keep", [(2, 1.0), (3, 1.0), (3, 0.5), (4, 1.0)])
@pytest.mark.parametrize("kernel,F", [("mid", F) for F in (16, 48, 64, 128, 256)]
                         + [("block4", F) for F in (64, 128, 256)])  # the 4x4-block kernel takes F in {64, 128, 256}
def test_ngram_transposed_bf16(pkg, cuda, n, keep, F, kernel):
    """bf16 transposed tile kernels (bf16 rows, fp32 sums, one rounding): the middle-tile kernel with the diagonal term
    in-kernel (pg_spmm3t_ngram_mid_bf16, PG_FLAG_MID_TRANSPOSED; F % 16 == 0) and the 4x4-block one
    (pg_spmm3t_ngram_bf16, the default; F in {64, 128, 256}), against the fp32 kernel on the widened bf16 input and against the bf16
    CSR kernel: within one bf16 ulp (|d| <= 2^-7 |ref| + 1e-6); the middle kernel's accumulate mode on a strided G,
    and determinism."""
    from protgram_directgcn_amd import ops
    from protgram_directgcn_amd._lib import PG_FLAG_MID_TRANSPOSED, load_library
    g = _graph(pkg, cuda, n, keep)
    N = g.n_rows
    G = torch.randn(N, 3 * F, generator=torch.Generator().manual_seed(n * 10 + F)).to(cuda).to(torch.bfloat16)
    fl = ops.default_flags() | (PG_FLAG_MID_TRANSPOSED if kernel == "mid" else 0)
    got = ops.spmm3_t(g, G, flags=fl)
    assert got.dtype == torch.bfloat16
    assert torch.equal(ops.spmm3_t(g, G, flags=fl), got)
    ref32 = ops.spmm3_t(g, G.float(), flags=_csr_flag())
    for other, tag in ((ref32, "fp32"), (ops.spmm3_t(g, G, flags=_csr_flag()).float(), "bf16 CSR")):
        d = (got.float() - other).abs()
        bad = d > 2.0 ** -7 * other.abs() + 1e-6
        assert not bool(bad.any()), (tag, int(bad.sum()), float(d.max()))
    if kernel == "mid":  # accumulate through the C ABI: dX += A^T G (fp32 sum, one rounding)
        lib = load_library()
        Gw = torch.zeros(N, 3 * F + 8, dtype=torch.bfloat16, device=cuda)
        Gw[:, :3 * F] = G
        dX = torch.randn(N, F, generator=torch.Generator().manual_seed(9)).to(cuda).to(torch.bfloat16)
        want = dX.float() + ref32
        ng = g.ngram
        rc = lib.pg_spmm3t_ngram_mid_bf16(ng.K, ng.n, N, ng.mplan.data_ptr(), Gw.data_ptr(), Gw.stride(0), F,
                                          dX.data_ptr(), dX.stride(0), 1, ops.default_flags(), ops._stream(dX))
        assert rc == 0
        d = (dX.float() - want).abs()
        bad = d > 2.0 ** -7 * want.abs() + 2.0 ** -7 * ref32.abs() + 1e-6
        assert not bool(bad.any()), ("accumulate", int(bad.sum()), float(d.max()))
    if kernel == "block4":
        # every features-per-lane variant (column pieces of a plan block on the waves of one workgroup) gives the
        # default's bits; then accumulate through the C ABI on a strided G
        from protgram_directgcn_amd._lib import PG_FLAG_NGRAMT_HALVES, PG_FLAG_NGRAMT_NARROW, PG_FLAG_NGRAMT_WIDE
        for vf in (PG_FLAG_NGRAMT_WIDE, PG_FLAG_NGRAMT_HALVES, PG_FLAG_NGRAMT_NARROW):
            assert torch.equal(ops.spmm3_t(g, G, flags=fl | vf), got), vf
        lib = load_library()
        Gw = torch.zeros(N, 3 * F + 8, dtype=torch.bfloat16, device=cuda)
        Gw[:, :3 * F] = G
        dX = torch.randn(N, F, generator=torch.Generator().manual_seed(9)).to(cuda).to(torch.bfloat16)
        want = dX.float() + ref32
        ng = g.ngram
        C = dX.clone()  # the addend, for the out-of-place form below
        rc = lib.pg_spmm3t_ngram_bf16(ng.K, ng.n, N, ng.plan.data_ptr(), Gw.data_ptr(), Gw.stride(0), F,
                                      dX.data_ptr(), dX.stride(0), 1, fl, ops._stream(dX))
        assert rc == 0
        d = (dX.float() - want).abs()
        bad = d > 2.0 ** -7 * want.abs() + 2.0 ** -7 * ref32.abs() + 1e-6
        assert not bool(bad.any()), ("accumulate", int(bad.sum()), float(d.max()))
        # pg_spmm3t_ngram_add_bf16: dX = C + A^T G with C read from its own rows -- the accumulate form's bits, C kept
        # (a strided C, and C = dX in place)
        Cw = torch.zeros(N, F + 8, dtype=torch.bfloat16, device=cuda)
        Cw[:, :F] = C
        out = torch.full((N, F), float("nan"), dtype=torch.bfloat16, device=cuda)
        rc = lib.pg_spmm3t_ngram_add_bf16(ng.K, ng.n, N, ng.plan.data_ptr(), Gw.data_ptr(), Gw.stride(0), F,
                                          Cw.data_ptr(), Cw.stride(0), out.data_ptr(), out.stride(0), fl,
                                          ops._stream(out))
        assert rc == 0
        assert torch.equal(out, dX) and torch.equal(Cw[:, :F], C)
        C2 = C.clone()
        rc = lib.pg_spmm3t_ngram_add_bf16(ng.K, ng.n, N, ng.plan.data_ptr(), Gw.data_ptr(), Gw.stride(0), F,
                                          C2.data_ptr(), C2.stride(0), C2.data_ptr(), C2.stride(0), fl,
                                          ops._stream(C2))
        assert rc == 0 and torch.equal(C2, dX)
        assert torch.equal(ops.spmm3t_ngram_acc_bf16(g, G, torch.empty_like(C), src=C), dX)
