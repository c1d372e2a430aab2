"""The middle partition's scatter-form backward (pg_spmm3t_ngram_scatter_*, pg_rows_gather_sum; shard.MiddleScatter):
a rank's transposed propagation sum_k A_k^T dZ_k from its owned rows only (the backward of protgram_directgcn.py:101-112
over the rank's column block), against the transposed CSR kernel over the same block (shard.middle_transpose, itself
checked against the oracle's autograd in tests/test_middle_partition.py).

Tolerances: the parts are fp32 MFMA sums of the same w*g terms in another order, then summed per row in fp32:
|d| <= 1e-5 + 1e-5 |ref| (BASELINE.json's fp32 bound); bf16 G is widened exactly, so the fp32 bound holds against the
CSR kernel on G.float(). pg_rows_gather_sum is a fixed-order fp32 sum: bit-exact against the same order on torch."""
import pytest
import torch

from test_gpu_parity import assert_close

pytestmark = pytest.mark.gpu


def _graph(pkg, cuda, n, keep=1.0, seed=0):
    import numpy as np
    N, s, d, c = pkg.synth.de_bruijn_edges(n)
    if keep < 1.0:
        m = np.random.default_rng(seed).random(s.size) < keep
        s, d, c = s[m], d[m], c[m]
    return pkg.build_propagation_csr(N, s, d, c, device=cuda)


def test_rows_gather_sum_order_and_dtypes(pkg, cuda):
    from protgram_directgcn_amd import ops
    gen = torch.Generator().manual_seed(3)
    F, nA, nB, n_out = 48, 300, 200, 257
    A = torch.randn(nA, F + 4, generator=gen).to(cuda)[:, :F]  # strided rows
    cnt = torch.randint(0, 6, (n_out,), generator=gen)
    ptr = torch.zeros(n_out + 1, dtype=torch.int64)
    ptr[1:] = torch.cumsum(cnt, 0)
    tot = int(ptr[-1])
    pick_b = torch.rand(tot, generator=gen) < 0.4
    idx = torch.where(pick_b, -1 - torch.randint(0, nB, (tot,), generator=gen), torch.randint(0, nA, (tot,), generator=gen))
    for b_bf in (False, True):
        B = torch.randn(nB, F, generator=gen).to(cuda)
        if b_bf:
            B = B.to(torch.bfloat16)
        ref = torch.zeros(n_out, F, device=cuda)
        rows = torch.repeat_interleave(torch.arange(n_out), cnt)
        k_of = torch.arange(tot) - torch.repeat_interleave(ptr[:-1], cnt)
        for k in range(int(cnt.max()) + 1):  # the same per-row order: entry k of every row, in turn
            sel = k_of == k
            r, v = rows[sel].to(cuda), idx[sel].to(cuda)
            src = torch.where((v >= 0).view(-1, 1), A[v.clamp(min=0)], B[(-1 - v).clamp(min=0)].float())
            ref[r] += src
        for out_dtype in (torch.float32, torch.bfloat16):
            got = ops.rows_gather_sum(A, ptr.to(cuda), idx.to(torch.int32).to(cuda), n_out, F, B=B, out_dtype=out_dtype)
            assert got.dtype == out_dtype
            assert torch.equal(got, ref.to(out_dtype)), (b_bf, out_dtype)
    got = ops.rows_gather_sum(A, ptr.to(cuda), idx.clamp(min=0).to(torch.int32).to(cuda), n_out, F)  # A only
    assert got.shape == (n_out, F)


@pytest.mark.parametrize("n,keep,world,rank", [(3, 1.0, 1, 0), (3, 0.5, 3, 1), (4, 1.0, 8, 0), (4, 0.7, 8, 7)])
@pytest.mark.parametrize("F", [16, 48, 128])
@pytest.mark.parametrize("bf16", [False, True])
def test_scatter_parts_vs_transposed_csr(pkg, cuda, n, keep, world, rank, F, bf16):
    """T's D / P / S parts summed at their global rows == the transposed CSR kernel over the rank's column block
    (every row it computes: the owned and the ghost rows), and the parts land only on those rows."""
    from protgram_directgcn_amd import ops, shard
    g = _graph(pkg, cuda, n, keep)
    mp_ = shard.middle_partition(g, rank, world)
    sc = shard.middle_scatter(mp_)
    assert sc is not None and sc.splan.shape == (mp_.m1 - mp_.m0, ops.SCATTER_PLAN_FLOATS)
    G = torch.randn(mp_.n_own, 3 * F, generator=torch.Generator().manual_seed(n * 1000 + F)).to(cuda)
    if bf16:
        G = G.to(torch.bfloat16)
    T = ops.spmm3t_scatter(sc.splan, G)
    assert T.shape == (3 * mp_.n_own, F) and T.dtype == torch.float32
    assert torch.equal(ops.spmm3t_scatter(sc.splan, G), T)  # deterministic
    mt = shard.middle_transpose(mp_)
    ref = ops.spmm3t_rows(mt.rowptr, mt.edges3, mt.rows, G.float(), mp_.n).float()
    rows = mt.rows.long()
    # every touched row's parts, summed by the gather-sum over all touched rows
    cnt = torch.zeros(mp_.n, dtype=torch.int64, device=cuda)
    K, Kn1, Kn2 = 20, 20 ** (n - 1), 20 ** (n - 2)
    M = torch.arange(mp_.m0, mp_.m1, device=cuda).view(-1, 1, 1)
    x = torch.arange(K, device=cuda).view(1, -1, 1)
    y = torch.arange(K, device=cuda).view(1, 1, -1)
    tgt = torch.cat([(x * Kn1 + M * K + y).reshape(-1), (M * K * K + x * K + y).reshape(-1),
                     (x * Kn1 + y * Kn2 + M).reshape(-1)])
    cnt.index_add_(0, tgt, torch.ones_like(tgt))
    assert torch.equal(torch.nonzero(cnt).view(-1), torch.sort(rows).values)  # parts land exactly on the touched rows
    dense = torch.zeros(mp_.n, F, dtype=torch.float64, device=cuda)
    dense.index_add_(0, tgt, T.double())
    assert_close(dense[rows].float(), ref[rows], f"n={n} keep={keep} world={world} rank={rank} F={F} bf16={bf16}")


class _Loop:
    """World-1 loopback collectives: the receive buffer is the send buffer (the identity exchange)."""

    def all_to_all(self, out, inp, out_splits, in_splits):
        out.copy_(inp)


@pytest.mark.parametrize("chunks", [1, 3])
@pytest.mark.parametrize("bf16", [False, True])
def test_exchange_propagate_backward_loopback(pkg, cuda, chunks, bf16):
    """_MidExchangePropagate (exchange -> owned-middle propagation; backward: scatter parts, ghost sums sent back,
    owned rows summed with the rows received) against the CSR composition _MidExchange -> _MidPropagate, on the
    loopback partition (world 1: every owned row goes through the send / receive lists)."""
    from protgram_directgcn_amd import shard
    g = _graph(pkg, cuda, 3, keep=0.8, seed=2)
    mp_ = shard.middle_partition(g, 0, 1, chunks=chunks, loopback=True)
    assert shard.middle_scatter(mp_) is not None
    F = 32
    dt = torch.bfloat16 if bf16 else torch.float32
    h = torch.randn(mp_.n_own, F, generator=torch.Generator().manual_seed(11)).to(cuda).to(dt)
    w = torch.randn(mp_.n_own, 3 * F, generator=torch.Generator().manual_seed(12)).to(cuda)
    grads, outs = [], []
    for fused in (True, False):
        hh = h.clone().requires_grad_(True)
        if fused:
            Z = shard._MidExchangePropagate.apply(hh, mp_, _Loop())
        else:
            Z = shard._MidPropagate.apply(shard._MidExchange.apply(hh, mp_, _Loop()), mp_)
        (Z.float() * w).sum().backward()
        outs.append(Z.detach())
        grads.append(hh.grad.float())
    assert torch.equal(outs[0], outs[1])
    if bf16:  # the two paths round to bf16 at different points: within one bf16 ulp of the larger
        d = (grads[0] - grads[1]).abs()
        assert not bool((d > 2.0 ** -7 * grads[1].abs() + 2.0 ** -7 * grads[0].abs() + 1e-6).any())
    else:
        assert_close(grads[0], grads[1], f"loopback chunks={chunks}")
