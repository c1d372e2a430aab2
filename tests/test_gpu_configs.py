"""BASELINE.json configs 3, 4 and 5 at their own sizes on the MI355X:

  config 3 -- 4-gram graph (N=160,000, 6,559,580 entries per adjacency), dims [128,128,128]: the trainer's loss
              (nll + 1e-7 * sum ||p||^2, protgram_directgcn_trainer.py:91-100) forward + backward against oracle
              autograd (loss, log-probs, embeddings, grad x, every parameter gradient), then one
              train.train_step + train.Adam step against torch.optim.Adam on the oracle's gradients;
  config 4 -- 5-gram graph (N=3.2M, 131,199,580 entries per adjacency: 64-bit row offsets, 32-bit column ids
              near their range): the 2-layer forward against the oracle on sampled output rows (the oracle runs
              on those rows' 2-hop neighbourhood with original_indices), and the halo-recompute partition for
              8 ranks bit-exact against the single-GPU forward;
  config 5 -- bf16 mode, dims [128,256,256,256] on the 4-gram graph: a training step of the trainer's loop
              against the fp32 model (loss, gradient directions), then train.train_step + train.Adam steps.

The oracle is oracle/directgcn_cpu.py with propagate_chunked (the reference's index_select -> mul ->
scatter_add_ per propagate, evaluated in row-aligned chunks: same values and gradients, bounded host memory).
Tolerances are the ones of tests/test_gpu_parity.py: outputs |d| <= 1e-5 + 1e-5|ref|; gradients
|d| <= 2e-5 max|ref| + 1e-4 |ref|.
"""
import dataclasses

import numpy as np
import pytest
import torch
import torch.nn.functional as Fn

from oracle import directgcn_cpu as oc
from test_gpu_parity import assert_close

pytestmark = pytest.mark.gpu
LAM = 1e-7   # l2_lambda, config.py:74
LR = 1e-3    # Adam lr of the trainer


def _model(pkg, dims, N, n, C=20, seed=0):
    """ProtGramDirectGCN with the reference init (torch.manual_seed) and randomised gates / biases (the
    reference init's C = 1, b = 0 would hide gate and bias bugs)."""
    torch.manual_seed(seed)
    m = pkg.ProtGramDirectGCN(dims, N, C, n, 0, 512, 0.5, True)
    gen = torch.Generator().manual_seed(seed + 11)
    with torch.no_grad():
        for name, p in m.named_parameters():
            leaf = name.split(".")[-1]
            if leaf.startswith("C_"):
                p.copy_(torch.rand(p.shape, generator=gen) + 0.5)
            elif "bias" in leaf:
                p.copy_(torch.rand(p.shape, generator=gen) * 0.2 - 0.1)
    return m


def _csr_coo(g):
    """The graph's CSR as the reference's COO inputs (ei = [source, destination], entries in CSR order) and the
    three weight vectors."""
    e = g.edges3.cpu().numpy()
    rp = g.rowptr.cpu().numpy()
    rows = torch.from_numpy(np.repeat(np.arange(g.n_rows, dtype=np.int64), np.diff(rp)))
    ei = torch.stack([torch.from_numpy(e[:, 0].astype(np.int64)), rows])
    w = [torch.from_numpy(e[:, 1 + j].copy().view(np.float32)) for j in range(3)]
    return ei, w


def _grad_close_or_as_exact(got, ref32, ref64, what):
    """The stated gradient tolerance against the fp32 oracle (|d| <= 2e-5 max|ref| + 1e-4 |ref|). Full-size
    gradients are sums over up to N rows chained through two layers, where the fp32 oracle's own rounding can
    exceed that bound: elements outside it pass only if the GPU gradient is at least as close to the float64
    gradient (same inputs) as the fp32 oracle is, up to 2x -- no less accurate than the reference itself."""
    got = got.detach().double().cpu()
    ref32, ref64 = ref32.detach().double(), ref64.detach().double()
    scale = float(ref32.abs().max()) if ref32.numel() else 0.0
    bad = (got - ref32).abs() > 2e-5 * scale + 1e-7 + 1e-4 * ref32.abs()
    if not bool(bad.any()):
        return
    e_gpu = float((got - ref64).abs().max())
    e_ref = float((ref32 - ref64).abs().max())
    i = int((got - ref64).abs().flatten().argmax())
    assert e_gpu <= 2 * e_ref + 1e-7 * float(ref64.abs().max()), (
        f"{what}: {int(bad.sum())} elements outside the fp32 tolerance (flat {bad.flatten().nonzero().flatten()[:8].tolist()}),"
        f" and max |gpu - f64| = {e_gpu:.3e} vs max |oracle fp32 - f64| = {e_ref:.3e}; worst flat index {i}: gpu "
        f"{float(got.flatten()[i]):.6e} fp32 oracle {float(ref32.flatten()[i]):.6e} f64 {float(ref64.flatten()[i]):.6e}")


def _count_tile_launches(monkeypatch):
    """Count the calls of the n-gram tile kernels' entry points (a dict, filled as they run)."""
    from collections import Counter
    from protgram_directgcn_amd import ops
    lib, calls = ops.load_library(), Counter()
    for name in ("pg_spmm3_ngram_f32", "pg_spmm3_ngram_mid_f32", "pg_spmm3t_ngram_f32", "pg_spmm3t_ngram_bf16",
                 "pg_spmm3t_ngram_mid_offdiag_f32", "pg_directgcn_dense_bwd_span_f32"):
        fn = getattr(lib, name)

        def wrap(*a, _fn=fn, _name=name):
            calls[_name] += 1
            return _fn(*a)
        monkeypatch.setattr(lib, name, wrap)
    return calls


def _fwd_tile(calls):
    """Forward n-gram tile launches: the middle-tile kernel (default) or the 4x4-block kernel."""
    return calls["pg_spmm3_ngram_mid_f32"] + calls["pg_spmm3_ngram_f32"]


def _labels(N, n):
    return torch.arange(N) // 20 ** (n - 1)  # the first letter


# ---------------------------------------------------------------------------------------------------------------
# config 3
# ---------------------------------------------------------------------------------------------------------------
@pytest.mark.timeout(1200)
def test_config3_4gram_training_step_vs_oracle(pkg, cuda, monkeypatch):
    from protgram_directgcn_amd import train
    n, F, dims = 4, 128, [128, 128, 128]
    N, s, d, c = pkg.synth.de_bruijn_edges(n)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    assert g.nnz == 6_559_580
    m = _model(pkg, dims, N, n).to(cuda).eval()  # eval: dropout off (its masks come from another RNG stream)
    x = torch.randn(N, F, generator=torch.Generator().manual_seed(1234))
    y = _labels(N, n)
    yd = y.to(cuda)

    xd = x.to(cuda).requires_grad_(True)
    # ProtGramDirectGCN.forward (eval) written out, to keep each layer's leaky_relu branch for the oracle
    h, masks = xd, []
    for conv in m.convs:  # identity residuals: res_projs are nn.Identity
        h = conv.fused_forward(h, g, None, res_x=h, act=True)
        masks.append((h > 0).detach().cpu())
    hook = m.decoder_fc[1].register_forward_hook(lambda mod, inp, out: masks.append((inp[0] > 0).detach().cpu()))
    lp, emb = m.head(h)  # decoder_fc: Linear, ReLU (its branches appended to masks), Dropout, Linear
    hook.remove()
    assert len(masks) == len(m.convs) + 1
    loss = Fn.nll_loss(lp, yd) + LAM * sum(p.norm(2).pow(2) for p in m.parameters())
    loss.backward()
    torch.cuda.synchronize()
    snap = {k: prm.grad.detach().cpu().clone() for k, prm in m.named_parameters()}
    snap["x"] = xd.grad.detach().cpu().clone()
    with torch.no_grad():
        lp_m, emb_m = m(pkg.Data(x=xd, graph=g))
    assert_close(lp_m, lp.detach(), "model forward vs the written-out forward")

    # the reference trainer's own wiring (protgram_directgcn_trainer.py:362-367): coalesced COO indices()/values() of
    # the three matrices, converted by csr_from_coo -- it must reach the same n-gram tile kernels (plan + schedule
    # attached) and give the prebuilt-graph path's bits
    data_coo = pkg.synth.trainer_data(g, x.to(cuda))
    gc = m.graph_of(data_coo)
    assert gc.ngram is not None and gc.symmetric and gc.row_order is not None
    assert torch.equal(gc.edges3, g.edges3) and torch.equal(gc.ngram.plan, g.ngram.plan)
    assert torch.equal(gc.row_order, g.row_order)  # closed-form schedule == locality_schedule on a complete graph
    calls = _count_tile_launches(monkeypatch)
    with torch.no_grad():
        lp_c, emb_c = m(data_coo)
    assert _fwd_tile(calls) == len(m.convs), calls
    assert torch.equal(lp_c, lp_m) and torch.equal(emb_c, emb_m)

    ei, w = _csr_coo(g)
    p = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    xr = x.clone().requires_grad_(True)
    pre = []
    lp_r, emb_r = oc.model_forward(p, dims, xr, ei, w[0], ei, w[1], ei, w[2], n_gram_len=n, prop=oc.propagate_chunked,
                                   act_masks=masks, pre_acts=pre)
    # the GPU's branch choices handed to the oracle may disagree with the oracle's own signs only where its
    # pre-activation is within the fp32 output tolerance of the kink (|z| <= 1e-5 + 1e-5|z|, i.e. rounding), and
    # only on a handful of elements
    for i, (mk, z) in enumerate(zip(masks, pre)):
        flip = mk != (z > 0)
        nflip = int(flip.sum())
        assert nflip <= 1e-5 * z.numel() + 8, (i, nflip, z.numel())
        if nflip:
            assert float(z[flip].abs().max()) <= 2e-5, (i, nflip, float(z[flip].abs().max()))
    loss_r = Fn.nll_loss(lp_r, y) + LAM * sum(v.norm(2).pow(2) for v in p.values())
    loss_r.backward()

    # the same in float64 on the same (fp32-valued) inputs: the exact gradients both fp32 paths approximate
    p64 = {k: v.detach().double().requires_grad_(True) for k, v in p.items()}
    x64 = x.double().requires_grad_(True)
    lp64, _ = oc.model_forward(p64, dims, x64, ei, w[0], ei, w[1], ei, w[2], n_gram_len=n, prop=oc.propagate_chunked,
                               act_masks=masks)
    (Fn.nll_loss(lp64, y) + LAM * sum(v.norm(2).pow(2) for v in p64.values())).backward()

    loss, loss_r = float(loss.detach()), float(loss_r.detach())
    assert abs(loss - loss_r) <= 1e-5 * abs(loss_r), (loss, loss_r)
    assert_close(lp, lp_r, "4-gram log_probs")
    assert_close(emb, emb_r, "4-gram embeddings")
    changed = [k for k, prm in m.named_parameters() if not torch.equal(prm.grad.detach().cpu(), snap[k])]
    assert not changed, f"gradients changed on the device after the backward: {changed}"
    fails = []
    for what, got, r32, r64 in [("x", snap["x"], xr.grad, x64.grad)] + [(k, snap[k], p[k].grad, p64[k].grad)
                                                                         for k, prm in m.named_parameters()]:
        try:
            _grad_close_or_as_exact(got, r32, r64, f"4-gram grad {what}")
        except AssertionError as ex:
            fails.append(str(ex).split("\n")[0])
    assert not fails, "\n".join(fails)

    # one step: train.train_step + train.Adam (GPU) vs torch.optim.Adam on the oracle's gradients (CPU)
    torch.optim.Adam(list(p.values()), lr=LR).step()
    m.zero_grad(set_to_none=True)
    opt = train.Adam(m.parameters(), lr=LR)
    p_pre = {k: prm.detach().cpu().clone() for k, prm in m.named_parameters()}
    # rows whose decoder pre-activation sits within fp32 rounding of ReLU's kink: there the head kernel and the oracle
    # may take different branches (as the layers' leaky_relu above, whose GPU choices the oracle was handed)
    with torch.no_grad():
        hb = m.body(data_coo).double().cpu()
    dec = m.decoder_fc[0]
    W1d, b1d = dec.weight.detach().double().cpu(), dec.bias.detach().double().cpu()
    zpre = hb @ W1d.t() + b1d
    zabs = hb.abs() @ W1d.abs().t() + b1d.abs()  # the size of the fp32 sum's terms: its rounding is ~1e-7 of this
    kink_rows = (zpre.abs() <= 2e-6 * zabs).any(1)
    assert int(kink_rows.sum()) <= 1e-3 * N, int(kink_rows.sum())
    calls.clear()
    loss_s = train.train_step(m, data_coo, yd, opt, l2_lambda=LAM, scaler=None)  # through the trainer's COO wiring
    # the gradients the step's Adam launch used: train_step's own (its head runs in one kernel, ops.head_train, whose
    # sums are ordered differently from the autograd path's g_gpu) plus the L2 gradient Adam folds in
    g_step = {k: prm.grad.detach().cpu() + 2 * LAM * p_pre[k] for k, prm in m.named_parameters()}
    fails = []
    for k in g_step:  # those gradients against the oracle, as the autograd path's above
        got, r32, r64 = g_step[k], p[k].grad, p64[k].grad
        if got.dim() >= 1 and got.size(0) == N:
            # per-node rows whose decoder pre-activation is within fp32 rounding of ReLU's kink (at most 1e-3 N,
            # asserted above) take the head kernel's own branch, which the oracle cannot be handed: excluded here
            keep = ~kink_rows
            got, r32, r64 = got[keep], r32[keep], r64[keep]
        try:
            _grad_close_or_as_exact(got, r32, r64, f"train_step grad {k}")
        except AssertionError as ex:
            fails.append(str(ex).split("\n")[0])
    assert not fails, "\n".join(fails)
    # the transposed propagation of every layer whose input needs a gradient: the span dense backward (diagonal term
    # and residual into E) + the off-diagonal transposed middle-tile kernel (ops.PropagateDense), not the 4x4 kernel
    assert _fwd_tile(calls) == len(m.convs), calls
    assert calls["pg_spmm3t_ngram_mid_offdiag_f32"] == len(m.convs) - 1, calls
    assert calls["pg_directgcn_dense_bwd_span_f32"] == len(m.convs) - 1 and calls["pg_spmm3t_ngram_f32"] == 0, calls
    assert abs(float(loss_s) - loss_r) <= 1e-5 * abs(loss_r)
    # The Adam step in two parts, each with a tolerance stated in advance (none taken from the observed errors):
    # (1) the update itself: the GPU parameters equal torch.optim.Adam (CPU, fp32) applied to the SAME gradients the
    #     launch used (g_step: train_step's gradients + the folded L2 term) within 3 ulp of the update's operands
    #     (max(|p|, lr, |p'|)), the kernel folding the L2 term by one FMA where torch adds a rounded product -- it restates
    #     torch's arithmetic, so this isolates it from the gradients' own error;
    # (2) against the oracle's step: a gradient within the stated gradient tolerance tol = 2e-5 max|g| + 1e-4 |g| of
    #     the oracle's moves Adam's first update lr g / (|g| + eps) by at most lr eps tol / (|g| - tol + eps)^2 (up
    #     to 2 lr where tol reaches |g|). Elements whose step gradient is outside tol -- accepted above only by the
    #     float64 criterion, or rows at the decoder's ReLU kink -- are covered by (1) and that gradient check; they
    #     are excluded here and their number is bounded.
    for k, prm in m.named_parameters():
        ref1 = p_pre[k].clone().requires_grad_(True)
        ref1.grad = g_step[k].clone()
        torch.optim.Adam([ref1], lr=LR).step()
        got = prm.detach().cpu()
        # the update's roundings that may differ (the device sqrt, the division, the final add: 1 ulp each of the
        # largest of p_pre, the step (|.| <= ~lr) and the result); plus the fold of the L2 gradient (one FMA in the
        # kernel, a rounded product and a sum here: g differs by <= 2 ulp of its larger term), which the first update
        # lr g / (|g| + eps) passes on with slope lr eps / (|g| + eps)^2
        eps32 = torch.finfo(torch.float32).eps
        ulp = 1.5 * eps32 * torch.maximum(torch.maximum(p_pre[k].abs(), got.abs()), torch.full_like(got, LR))
        dg = 2 * eps32 * torch.maximum(g_step[k].abs(), (2 * LAM * p_pre[k]).abs()) + 2 * eps32 * g_step[k].abs()
        fold = LR * 1e-8 * dg / (g_step[k].abs() + 1e-8) ** 2
        d1 = (got - ref1.detach()).abs()
        lim = 2 * ulp + fold + 1e-30
        if not bool((d1 <= lim).all()):
            i = int((d1 / lim).flatten().argmax())
            f = lambda t: float(t.flatten()[i])  # noqa: E731
            raise AssertionError(f"{k}: Adam update off by {f(d1):.3e} (limit {f(lim):.3e}) vs torch Adam at flat {i}: "
                                 f"p_pre {f(p_pre[k]):.9e} grad {f(prm.grad.detach().cpu()):.9e} g_step {f(g_step[k]):.9e}"
                                 f" got {f(got):.9e} torch {f(ref1.detach()):.9e}")
        gref = p[k].grad
        tol = 2e-5 * float(gref.abs().max()) + 1e-4 * gref.abs()
        inside = (g_step[k] - gref).abs() <= tol
        assert int((~inside).sum()) <= max(8, 1e-3 * gref.numel()), (k, int((~inside).sum()))
        sens = torch.where(gref.abs() > tol, LR * 1e-8 * tol / (gref.abs() - tol + 1e-8) ** 2,
                           torch.full_like(gref, 2 * LR))
        err = (got - p[k].detach()).abs()
        bad = inside & (err > sens + 2 * ulp)
        assert not bool(bad.any()), f"{k}: {int(bad.sum())} parameters off, max |d| {float(err[inside].max()):.3e}"


# ---------------------------------------------------------------------------------------------------------------
# config 4
# ---------------------------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def five_gram(pkg, cuda):
    n, F = 5, 128
    N, s, d, c = pkg.synth.de_bruijn_edges(n)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    del s, d, c
    m = _model(pkg, [F, F, F], N, n).to(cuda).eval()
    x = torch.randn(N, F, generator=torch.Generator().manual_seed(1234))
    xd = x.to(cuda)
    with torch.no_grad():
        lp, emb = m(pkg.Data(x=xd, graph=g))
        # the same forward on the CSR kernels alone: what a halo rank's subgraph (no n-gram tile plan) runs
        lp_c, emb_c = m(pkg.Data(x=xd, graph=dataclasses.replace(g, ngram=None)))
    assert g.ngram is not None
    assert_close(lp, lp_c, "5-gram forward: n-gram tile kernels vs CSR kernels")
    return {"N": N, "n": n, "F": F, "g": g, "m": m, "x": x, "xd": xd, "lp": lp, "emb": emb, "lp_csr": lp_c,
            "emb_csr": emb_c}


@pytest.mark.timeout(1200)
def test_config4_5gram_csr_matches_host_build(pkg, cuda, five_gram):
    """The GPU-built 5-gram CSR (torch GPU integer ops + pg_edges_normalize_f32) against the same construction
    on the host (torch CPU ops; the IEEE closed form in numpy for the weights), bit for bit: the sampled-row
    oracle check below reads the GPU-built weights, so this is what pins them at this size. (ROCm torch's
    index gather silently drops output past 1 GiB -- DESIGN.md §5a -- which is why this is checked at size.)"""
    from test_host import _closed_form
    f = five_gram
    g, N = f["g"], f["N"]
    _, s, d, c = pkg.synth.de_bruijn_edges(f["n"])
    rc = pkg.graph.ngram_raw_csr(N, s, d, c, device="cpu", schedule=False)
    del s, d, c
    assert rc.nnz == g.nnz
    assert torch.equal(g.rowptr.cpu(), rc.rowptr)
    assert torch.equal(g.raw.cpu(), rc.raw)
    assert torch.equal(g.node_norm.cpu(), rc.node_norm)
    rows, col, w = _closed_form(rc.raw.numpy(), rc.node_norm.numpy(), rc.rowptr.numpy())
    del rows, col
    e = g.edges3.cpu().numpy()
    assert np.array_equal(e[:, 0], rc.raw[:, 0].numpy())
    for j, k in enumerate(("in", "out", "und")):
        ulp = np.abs(e[:, 1 + j].astype(np.int64) - w[k].view(np.int32).astype(np.int64))
        bad = np.flatnonzero(ulp)
        assert bad.size == 0, (k, bad.size, int(ulp.max()), [(int(i), int(rc.raw[i, 0]), e[i, 1 + j].view(np.float32).item(),
                                                          w[k][i].item(), rc.raw[i, 1:].numpy().view(np.float32).tolist())
                                                         for i in bad[:4]])


@pytest.mark.timeout(1200)
def test_config4_5gram_forward_sampled_rows_vs_oracle(pkg, cuda, five_gram):
    f = five_gram
    N, n, g, m, x = f["N"], f["n"], f["g"], f["m"], f["x"]
    assert N == 3_200_000 and g.nnz == 131_199_580
    rp = g.rowptr.cpu()
    assert rp.dtype == torch.int64 and int(rp[-1]) == g.nnz  # offsets past 2^31 bytes of records
    e = g.edges3.cpu()
    gen = torch.Generator().manual_seed(5)
    R = torch.cat([torch.tensor([0, 1, N // 2, N - 2, N - 1]), torch.randint(0, N, (43,), generator=gen)]).unique()

    def entries(rows):  # CSR entries of these destination rows, in CSR order
        cnt = rp[rows + 1] - rp[rows]
        starts = torch.repeat_interleave(rp[rows], cnt)
        off = torch.arange(int(cnt.sum())) - torch.repeat_interleave(torch.cumsum(cnt, 0) - cnt, cnt)
        return torch.repeat_interleave(rows, cnt), e[starts + off]

    d2, e2 = entries(R)                                     # layer 2 reads layer-1 rows S1
    S1 = torch.cat([R, e2[:, 0].long()]).unique()
    d1, e1 = entries(S1)                                    # layer 1 reads input rows S0
    S0 = torch.cat([S1, e1[:, 0].long()]).unique()          # sorted: relabelling keeps column order
    assert int(e1[:, 0].max()) < N and int(e1[:, 0].min()) >= 0
    loc = lambda ids: torch.searchsorted(S0, ids)  # noqa: E731
    p = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    xs = x[S0]

    def layer(prefix, h, dst, ent):
        ei = torch.stack([loc(ent[:, 0].long()), loc(dst)])
        w = [ent[:, 1 + j].contiguous().view(torch.float32) for j in range(3)]
        return oc.layer_forward(p, h, ei, w[0], ei, w[1], ei, w[2], original_indices=S0, prefix=prefix)

    with torch.no_grad():
        h1 = Fn.leaky_relu(layer("convs.0.", xs, d1, e1) + xs)   # identity residual (128 -> 128)
        h2 = Fn.leaky_relu(layer("convs.1.", h1, d2, e2) + h1)[loc(R)]
        z = Fn.relu(oc.linear(h2, p["decoder_fc.0.weight"], p["decoder_fc.0.bias"]))
        lp_r = Fn.log_softmax(oc.linear(z, p["decoder_fc.3.weight"], p["decoder_fc.3.bias"]), dim=-1)
        emb_r = oc.l2_normalize(h2)
    Rd = R.to(cuda)
    assert_close(f["lp"][Rd], lp_r, "5-gram log_probs (sampled rows)")
    assert_close(f["emb"][Rd], emb_r, "5-gram embeddings (sampled rows)")
    assert bool(torch.isfinite(f["lp"]).all()) and bool(torch.isfinite(f["emb"]).all())


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("rank", [0, 7])
def test_config4_5gram_halo_partition_bitexact(pkg, cuda, five_gram, rank):
    """The 8-way halo-recompute partition at 5-gram (the multi-GPU forward bench.py --gpus 8 runs), one rank at a
    time on this GPU: its rows equal the single-GPU forward's bit for bit (on the CSR kernels; the single-GPU
    default runs the n-gram tile kernels, within fp32 summation rounding of those -- checked in the fixture)."""
    from protgram_directgcn_amd import shard
    f = five_gram
    hp = shard.halo_partition(f["g"], rank, 8, 2)
    assert hp.layer_rows[-1] in (f["N"] // 8, f["N"] // 8 + 1)
    inp = shard.halo_inputs(f["m"], hp, f["xd"])
    lp, emb = shard.halo_forward(f["m"], hp, inp)
    rows = hp.global_rows
    assert torch.equal(lp, f["lp_csr"][rows]) and torch.equal(emb, f["emb_csr"][rows])


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("rank", [0, 7])
def test_config4_5gram_exchange_partition_bitexact(pkg, cuda, five_gram, rank, monkeypatch):
    """The node-range exchange partition (config 4's RCCL design: shard.sharded_forward, chunked all-gather between
    the layers) at 5-gram for ranks 0 and 7 of P = 8, on this one GPU: the all-gather is replaced by a copy that
    fills the other ranks' rows from the single-GPU layer-1 output (this rank's own chunk is what it computed), so
    the rank runs exactly its production code -- row-chunked layer 1 on the row-sliced CSR, remapped CSR reading the
    chunk-major gathered buffer in layer 2, dense layer on row slices of the per-node parameters. Its rows equal the
    single-GPU forward on the same (CSR, ungated) kernels bit for bit, layer 1 and the outputs."""
    from protgram_directgcn_amd import ops, shard
    f = five_gram
    g, m, xd, N = f["g"], f["m"], f["xd"], f["N"]
    gc = dataclasses.replace(g, ngram=None)  # a rank's row-sliced CSR has no tile plan: compare on the CSR kernels
    monkeypatch.setattr(ops, "PREGATED_INFERENCE", False)  # sharded_forward gates in the dense kernel
    with torch.no_grad():
        h1 = m.convs[0].fused_forward(xd, gc, None, res_x=xd, act=True)
        h2 = m.convs[1].fused_forward(h1, gc, None, res_x=h1, act=True)
        lp_ref, emb_ref = m.head(h2)
    part = shard.partition(g, rank, 8)
    calls = [0]
    own_ok = []

    def fake_gather(send, dst, prt, group=None):
        k = calls[0]
        calls[0] += 1
        W, cs = prt.world, send.size(0)
        v = dst.view(W, cs, -1)
        for q in range(W):
            lo = q * prt.per + k * cs
            hi = min(lo + cs, (q + 1) * prt.per, prt.n)
            if q == prt.rank:
                v[q].copy_(send)
                if hi > lo:
                    own_ok.append(torch.equal(send[:hi - lo], h1[lo:hi]))
            elif hi > lo:
                v[q, :hi - lo] = h1[lo:hi]
        return None

    monkeypatch.setattr(shard, "_all_gather_chunk", fake_gather)
    lp, emb = shard.sharded_forward(m, part, xd, chunks=4)
    assert calls[0] == 4 and own_ok and all(own_ok)  # layer 1's own rows: bit-exact
    assert lp.shape[0] == part.n_local
    assert torch.equal(lp, lp_ref[part.r0:part.r1]) and torch.equal(emb, emb_ref[part.r0:part.r1])


def _middle_rank_check(pkg, m, g, xd, lp_ref, emb_ref, rank, world, monkeypatch):
    """One rank of the middle partition (shard.middle_forward) on this GPU, the ghost-row exchange replaced by a
    copy from the single-GPU layer-1 output into a NaN-filled buffer (so a read outside the rank's own + ghost
    rows would show): its layer-1 rows and its outputs must equal the single-GPU forward's bit for bit (the same
    middle-tile kernel over the rank's middles, the same dense kernel on its rows)."""
    from protgram_directgcn_amd import ops, shard
    conv = m.convs[0]
    vec = conv.use_vector_coeffs
    prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in conv._dense_params())))
    with torch.no_grad():
        h0 = m._apply_pe(xd)
        h1 = ops.layer_dense(ops.spmm3(g, h0), prm, 0 if vec else 1,
                             constant=conv.constant.detach() if vec else None, res_x=h0, act=True)
    mp = shard.middle_partition(g, rank, world)
    calls, own_ok = [0], []

    def fake_exchange(mp_, h_own, group=None):
        calls[0] += 1
        own_ok.append(torch.equal(h_own, h1[mp_.own]))
        X = torch.full_like(h1, float("nan"))
        X[mp_.own] = h_own
        X[mp_.recv_ids] = h1[mp_.recv_ids]
        return X

    hits = []
    real = ops.spmm3_middles
    with monkeypatch.context() as mpc:
        mpc.setattr(shard, "_exchange_rows", fake_exchange)
        mpc.setattr(ops, "spmm3_middles", lambda *a, **k: hits.append(1) or real(*a, **k))
        lp, emb = shard.middle_forward(m, mp, xd)
    assert calls[0] == len(m.convs) - 1 and own_ok and all(own_ok)
    assert len(hits) == len(m.convs)  # every layer on the middle-tile kernel
    rows = mp.global_rows
    assert torch.equal(lp, lp_ref[rows]) and torch.equal(emb, emb_ref[rows])
    # the same rank through MiddleRunner (the bench's path): layer 1 in 3 middle sub-ranges, each compute segment
    # captured as a HIP graph; the per-sub-range exchange (outside the graphs) fills the receive slices from the
    # single-GPU layer-1 output
    def fill(self, i, c):
        r0, r1 = self.recv_slices[c]
        self.recv[i][r0:r1] = h1[self.mp.recv_ids[r0:r1]]

    mpc_ = shard.middle_partition(g, rank, world, chunks=3)
    with monkeypatch.context() as mpc:
        mpc.setattr(shard.MiddleRunner, "_exchange", fill)
        run = shard.MiddleRunner(m, mpc_, xd)
        assert run.graphs is not None and len(run.graphs) == 3 * (len(m.convs) - 1) + 1
        assert run.mapped == (xd.size(1) == 128)  # 128-wide fp32 layers: the dense kernel maps its rows itself
        for _ in range(2):
            lp2, emb2 = run()
            torch.cuda.synchronize()
            assert torch.equal(lp2, lp) and torch.equal(emb2, emb)
    # replicated first layer (the bench's partition at 2 ranks): layer 1 over every row on this rank, the last layer
    # over its middles; no exchange at all
    with monkeypatch.context() as mpc:
        mpc.setattr(shard.MiddleRunner, "_exchange", lambda *a: pytest.fail("replicate must not exchange"))
        run = shard.MiddleRunner(m, mp, xd, replicate=True)
        assert len(run.graphs) == len(m.convs)
        lp3, emb3 = run()
        torch.cuda.synchronize()
        assert torch.equal(run.bufs[0], h1)
        assert torch.equal(lp3, lp) and torch.equal(emb3, emb)
    return mp


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("rank", [0, 7])
def test_config4_5gram_middle_partition_bitexact(pkg, cuda, five_gram, rank, monkeypatch):
    """The middle partition (bench.py --gpus N's default multi-GPU forward) at 5-gram, ranks 0 and 7 of P = 8."""
    f = five_gram
    mp = _middle_rank_check(pkg, f["m"], f["g"], f["xd"], f["lp"], f["emb"], rank, 8, monkeypatch)
    assert mp.n_own == f["N"] // 8
    assert mp.recv_ids.numel() < 0.35 * f["N"]  # ghost rows: about a third of N at P = 8


@pytest.mark.timeout(600)
def test_middle_partition_4gram_every_rank_bitexact(pkg, cuda, monkeypatch):
    """The same for every rank of P = 8 at 4-gram (the bench graph); together the ranks' rows tile the graph."""
    n, F = 4, 128
    N, s, d, c = pkg.synth.de_bruijn_edges(n)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    m = _model(pkg, [F, F, F], N, n).to(cuda).eval()
    xd = torch.randn(N, F, generator=torch.Generator().manual_seed(1234)).to(cuda)
    with torch.no_grad():
        lp, emb = m(pkg.Data(x=xd, graph=g))
    seen = torch.zeros(N, dtype=torch.int64, device=cuda)
    for rank in range(8):
        mp = _middle_rank_check(pkg, m, g, xd, lp, emb, rank, 8, monkeypatch)
        seen[mp.own] += 1
    assert bool((seen == 1).all())


@pytest.mark.timeout(600)
def test_middle_partition_bf16_rank_bitexact(pkg, cuda, monkeypatch):
    """bf16 mode through the middle partition (the bf16 middle-tile kernel over the rank's middles, bf16 ghost
    rows): ranks 0 and 3 of P = 4 at 4-gram match the single-GPU bf16 forward. The propagation rows are
    bit-identical (the same kernel, the same per-row sums, over the rank's middle range); the bf16 dense kernel's
    accumulation order depends on the row count, so its layer outputs agree to one bf16 rounding (1 ulp: up to
    0.44 on layer-1 values of ~100 here), not bit for bit, and those ulps carry through layer 2 and the decoder:
    |d| <= 5e-2 + 5e-2|ref| on the log-probs (measured max 0.09 on values ~ -3) and 2e-2 + 2e-2|ref| on the
    embeddings (measured max 0.004)."""
    from protgram_directgcn_amd import ops, shard
    n, F = 4, 128
    N, s, d, c = pkg.synth.de_bruijn_edges(n)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    m = _model(pkg, [F, F, F], N, n).to(cuda).eval()
    m.compute_dtype = torch.bfloat16
    xd = torch.randn(N, F, generator=torch.Generator().manual_seed(1234)).to(cuda).to(torch.bfloat16)
    conv = m.convs[0]
    prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in conv._dense_params())))
    with torch.no_grad():
        lp, emb = m(pkg.Data(x=xd, graph=g))
        h1 = ops.layer_dense(ops.spmm3(g, xd), prm, 0, constant=conv.constant.detach(), res_x=xd, act=True)
    assert h1.dtype == torch.bfloat16

    def fill(self, i, c):
        r0, r1 = self.recv_slices[c]
        assert self.recv[i].dtype == torch.bfloat16  # bf16 rows on the wire in bf16 mode
        self.recv[i][r0:r1] = h1[self.mp.recv_ids[r0:r1]]

    monkeypatch.setattr(shard.MiddleRunner, "_exchange", fill)
    for rank in (0, 3):
        mp = shard.middle_partition(g, rank, 4, chunks=2)
        lp2, emb2 = shard.MiddleRunner(m, mp, xd)()
        torch.cuda.synchronize()
        assert torch.equal(ops.spmm3_middles(g, xd, mp.m0, mp.m1), ops.spmm3(g, xd)[mp.own])  # bit-identical
        for got, ref, tol in ((lp2, lp[mp.global_rows], 5e-2), (emb2, emb[mp.global_rows], 2e-2)):
            assert bool(((got.float() - ref.float()).abs() <= tol + tol * ref.float().abs()).all()), rank


# ---------------------------------------------------------------------------------------------------------------
# config 5
# ---------------------------------------------------------------------------------------------------------------
@pytest.mark.timeout(900)
def test_config5_bf16_4gram_256_training_vs_fp32(pkg, cuda):
    from protgram_directgcn_amd import train
    n, dims = 4, [128, 256, 256, 256]
    N, s, d, c = pkg.synth.de_bruijn_edges(n)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    x = torch.randn(N, dims[0], generator=torch.Generator().manual_seed(1234)).to(cuda)
    y = _labels(N, n).to(cuda)
    data = pkg.Data(x=x, graph=g)
    grads, losses = [], []
    for dt in (torch.float32, torch.bfloat16):
        m = _model(pkg, dims, N, n).to(cuda).eval()
        m.compute_dtype = dt
        with torch.amp.autocast("cuda", enabled=True):  # the trainer's loop (trainer :91-100)
            lp, emb = m(data)
            loss = Fn.nll_loss(lp, y) + LAM * sum(p.norm(2).pow(2) for p in m.parameters())
        assert lp.dtype == torch.float32 and emb.dtype == torch.float32
        loss.backward()
        losses.append(float(loss.detach()))
        grads.append({k: p.grad.detach().float().clone() for k, p in m.named_parameters()})
    assert abs(losses[0] - losses[1]) < 2e-2 * abs(losses[0]), losses
    for k, g32 in grads[0].items():
        g16 = grads[1][k]
        cos = float((g32 * g16).sum() / (g32.norm() * g16.norm() + 1e-30))
        assert cos > 0.99, (k, cos)
    # the full step in bf16 mode: train_step + train.Adam under autocast + GradScaler; the loss goes down
    m = _model(pkg, dims, N, n).to(cuda).eval()
    m.compute_dtype = torch.bfloat16
    opt = train.Adam(m.parameters(), lr=LR)
    scaler = torch.amp.GradScaler("cuda", enabled=True)
    ls = [float(train.train_step(m, data, y, opt, l2_lambda=LAM, scaler=scaler)) for _ in range(5)]
    assert all(np.isfinite(ls)) and ls[-1] < ls[0], ls


# bf16 model-level tolerance, stated here and in DESIGN.md §10: against float64 autograd on the same
# bf16-rounded input (fp32 parameters and edge weights, exact in float64), every element d of an output or gradient obeys
#   |d| <= 2^-8 (C_REL |ref| + C_MAX max|ref|)      (max over the tensor)
# bf16 mode rounds each stored tensor once (RNE, unit roundoff 2^-8 of the stored value): forward x, then per layer Z
# and h (7 roundings on the path to the log-probs of a 3-layer model): (C_REL, C_MAX) = (8, 2). The backward also rounds
# dZ (3F wide), dpre and the layer gradient dY per layer, and dY is a sum of the transposed propagation and the
# residual's gradient: where those cancel, a rounding of 2^-8 of an addend is large against the result, so the per-node
# gradients (the constant's is dpre itself, elementwise) carry errors proportional to the addends, not to the element:
# (16, 16) for gradients. Measured on config 5 (profiles/r06_bf16_elementwise.txt): forward max |d| <= 1.4 x 2^-8
# max|ref|, weight / bias / gate gradients <= 4, the per-node constants' gradients up to 10.4.
BF16_TOL = {"forward": (8.0, 2.0), "grad": (16.0, 16.0)}


def _bf16_close(got, ref, kind, what):
    """(failure message or None, the largest |d| / 2^-8 max|ref|, the largest |d| / 2^-8 |ref| where |ref| >= max|ref|/16)
    of one tensor against the stated bf16 tolerance."""
    c_rel, c_max = BF16_TOL[kind]
    got, ref = got.detach().double(), ref.detach().double()
    mx = float(ref.abs().max())
    bound = 2.0 ** -8 * (c_rel * ref.abs() + c_max * mx)
    d = (got - ref).abs()
    r_max = float(d.max()) / (2.0 ** -8 * mx + 1e-300)
    big = ref.abs() >= mx / 16
    r_rel = float((d[big] / (2.0 ** -8 * ref.abs()[big])).max()) if bool(big.any()) else 0.0
    bad = d > bound
    msg = None
    if bool(bad.any()):
        msg = (f"{what}: {int(bad.sum())} of {d.numel()} outside 2^-8 ({c_rel} |ref| + {c_max} max|ref|); max |d| "
               f"{float(d.max()):.3e}, max|ref| {mx:.3e}")
    return msg, round(r_max, 3), round(r_rel, 3)


@pytest.mark.timeout(900)
def test_config5_bf16_elementwise_vs_float64(pkg, cuda):
    """Config 5's model in bf16 mode (4-gram, dims [128, 256, 256, 256], eval-mode dropout): log-probs, embeddings, the
    input's gradient and EVERY parameter gradient of the trainer's loss (nll + 1e-7 sum ||p||^2), elementwise within
    the stated bf16 tolerance of float64 autograd (the oracle, on the GPU) on the same bf16-rounded input. The GPU's
    leaky_relu / ReLU branch choices are handed to the oracle (act_masks) as in config 3: a pre-activation within
    bf16 rounding of 0 may sit on either side of the kink."""
    n, dims = 4, [128, 256, 256, 256]
    N, s, d, c = pkg.synth.de_bruijn_edges(n)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    m = _model(pkg, dims, N, n).to(cuda).eval()
    m.compute_dtype = torch.bfloat16
    xb = torch.randn(N, dims[0], generator=torch.Generator().manual_seed(1234)).to(torch.bfloat16).to(cuda)
    y = _labels(N, n).to(cuda)
    xd = xb.clone().requires_grad_(True)
    h, masks = xd, []
    for conv, res in zip(m.convs, m.res_projs):  # ProtGramDirectGCN.body (eval) written out, keeping the branches
        if isinstance(res, torch.nn.Linear):
            h = conv.fused_forward(h, g, None, res_x=h, W_res=res.weight, b_res=res.bias, act=True)
        else:
            h = conv.fused_forward(h, g, None, res_x=h, act=True)
        assert h.dtype == torch.bfloat16
        masks.append((h > 0).detach())
    hook = m.decoder_fc[1].register_forward_hook(lambda mod, inp, out: masks.append((inp[0] > 0).detach()))
    lp, emb = m.head(h)
    hook.remove()
    loss = Fn.nll_loss(lp, y) + LAM * sum(p.norm(2).pow(2) for p in m.parameters())
    loss.backward()
    torch.cuda.synchronize()

    ei, w = _csr_coo(g)
    ei = ei.to(cuda)
    w64 = [t.to(cuda).double() for t in w]
    p64 = {k: v.detach().double().requires_grad_(True) for k, v in m.state_dict().items()}
    x64 = xb.double().requires_grad_(True)
    lp64, emb64 = oc.model_forward(p64, dims, x64, ei, w64[0], ei, w64[1], ei, w64[2], n_gram_len=n,
                                   prop=oc.propagate_chunked, act_masks=masks)
    loss64 = Fn.nll_loss(lp64, y) + LAM * sum(v.norm(2).pow(2) for v in p64.values())
    loss64.backward()
    assert abs(float(loss) - float(loss64)) <= 2.0 ** -8 * 8.0 * abs(float(loss64)), (float(loss), float(loss64))
    res = {"log_probs": _bf16_close(lp, lp64, "forward", "log_probs"),
           "emb": _bf16_close(emb, emb64, "forward", "embeddings"),
           "grad x": _bf16_close(xd.grad, x64.grad, "grad", "grad x")}
    for k, prm in m.named_parameters():
        res[k] = _bf16_close(prm.grad, p64[k].grad, "grad", f"grad {k}")
    # the margins against the stated constants: max |d| / 2^-8 max|ref|, and max |d| / 2^-8 |ref| over the elements
    # with |ref| >= max|ref| / 16
    print("bf16 vs float64 (max |d| / 2^-8 max|ref|, max |d| / 2^-8 |ref| on large elements):",
          {k: v[1:] for k, v in res.items()})
    fails = [v[0] for v in res.values() if v[0]]
    assert not fails, "\n".join(fails)
