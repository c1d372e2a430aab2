"""The middle partition with its ghost-row exchange (shard.middle_partition / middle_forward), on the CPU:
  * structure: the ranks' owned rows tile the graph; what rank q sends rank p is exactly what p receives from q, in
    the same order; a rank's own rows plus the ghost rows it receives are exactly the rows its middles read;
  * the forward at world sizes 2 and 3 with gloo (the product's all_to_all_single) against the single-process
    oracle, with CPU stand-ins for the HIP kernels (the product has no CPU path)."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _graph(pkg, n):
    from oracle import graph_cpu as og
    N, s, d, c = pkg.synth.de_bruijn_edges(n)
    m = og.build_matrices(N, s, d, c)
    return N, m, pkg.graph.csr_from_coo(N, *m["in"], *m["out"], *m["und"], cache=False)


@pytest.mark.parametrize("n,world", [(3, 1), (3, 2), (3, 3), (3, 8), (4, 8)])
def test_middle_partition_structure(pkg, n, world):
    from protgram_directgcn_amd import shard
    N, _, g = _graph(pkg, n)
    parts = [shard.middle_partition(g, r, world) for r in range(world)]
    owned = torch.cat([p.own for p in parts])
    assert torch.equal(torch.sort(owned).values, torch.arange(N))
    K = 20
    for p in parts:
        assert p.n_own == (p.m1 - p.m0) * K * K
        assert p.send_counts[p.rank] == 0 and p.recv_counts[p.rank] == 0
        assert sum(p.send_counts) == p.send_pos.numel() and sum(p.recv_counts) == p.recv_ids.numel()
        reads = shard._middle_reads(K, n, p.m0, p.m1, torch.device("cpu"))
        got = torch.sort(torch.cat([p.own, p.recv_ids])).values
        assert torch.equal(got, reads)  # own rows + ghosts == the rows its middles read, each once
        cols = torch.unique(p.own_csr.edges3[:, 0].long())
        assert bool(torch.isin(cols, reads).all())
    for q in parts:  # q -> p: q's send list (as global ids) == p's receive list from q
        off_s = [0]
        for c in q.send_counts:
            off_s.append(off_s[-1] + c)
        for p in parts:
            if p.rank == q.rank:
                continue
            sent = q.own[q.send_pos[off_s[p.rank]:off_s[p.rank + 1]]]
            off_r = sum(p.recv_counts[:q.rank])
            assert torch.equal(sent, p.recv_ids[off_r:off_r + p.recv_counts[q.rank]]), (q.rank, p.rank)
    if world == 8 and n == 4:  # ghost rows received per rank: well below the (P-1)/P N of a node-range all-gather
        assert max(p.recv_ids.numel() for p in parts) < 0.5 * N


@pytest.mark.parametrize("n,world,chunks", [(3, 2, 2), (3, 3, 3), (4, 8, 4)])
def test_middle_partition_chunked_lists(pkg, n, world, chunks):
    """With the owned middles in sub-ranges, sub-range c of rank q sends p exactly what p receives from q in c (same
    order), the sub-ranges tile the owned middles, and the per-pair totals equal the unchunked partition's."""
    from protgram_directgcn_amd import shard
    N, _, g = _graph(pkg, n)
    parts = [shard.middle_partition(g, r, world, chunks=chunks) for r in range(world)]
    flat = [shard.middle_partition(g, r, world) for r in range(world)]
    for p, f in zip(parts, flat):
        assert p.chunks == chunks and p.chunk_bounds[0][0] == p.m0 and p.chunk_bounds[-1][1] == p.m1
        assert all(a[1] == b[0] for a, b in zip(p.chunk_bounds, p.chunk_bounds[1:]))
        assert p.send_counts == f.send_counts and p.recv_counts == f.recv_counts
        assert torch.equal(torch.sort(p.recv_ids).values, torch.sort(f.recv_ids).values)

    def seg(counts, c, r):  # offset of (chunk c, rank r) in a chunk-major, rank-minor list
        off = sum(sum(counts[cc]) for cc in range(c)) + sum(counts[c][:r])
        return off, off + counts[c][r]

    for q in parts:
        for p in parts:
            if p.rank == q.rank:
                continue
            for c in range(chunks):
                a, b = seg(q.chunk_send, c, p.rank)
                sent = q.own[q.send_pos[a:b]]
                a2, b2 = seg(p.chunk_recv, c, q.rank)
                assert torch.equal(sent, p.recv_ids[a2:b2]), (q.rank, p.rank, c)
                lo, hi = q.chunk_bounds[c]  # every row q sends in sub-range c comes from one of its middles
                mids = (sent % 20 ** (n - 1)) // 20
                assert bool(((mids >= lo) & (mids < hi)).all())


def test_middle_partition_rejects_other_graphs(pkg):
    from protgram_directgcn_amd import shard
    _, _, g2 = _graph(pkg, 2)
    with pytest.raises(NotImplementedError):
        shard.middle_partition(g2, 0, 2)  # a single middle
    from oracle import graph_cpu as og
    N, s, d, c = pkg.synth.de_bruijn_edges(3)
    s, d = s.copy(), d.copy()
    d[0] = (s[0] + 4210) % N  # 0 -> 4210 = 10.10.10: not a row that middles 0..9 (rank 0) read
    m = og.build_matrices(N, s, d, c)
    g = pkg.graph.csr_from_coo(N, *m["in"], *m["out"], *m["und"], cache=False)
    with pytest.raises(ValueError):
        shard.middle_partition(g, 0, 2)


def _worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [REPO, HERE]
    from __graft_entry__ import load_package
    pkg = load_package()
    from protgram_directgcn_amd import ops, shard
    from oracle import directgcn_cpu as oc
    from test_shard_gloo import _cpu_layer_dense, _cpu_spmm3
    ops.spmm3 = _cpu_spmm3
    ops.layer_dense = _cpu_layer_dense
    ops.rows_gather = lambda src, idx, out=None, check_idx=True: src[idx] if out is None else out.copy_(src[idx])
    ops.rows_scatter = lambda src, idx, dst, check_idx=True: dst.index_copy_(0, idx, src)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        N, m, g = _graph(pkg, 3)
        dims = [16, 16, 12, 12]
        torch.manual_seed(0)
        model = pkg.ProtGramDirectGCN(dims, N, 5, 3, 0, 512, 0.5, True).eval()
        with torch.no_grad():
            for name, p in model.named_parameters():
                if name.split(".")[-1].startswith("C_"):
                    p.uniform_(0.5, 1.5)
        x = torch.randn(N, 16, generator=torch.Generator().manual_seed(1234))
        mp_ = shard.middle_partition(g, rank, world)
        p = {k: v.detach() for k, v in model.state_dict().items()}
        lp_r, emb_r = oc.model_forward(p, dims, x, *m["in"], *m["out"], *m["und"], n_gram_len=3)
        lp, emb = shard.middle_forward(model, mp_, x)
        rows = mp_.global_rows
        ok = (torch.allclose(lp, lp_r[rows], rtol=1e-5, atol=1e-5)
              and torch.allclose(emb, emb_r[rows], rtol=1e-5, atol=1e-5))
        run = shard.MiddleRunner(model, mp_, x)  # CPU input: its segments run eagerly
        lp2, emb2 = run()
        ok = ok and torch.equal(lp2, lp) and torch.equal(emb2, emb)
        mpc = shard.middle_partition(g, rank, world, chunks=2)  # layer 1 in two sub-ranges, exchanged per sub-range
        lp3, emb3 = shard.MiddleRunner(model, mpc, x)()
        ok = ok and torch.equal(lp3, lp) and torch.equal(emb3, emb)
        # middle_forward on the chunked partition: its lists are (chunk, rank)-grouped (at world >= 3
        # one all_to_all over all chunks sent rows to the wrong ranks)
        lp5, emb5 = shard.middle_forward(model, mpc, x)
        ok = ok and torch.equal(lp5, lp) and torch.equal(emb5, emb)
        lp4, emb4 = shard.MiddleRunner(model, mp_, x, replicate=True)()  # layer 1 on every row, no exchange
        ok = ok and torch.allclose(lp4, lp, rtol=1e-5, atol=1e-6) and torch.allclose(emb4, emb, rtol=1e-5, atol=1e-6)
        out_q.put((rank, int(rows.numel()), bool(ok), float((lp - lp_r[rows]).abs().max())))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_middle_forward_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=280) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert sum(r[1] for r in res) == 8000
    assert all(r[2] for r in res), res


def _cpu_spmm3t_rows(rowptr_t, edges3_t, rows, G, n_out, flags=None):
    """CPU stand-in for ops.spmm3t_rows (pg_spmm3t_f32 over a row list); rows outside the list stay NaN."""
    n = rowptr_t.numel() - 1
    r = torch.repeat_interleave(torch.arange(n), rowptr_t[1:] - rowptr_t[:-1])
    col = edges3_t[:, 0].long()
    F = G.size(1) // 3
    dX = torch.zeros(n_out, F, dtype=torch.float32)
    for k in range(3):
        w = edges3_t[:, 1 + k].contiguous().view(torch.float32)
        dX.index_add_(0, r, w[:, None] * G[col, k * F:(k + 1) * F].float())
    keep = torch.zeros(n_out, dtype=torch.bool)
    keep[rows.long()] = True
    dX[~keep] = float("nan")
    return dX.to(G.dtype)


def _mid_train_worker(rank, world, port, out_q, chunks, bf16):
    """shard.MiddleTrainer (middle partition: owned-middle propagation, ghost-row exchange forward and its transpose
    backward, owned-row per-node state, replicated-gradient all-reduce) for two steps against the single-process
    oracle's autograd + Adam; also the exchange's adjointness <E h, g> = <h, E^T g> summed over ranks."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [REPO, HERE]
    from __graft_entry__ import load_package
    pkg = load_package()
    from protgram_directgcn_amd import ops, shard, train
    from oracle import directgcn_cpu as oc
    import torch.nn.functional as F
    from test_shard_gloo import (_any_dtype, _cpu_layer_dense, _cpu_layer_dense_backward, _cpu_spmm3)
    ops.spmm3 = _any_dtype(_cpu_spmm3)
    ops.spmm3t_rows = _cpu_spmm3t_rows
    ops.layer_dense = _any_dtype(_cpu_layer_dense)
    ops.layer_dense_backward = _any_dtype(_cpu_layer_dense_backward, out_keys=("dpre", "dZ", "dres"))
    train.l2_sqsum = lambda ps: sum((p.detach().float() ** 2).sum() for p in ps)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bad = []
    try:
        N, m, g = _graph(pkg, 3)
        g.symmetric = True  # the n-gram matrices are symmetric (csr_from_coo on the CPU keeps a separate transpose)
        mp_ = shard.middle_partition(g, rank, world, chunks=chunks)
        comm = shard.TorchComm()
        # adjointness of the exchange (F = 3)
        gen = torch.Generator().manual_seed(100 + rank)
        h = torch.randn(mp_.n_own, 3, generator=gen, dtype=torch.float64)
        G = torch.randn(N, 3, generator=gen, dtype=torch.float64)
        X = shard.forward_exchange(mp_, h, comm)
        valid = torch.cat([mp_.own, mp_.recv_ids])
        lhs = (X[valid] * G[valid]).sum()
        d = G[mp_.own] + shard.reverse_exchange(mp_, G, comm).double()
        rhs = (h * d).sum()
        t = torch.stack([lhs, rhs])
        dist.all_reduce(t)
        if abs(float(t[0] - t[1])) > 1e-9 * abs(float(t[0])):
            bad.append(("adjoint", float(t[0]), float(t[1])))
        mt = shard.middle_transpose(mp_)
        if not torch.equal(torch.sort(mt.rows.long()).values, torch.sort(valid).values):
            bad.append("transpose rows != own + ghost rows")
        # the training step
        dims = [16, 16, 16, 12]
        torch.manual_seed(0)
        model = pkg.ProtGramDirectGCN(dims, N, 5, 3, 0, 512, 0.5, True).eval()
        with torch.no_grad():
            gen = torch.Generator().manual_seed(5)
            for name, p in model.named_parameters():
                leaf = name.split(".")[-1]
                if leaf.startswith("C_"):
                    p.copy_(torch.rand(p.shape, generator=gen) + 0.5)
                elif "bias" in leaf:
                    p.copy_(torch.rand(p.shape, generator=gen) * 0.2 - 0.1)
        if bf16:
            model.compute_dtype = torch.bfloat16
        ref = {k: v.detach().clone().requires_grad_(True) for k, v in model.state_dict().items()}
        x = torch.randn(N, 16, generator=torch.Generator().manual_seed(1234))
        y = (torch.arange(N) // 400) % 5
        lam, steps, lr = 1e-3, 2, 1e-2
        tr = shard.MiddleTrainer(model, mp_, l2_lambda=lam, comm=comm,
                                 optimizer_factory=lambda ps: torch.optim.Adam(ps, lr=lr))
        losses, grads = [], []
        for _ in range(steps):
            loss = tr.step(x, y[mp_.own])
            losses.append(float(loss))
            gd = {}
            for name, p in model.named_parameters():
                if shard._is_node_param(name, p, N):
                    gd[name] = tr.own[int(name.split(".")[1])][name.split(".")[-1]].grad.clone()
                else:
                    gd[name] = p.grad.clone()
            grads.append(gd)
        ropt = torch.optim.Adam(list(ref.values()), lr=lr)
        rlosses, rgrads = [], []
        for _ in range(steps):
            ropt.zero_grad()
            lp, _ = oc.model_forward(ref, dims, x, *m["in"], *m["out"], *m["und"], n_gram_len=3)
            loss = F.nll_loss(lp, y) + lam * sum(v.norm(2).pow(2) for v in ref.values())
            loss.backward()
            rgrads.append({k: v.grad.clone() for k, v in ref.items()})
            ropt.step()
            rlosses.append(float(loss))
        for st in range(steps):
            tol = 2e-2 * abs(rlosses[st]) if bf16 else 1e-5 * abs(rlosses[st]) + 1e-6
            if abs(losses[st] - rlosses[st]) > tol:
                bad.append(("loss", st, losses[st], rlosses[st]))
        for name, gg in grads[0].items():
            r = rgrads[0][name]
            if shard._is_node_param(name, r, N):
                r = r[mp_.own]
            if bf16:
                cos = float((gg.float() * r).sum() / (gg.float().norm() * r.norm() + 1e-30))
                if cos < 0.99:
                    bad.append((name, "cos", cos))
            else:
                err = float((gg - r).abs().max())
                if err > 2e-5 * float(r.abs().max()) + 1e-6:
                    bad.append((name, "grad", err))
        tr.gather()  # every rank's rows, on every rank
        if not bf16:
            for name, p in model.named_parameters():
                err = float((p.detach() - ref[name].detach()).abs().max())
                if err > 2e-5:
                    bad.append(("param " + name, err))
        out_q.put((rank, mp_.n_own, not bad, str(bad[:4])))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,chunks,bf16", [(2, 1, False), (3, 2, False), (3, 1, True)])
def test_middle_trainer_gloo(world, chunks, bf16):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mid_train_worker, args=(r, world, port, q, chunks, bf16)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=280) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert sum(r[1] for r in res) == 8000
    for r in res:
        assert r[2], f"rank {r[0]}: {r[3]}"


def _cpu_scatter_parts(mp_):
    """CPU stand-in for ops.spmm3t_scatter on partition mp_: T [3 n_own, F] (D | P | S) from the owned rows' CSR,
    each entry (i = a.M.b <- j) to the part row of j that the kernel writes (prefix M: P, suffix M: S, else D = i)."""
    def fn(splan, G, flags=None):
        oc = mp_.own_csr
        K, n = mp_.K, mp_.ngram
        Kn1, Kn2 = K ** (n - 1), K ** (n - 2)
        n_own, F = mp_.n_own, G.size(1) // 3
        ipos = torch.repeat_interleave(torch.arange(n_own), oc.rowptr[1:] - oc.rowptr[:-1])
        j = oc.edges3[:, 0].long()
        l = ipos // (K * K)
        M = mp_.m0 + l
        P_row = n_own + l * K * K + ((j // K) % K) * K + j % K
        S_row = 2 * n_own + l * K * K + (j // Kn1) * K + (j // Kn2) % K
        t = torch.where(j // (K * K) == M, P_row, torch.where(j % Kn2 == M, S_row, ipos))
        d_ok = (j // (K * K) == M) | (j % Kn2 == M) | (j == mp_.own[ipos])
        assert bool(d_ok.all()), "an entry outside the out / in / diagonal slots"
        T = torch.zeros(3 * n_own, F, dtype=torch.float64)
        Gd = G.double()
        for k in range(3):
            w = oc.edges3[:, 1 + k].contiguous().view(torch.float32).double()
            T.index_add_(0, t, w[:, None] * Gd[ipos, k * F:(k + 1) * F])
        return T.float()
    return fn


def _cpu_gather_sum(A, rowptr, idx, n_out, F, B=None, out_dtype=torch.float32):
    """CPU stand-in for ops.rows_gather_sum (fp32 sum in entry order)."""
    out = torch.zeros(n_out, F)
    cnt = rowptr[1:] - rowptr[:-1]
    rows = torch.repeat_interleave(torch.arange(n_out), cnt)
    k_of = torch.arange(int(rowptr[-1])) - torch.repeat_interleave(rowptr[:-1], cnt)
    v = idx.long()
    for k in range(int(cnt.max()) + 1 if n_out and cnt.numel() and int(cnt.max()) > 0 else 0):
        sel = k_of == k
        vv = v[sel]
        src = A[vv.clamp(min=0)].float()
        if B is not None:
            src = torch.where((vv >= 0).view(-1, 1), src, B[(-1 - vv).clamp(min=0)].float())
        out[rows[sel]] += src[:, :F]
    return out.to(out_dtype)


def _scatter_bwd_worker(rank, world, port, out_q, chunks):
    """The scatter-form backward (_MidExchangePropagate: part rows, ghost sums sent back, owned rows summed with the
    rows received) against the CSR composition (_MidExchange -> _MidPropagate) on the same rank, the kernels replaced
    by CPU stand-ins; the lists (shard.scatter_lists) and the exchange are the product's."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [REPO, HERE]
    from __graft_entry__ import load_package
    pkg = load_package()
    from protgram_directgcn_amd import ops, shard
    from test_shard_gloo import _cpu_spmm3
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bad = []
    try:
        N, m, g = _graph(pkg, 3)
        g.symmetric = True
        mp_ = shard.middle_partition(g, rank, world, chunks=chunks)
        comm = shard.TorchComm()
        ops.spmm3 = _cpu_spmm3
        ops.spmm3t_rows = _cpu_spmm3t_rows
        ops.spmm3t_scatter = _cpu_scatter_parts(mp_)
        ops.rows_gather_sum = _cpu_gather_sum
        shard.middle_scatter = lambda mp: shard.MiddleScatter(None, *shard.scatter_lists(mp))
        F = 8
        gen = torch.Generator().manual_seed(50 + rank)
        h = torch.randn(mp_.n_own, F, generator=gen)
        w = torch.randn(mp_.n_own, 3 * F, generator=gen)
        grads = []
        for fused in (True, False):
            hh = h.clone().requires_grad_(True)
            if fused:
                Z = shard._MidExchangePropagate.apply(hh, mp_, comm)
            else:
                Z = shard._MidPropagate.apply(shard._MidExchange.apply(hh, mp_, comm), mp_)
            (Z * w).sum().backward()
            grads.append(hh.grad)
        err = float((grads[0] - grads[1]).abs().max())
        if err > 1e-5 * float(grads[1].abs().max()) + 1e-6:
            bad.append(("grad", err))
        out_q.put((rank, not bad, str(bad)))
    except Exception as e:
        out_q.put((rank, False, repr(e)[:300]))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,chunks", [(3, 1), (3, 2)])
def test_scatter_backward_gloo(world, chunks):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_scatter_bwd_worker, args=(r, world, port, q, chunks)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=280) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for r in res:
        assert r[1], f"rank {r[0]}: {r[2]}"
