"""Halo-recompute partition (shard.halo_partition / halo_forward): the communication-free multi-GPU forward.

CPU tests: the partition's structure (every layer's rows are a prefix of the rank's node order, later layers
read only rows the previous layer computed, the relabelled CSR keeps each row's entries in order, the owned
rows of all ranks tile the graph) and the forward with CPU stand-ins for the HIP kernels against the
single-process oracle, in one process and in world_size-2 gloo processes (the bench's N>1 launch shape).
The GPU parity test (bit-identical to the single-GPU forward) is in test_gpu_parity.py."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [REPO, HERE]

from test_shard_gloo import _cpu_layer_dense_impl, _cpu_spmm3, _free_port  # noqa: E402


def _cpu_spmm3_gated(g, x, prm, gate_mode, flags=None, out=None):
    Z = _cpu_spmm3(g, x)
    M, F = g.n_rows, x.size(1)

    def gate(k):
        v = prm[k]
        return v.reshape(1, 1).expand(M, 1) if gate_mode == 1 else v[:M]

    ci, co, cd, cu, ca = (gate(k) for k in ("C_in", "C_out", "C_directed", "C_undirected", "C_all"))
    for q, s in enumerate((ca * cd * ci, ca * cd * co, ca * cu)):
        Z[:, q * F:(q + 1) * F] *= s
    return Z


def _cpu_layer_dense_pregated(Z, prm, gate_mode, rows=None, constant=None, res_x=None, W_res=None, b_res=None,
                              act=False, slope=0.01, flags=None, out=None, pregated=False, packs=None, drop=None):
    assert drop is None, "the CPU stand-in has no fused dropout"
    if not pregated:
        return _cpu_layer_dense_impl(Z, prm, gate_mode, rows, constant, res_x, W_res, b_res, act, slope)
    # pre-gated operand: sum_q Zg_q W_q^T + sum_q s_q b_q (the gates still scale the biases)
    M, F = Z.size(0), Z.size(1) // 3

    def gate(k):
        v = prm[k]
        return v.reshape(1, 1).expand(M, 1) if gate_mode == 1 else v[:M]

    ci, co, cd, cu, ca = (gate(k) for k in ("C_in", "C_out", "C_directed", "C_undirected", "C_all"))
    s = [ca * cd * ci, ca * cd * co, ca * cu]
    Ws = prm["W_shared"]
    W = [prm["W_main_in"] + Ws, prm["W_main_out"] + Ws, prm["W_undirected"] + Ws]
    b = [prm["b_main_in"] + prm["b_dir_shared_in"], prm["b_main_out"] + prm["b_dir_shared_out"],
         prm["b_undirected"] + prm["b_undirected_shared"]]
    y = sum(Z[:, q * F:(q + 1) * F] @ W[q].t() + s[q] * b[q] for q in range(3))
    if constant is not None and gate_mode == 0:
        y = y + constant[:M]
    if res_x is not None:
        y = y + (res_x @ W_res.t() + b_res if W_res is not None else res_x)
    return torch.nn.functional.leaky_relu(y, slope) if act else y


def _setup(pkg, n=2, dims=(16, 16, 12, 12), vec=True):
    from oracle import graph_cpu as og
    N, s, d, c = pkg.synth.de_bruijn_edges(n)
    m = og.build_matrices(N, s, d, c)
    g = pkg.graph.csr_from_coo(N, *m["in"], *m["out"], *m["und"], cache=False)
    g.row_order = pkg.graph.locality_schedule(N, torch.from_numpy(s), torch.from_numpy(d))
    torch.manual_seed(0)
    model = pkg.ProtGramDirectGCN(list(dims), N, 5, n, 0, 512, 0.5, vec).eval()
    with torch.no_grad():
        gen = torch.Generator().manual_seed(7)
        for name, p in model.named_parameters():
            leaf = name.split(".")[-1]
            if leaf.startswith("C_"):
                p.copy_(torch.rand(p.shape, generator=gen) + 0.5)
            elif "bias" in leaf:
                p.copy_(torch.rand(p.shape, generator=gen) * 0.2 - 0.1)
    x = torch.randn(N, dims[0], generator=torch.Generator().manual_seed(1234))
    return N, m, g, model, x


def _patch(ops):
    ops.spmm3 = _cpu_spmm3
    ops.spmm3_gated = _cpu_spmm3_gated
    ops.layer_dense = _cpu_layer_dense_pregated


@pytest.fixture(scope="module")
def pkg():
    from __graft_entry__ import load_package
    return load_package()


@pytest.mark.parametrize("world,layers", [(1, 2), (2, 2), (3, 1), (4, 3), (8, 2)])
def test_halo_partition_structure(pkg, world, layers):
    from protgram_directgcn_amd import shard
    N, m, g, model, x = _setup(pkg, n=3)
    rp, e = g.rowptr, g.edges3
    owned = []
    for rank in range(world):
        hp = shard.halo_partition(g, rank, world, layers)
        perm = hp.perm
        assert torch.equal(torch.sort(perm).values, torch.arange(N))
        rows = hp.layer_rows
        assert len(rows) == layers and all(a >= b for a, b in zip(rows, rows[1:]))
        for i, gi in enumerate(hp.graphs):
            assert gi.n_rows == rows[i]
            col = gi.edges3[:, 0].long()
            assert int(col.max()) < (N if i == 0 else rows[i - 1])  # a layer reads only rows computed before
            if gi.row_order is not None:
                assert torch.equal(torch.sort(gi.row_order.long()).values, torch.arange(rows[i]))
        g0 = hp.graphs[0]
        inv = torch.empty(N, dtype=torch.long)
        inv[perm] = torch.arange(N)
        for j in range(0, rows[0], max(1, rows[0] // 97)):  # relabelled rows keep their entries in order
            o = int(perm[j])
            ref = e[rp[o]:rp[o + 1]].clone()
            ref[:, 0] = inv[ref[:, 0].long()].int()
            assert torch.equal(g0.edges3[g0.rowptr[j]:g0.rowptr[j + 1]], ref)
        owned.append(hp.global_rows)
    allr = torch.cat(owned)
    assert torch.equal(torch.sort(allr).values, torch.arange(N))  # the owned rows tile the graph
    if world == 8 and layers == 2:  # locality-schedule ownership: the 1-hop halo is far below N
        assert max(shard.halo_partition(g, r, world, 2).layer_rows[0] for r in range(world)) < 0.6 * N


@pytest.mark.parametrize("world,dims,vec", [(2, (16, 16, 12, 12), True), (3, (16, 12, 12), True),
                                            (5, (16, 16, 16), False)])
def test_halo_forward_matches_oracle(pkg, world, dims, vec):
    from oracle import directgcn_cpu as oc
    from protgram_directgcn_amd import ops, shard
    saved = (ops.spmm3, ops.spmm3_gated, ops.layer_dense)
    _patch(ops)
    try:
        N, m, g, model, x = _setup(pkg, n=2, dims=dims, vec=vec)
        p = {k: v.detach() for k, v in model.state_dict().items()}
        lp_r, emb_r = oc.model_forward(p, list(dims), x, *m["in"], *m["out"], *m["und"], n_gram_len=2,
                                       use_vector_coeffs=vec)
        L = len(dims) - 1
        for rank in range(world):
            hp = shard.halo_partition(g, rank, world, L)
            lp, emb = shard.halo_forward(model, hp, shard.halo_inputs(model, hp, x))
            gr = hp.global_rows
            assert lp.shape == (hp.owned, 5)
            torch.testing.assert_close(lp, lp_r[gr], rtol=1e-5, atol=1e-5)
            torch.testing.assert_close(emb, emb_r[gr], rtol=1e-5, atol=1e-5)
    finally:
        ops.spmm3, ops.spmm3_gated, ops.layer_dense = saved


def _gloo_worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [REPO, HERE]
    from __graft_entry__ import load_package
    pkg = load_package()
    from oracle import directgcn_cpu as oc
    from protgram_directgcn_amd import ops, shard
    _patch(ops)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dims = [16, 16, 12, 12]
        N, m, g, model, x = _setup(pkg, n=2, dims=dims)
        hp = shard.halo_partition(g, rank, world, len(dims) - 1)
        inputs = shard.halo_inputs(model, hp, x)
        dist.barrier()
        lp, emb = shard.halo_forward(model, hp, inputs)  # no collective inside
        dist.barrier()
        # test-only reassembly: every rank's rows and ids to rank 0's view
        n_max = torch.tensor([hp.owned])
        dist.all_reduce(n_max, op=dist.ReduceOp.MAX)
        pad = int(n_max)
        ids = torch.full((pad,), -1, dtype=torch.long)
        ids[:hp.owned] = hp.global_rows
        lpp = torch.zeros(pad, lp.size(1))
        lpp[:hp.owned] = lp
        all_ids = [torch.empty_like(ids) for _ in range(world)]
        all_lp = [torch.empty_like(lpp) for _ in range(world)]
        dist.all_gather(all_ids, ids)
        dist.all_gather(all_lp, lpp)
        p = {k: v.detach() for k, v in model.state_dict().items()}
        lp_r, _ = oc.model_forward(p, dims, x, *m["in"], *m["out"], *m["und"], n_gram_len=2)
        full = torch.full_like(lp_r, float("nan"))
        for i, l in zip(all_ids, all_lp):
            k = i >= 0
            full[i[k]] = l[k]
        ok = bool(torch.allclose(full, lp_r, rtol=1e-5, atol=1e-5))
        out_q.put((rank, ok, float((full - lp_r).abs().max())))
    finally:
        dist.destroy_process_group()


def test_halo_forward_gloo_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in res:
        assert r[1], f"rank {r[0]}: max |d| {r[2]:.2e}"
