"""Multi-process (world_size 2 and 3, gloo, CPU) tests of the node-range partition (shard.py):
row slicing of the CSR, global-row gate/constant gathering, padded all-gather between layers; and the
sharded training step (reduce-scatter backward through the transposed column block, dense-gradient
all-reduce, communication-free per-node parameters) against the single-process oracle + Adam.
The two HIP kernels are replaced by CPU stand-ins inside this test (the product has no CPU path);
the result on every rank must equal the single-process oracle model forward."""
import os
import socket
import sys

import numpy as np
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


def _cpu_spmm3(g, x, out=None, fused=False, flags=None):
    rp, e = g.rowptr, g.edges3
    rows = torch.repeat_interleave(torch.arange(g.n_rows), rp[1:] - rp[:-1])
    col = e[:, 0].long()
    F = x.size(1)
    Z = torch.zeros(g.n_rows, 3 * F)
    for k in range(3):
        w = e[:, 1 + k].contiguous().view(torch.float32)
        Z[:, k * F:(k + 1) * F].index_add_(0, rows, w[:, None] * x[col])
    return Z


def _cpu_spmm3_t(g, G, flags=None):
    rp, e = g.rowptr_t, g.edges3_t
    n = rp.numel() - 1
    rows = torch.repeat_interleave(torch.arange(n), rp[1:] - rp[:-1])
    col = e[:, 0].long()
    F = G.size(1) // 3
    dX = torch.zeros(n, F)
    for k in range(3):
        w = e[:, 1 + k].contiguous().view(torch.float32)
        dX.index_add_(0, rows, w[:, None] * G[col, k * F:(k + 1) * F])
    return dX


def _cpu_layer_dense(Z, prm, gate_mode, rows=None, constant=None, res_x=None, W_res=None, b_res=None, act=False,
                     slope=0.01, flags=None, out=None, packs=None, drop=None):
    assert drop is None, "the CPU stand-in has no fused dropout"
    y = _cpu_layer_dense_impl(Z, prm, gate_mode, rows, constant, res_x, W_res, b_res, act, slope)
    if out is not None:
        out.copy_(y)
        return out
    return y


def _cpu_layer_dense_impl(Z, prm, gate_mode, rows=None, constant=None, res_x=None, W_res=None, b_res=None, act=False,
                          slope=0.01):
    M, F = Z.size(0), Z.size(1) // 3

    def gate(name):
        v = prm[name]
        return v.reshape(1, 1).expand(M, 1) if gate_mode == 1 else (v[rows] if rows is not None else v[:M])

    ci, co, cd, cu, ca = (gate(k) for k in ("C_in", "C_out", "C_directed", "C_undirected", "C_all"))
    s = [ca * cd * ci, ca * cd * co, ca * cu]
    Ws = prm["W_shared"]
    W = [prm["W_main_in"] + Ws, prm["W_main_out"] + Ws, prm["W_undirected"] + Ws]
    b = [prm["b_main_in"] + prm["b_dir_shared_in"], prm["b_main_out"] + prm["b_dir_shared_out"],
         prm["b_undirected"] + prm["b_undirected_shared"]]
    y = sum(s[k] * (Z[:, k * F:(k + 1) * F] @ W[k].t() + b[k]) for k in range(3))
    if constant is not None and gate_mode == 0:
        y = y + (constant[rows] if rows is not None else constant[:M])
    if res_x is not None:
        y = y + (res_x @ W_res.t() + b_res if W_res is not None else res_x)
    return torch.nn.functional.leaky_relu(y, slope) if act else y


def _cpu_layer_dense_backward(dY, Z, Y, prm, gate_mode, rows=None, res_x=None, W_res=None, b_res=None, act=False,
                              slope=0.01, flags=None, need_dZ=True, packs=None, drop_p=0.0, dpre_f32=False):
    """CPU stand-in for ops.layer_dense_backward (pg_directgcn_dense_bwd_f32): the same outputs from torch ops."""
    assert drop_p == 0.0, "the CPU stand-in has no fused dropout"
    M, F_in = Z.size(0), Z.size(1) // 3
    dpre = dY * torch.where(Y > 0, 1.0, slope) if act else dY

    def gate(name):
        v = prm[name]
        if gate_mode == 1:
            return v.reshape(1, 1).expand(M, 1)
        return (v[rows] if rows is not None else v[:M]).reshape(M, 1)

    ci, co, cd, cu, ca = (gate(k) for k in ("C_in", "C_out", "C_directed", "C_undirected", "C_all"))
    cad = ca * cd
    s = [cad * ci, cad * co, ca * cu]
    Wp = [prm["W_main_in"] + prm["W_shared"], prm["W_main_out"] + prm["W_shared"],
          prm["W_undirected"] + prm["W_shared"]]
    bp = [prm["b_main_in"] + prm["b_dir_shared_in"], prm["b_main_out"] + prm["b_dir_shared_out"],
          prm["b_undirected"] + prm["b_undirected_shared"]]
    dZ = torch.empty_like(Z)
    ds, dB, db = [], [], []
    for k in range(3):
        Zk = Z[:, k * F_in:(k + 1) * F_in]
        Gk = dpre @ Wp[k]
        dZ[:, k * F_in:(k + 1) * F_in] = s[k] * Gk
        ds.append((Gk * Zk).sum(1, keepdim=True) + dpre @ bp[k].reshape(-1, 1))
        sd = s[k] * dpre
        dB.append(sd.t() @ Zk)
        db.append(sd.sum(0))
    dres = None
    if W_res is not None:
        dres = dpre @ W_res
        dB.append(dpre.t() @ res_x)
    db.append(dpre.sum(0) if W_res is not None else torch.zeros_like(db[0]))
    dgate = torch.stack([(ds[0] * cad).reshape(M), (ds[1] * cad).reshape(M),
                         (ds[0] * ca * ci + ds[1] * ca * co).reshape(M), (ds[2] * ca).reshape(M),
                         (ds[0] * cd * ci + ds[1] * cd * co + ds[2] * cu).reshape(M)])
    return {"dpre": dpre, "dZ": dZ, "dres": dres, "dgate": dgate, "dB": torch.cat(dB, 1), "dbsum": torch.stack(db)}


def _worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [REPO, HERE]
    from __graft_entry__ import load_package
    pkg = load_package()
    from protgram_directgcn_amd import ops, shard
    from oracle import directgcn_cpu as oc
    from oracle import graph_cpu as og
    ops.spmm3 = _cpu_spmm3
    ops.layer_dense = _cpu_layer_dense
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        N, s, d, c = pkg.synth.de_bruijn_edges(2)
        m = og.build_matrices(N, s, d, c)
        g = pkg.graph.csr_from_coo(N, *m["in"], *m["out"], *m["und"], cache=False)
        torch.manual_seed(0)
        model = pkg.ProtGramDirectGCN([16, 16, 12, 12], N, 5, 2, 0, 512, 0.5, True).eval()
        with torch.no_grad():
            for name, p in model.named_parameters():
                if name.split(".")[-1].startswith("C_"):
                    p.uniform_(0.5, 1.5)
        x = torch.randn(N, 16, generator=torch.Generator().manual_seed(1234))
        part = shard.partition(g, rank, world)
        p = {k: v.detach() for k, v in model.state_dict().items()}
        lp_r, emb_r = oc.model_forward(p, [16, 16, 12, 12], x, *m["in"], *m["out"], *m["und"], n_gram_len=2)
        ok, err, first = True, 0.0, None
        for chunks in (1, 3):  # unchunked and chunked (overlapped) layer-boundary exchange
            lp, emb = shard.sharded_forward(model, part, x, chunks=chunks)
            ok = ok and (torch.allclose(lp, lp_r[part.r0:part.r1], rtol=1e-5, atol=1e-5)
                         and torch.allclose(emb, emb_r[part.r0:part.r1], rtol=1e-5, atol=1e-5))
            if first is None:
                first = lp
            else:
                ok = ok and torch.equal(first, lp)  # chunking changes the schedule, never the values
            err = max(err, float((lp - lp_r[part.r0:part.r1]).abs().max()))
        out_q.put((rank, part.r0, part.r1, bool(ok), err))
    finally:
        dist.destroy_process_group()


def _train_worker(rank, world, port, out_q):
    """Two sharded training steps (eval-mode dropout, L2 term on) vs the single-process oracle + Adam."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [REPO, HERE]
    from __graft_entry__ import load_package
    pkg = load_package()
    from protgram_directgcn_amd import ops, shard
    from oracle import directgcn_cpu as oc
    from oracle import graph_cpu as og
    import torch.nn.functional as F
    ops.spmm3 = _cpu_spmm3
    ops.spmm3_t = _cpu_spmm3_t
    ops.layer_dense = _cpu_layer_dense
    ops.layer_dense_backward = _cpu_layer_dense_backward
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        N, s, d, c = pkg.synth.de_bruijn_edges(2)
        m = og.build_matrices(N, s, d, c)
        g = pkg.graph.csr_from_coo(N, *m["in"], *m["out"], *m["und"], cache=False)
        dims = [16, 16, 12, 12]
        torch.manual_seed(0)
        model = pkg.ProtGramDirectGCN(dims, N, 5, 2, 0, 512, 0.5, True).eval()
        with torch.no_grad():
            gen = torch.Generator().manual_seed(5)
            for name, p in model.named_parameters():
                leaf = name.split(".")[-1]
                if leaf.startswith("C_"):
                    p.copy_(torch.rand(p.shape, generator=gen) + 0.5)
                elif "bias" in leaf:
                    p.copy_(torch.rand(p.shape, generator=gen) * 0.2 - 0.1)
        ref = {k: v.detach().clone().requires_grad_(True) for k, v in model.state_dict().items()}
        x = torch.randn(N, 16, generator=torch.Generator().manual_seed(1234))
        y = (torch.arange(N) // 20) % 5
        lam, steps = 1e-3, 2
        part = shard.partition(g, rank, world, transpose=True)
        opt = torch.optim.Adam(model.parameters(), lr=1e-2)
        losses = [shard.sharded_train_step(model, part, x, y[part.r0:part.r1], opt, l2_lambda=lam)
                  for _ in range(steps)]
        ropt = torch.optim.Adam(list(ref.values()), lr=1e-2)
        rlosses = []
        for _ in range(steps):
            ropt.zero_grad()
            lp, _ = oc.model_forward(ref, dims, x, *m["in"], *m["out"], *m["und"], n_gram_len=2)
            loss = F.nll_loss(lp, y) + lam * sum(v.norm(2).pow(2) for v in ref.values())
            loss.backward()
            ropt.step()
            rlosses.append(float(loss))
        bad = []
        if not np.allclose(losses, rlosses, rtol=1e-5, atol=1e-6):
            bad.append(("loss", losses, rlosses))
        for name, p in model.named_parameters():
            r = ref[name].detach()
            if shard._is_node_param(name, p, N):
                p, r = p[part.r0:part.r1], r[part.r0:part.r1]
            err = float((p.detach() - r).abs().max())
            if err > 2e-5:
                bad.append((name, err))
        shard.gather_node_params(model, part)
        for name, p in model.named_parameters():
            err = float((p.detach() - ref[name].detach()).abs().max())
            if err > 2e-5:
                bad.append(("gathered " + name, err))
        out_q.put((rank, part.r0, part.r1, not bad, str(bad[:4])))
    finally:
        dist.destroy_process_group()


def _any_dtype(fn, out_keys=None):
    """A CPU stand-in run in fp32 on bf16 inputs, its outputs rounded back to bf16 (the kernels' bf16 storage)."""
    def wrapped(*args, **kw):
        dt = next((a.dtype for a in args if torch.is_tensor(a) and a.is_floating_point()), torch.float32)
        args = [a.float() if torch.is_tensor(a) and a.dtype == torch.bfloat16 else a for a in args]
        kw = {k: (v.float() if torch.is_tensor(v) and v.dtype == torch.bfloat16 else v) for k, v in kw.items()}
        r = fn(*args, **kw)
        if dt != torch.bfloat16:
            return r
        if isinstance(r, dict):
            return {k: (v.to(dt) if k in out_keys and v is not None else v) for k, v in r.items()}
        return r.to(dt)
    return wrapped


def _trainer_worker(rank, world, port, out_q, bf16):
    """shard.ShardedTrainer (owned-row per-node state, flat-buffer all-reduce, device-side loss) for two steps, fp32
    or bf16 mode, against the single-process oracle's autograd + Adam (fp32): fp32 within the gradient tolerance,
    bf16 within bf16 rounding (loss within 2 %, gradient cosine > 0.99)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [REPO, HERE]
    from __graft_entry__ import load_package
    pkg = load_package()
    from protgram_directgcn_amd import ops, shard, train
    from oracle import directgcn_cpu as oc
    from oracle import graph_cpu as og
    import torch.nn.functional as F
    ops.spmm3 = _any_dtype(_cpu_spmm3)
    ops.spmm3_t = _any_dtype(_cpu_spmm3_t)
    ops.layer_dense = _any_dtype(_cpu_layer_dense)
    ops.layer_dense_backward = _any_dtype(_cpu_layer_dense_backward, out_keys=("dpre", "dZ", "dres"))
    train.l2_sqsum = lambda ps: sum((p.detach().float() ** 2).sum() for p in ps)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        N, s, d, c = pkg.synth.de_bruijn_edges(2)
        m = og.build_matrices(N, s, d, c)
        g = pkg.graph.csr_from_coo(N, *m["in"], *m["out"], *m["und"], cache=False)
        dims = [16, 16, 16, 12]
        torch.manual_seed(0)
        model = pkg.ProtGramDirectGCN(dims, N, 5, 2, 0, 512, 0.5, True).eval()
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
        y = (torch.arange(N) // 20) % 5
        lam, steps, lr = 1e-3, 2, 1e-2
        part = shard.partition(g, rank, world, transpose=True)
        tr = shard.ShardedTrainer(model, part, l2_lambda=lam,
                                  optimizer_factory=lambda ps: torch.optim.Adam(ps, lr=lr))
        # the node state is owned-row sized
        owned = [p for d in tr.own for p in d.values()]
        assert owned and all(p.size(0) == part.n_local for p in owned)
        losses, grads = [], []
        for _ in range(steps):
            loss = tr.step(x, y[part.r0:part.r1])
            assert torch.is_tensor(loss) and loss.dim() == 0
            losses.append(float(loss))
            gd = {}
            for name, p in model.named_parameters():
                if shard._is_node_param(name, p, N):
                    conv = model.convs[int(name.split(".")[1])]
                    gd[name] = tr.own[list(model.convs).index(conv)][name.split(".")[-1]].grad.clone()
                else:
                    gd[name] = p.grad.clone()
            grads.append(gd)
        ropt = torch.optim.Adam(list(ref.values()), lr=lr)
        rlosses, rgrads = [], []
        for _ in range(steps):
            ropt.zero_grad()
            lp, _ = oc.model_forward(ref, dims, x, *m["in"], *m["out"], *m["und"], n_gram_len=2)
            loss = F.nll_loss(lp, y) + lam * sum(v.norm(2).pow(2) for v in ref.values())
            loss.backward()
            rgrads.append({k: v.grad.clone() for k, v in ref.items()})
            ropt.step()
            rlosses.append(float(loss))
        bad = []
        for st in range(steps):
            if bf16:
                if abs(losses[st] - rlosses[st]) > 2e-2 * abs(rlosses[st]):
                    bad.append(("loss", st, losses[st], rlosses[st]))
            elif abs(losses[st] - rlosses[st]) > 1e-5 * abs(rlosses[st]) + 1e-6:
                bad.append(("loss", st, losses[st], rlosses[st]))
            if st:  # the second step's gradients depend on the first update: compare step 0 only
                continue
            for name, gg in grads[st].items():
                r = rgrads[st][name]
                if shard._is_node_param(name, r, N):
                    r = r[part.r0:part.r1]
                if bf16:
                    cos = float((gg * r).sum() / (gg.norm() * r.norm() + 1e-30))
                    if cos < 0.99:
                        bad.append((name, "cos", cos))
                else:
                    err = float((gg - r).abs().max())
                    if err > 2e-5 * float(r.abs().max()) + 1e-6:
                        bad.append((name, "grad", err))
        tr.gather()
        if not bf16:
            for name, p in model.named_parameters():
                err = float((p.detach() - ref[name].detach()).abs().max())
                if err > 2e-5:
                    bad.append(("gathered " + name, err))
        out_q.put((rank, part.r0, part.r1, not bad, str(bad[:4])))
    finally:
        dist.destroy_process_group()


def _untouched_worker(rank, world, port, out_q):
    """ShardedTrainer with l2_lambda = 0 steps only the parameters autograd reached: a positional
    embedding that the forward does not apply (x width != n * one_gram_dim) keeps its value and gets no Adam state,
    as torch.optim.Adam skips grad None in the reference loop; with l2_lambda > 0 its L2 gradient steps it."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [REPO, HERE]
    from __graft_entry__ import load_package
    pkg = load_package()
    from protgram_directgcn_amd import ops, shard, train
    from oracle import graph_cpu as og
    ops.spmm3 = _cpu_spmm3
    ops.spmm3_t = _cpu_spmm3_t
    ops.layer_dense = _cpu_layer_dense
    ops.layer_dense_backward = _cpu_layer_dense_backward
    train.l2_sqsum = lambda ps: sum((p.detach().float() ** 2).sum() for p in ps)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        N, s, d, c = pkg.synth.de_bruijn_edges(2)
        m = og.build_matrices(N, s, d, c)
        g = pkg.graph.csr_from_coo(N, *m["in"], *m["out"], *m["und"], cache=False)
        x = torch.randn(N, 16, generator=torch.Generator().manual_seed(1234))
        y = (torch.arange(N) // 20) % 5
        part = shard.partition(g, rank, world, transpose=True)
        res = []
        for lam in (0.0, 1e-3):
            torch.manual_seed(0)
            model = pkg.ProtGramDirectGCN([16, 16, 12], N, 5, 2, 3, 4, 0.5, True).eval()  # PE 2 x 3 != 16: unused
            pe0 = model.pe_layer.weight.detach().clone()
            w0 = model.convs[0].lin_shared.weight.detach().clone()
            tr = shard.ShardedTrainer(model, part, l2_lambda=lam,
                                      optimizer_factory=lambda ps: torch.optim.Adam(ps, lr=1e-2))
            for _ in range(2):
                tr.step(x, y[part.r0:part.r1])
            pe_moved = not torch.equal(model.pe_layer.weight.detach(), pe0)
            res.append((lam, pe_moved, len(tr.opt.state.get(model.pe_layer.weight, {})) > 0,
                        not torch.equal(model.convs[0].lin_shared.weight.detach(), w0)))
        ok = res[0][1:] == (False, False, True) and res[1][1:] == (True, True, True)
        out_q.put((rank, ok, str(res)))
    finally:
        dist.destroy_process_group()


def test_sharded_trainer_skips_untouched_without_l2():
    for r in _run(_untouched_worker, 2):
        assert r[1], f"rank {r[0]}: {r[2]}"


def _run(target, world, *extra):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q, *extra)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res)


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_training_gloo(world):
    res = _run(_train_worker, world)
    for r in res:
        assert r[3], f"rank {r[0]}: {r[4]}"


@pytest.mark.parametrize("world", [2, 3])
def test_node_range_partition_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    assert res[0][1] == 0 and res[-1][2] == 400
    for a, b in zip(res, res[1:]):
        assert a[2] == b[1]
    for r in res:
        assert r[3], f"rank {r[0]} mismatch (max |d| {r[4]:.2e})"


@pytest.mark.parametrize("world,bf16", [(2, False), (3, False), (2, True), (3, True)])
def test_sharded_trainer_gloo(world, bf16):
    """Config 5's multi-GPU training path (ShardedTrainer: owned-row per-node state, fp32 / bf16) on gloo ranks."""
    res = _run(_trainer_worker, world, bf16)
    for r in res:
        assert r[3], f"rank {r[0]}: {r[4]}"
