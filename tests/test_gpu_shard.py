"""Sharded training step (shard.py) with the HIP kernels: 2 gloo ranks sharing cuda:0 (rehearsal of the
RCCL path; the collectives are the same calls) against the single-GPU model's step on the 3-gram graph."""
import dataclasses
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _collect(q, procs, timeout=300):
    """The ranks' results; on the first failure the others (which may wait in a collective) are terminated."""
    res = []
    for _ in procs:
        r = q.get(timeout=timeout)
        res.append(r)
        if not r[1]:
            for p in procs:
                if p.is_alive():
                    p.terminate()
            break
    return sorted(res)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _setup(pkg, dev):
    N, s, d, c = pkg.synth.de_bruijn_edges(3)
    g = pkg.build_propagation_csr(N, s, d, c, device=dev)
    dims = [64, 64, 32]
    torch.manual_seed(0)
    model = pkg.ProtGramDirectGCN(dims, N, 20, 3, 0, 512, 0.5, True)
    with torch.no_grad():
        gen = torch.Generator().manual_seed(5)
        for name, p in model.named_parameters():
            leaf = name.split(".")[-1]
            if leaf.startswith("C_"):
                p.copy_(torch.rand(p.shape, generator=gen) + 0.5)
            elif "bias" in leaf:
                p.copy_(torch.rand(p.shape, generator=gen) * 0.2 - 0.1)
    model = model.to(dev).eval()
    x = torch.randn(N, 64, generator=torch.Generator().manual_seed(1234)).to(dev)
    y = (torch.arange(N, device=dev) // 400) % 20
    return N, g, model, x, y


def _worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [REPO, HERE]
    import torch.distributed as dist
    import torch.nn.functional as F
    from __graft_entry__ import load_package
    pkg = load_package()
    from protgram_directgcn_amd import shard
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        N, g, model, x, y = _setup(pkg, dev)
        ref = {k: v.detach().clone() for k, v in model.state_dict().items()}
        lam, steps = 1e-3, 2
        part = shard.partition(g, rank, world, transpose=True)
        opt = torch.optim.SGD(model.parameters(), lr=0.1)  # linear in the gradients (Adam's
        # first steps are ~lr*sign(g) and amplify rounding-level differences of near-zero gradients)
        losses = [shard.sharded_train_step(model, part, x, y[part.r0:part.r1], opt, l2_lambda=lam)
                  for _ in range(steps)]
        shard.gather_node_params(model, part)
        # single-GPU reference: the model itself with the same loop
        _, g1, m1, _, _ = _setup(pkg, dev)
        m1.load_state_dict(ref)
        opt1 = torch.optim.SGD(m1.parameters(), lr=0.1)
        rl = []
        for _ in range(steps):
            opt1.zero_grad()
            lp, _ = m1(pkg.Data(x=x, graph=g1))
            loss = F.nll_loss(lp, y) + lam * sum(p.norm(2).pow(2) for p in m1.parameters())
            loss.backward()
            opt1.step()
            rl.append(float(loss))
        bad = []
        for a, b in zip(losses, rl):
            if abs(a - b) > 1e-5 * abs(b) + 1e-6:
                bad.append(("loss", losses, rl))
        p1 = dict(m1.named_parameters())
        for name, p in model.named_parameters():
            r = p1[name].detach()
            tol = 2e-5 * float(r.abs().max()) + 1e-6
            err = float((p.detach() - r).abs().max())
            if err > tol:
                bad.append((name, err, tol))
        out_q.put((rank, not bad, str(bad[:4])))
    except Exception as e:  # report at once (the parent would otherwise wait out its queue timeout)
        out_q.put((rank, False, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def test_sharded_training_two_ranks_one_gpu(pkg, cuda):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = _collect(q, procs)
    for r in res:
        assert r[1], f"rank {r[0]}: {r[2]}"
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0


def _trainer_worker(rank, world, port, out_q, bf16):
    """shard.ShardedTrainer (config 5's multi-GPU step: owned-row per-node state, flat all-reduce, device-side loss)
    with the HIP kernels on 2 gloo ranks sharing cuda:0, against the single-GPU train.train_step: fp32 with SGD
    (linear in the gradients) to the gradient tolerance; bf16 mode with train.Adam: loss within 2 % and gradient
    cosine > 0.99 (different bf16 rounding points: the exchange and the ranks' partial sums)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [REPO, HERE]
    import torch.distributed as dist
    from __graft_entry__ import load_package
    pkg = load_package()
    from protgram_directgcn_amd import shard, train
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        N, g, model, x, y = _setup(pkg, dev)
        ref = {k: v.detach().clone() for k, v in model.state_dict().items()}
        lam = 1e-3
        dt = torch.bfloat16 if bf16 else torch.float32
        model.compute_dtype = dt
        part = shard.partition(g, rank, world, transpose=True)
        fac = None if bf16 else (lambda ps: torch.optim.SGD(ps, lr=0.1))
        tr = shard.ShardedTrainer(model, part, lr=1e-3, l2_lambda=lam, optimizer_factory=fac)
        for d in tr.own:
            for leaf in d.values():
                assert leaf.size(0) == part.n_local and leaf.data_ptr() != 0
        steps = 1 if bf16 else 2
        losses, grads = [], {}
        for _ in range(steps):
            losses.append(float(tr.step(x, y[part.r0:part.r1])))
        if bf16:  # the per-node Adam moments cover the owned rows only
            for leaf in tr.node:
                assert tr.opt.state[leaf]["exp_avg"].shape == leaf.shape
            for li, conv in enumerate(model.convs):
                for k, leaf in tr.own[li].items():
                    grads[f"convs.{li}.{k}"] = leaf.grad.detach().float().clone()
            for name, p in model.named_parameters():
                if name not in grads:
                    grads[name] = p.grad.detach().float().clone()
        tr.gather()
        # single-GPU reference: train.train_step on the whole graph
        _, g1, m1, _, _ = _setup(pkg, dev)
        m1.load_state_dict(ref)
        m1.compute_dtype = dt
        opt1 = train.Adam(m1.parameters(), lr=1e-3) if bf16 else torch.optim.SGD(m1.parameters(), lr=0.1)
        train.DEFER_CONST_GRAD = False  # the comparison below reads every parameter's .grad
        rl = [float(train.train_step(m1, pkg.Data(x=x, graph=g1), y, opt1, l2_lambda=lam, scaler=None))
              for _ in range(steps)]
        bad = []
        for a, b in zip(losses, rl):
            if abs(a - b) > (2e-2 if bf16 else 1e-5) * abs(b) + 1e-6:
                bad.append(("loss", losses, rl))
        if bf16:
            for name, p in m1.named_parameters():
                r = p.grad.detach().float()
                if shard._is_node_param(name, p, N):
                    r = r[part.r0:part.r1]
                gg = grads[name]
                cos = float((gg * r).sum() / (gg.norm() * r.norm() + 1e-30))
                if cos < 0.99:
                    bad.append((name, "cos", cos))
        else:
            p1 = dict(m1.named_parameters())
            for name, p in model.named_parameters():
                r = p1[name].detach()
                tol = 2e-5 * float(r.abs().max()) + 1e-6
                err = float((p.detach() - r).abs().max())
                if err > tol:
                    bad.append((name, err, tol))
        out_q.put((rank, not bad, str(bad[:4])))
    except Exception as e:  # report at once (the parent would otherwise wait out its queue timeout)
        out_q.put((rank, False, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bf16", [False, True])
def test_sharded_trainer_two_ranks_one_gpu(pkg, cuda, bf16):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_trainer_worker, args=(r, 2, port, q, bf16)) for r in range(2)]
    for p in procs:
        p.start()
    res = _collect(q, procs)
    for r in res:
        assert r[1], f"rank {r[0]}: {r[2]}"
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0


@pytest.mark.parametrize("n,dims", [(3, [128, 128, 128]), (3, [64, 64, 32]), (2, [32, 32, 32, 16])])
def test_halo_forward_bitexact_vs_single_gpu(pkg, cuda, n, dims):
    """Every rank of the halo-recompute partition (world 2, 3, 8; each rank run in turn on cuda:0, which is
    exactly what that rank computes: the path has no collective) reproduces its rows of the single-GPU
    forward bit for bit: same kernels, same per-row entry order."""
    from protgram_directgcn_amd import shard
    N, s, d, c = pkg.synth.de_bruijn_edges(n)
    g = pkg.build_propagation_csr(N, s, d, c, device=cuda)
    torch.manual_seed(0)
    model = pkg.ProtGramDirectGCN(dims, N, 20, n, 0, 512, 0.5, True)
    with torch.no_grad():
        gen = torch.Generator().manual_seed(5)
        for name, p in model.named_parameters():
            leaf = name.split(".")[-1]
            if leaf.startswith("C_"):
                p.copy_(torch.rand(p.shape, generator=gen) + 0.5)
            elif "bias" in leaf:
                p.copy_(torch.rand(p.shape, generator=gen) * 0.2 - 0.1)
    model = model.to(cuda).eval()
    x = torch.randn(N, dims[0], generator=torch.Generator().manual_seed(1234)).to(cuda)
    with torch.no_grad():
        # CSR kernels (a halo subgraph has no n-gram tile plan; the tile kernels sum in another order)
        lp_r, emb_r = model(pkg.Data(x=x, graph=dataclasses.replace(g, ngram=None)))
    L = len(dims) - 1
    for world in (2, 3, 8):
        seen = torch.zeros(N, dtype=torch.bool, device=cuda)
        for rank in range(world):
            hp = shard.halo_partition(g, rank, world, L)
            lp, emb = shard.halo_forward(model, hp, shard.halo_inputs(model, hp, x))
            torch.cuda.synchronize()
            gr = hp.global_rows
            assert torch.equal(lp, lp_r[gr]), (world, rank, float((lp - lp_r[gr]).abs().max()))
            assert torch.equal(emb, emb_r[gr]), (world, rank)
            seen[gr] = True
        assert bool(seen.all())
