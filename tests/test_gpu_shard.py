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
    finally:
        dist.destroy_process_group()


def test_sharded_training_two_ranks_one_gpu(pkg, cuda):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in res:
        assert r[1], f"rank {r[0]}: {r[2]}"


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
