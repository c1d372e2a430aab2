"""BASELINE config 5 (3-layer DirectGCN, 4-gram graph, dims [128, 256, 256, 256], the trainer's full-batch step on
8 MI355X) through shard.MiddleTrainer at its size: P = 8 ranks as 8 processes sharing this one GPU, gloo carrying
the ghost-row exchanges, their transposes and the gradient all-reduce (the same calls RCCL runs on the 8-GPU node;
tests/test_gpu_rccl.py runs the RCCL branch itself). Every rank propagates its middles on the middle-tile kernel
(launches counted) and backpropagates in scatter form (pg_spmm3t_ngram_scatter_*: its middles' dZ to the D / P / S
row sets, the ghost rows' sums back to their owners).

Each rank checks its own share against the single-GPU step on the same model and inputs (computed once in the test's
process and loaded by the ranks): the global loss, every replicated parameter gradient after the all-reduce and the
owned rows of every per-node parameter gradient (plus the L2 term 2 lam p, which the trainer's train.Adam folds
into its update instead of the gradient). fp32: |d| <= 1e-4 max|ref| + 1e-4 |ref| (the kernels sum in
other orders than the single-GPU step's); bf16 mode against the fp32 step (as test_gpu_configs' config-5 test):
loss within 2 %, gradient cosine > 0.99. Reference loop: protgram_directgcn_trainer.py:76-108; dims: config.py:63."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
WORLD = 8


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _reference(pkg, path):
    """The single-GPU fp32 step (loss and every parameter gradient) on the config-5 model and inputs, computed ONCE
    in the test's own process and saved for the ranks (round 4 had every rank compute it: 8 full-graph steps at once
    on one GPU, 14-73 s, whose slow runs crossed the ranks' 150 s watchdog -- the intermittent 'stall')."""
    from protgram_directgcn_amd import train
    from test_gpu_configs import _labels, _model
    n, dims, lam = 4, [128, 256, 256, 256], 1e-7
    dev = torch.device("cuda", 0)
    N, s, d, c = pkg.synth.de_bruijn_edges(n)
    g = pkg.build_propagation_csr(N, s, d, c, device=dev)
    x = torch.randn(N, dims[0], generator=torch.Generator().manual_seed(1234)).to(dev)
    y = _labels(N, n).to(dev)
    out = {}
    for tag, dt in (("", torch.float32), ("bf16_", torch.bfloat16)):  # the fp32 step, and the same step in bf16 mode
        ref = _model(pkg, dims, N, n).to(dev).eval()
        ref.compute_dtype = dt
        lp, _ = ref(pkg.Data(x=x, graph=g))
        loss_r = train.nll_mean(lp.float(), y) + lam * sum(p.norm(2).pow(2) for p in ref.parameters())
        loss_r.backward()
        out[tag + "loss"] = float(loss_r.detach())
        out[tag + "grads"] = {k: p.grad.detach().float().cpu() for k, p in ref.named_parameters()}
        del ref, lp
    torch.save(out, path)
    del g
    torch.cuda.empty_cache()


def _worker(rank, world, port, out_q, bf16, ref_path):
    import faulthandler
    import time
    t_start = time.time()
    faulthandler.dump_traceback_later(300, exit=True)  # a stuck rank prints where it is and exits (the parent fails)

    def phase(what):  # per-rank progress on stderr (pytest -s shows it): where the time of a slow run goes
        print(f"[p8 rank {rank} bf16={bf16}] {what} at {time.time() - t_start:.1f}s", file=sys.stderr, flush=True)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [REPO, HERE]
    import torch.distributed as dist
    from __graft_entry__ import load_package
    pkg = load_package()
    from protgram_directgcn_amd import ops, shard
    from test_gpu_configs import _labels, _model
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    phase("process group up")
    bad = []
    try:
        n, dims, lam = 4, [128, 256, 256, 256], 1e-7
        N, s, d, c = pkg.synth.de_bruijn_edges(n)
        g = pkg.build_propagation_csr(N, s, d, c, device=dev)
        x = torch.randn(N, dims[0], generator=torch.Generator().manual_seed(1234)).to(dev)
        y = _labels(N, n).to(dev)
        saved = torch.load(ref_path, weights_only=True, mmap=True)  # the single-GPU step, from the parent
        loss_r, rgrad, rgrad_bf = saved["loss"], saved["grads"], saved["bf16_grads"]
        phase("reference loaded")
        # this rank of the middle partition
        mp_ = shard.middle_partition(g, rank, world)
        m = _model(pkg, dims, N, n).to(dev).eval()
        if bf16:
            m.compute_dtype = torch.bfloat16
        tr = shard.MiddleTrainer(m, mp_, l2_lambda=lam)
        # pre-step values (the model's full per-node parameters are not written by the trainer: its leaves are)
        pre_dense = {k: p.detach().float().clone() for k, p in m.named_parameters()}
        hits = []
        real = ops.spmm3_middles
        ops.spmm3_middles = lambda *a, **k: hits.append(1) or real(*a, **k)
        # bf16: the per-node constants' gradients go to Adam as the layers' bf16 dpre (train.DEFER_CONST_GRAD), not
        # as .grad; keep a widened copy of each as the backward files it
        filed = {}
        real_file = ops._file_deferred

        def spy(constant, dpre):
            ok = real_file(constant, dpre)
            if ok:
                filed[constant.data_ptr()] = dpre.float()
            return ok
        ops._file_deferred = spy
        phase("trainer built")
        loss = float(tr.step(x, y[mp_.own]))
        torch.cuda.synchronize()
        phase("trainer step done")
        if len(hits) != len(dims) - 1:
            bad.append(("middle-tile launches", len(hits)))
        if bf16:
            if abs(loss - loss_r) > 2e-2 * abs(loss_r):
                bad.append(("loss", loss, loss_r))
        elif abs(loss - loss_r) > 1e-5 * abs(loss_r):
            bad.append(("loss", loss, loss_r))
        own = mp_.own
        for name, p in m.named_parameters():
            r = rgrad[name]
            if shard._is_node_param(name, p, N):
                leaf = tr.own[int(name.split(".")[1])][name.split(".")[-1]]
                gg = leaf.grad if leaf.grad is not None else filed.get(leaf.data_ptr())
                r = r[own.cpu()]
            else:
                gg = p.grad
            r = r.to(dev)
            if gg is None:
                bad.append((name, "no grad"))
                continue
            pre = p.detach().float()[own] if shard._is_node_param(name, p, N) else pre_dense[name]
            gg = gg.detach().float() + 2 * lam * pre  # train.Adam folds the L2 gradient into its update
            if bf16:
                cos = float((gg * r).sum() / (gg.norm() * r.norm() + 1e-30))
                if cos < 0.99:
                    bad.append((name, "cos", cos))
                # elementwise against the single-GPU step in bf16 mode (itself bounded elementwise against float64 by
                # test_gpu_configs.test_config5_bf16_elementwise_vs_float64): |d| <= 2^-8 (16 |ref| + 16 max|ref|),
                # except at most max(8, 1e-3 n) elements -- a pre-activation within a bf16 rounding of 0 may take the
                # other leaky-ReLU branch when the rank sums in another order
                rb = rgrad_bf[name]
                if shard._is_node_param(name, p, N):
                    rb = rb[own.cpu()]
                rb = rb.to(dev).double() + 2 * lam * pre.double()
                dd = (gg.double() - rb).abs()
                nout = int((dd > 2.0 ** -8 * (16 * rb.abs() + 16 * float(rb.abs().max()))).sum())
                if nout > max(8, int(1e-3 * dd.numel())):
                    bad.append((name, "elementwise vs bf16 step", nout, dd.numel(), float(dd.max())))
            else:
                err = (gg - r).abs()
                if bool((err > 1e-4 * float(r.abs().max()) + 1e-4 * r.abs()).any()):
                    bad.append((name, "grad", float(err.max()), float(r.abs().max())))
        faulthandler.cancel_dump_traceback_later()
        out_q.put((rank, mp_.n_own, int(mp_.recv_ids.numel()), not bad, str(bad[:4]), loss, loss_r))
    except Exception as e:  # report instead of hanging the parent
        out_q.put((rank, 0, 0, False, repr(e)[:400], 0.0, 0.0))
        raise
    finally:
        dist.destroy_process_group()


def _collect(q, procs, n, limit):
    """The n ranks' results; fails fast (terminating the others) when a rank reports an error or dies, instead of
    leaving the surviving ranks blocked in a collective until the time limit."""
    import queue
    import time
    res, t0 = [], time.time()
    while len(res) < n:
        try:
            r = q.get(timeout=5)
        except queue.Empty:
            r = None
        if r is not None:
            res.append(r)
            if not r[3] and r[1] == 0:  # an exception in the rank (see _worker)
                break
        dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
        if dead or time.time() - t0 > limit:
            break
    if len(res) < n or any(not r[3] and r[1] == 0 for r in res):
        for p in procs:
            if p.is_alive():
                p.terminate()
        pytest.fail(f"ranks incomplete: {len(res)} of {n} results, exit codes {[p.exitcode for p in procs]}, "
                    f"errors {[r[4] for r in res if not r[3]]}")
    return res


_REF = {}


@pytest.mark.timeout(900)
@pytest.mark.parametrize("bf16", [False, True])
def test_config5_middle_trainer_p8_one_gpu(pkg, cuda, bf16, tmp_path_factory):
    if "path" not in _REF:  # one single-GPU reference step for both cases
        _REF["path"] = str(tmp_path_factory.mktemp("p8ref") / "ref.pt")
        _reference(pkg, _REF["path"])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    env_keep = os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q, bf16, _REF["path"])) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = sorted(_collect(q, procs, WORLD, 840))
    for p in procs:
        p.join(timeout=120)
    assert env_keep is None or os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY") == env_keep
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert sum(r[1] for r in res) == 160_000
    for r in res:
        assert r[3], f"rank {r[0]}: {r[4]}"
    print("ranks (rank, own rows, ghost rows, loss, single-GPU loss):", [(r[0], r[1], r[2], r[5], r[6]) for r in res])


class _NoComm:
    """No-op collectives that can be captured (a rank's own work alone)."""
    capturable = True

    def all_to_all(self, out, inp, out_splits, in_splits):
        out.zero_()

    def all_reduce(self, t):
        pass


@pytest.mark.timeout(300)
@pytest.mark.parametrize("bf16", [False, True])
def test_middle_trainer_hip_graph_matches_eager(pkg, cuda, bf16):
    """MiddleTrainer(graphs=True): after its eager warm-up steps the whole step is captured as a HIP graph and
    replayed. Six steps from the same start give the same losses and parameters, bit for bit, as six eager steps
    (rank 0 of 2 at 3-gram, the collectives no-ops)."""
    from protgram_directgcn_amd import shard
    from test_gpu_configs import _labels, _model
    n, dims = 3, [64, 64, 32]
    N, s_, d, c = pkg.synth.de_bruijn_edges(n)
    g = pkg.build_propagation_csr(N, s_, d, c, device=cuda)
    x = torch.randn(N, dims[0], generator=torch.Generator().manual_seed(5)).to(cuda)
    y = _labels(N, n).to(cuda)
    mp_ = shard.middle_partition(g, 0, 2)
    res = []
    for graphs in (False, True):
        m = _model(pkg, dims, N, n).to(cuda).eval()
        if bf16:
            m.compute_dtype = torch.bfloat16
        tr = shard.MiddleTrainer(m, mp_, l2_lambda=1e-3, comm=_NoComm(), graphs=graphs)
        losses = [float(tr.step(x, y[mp_.own])) for _ in range(6)]
        torch.cuda.synchronize()
        assert (tr._graph is not None) == graphs
        res.append((losses, [p.detach().clone() for p in tr.params]))
    assert res[0][0] == res[1][0], res
    assert all(torch.equal(a, b) for a, b in zip(res[0][1], res[1][1]))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("bf16", [False, True])
def test_middle_trainer_hip_graph_follows_lr_schedule(pkg, cuda, bf16):
    """VERDICT r05 item 1 for config 5's fast path: train.fit (the reference loop's ReduceLROnPlateau + EarlyStopper,
    protgram_directgcn_trainer.py:76-108) around MiddleTrainer.step, the scheduler forced to halve the learning rate
    after every epoch. With graphs=True the step is captured once and every replay reads the refreshed device lr: the
    losses, learning rates and parameters equal the eager steps' bit for bit (rank 0 of 2 at 3-gram, the collectives
    no-ops). Early stopping ends both runs at the same epoch."""
    from protgram_directgcn_amd import shard, train
    from test_gpu_configs import _labels, _model
    n, dims = 3, [64, 64, 32]
    N, s_, d, c = pkg.synth.de_bruijn_edges(n)
    g = pkg.build_propagation_csr(N, s_, d, c, device=cuda)
    x = torch.randn(N, dims[0], generator=torch.Generator().manual_seed(5)).to(cuda)
    y = _labels(N, n).to(cuda)
    mp_ = shard.middle_partition(g, 0, 2)
    res = []
    for graphs in (False, True):
        m = _model(pkg, dims, N, n).to(cuda).eval()
        if bf16:
            m.compute_dtype = torch.bfloat16
        tr = shard.MiddleTrainer(m, mp_, lr=1e-2, l2_lambda=1e-3, comm=_NoComm(), graphs=graphs)
        sched = torch.optim.lr_scheduler.ReduceLROnPlateau(tr.opt, "min", patience=0, factor=0.5, threshold=0.99)
        yo = y[mp_.own]
        hist = train.fit(lambda: tr.step(x, yo), tr.opt, 9, scheduler=sched, es_patience=7, es_min_delta=0.0)
        torch.cuda.synchronize()
        assert (tr._graph is not None) == graphs
        res.append((hist, [p.detach().clone() for p in tr.params]))
        tr.close()
    lrs = [h["lr"][0] for h in res[0][0]]
    assert lrs[:4] == [1e-2, 1e-2, 5e-3, 2.5e-3], lrs
    assert res[0][0] == res[1][0], res
    assert all(torch.equal(a, b) for a, b in zip(res[0][1], res[1][1]))


@pytest.mark.parametrize("graphs", [False, True])
def test_middle_trainer_bf16_deferred_constant_grads_bit_identical(pkg, cuda, graphs):
    """bf16 MiddleTrainer with train.Adam: the owned per-node constants' gradients go to Adam as the layers' bf16
    dpre (train.DEFER_CONST_GRAD) instead of fp32 .grad copies moved into home buffers. 4 steps (eager, or captured
    after the warm-up and replayed), training mode with the fused dropout: losses and every parameter bit-identical
    to the run without deferral (rank 0 of 2 at 3-gram, the collectives no-ops); the constants' .grad stay None."""
    from protgram_directgcn_amd import ops, shard, train
    from test_gpu_configs import _labels, _model
    n, dims = 3, [64, 256, 256]
    N, s_, d, c = pkg.synth.de_bruijn_edges(n)
    g = pkg.build_propagation_csr(N, s_, d, c, device=cuda)
    x = torch.randn(N, dims[0], generator=torch.Generator().manual_seed(5)).to(cuda)
    y = _labels(N, n).to(cuda)
    mp_ = shard.middle_partition(g, 0, 2)
    res = []
    filed = []
    real_file = ops._file_deferred
    try:
        for defer in (False, True):
            train.DEFER_CONST_GRAD = defer
            ops._file_deferred = lambda cst, dp: (filed.append(defer), real_file(cst, dp))[1]
            torch.manual_seed(0)
            m = _model(pkg, dims, N, n).to(cuda).train()
            m.compute_dtype = torch.bfloat16
            tr = shard.MiddleTrainer(m, mp_, lr=1e-2, l2_lambda=1e-3, comm=_NoComm(), graphs=graphs)
            yo = y[mp_.own]
            losses = [float(tr.step(x, yo)) for _ in range(4 + 3 * graphs)]
            torch.cuda.synchronize()
            if defer:
                assert all(d["constant"].grad is None for d in tr.own if "constant" in d)
                assert not ops._DEFERRED_GRADS and not ops._DEFER_CONST_GRAD
            res.append((losses, [p.detach().clone() for p in tr.params]))
            tr.close()
    finally:
        train.DEFER_CONST_GRAD = True
        ops._file_deferred = real_file
    assert filed and all(filed)  # filed in the deferring run only
    assert res[0][0] == res[1][0], res
    assert all(torch.equal(a, b) for a, b in zip(res[0][1], res[1][1]))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("bf16", [False, True])
def test_middle_trainer_fused_dropout_matches_masked(pkg, cuda, bf16, monkeypatch):
    """MiddleTrainer.forward in training mode with the layer dropout fused into the rank's dense launches
    (ops.FUSED_DROPOUT, seeds salted by the rank's first middle) against the same forward with F.dropout replaced by
    the host restatement of the kernel's mask on those seeds: at p = 0.5 the log-probs are bit-identical (rank 0 of 2
    at 3-gram, the collectives no-ops; the decoder's own dropout set to 0)."""
    from protgram_directgcn_amd import ops, shard
    from test_gpu_configs import _model
    from test_gpu_parity import _layer_drop_keep
    n, dims = 3, [64, 64, 32]
    N, s_, d, c = pkg.synth.de_bruijn_edges(n)
    g = pkg.build_propagation_csr(N, s_, d, c, device=cuda)
    x = torch.randn(N, dims[0], generator=torch.Generator().manual_seed(8)).to(cuda)
    mp_ = shard.middle_partition(g, 0, 2)

    def trainer():
        m = _model(pkg, dims, N, n).to(cuda).train()
        m.decoder_fc[2].p = 0.0
        if bf16:
            m.compute_dtype = torch.bfloat16
        return shard.MiddleTrainer(m, mp_, l2_lambda=0.0, comm=_NoComm())

    assert ops.FUSED_DROPOUT
    randint, drawn = torch.randint, []

    def rec(*a, **k):
        t = randint(*a, **k)
        drawn.append(t)
        return t
    monkeypatch.setattr(torch, "randint", rec)
    with torch.no_grad():
        lp, _ = trainer().forward(x, need_emb=False)
    monkeypatch.setattr(torch, "randint", randint)
    assert len(drawn) == 1
    seeds = [int(v) for v in drawn[0].cpu()]  # salted in place by the trainer
    calls = []
    dropout = torch.nn.functional.dropout

    def masked(inp, p=0.5, training=True, inplace=False):
        if p == 0.0 or not training:
            return inp
        i = len(calls)
        calls.append(i)
        keep = _layer_drop_keep(seeds[i], inp.size(0), inp.size(1), p).to(inp.device)
        return inp * keep.to(inp.dtype) * (1.0 / (1.0 - p))
    monkeypatch.setattr(ops, "FUSED_DROPOUT", False)
    monkeypatch.setattr(torch.nn.functional, "dropout", masked)
    with torch.no_grad():
        lp_ref, _ = trainer().forward(x, need_emb=False)
    monkeypatch.setattr(torch.nn.functional, "dropout", dropout)
    assert len(calls) == len(dims) - 1
    assert torch.equal(lp, lp_ref)


def _fit_worker(rank, world, port, q, argv):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path[:0] = [REPO, os.path.join(REPO, "tools")]
    try:
        import fit_config5
        rec = fit_config5.run(argv)
        if rank == 0:
            q.put(("ok", rec))
    except Exception as e:  # report instead of leaving the parent to its timeout
        q.put(("error", repr(e)[:400]))
        raise


@pytest.mark.timeout(600)
def test_fit_config5_driver_two_ranks_matches_one():
    """tools/fit_config5.py, the multi-GPU epoch loop of config 5 (train.fit around MiddleTrainer.step: the reference
    loop's ReduceLROnPlateau + EarlyStopper, protgram_directgcn_trainer.py:76-108), on 2 gloo ranks sharing cuda:0
    against the same loop on 1 rank: 8 epochs at 3-gram, fp32, no dropout; the same number of epochs, the same
    learning rates, and the per-epoch losses within 1e-5 relative (the ranks' partial sums are added in another
    order)."""
    argv = ["--backend", "gloo", "--n", "3", "--dims", "64,64,32", "--epochs", "8", "--fp32", "--eval",
            "--lr", "1e-2", "--l2", "1e-3"]
    ctx = mp.get_context("spawn")
    recs = []
    for world in (1, 2):
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_fit_worker, args=(r, world, port, q, argv)) for r in range(world)]
        for p in procs:
            p.start()
        status, rec = q.get(timeout=300)
        for p in procs:
            p.join(timeout=120)
        assert status == "ok", rec
        assert all(p.exitcode == 0 for p in procs)
        recs.append(rec)
    (a, b) = recs
    assert a["epochs_run"] == b["epochs_run"] == 8
    assert [h["lr"] for h in a["history"]] == [h["lr"] for h in b["history"]]
    for ha, hb in zip(a["history"], b["history"]):
        assert abs(ha["loss"] - hb["loss"]) <= 1e-5 * abs(ha["loss"]), (ha, hb)
    assert a["history"][-1]["loss"] < a["history"][0]["loss"]

