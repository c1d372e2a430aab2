#!/usr/bin/env python3
"""Bench: edges/sec propagated, DirectGCN forward on the 4-gram graph (BASELINE.json metric).

Workload: complete n-gram graph B(20,4) in the reference's node order (N=160,000,
E=3,200,000 transitions, 6,559,580 entries per adjacency, shared pattern), synthetic features
X = randn(N, 128) (seed 1234), ProtGramDirectGCN with layer_dims [128,128,128] (2 DirectGCN layers,
identity residuals), C=20 classes, eval mode, fp32. One step = one full model forward (both layers,
decoder, log_softmax, L2-normalised embeddings), inputs resident in HBM.
  edges/s = 3 * nnz * L / t_step   (each adjacency entry counted once per layer)

--gpus N (torchrun, one process per GPU; "scaling": "strong": total work fixed). --partition middle (complete
n-gram graphs, n >= 3): rank p owns the nodes a.M.b of a contiguous range of middle (n-2)-grams M and runs the
middle-tile kernel over them; between the layers each rank receives exactly the ghost rows its middles read from
their owners (one RCCL all_to_all_single; shard.middle_partition / MiddleRunner). --partition halo: each rank
recomputes the 1-hop halo of its rows in layer 1 on the CSR kernels, no collective (shard.halo_partition).
--partition exchange: node-range rows and an RCCL all-gather of all layer-1 rows (shard.sharded_forward).
--partition replicate: every rank runs the layers before the last over all rows (the single-GPU kernels) and the
last layer over its middles only; no collective (MiddleRunner(replicate=True)).
Default (auto): AUTO_PARTITION below (by rank count, from the round-3 per-rank measurements).
Timing: W warmup steps, then exactly K steps between barrier + synchronize on both sides; the max
over ranks is reported. Rank 0 prints one JSON line.

At N = 1 the forward is captured once as a HIP graph and replayed in the timed loop, as each rank's work is at
N > 1 (MiddleRunner), so the 1 -> N curve compares like with like (--no-graphs: eager everywhere).

Extra fields: "roofline" for the dominant kernel, chosen by measured time per step, with "roofline.kernels" holding
one entry per hot-path kernel (the propagation -- pg_spmm3_ngram_mid_f32 at B(20,4) --, the dense layer
pg_directgcn_dense_f32 and the head): compulsory bytes per launch / its average launch duration from HIP events
recorded on its launch stream (eager steps right after the timed region), and the L2-miss traffic of each measured by
two rocprofv3 --pmc passes in the same run; "cpu_baseline" (the oracle = the reference's CPU algorithm, timed on
this host, rank 0 at N=1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
# --partition auto by rank count (absent: middle). Per-rank 4-gram times measured on one MI355X
AUTO_PARTITION = {2: "replicate", 3: "replicate", 4: "halo"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults: 50 warmup steps let the GPU clocks ramp (5 warmups measured 0.915 ms/step, 50 or 200:
    # 0.846 ms at B(20,4)); the whole default run is still well under a second of GPU work
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--clock-warmup-s", type=float, default=1.0,
                    help="untimed seconds of steps before the warm-up steps (clock ramp)")
    ap.add_argument("--ngram", type=int, default=4)
    ap.add_argument("--graph", choices=("debruijn", "fasta"), default="debruijn",
                    help="debruijn (default): the complete n-gram graph B(20,n); fasta: a builder-produced level "
                    "(ngram.ngram_transitions on seeded protein-like sequences with the builder's ' ' padding and "
                    "rare X/U/B/Z, sorted-string node ids: not the complete grid) on the mapped middle-tile plan")
    ap.add_argument("--fasta-seqs", type=int, default=8000, help="--graph fasta: sequences (mean length 350)")
    ap.add_argument("--feat", type=int, default=128)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--fused-norm", action="store_true", help="compute edge weights inside the SpMM")
    ap.add_argument("--bf16", action="store_true", help="bf16 mode (config 5): bf16 features/activations, fp32 sums")
    ap.add_argument("--entry", choices=("coo", "graph"), default="coo",
                    help="coo (default): the model reads the reference trainer's COO wiring (Data.edge_index_* = "
                    "mathcal_A_*.indices(), edge_weight_* = .values(), protgram_directgcn_trainer.py:362-367) through "
                    "csr_from_coo; graph: a prebuilt Data.graph (build_propagation_csr)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-layers", type=int, default=1)
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 FETCH_SIZE/WRITE_SIZE passes that "
                    "measure roofline.traffic (N=1 only)")
    ap.add_argument("--extra", action="store_true", help="also time kernel variants / training step (stderr)")
    ap.add_argument("--chunks", type=int, default=0, help="N>1: layer-boundary exchange in this many pieces, "
                    "overlapped with the compute (1 = one exchange after the layer; 0 = by the rank's share)")
    ap.add_argument("--partition", choices=("auto", "middle", "replicate", "halo", "exchange"), default="auto",
                    help="N>1: 'middle' = middle (n-2)-gram ranges + RCCL ghost-row all_to_all per layer boundary "
                    "(falls back to 'halo' on graphs it does not take); 'halo' = each rank recomputes the (L-1)-hop "
                    "halo of its rows (no collective on the data path); 'exchange' = node-range rows + RCCL "
                    "all-gather of all rows per layer; 'replicate' = layers before the last over all rows on every "
                    "rank, the last over the rank's middles (no collective); 'auto' (default) = AUTO_PARTITION by rank "
                    "count (at few ranks a rank's ghost rows go over few links: the exchange costs more than "
                    "recomputing, DESIGN.md 5c)")
    ap.add_argument("--no-graphs", action="store_true", help="eager launches instead of HIP graph replays (N=1: the "
                    "whole forward captured once; N>1 middle partition: the per-segment graphs)")
    ap.add_argument("--kernel-reps", type=int, default=10, help="eager steps after the timed region whose launches "
                    "are timed with HIP events (per-kernel roofline)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL); 'gloo' only to rehearse N>1 on one GPU")
    ap.add_argument("--one-device", action="store_true", help="all ranks on cuda:0 (rehearsal with gloo only)")
    ap.add_argument("--launch-check", action="store_true", help="N>1 plumbing check without a GPU: start the ranks, "
                    "all-reduce over --dist-backend, print one JSON line, exit")
    return ap.parse_args()


def launch_workers(n: int) -> int:
    """--gpus N without an outside launcher: start N ranks with torch.distributed.run (127.0.0.1, a free port) as
    CHILD processes and return their exit code. Called before anything touches the GPU."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def launch_check(args, world: int, rank: int) -> None:
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group(args.dist_backend)
    t = torch.tensor([float(rank), 1.0])
    if world > 1:
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"launch_check": True, "world_size": world, "rank_sum": float(t[0]),
                          "ranks": int(t[1]), "backend": args.dist_backend}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_workers(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.launch_check:
        return launch_check(args, world, rank)

    import numpy as np
    import torch
    import torch.distributed as dist

    from __graft_entry__ import load_package
    pkg = load_package()
    from protgram_directgcn_amd import ops, shard

    dev_index = 0 if args.one_device else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    def log(*a):
        if rank == 0:
            print(*a, file=sys.stderr, flush=True)

    n, Fd, L = args.ngram, args.feat, args.layers
    t0 = time.time()
    wl = build_workload(pkg, args, dev, keep_raw=args.fused_norm or args.extra)
    N, g, tr = wl["N"], wl["graph"], wl["transitions"]
    torch.cuda.synchronize()
    log(f"[bench] graph {wl['desc']}: N={N} E={wl['E']} nnz/adj={g.nnz} built in {time.time() - t0:.1f}s"
        + (f"; mapped plan: {g.ngram_map.n_grid} grid nodes, {g.ngram_map.n_off} off-grid rows, "
           f"{g.ngram_map.n_acc} grid rows with {g.ngram_map.nnz_res} residual entries" if g.ngram_map is not None
           else ""))

    model = bench_model(pkg, N, Fd, L, n).to(dev).eval()
    dims = [Fd] * (L + 1)
    C = 20
    model.fused_norm = args.fused_norm
    x = torch.randn(N, Fd, generator=torch.Generator().manual_seed(1234)).to(dev)
    if args.bf16:
        if args.fused_norm:
            raise SystemExit("--bf16 uses precomputed weights (no fused-norm bf16 kernel)")
        model.compute_dtype = torch.bfloat16
        x = x.to(torch.bfloat16)  # inputs resident in HBM in the compute dtype
    entry = "graph" if args.fused_norm else args.entry  # fused-norm reads the raw counts only the builder keeps
    if entry == "coo":
        # the trainer's wiring: coalesced COO indices()/values() of the three matrices; the model converts them once
        # (csr_from_coo: CSR + n-gram tile plan + schedule, cached by tensor identity) in the first, untimed, call
        data = pkg.synth.trainer_data(g, x)
        del g
        with torch.no_grad():
            g = model.graph_of(data)
            if tr is not None:  # a builder-produced level: the trainer hands its node map over once
                pkg.attach_ngram_map(g, tr)
        torch.cuda.synchronize()
        log(f"[bench] entry coo: csr_from_coo -> plan "
            + ("attached" if g.ngram is not None else "mapped" if g.ngram_map is not None else "NOT attached"))
    else:
        data = pkg.Data(x=x, graph=g)

    part = hp = mp = None
    partition = args.partition
    if partition == "auto":
        partition = AUTO_PARTITION.get(world, "middle")
    if (world > 1 and partition in ("middle", "replicate")
            and (shard.ngram_shape(g) is None or shard.ngram_shape(g)[1] < 3)):
        partition = "halo"
    if world > 1 and partition == "replicate":
        mp = shard.middle_partition(g, rank, world)
        mid_in = shard.middle_inputs(model, mp)
        mid_run = shard.MiddleRunner(model, mp, x, mid_in, graphs=not args.no_graphs, replicate=True)
        log(f"[bench] replicate: every rank runs layers 1..{L - 1} over all {N} rows, rank {rank} the last layer "
            f"over middles [{mp.m0}, {mp.m1}) = {mp.n_own} rows")
    elif world > 1 and partition == "middle":
        # sub-ranges for the overlapped exchange only where a rank's share is large enough that a sub-range still
        # fills the GPU (a middle-tile launch has a fixed ~10 us start; at 4-gram, 8 ranks, 20k rows each, one
        # range is faster; at 5-gram, 400k rows each, four)
        n_own = N // world
        chunks = args.chunks if args.chunks > 0 else max(1, min(4, n_own // 100_000))
        mp = shard.middle_partition(g, rank, world, chunks=chunks)
        mid_in = shard.middle_inputs(model, mp)
        mid_run = shard.MiddleRunner(model, mp, x, mid_in, graphs=not args.no_graphs)  # setup: HIP graphs captured
        log(f"[bench] middle partition: rank {rank} owns middles [{mp.m0}, {mp.m1}) = {mp.n_own} rows, receives "
            f"{int(mp.recv_ids.numel())} ghost rows per layer boundary (N={N})")
    elif world > 1 and partition == "halo":
        hp = shard.halo_partition(g, rank, world, L)
        halo_in = shard.halo_inputs(model, hp, x)  # this rank's resident inputs in its node order (setup)
        log(f"[bench] halo partition: rank 0 computes {hp.layer_rows} rows per layer (N={N})")
    elif world > 1:
        part = shard.partition(g, rank, world)

    def eager_step():
        with torch.no_grad():
            if mp is not None:
                return mid_run._run_eager()
            if hp is not None:
                return shard.halo_forward(model, hp, halo_in)
            if part is None:
                return model(data)
            return shard.sharded_forward(model, part, x, chunks=args.chunks or 4)

    # The timed step. At N = 1 the forward is captured once as a HIP graph and replayed, as a rank's work is at
    # N > 1 (MiddleRunner's per-segment graphs): the 1 -> N ratio compares like with like. --no-graphs: eager.
    graph_step = None
    if mp is not None:
        step = mid_run  # replays its captured segments (eager with --no-graphs)
    elif world == 1 and not args.no_graphs:
        graph_step = GraphStep(eager_step)
        step = graph_step
    else:
        step = eager_step

    # untimed clock ramp: the GPU's clocks take ~100 ms of load to settle (5 warm-up steps measured 0.915 ms/step,
    # 50 or 200 gave 0.62): run steps for args.clock_warmup_s seconds before the W counted warm-up steps, so a short
    # --warmup (the driver passes 5) does not time a cold GPU. Outside the timed region, like every warm-up step.
    t_ramp = time.perf_counter()
    while time.perf_counter() - t_ramp < args.clock_warmup_s:
        for _ in range(10):
            step()
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    # per-kernel launch durations: HIP events recorded on each launch's stream around every propagation, dense and
    # head launch of eager runs of the same step right after the timed region (graph replays carry no per-launch
    # events; the kernels are the same). rocprofv3's kernel trace of the same command agrees (profiles/).
    # The eager steps themselves are bracketed by events on the current stream too (eager_ms_per_step): the
    # per-kernel times are checked against the step of the same mode (their sum cannot exceed it).
    ops.SPMM_EVENTS, ops.DENSE_EVENTS, ops.HEAD_EVENTS = [], [], []
    step_evs = []
    for _ in range(args.kernel_reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        eager_step()
        e1.record()
        step_evs.append((e0, e1))
    torch.cuda.synchronize()
    evs = {"propagation": ops.SPMM_EVENTS, "dense": ops.DENSE_EVENTS, "head": ops.HEAD_EVENTS}
    ops.SPMM_EVENTS = ops.DENSE_EVENTS = ops.HEAD_EVENTS = None
    kms = {k: [e0.elapsed_time(e1) for e0, e1 in v] for k, v in evs.items()}
    eager_ms = sum(e0.elapsed_time(e1) for e0, e1 in step_evs) / max(1, len(step_evs))
    t_local = torch.tensor([elapsed, eager_ms] + [sum(v) / max(1, len(v)) for v in kms.values()], dtype=torch.float64,
                           device=dev)
    if world > 1:
        dist.all_reduce(t_local, op=dist.ReduceOp.MAX)
    elapsed = float(t_local[0])
    eager_ms = float(t_local[1])
    avg_ms = dict(zip(kms, (float(v) for v in t_local[2:].tolist())))
    spmm_avg_ms = avg_ms["propagation"]
    ms_per_step = elapsed / args.steps * 1e3
    edges_per_step = 3 * g.nnz * L
    value = edges_per_step * args.steps / elapsed

    # roofline of each hot-path kernel, priced on SURVEY 8(d)'s COMPULSORY bytes per launch (its inputs once, its
    # outputs once): the floor of HBM traffic for one launch
    el = 2 if args.bf16 else 4
    gated = (world == 1 or hp is not None) and ops.PREGATED_INFERENCE and not args.fused_norm and not args.bf16
    if mp is not None:
        launch_graphs = [g]
    elif hp is not None:  # launches alternate over the layers' row prefixes: their mean
        launch_graphs = hp.graphs
    elif part is None:
        launch_graphs = [g]
    else:
        launch_graphs = [part.local]
    ngram = (all(gi.ngram is not None for gi in launch_graphs) and not args.bf16 and not args.fused_norm
             and Fd in (64, 128, 256))
    mapped = (all(gi.ngram_map is not None for gi in launch_graphs) and not args.bf16 and not args.fused_norm
              and Fd % 16 == 0)
    if mapped:  # builder-produced graph: mapped middle-tile kernel + the residual CSR pass (one propagation)
        gated = False
        kname = "pg_spmm3_ngram_mid_map_f32 + pg_spmm3_resid_f32"
    elif args.bf16:
        kname = ("pg_spmm3_ngram_mid_bf16" if all(gi.ngram is not None and gi.ngram.mplan is not None
                                                  for gi in launch_graphs) and Fd % 16 == 0 else "pg_spmm3_bf16")
    elif args.fused_norm:
        kname = "pg_spmm3_fusednorm_f32"
    elif ngram:  # n-gram tile kernel; inference gates the aggregates at its store
        mid = all(gi.ngram.mplan is not None for gi in launch_graphs) and Fd % 16 == 0
        gated = gated and not mid  # the middle-tile kernel stores ungated aggregates (the dense kernel gates)
        kname = ("pg_spmm3_ngram_mid_f32" if mid else "pg_spmm3_ngram_f32") + (" (gated)" if gated else "")
    else:
        kname = "pg_spmm3_gated_f32" if gated else "pg_spmm3_f32"
    comp = sum(gi.compulsory_bytes(Fd, elem=el, gated=gated) for gi in launch_graphs) // len(launch_graphs)
    if mp is not None:  # a rank's launch: its middles' plan share, the rows they read once, its rows' aggregates
        mid_launch = (g.ngram is not None and g.ngram.mplan is not None and Fd % 16 == 0 and not args.fused_norm
                      and (args.bf16 or ngram))
        if mid_launch:
            kname = "pg_spmm3_ngram_mid_rows_" + ("bf16" if args.bf16 else "f32")
            reads = shard._middle_reads(mp.K, mp.ngram, mp.m0, mp.m1, mp.own.device).numel()
            comp = (g.ngram.mplan.numel() * 4 * (mp.m1 - mp.m0) // (N // mp.K ** 2) + reads * Fd * el
                    + mp.n_own * 3 * Fd * el)
            if mid_run.replicate:  # L-1 whole-graph launches, then one over the rank's middles: their mean
                sfx = "bf16" if args.bf16 else "f32"
                kname = f"pg_spmm3_ngram_mid_{sfx} x{L - 1} + pg_spmm3_ngram_mid_rows_{sfx}"
                comp = ((L - 1) * g.compulsory_bytes(Fd, elem=el, gated=False) + comp) // L
        else:
            kname = "pg_spmm3_bf16" if args.bf16 else "pg_spmm3_f32"
            comp = mp.own_csr.compulsory_bytes(Fd, elem=el, gated=False)
    noreuse = sum(gi.algorithmic_bytes(Fd, elem=el) for gi in launch_graphs) // len(launch_graphs)
    # rows per dense launch (mean over the step's L launches) and per head launch
    if mp is not None:
        own = mp.n_own
        dense_rows = ((L - 1) * N + own) / L if mid_run.replicate else own
        head_rows = own
    elif hp is not None:
        dense_rows, head_rows = sum(hp.layer_rows) / L, hp.owned
    elif part is not None:
        dense_rows = head_rows = part.n_local
    else:
        dense_rows = head_rows = N
    C = 20
    # dense: Z (3F) + residual row (F) + constant (F_out fp32) + 5 gates (fp32; pre-gated Z: none) + Y, + weights;
    # head: h row + log-probs + embedding row (fp32), + decoder weights
    dense_comp = int(dense_rows * (3 * Fd * el + Fd * el + Fd * 4 + (0 if gated else 20) + Fd * el)
                     + 4 * (4 * Fd * Fd + 6 * Fd))
    H = Fd // 2
    head_comp = int(head_rows * (Fd * el + C * 4 + Fd * 4) + 4 * (H * Fd + H + C * H + C))
    dense_name = ("pg_directgcn_dense_ngram_rows_f32" if mp is not None and getattr(mid_run, "mapped", False)
                  else "pg_directgcn_dense_" + ("bf16" if args.bf16 else "f32"))
    head_name = "pg_directgcn_head_" + ("bf16" if args.bf16 else "f32")
    per_step = {"propagation": L, "dense": L, "head": 1}

    def kernel_entry(cls, name, nbytes, extra=None):
        # every derived field is computed from the EMITTED avg_launch_ms (rounded to 1 ns), so a reader recomputing
        # achieved / frac from the line gets the same numbers up to the 0.1 GB/s rounding of achieved
        ms = round(avg_ms[cls], 6)
        ach = nbytes / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
        e = {"kernel": name, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": None, "algorithmic_bytes_per_launch": int(nbytes),
             "avg_launch_ms": ms, "launches_timed": len(kms[cls]), "launches_per_step": per_step[cls],
             "ms_per_step": round(ms * per_step[cls], 6)}
        if extra:
            e.update(extra)
        return e

    kernels = {
        "propagation": kernel_entry("propagation", kname, comp,
                             {"no_reuse_bytes_per_launch": noreuse,
                              "no_reuse_gbs": (round(noreuse / (round(spmm_avg_ms, 6) * 1e-3) / 1e9, 1)
                                               if round(spmm_avg_ms, 6) else None),
                              "bytes_model": "compulsory: the kernel's own inputs once (n-gram tile kernel: its plan "
                                             "weights; CSR kernels: 8(N+1) rowptr + 16 B records per entry, SURVEY "
                                             "8d) + X once + 3 output rows (+ 20 B/row gates)"}),
        "dense": kernel_entry("dense", dense_name, dense_comp,
                       {"bytes_model": "Z (3F) + residual row (F) + per-node constant (F_out, fp32) + 5 gates (fp32) "
                                       "+ output row, per row; + the layer's weights"}),
        "head": kernel_entry("head", head_name, head_comp,
                      {"bytes_model": "h row + log-probs + L2-normalised embedding (fp32), per row; + the decoder"}),
    }
    dominant = max(kernels, key=lambda k: kernels[k]["ms_per_step"])
    roofline = dict(kernels[dominant])
    roofline["dominant_by"] = ("measured time per step (avg launch ms x launches per step, HIP events): "
                               + ", ".join(f"{k} {v['ms_per_step']} ms" for k, v in kernels.items()))
    roofline["kernels"] = kernels
    roofline["timing"] = ("step: " + ("HIP graph replays" if (graph_step is not None or (mp is not None and
                                                                                     mid_run.graphs is not None))
                                      else "eager launches")
                          + f"; per-kernel: HIP events around each launch of {args.kernel_reps} eager steps "
                            "after the timed region, on the launch stream (eager_ms_per_step: those steps' own "
                            "duration, the bound their per-kernel times sum under)")
    roofline["eager_ms_per_step"] = round(eager_ms, 6)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(g, model, x, args.cpu_sample_layers, log)

    if rank == 0 and world == 1 and not args.no_pmc:
        pmc = pmc_traffic(args, log)
        if pmc is not None:
            for cls, ent in list(kernels.items()) + [(dominant, roofline)]:
                hit = pmc["by_class"].get(cls)
                if not hit:
                    continue
                ent["traffic"] = hit["bytes_per_launch"]
                ent["traffic_kernel"] = hit["kernel"]
                ent["traffic_source"] = pmc["traffic_source"]
                ms = ent["avg_launch_ms"]
                ent["traffic_gbs"] = round(ent["traffic"] / (ms * 1e-3) / 1e9, 1) if ms else None
                ent["traffic_frac"] = round(ent["traffic"] / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5) if ms else None
                ent["traffic_over_compulsory"] = round(ent["traffic"] / ent["algorithmic_bytes_per_launch"], 3)

    extra = {}
    if args.extra and world == 1:
        extra = extra_measurements(pkg, ops, g, model, x, data, log)

    if rank == 0:
        line = {
            "metric": "edges/sec propagated, DirectGCN fwd on 4-gram graph, 1/2/4/8 MI355X",
            "value": round(value, 1), "unit": "edges/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 6), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "bf16" if args.bf16 else "f32", "data": "synthetic",
            "config": {"workload": wl["workload"], "graph": wl["desc"],
                       "num_nodes": N, "transitions": int(wl["E"]), "nnz_per_adjacency": g.nnz, "feat_dim": Fd,
                       "layers": L, "layer_dims": dims, "classes": C,
                       "propagation": "fused-norm" if args.fused_norm else "precomputed-weights",
                       "entry": ("trainer COO (edge_index_*/edge_weight_* -> csr_from_coo)" if entry == "coo"
                                 else "prebuilt Data.graph (build_propagation_csr)"),
                       "parallelism": ("single" if world == 1
                                       else f"replicate_then_middle_x{world}" if mp is not None and mid_run.replicate
                                       else f"middle_ghost_a2a_x{world}" if mp is not None
                                       else f"halo_recompute_x{world}" if hp is not None else f"node_range_x{world}"),
                       "ghost_rows_rank0": (int(mp.recv_ids.numel()) if mp is not None and not mid_run.replicate
                                            else None),
                       "exchange_chunks": (mp.chunks if mp is not None and not mid_run.replicate
                                           else (args.chunks or 4) if part is not None else None),
                       "halo_rows_rank0": hp.layer_rows if hp is not None else None},
            "nodes_per_sec": round(N * L * args.steps / elapsed, 1),
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        if extra:
            line["extra"] = extra
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def build_workload(pkg, args, dev, keep_raw=False):
    """The bench graph: the complete B(20, n) (--graph debruijn) or a builder-produced level (--graph fasta:
    ngram.ngram_transitions over synth.protein_sequences(args.fasta_seqs, 350, seed=1) -- the padding ' ' of
    data_builder.py:29-35, rare X/U/B/Z, sorted-string ids -- with the mapped middle-tile plan attached).
    Shared with tools/kprobe.py (the PMC passes run the same workload)."""
    n = args.ngram
    if getattr(args, "graph", "debruijn") == "debruijn":
        N, s, d, c = pkg.synth.de_bruijn_edges(n)
        g = pkg.build_propagation_csr(N, s, d, c, device=dev, keep_raw=keep_raw)
        return {"N": N, "E": int(s.size), "graph": g, "transitions": None,
                "desc": f"complete n-gram de Bruijn B(20,{n})", "workload": f"directgcn_fwd_B(20,{n})"}
    seqs = pkg.synth.protein_sequences(args.fasta_seqs, 350, seed=1)
    tr = pkg.ngram.ngram_transitions(seqs, n, device=dev)
    g = pkg.build_propagation_csr(tr.num_nodes, tr.src.cpu().numpy(), tr.dst.cpu().numpy(), tr.cnt.cpu().numpy(),
                                  device=dev, keep_raw=keep_raw, transitions=tr)
    res = sum(len(q) for q in seqs)
    return {"N": tr.num_nodes, "E": int(tr.src.numel()), "graph": g, "transitions": tr,
            "desc": (f"builder-produced {n}-gram level: {args.fasta_seqs} padded protein-like sequences ({res} "
                     f"residues, Swiss-Prot composition, 0.1% X/U/B/Z), sorted-string ids"),
            "workload": f"directgcn_fwd_fasta{n}"}


class GraphStep:
    """A step captured once as a HIP graph (torch.cuda.CUDAGraph) and replayed; returns the graph's static outputs
    (overwritten by the next replay). Two eager runs first (lazy library state, allocator pools, the COO -> CSR
    cache); the capture mode is thread-local."""

    def __init__(self, fn):
        import torch
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
            self.out = fn()
        torch.cuda.synchronize()

    def __call__(self):
        self.graph.replay()
        return self.out


def bench_model(pkg, N, Fd, L, n, C=20):
    """ProtGramDirectGCN([Fd]*(L+1), N, C) with the reference init (torch.manual_seed(0)) and non-trivial gates /
    biases (the reference init has C=1, b=0), on the CPU."""
    import torch
    torch.manual_seed(0)
    model = pkg.ProtGramDirectGCN([Fd] * (L + 1), N, C, n, 0, 512, 0.5, True)
    with torch.no_grad():
        gen = torch.Generator().manual_seed(11)
        for name, p in model.named_parameters():
            leaf = name.split(".")[-1]
            if leaf.startswith("C_"):
                p.copy_(torch.rand(p.shape, generator=gen) + 0.5)
            elif "bias" in leaf:
                p.copy_(torch.rand(p.shape, generator=gen) * 0.2 - 0.1)
    return model


def pmc_traffic(args, log, timeout=240):
    """roofline.traffic measured live: two rocprofv3 counter passes (FETCH_SIZE, then WRITE_SIZE: one TCC group
    each, --kernel-trace only) over tools/kprobe.py --forward, i.e. this bench's own step on the same workload
    from this same tree, corrected as MI355X_MICROARCH.md prescribes (read = 2 x FETCH_SIZE KiB on gfx950,
    write = WRITE_SIZE KiB). The dominant kernel is the one with the largest total duration in the pass."""
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        log("[bench] rocprofv3 not found: roofline.traffic = null")
        return None
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import pmc_traffic as pt
    out = tempfile.mkdtemp(prefix="pg_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    child = [sys.executable, os.path.join(REPO, "tools", "kprobe.py"), "--forward", "3", "--ngram", str(args.ngram),
             "--feat", str(args.feat), "--layers", str(args.layers), "--entry", args.entry,
             "--graph", args.graph, "--fasta-seqs", str(args.fasta_seqs)] \
        + (["--bf16"] if args.bf16 else []) \
        + (["--fused-norm"] if args.fused_norm else [])
    env = dict(os.environ)
    env.setdefault("TMPDIR", "/tmp")
    t0 = time.time()
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        cmd = [prof, "--pmc", counter, "--kernel-trace", "-d", os.path.join(out, counter), "-o", "k",
               "--output-format", "csv", "--"] + child
        try:
            r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=timeout)
        except subprocess.TimeoutExpired:
            log(f"[bench] rocprofv3 --pmc {counter} timed out: roofline.traffic = null")
            return None
        if r.returncode != 0:
            log(f"[bench] rocprofv3 --pmc {counter} failed (rc={r.returncode}): roofline.traffic = null\n"
                + r.stdout.decode(errors="replace")[-2000:])
            return None
    res = pt.reduce(os.path.join(out, "FETCH_SIZE"), os.path.join(out, "WRITE_SIZE"))
    shutil.rmtree(out, ignore_errors=True)
    if not res.get("kernel"):
        return None
    log(f"[bench] PMC traffic ({time.time() - t0:.0f}s): " + "; ".join(
        f"{k}: {v['kernel'][:60]} {v['bytes_per_launch'] / 1e6:.1f} MB per launch"
        for k, v in res.get("by_class", {}).items()))
    return {"by_class": res.get("by_class", {}),
            "traffic_source": "measured in this run: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over "
                              "tools/kprobe.py --forward (this bench's step), read = 2 x FETCH_SIZE KiB, "
                              "write = WRITE_SIZE KiB, per launch"}


def usable_cpus() -> int:
    """CPUs this process may run on: its affinity set, capped by a cgroup-v2 CPU quota if there is one."""
    import math
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, math.ceil(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(g, model, x, layers, log, max_msg_bytes=6 << 30):
    """The reference algorithm on this host's CPU (oracle = op-for-op restatement of
    protgram_directgcn.py:93-135 with PyG's propagate), on the same graph / weights / features:
    ``layers`` DirectGCN layer forward(s). When one propagate's [nnz, F] message tensor would exceed
    ``max_msg_bytes`` (5-gram: 67 GB), a bounded sample is timed instead: the entries of the first R
    destination rows (all source rows stay available), and edges/s counts the entries processed.

    Threads (SURVEY 8d / BASELINE.md: all host cores): torch is tried at os.cpu_count() threads and at the CPUs
    this process may actually use (affinity / cgroup quota) on one propagate, and the faster count runs the
    measurement; the previous setting is restored afterwards."""
    import numpy as np
    import torch

    from oracle import directgcn_cpu as oc

    prev_threads = torch.get_num_threads()
    e = g.edges3.cpu().numpy()
    rp = g.rowptr.cpu().numpy()
    N = g.n_rows
    F = x.size(1)
    nnz_keep = e.shape[0]
    if nnz_keep * F * 4 > max_msg_bytes:
        limit = max_msg_bytes // (F * 4)
        R = int(np.searchsorted(rp, limit, side="right")) - 1
        nnz_keep = int(rp[R])
    rows = torch.from_numpy(np.repeat(np.arange(N, dtype=np.int64), np.diff(rp))[:nnz_keep])
    ei = torch.stack([torch.from_numpy(e[:nnz_keep, 0].astype(np.int64)), rows])
    w = [torch.from_numpy(e[:nnz_keep, 1 + j].copy().view(np.float32)) for j in range(3)]
    xc = x.float().cpu()
    usable, total = usable_cpus(), os.cpu_count() or 1
    cands = sorted({usable, total})
    probe = {}
    try:
        with torch.no_grad():
            if len(cands) > 1:
                k = min(nnz_keep, 1 << 20)  # probe on a bounded slice: an oversubscribed count can be slow
                for th in cands:  # one warm + one timed propagate per candidate thread count
                    torch.set_num_threads(th)
                    oc.propagate(ei[:, :k], xc, w[0][:k])
                    t0 = time.perf_counter()
                    oc.propagate(ei[:, :k], xc, w[0][:k])
                    probe[th] = time.perf_counter() - t0
                threads = min(probe, key=probe.get)
            else:
                threads = cands[0]
            torch.set_num_threads(threads)
            times = []
            reps = 3
            for i, conv in enumerate(model.convs[:layers]):
                p = {k: v.detach().float().cpu() for k, v in conv.state_dict().items()}
                ts = []
                for rep in range(reps + 1):  # 1 warm-up + `reps` timed runs per layer, median
                    t0 = time.perf_counter()
                    y = oc.layer_forward(p, xc, ei, w[0], ei, w[1], ei, w[2])
                    dt = time.perf_counter() - t0
                    if rep:
                        ts.append(dt)
                times.append(sorted(ts)[len(ts) // 2])
                xc = torch.nn.functional.leaky_relu(y + xc)
    finally:
        torch.set_num_threads(prev_threads)
    t = sum(times)
    val = 3 * nnz_keep * len(times) / t
    full = nnz_keep == e.shape[0]
    log(f"[bench] cpu baseline: {len(times)} layer(s) over {nnz_keep} entries/adj in {t:.2f}s on {threads} threads "
        f"(probe s/propagate by threads: {({k: round(v, 3) for k, v in probe.items()})}) -> {val:.3e} edges/s")
    what = (f"full graph (N={N}, 3x{e.shape[0]} entries)" if full else
            f"row sample: first {int(rows[-1]) + 1 if nnz_keep else 0} of {N} destination rows (3x{nnz_keep} of "
            f"3x{e.shape[0]} entries; a full propagate would materialise {e.shape[0] * F * 4 / 1e9:.0f} GB)")
    cpu_model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": round(val, 1), "unit": "edges/s", "cores": threads, "kind": "port",
            "sample": f"{len(times)} DirectGCN layer forward(s), {what}; oracle = reference CPU algorithm "
                      f"(6 Linear + 6 index_select/mul/scatter_add_), torch {torch.__version__} CPU, {threads} threads "
                      f"(faster of os.cpu_count()={total} and the {usable} CPUs usable by this process "
                      f"[affinity/cgroup quota] on one timed propagate of <=2^20 entries: {({k: round(v, 3) for k, v in probe.items()})} s) "
                      f"on {cpu_model}, median of {reps} timed runs per layer after 1 warm-up",
            "threads_probe_s": {str(k): round(v, 3) for k, v in probe.items()},
            "host_cpus": total, "usable_cpus": usable, "seconds": round(t, 3)}


def extra_measurements(pkg, ops, g, model, x, data, log):
    """Kernel-variant timings and a training step (diagnostics, stderr + 'extra' field)."""
    import torch
    res = {}

    def timeit(fn, reps=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    from protgram_directgcn_amd._lib import (PG_FLAG_MID_NO_PAIRS, PG_FLAG_NGRAM_BLOCK4, PG_FLAG_NO_NGRAM,
                                             PG_FLAG_UNROLL4)
    Fd = x.size(1)
    comp = g.compulsory_bytes(Fd)
    conv0 = model.convs[0]
    prm0 = dict(zip(ops._DENSE_KEYS, (p.detach() for p in conv0._dense_params())))
    df = ops.default_flags()
    variants = [(df, "ngram" if g.ngram is not None else "csr")]
    if g.ngram is not None:
        variants += [(df | PG_FLAG_MID_NO_PAIRS, "ngram_mid_no_pairs"), (df | PG_FLAG_NGRAM_BLOCK4, "ngram_block4")]
    variants += [(df | PG_FLAG_NO_NGRAM, "csr_window_u4"), (df | PG_FLAG_NO_NGRAM | PG_FLAG_UNROLL4, "csr_window_u8")]
    for fl, name in variants:
        ms = timeit(lambda: ops.spmm3(g, x, flags=fl))
        res[f"spmm3_{name}_ms"] = round(ms, 4)
        res[f"spmm3_{name}_compulsory_GBs"] = round(comp / ms / 1e6, 1)
        if ops.spmm3_gated(g, x, prm0, 0, flags=fl) is not None:  # kernels with a gated store (not the middle one)
            res[f"spmm3_gated_{name}_ms"] = round(timeit(lambda: ops.spmm3_gated(g, x, prm0, 0, flags=fl)), 4)
        if g.raw is not None and fl:
            res[f"spmm3_fused_{name}_ms"] = round(timeit(lambda: ops.spmm3(g, x, fused=True, flags=fl)), 4)
    Z = ops.spmm3(g, x)
    conv = model.convs[0]
    prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in conv._dense_params())))
    flops = 2 * x.size(0) * 3 * Fd * conv.out_channels
    ms = timeit(lambda: ops.layer_dense(Z, prm, 0, constant=conv.constant.detach(), res_x=x, act=True))
    res["dense_ms"] = round(ms, 4)
    res["dense_TFLOPs"] = round(flops / ms / 1e9, 2)
    dec = model.decoder_fc
    res["head_ms"] = round(timeit(lambda: ops.head(x, dec[0].weight, dec[0].bias, dec[3].weight, dec[3].bias,
                                                   1e-12)), 4)
    G = torch.randn_like(Z)
    for fl, name in ((0, "ngram" if g.ngram is not None else "csr"), (PG_FLAG_NO_NGRAM, "csr_window_u4")):
        res[f"spmm3t_{name}_ms"] = round(timeit(lambda: ops.spmm3_t(g, G, flags=fl)), 4)
    # copy-kernel bandwidth reference
    a = torch.empty(512 * 1024 * 1024 // 4, device=x.device)
    b = torch.empty_like(a)
    ms = timeit(lambda: b.copy_(a))
    res["copy_GBs"] = round(2 * a.numel() * 4 / ms / 1e6, 1)
    # training step: the reference trainer's loop (protgram_directgcn_trainer.py:91-100: autocast +
    # GradScaler + L2 term + Adam(wd=0)), and the same without autocast/GradScaler
    model.train()
    y = (torch.arange(x.size(0), device=x.device) // (20 ** 3)).clamp(max=19)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=0.0)
    scaler = torch.amp.GradScaler("cuda", enabled=True)
    import torch.nn.functional as F

    def train_step(amp):
        opt.zero_grad()
        with torch.amp.autocast("cuda", enabled=amp):
            lp, _ = model(data)
            loss = F.nll_loss(lp, y) + 1e-7 * sum(p.norm(2).pow(2) for p in model.parameters() if p.requires_grad)
        if amp:
            scaler.scale(loss).backward()
            scaler.step(opt)
            scaler.update()
        else:
            loss.backward()
            opt.step()

    if x.dtype == torch.float32 or getattr(ops, "BF16_BACKWARD", False):
        res["train_step_ms"] = round(timeit(lambda: train_step(False), reps=5), 3)
        res["train_step_trainer_amp_ms"] = round(timeit(lambda: train_step(True), reps=5), 3)
    model.eval()
    log(f"[bench] extra: {json.dumps(res)}")
    return res


if __name__ == "__main__":
    main()
