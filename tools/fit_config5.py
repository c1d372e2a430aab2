#!/usr/bin/env python3
"""The reference's full-batch training loop (protgram_directgcn_trainer.py:76-108: per epoch zero_grad -> forward ->
nll + l2_lambda * sum ||p||^2 -> backward -> Adam step -> ReduceLROnPlateau.step(loss) -> EarlyStopper) for config 5
on P GPUs: one process per GPU, each rank a shard.MiddleTrainer over its range of middle (n-2)-grams (the ghost rows
and their gradients exchanged with all_to_all_single, the replicated gradients all-reduced: RCCL over xGMI), driven by
train.fit with the reference configuration's scheduler and early-stopping defaults (config.py:77-83). With --graphs the
rank's step is captured as a HIP graph after its warm-up steps and replayed; the learning rate the scheduler sets
reaches the replays through train.Adam's device scalars.

  python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29500 \\
      tools/fit_config5.py --epochs 100 --graphs
  (--backend gloo: ranks may share one GPU, the collectives staged through host memory; not capturable)

Synthetic data of config 5's shape (BASELINE.json): the complete 4-gram graph over 20 letters (N = 160,000, random
transition counts), random features, labels = the first letter; model dims [128, 256, 256, 256] in bf16. Rank 0 prints
one JSON line: the per-epoch history (loss, learning rate, early stop) and the wall time per epoch."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402


def run(argv=None):
    """Parse argv, train, return rank 0's record (None on the other ranks)."""
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=50)
    ap.add_argument("--n", type=int, default=4, help="n-gram order (the graph is the complete K^n grid, K = 20)")
    ap.add_argument("--dims", default="128,256,256,256")
    ap.add_argument("--fp32", action="store_true", help="fp32 instead of config 5's bf16")
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--l2", type=float, default=1e-7, help="the trainer's L2 lambda")
    ap.add_argument("--graphs", action="store_true", help="replay each rank's step from a HIP graph")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl")
    ap.add_argument("--eval", action="store_true", help="no dropout (model.eval()): runs comparable across world sizes")
    ap.add_argument("--lr-patience", type=int, default=10)
    ap.add_argument("--lr-factor", type=float, default=0.5)
    ap.add_argument("--es-patience", type=int, default=25)
    ap.add_argument("--es-min-delta", type=float, default=1e-5)
    args = ap.parse_args(argv)
    pkg = load_package()
    from protgram_directgcn_amd import shard, train
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    dev = torch.device("cuda", local if args.backend == "nccl" else local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    kw = {"device_id": dev} if args.backend == "nccl" else {}
    dist.init_process_group(args.backend, rank=rank, world_size=world, **kw)
    try:
        dims = [int(v) for v in args.dims.split(",")]
        N, s, d, c = pkg.synth.de_bruijn_edges(args.n)
        g = pkg.build_propagation_csr(N, s, d, c, device=dev)
        x = torch.randn(N, dims[0], generator=torch.Generator().manual_seed(1234)).to(dev)
        y = (torch.arange(N) // 20 ** (args.n - 1)).to(dev)
        torch.manual_seed(0)  # every rank builds the same model (the reference init)
        model = pkg.ProtGramDirectGCN(dims, N, 20, args.n, 0, 512, 0.5, True).to(dev)
        model.train(not args.eval)
        model.compute_dtype = torch.float32 if args.fp32 else torch.bfloat16
        mp = shard.middle_partition(g, rank, world)
        tr = shard.MiddleTrainer(model, mp, lr=args.lr, l2_lambda=args.l2, graphs=args.graphs)
        y_own = y[mp.own]
        t0 = time.time()
        hist = train.fit(lambda: tr.step(x, y_own), tr.opt, args.epochs, lr_patience=args.lr_patience,
                         lr_factor=args.lr_factor, es_patience=args.es_patience, es_min_delta=args.es_min_delta)
        torch.cuda.synchronize()
        wall = time.time() - t0
        tr.close()
        if rank != 0:
            return None
        return {"config": f"{args.n}-gram, dims {dims}, {'fp32' if args.fp32 else 'bf16'}", "world": world,
                "backend": args.backend, "graphs": args.graphs, "epochs_run": len(hist),
                "s_per_epoch": round(wall / max(1, len(hist)), 5), "history": hist}
    finally:
        dist.destroy_process_group()


def main(argv=None):
    rec = run(argv)
    if rec is not None:
        print(json.dumps(rec), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
