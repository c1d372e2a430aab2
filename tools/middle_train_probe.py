#!/usr/bin/env python3
"""Per-rank step time of config 5's 8-GPU training (shard.MiddleTrainer) measured on one MI355X.

BASELINE config 5: 3-layer DirectGCN, 4-gram graph (N = 160,000), dims [128, 256, 256, 256], bf16, the trainer's
full-batch step (protgram_directgcn_trainer.py:91-100). For ranks of P = 8 (default 0 and 7) the probe runs that rank's
MiddleTrainer.step with the collectives replaced by local no-ops (the received buffers zeroed, the all-reduce skipped):
the compute a rank does per step. It prints the per-rank step time (HIP events, median of --reps after warm-up), the
bytes the rank would move per step over xGMI (forward ghost rows + their gradients, per layer boundary, and the
all-reduce of the replicated gradients), the single-GPU step of the same model (train.train_step + train.Adam, the
same rank-less kernels), and the projected 8-GPU step at a stated link rate.
  python tools/middle_train_probe.py [--ranks 0 7] [--fp32] [--reps 20] [--link-gbs 50]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import shard, train  # noqa: E402
from test_gpu_configs import _labels, _model  # noqa: E402


class SoloComm:
    """No-op collectives: a rank's compute alone (received rows / gradients zero, no all-reduce)."""
    capturable = True

    def all_to_all(self, out, inp, out_splits, in_splits):
        out.zero_()

    def all_reduce(self, t):
        pass


class RcclVolumeComm:
    """Real RCCL collectives at world size 1 moving the P-rank exchange's byte volume: each all_to_all sends the
    rank's rows to itself through RCCL (min(send, receive) rows of the chunk), the all-reduce runs on RCCL. The
    per-rank step then carries the product's TorchComm call pattern and RCCL's per-call costs (not xGMI transfer)."""
    capturable = True

    def all_to_all(self, out, inp, out_splits, in_splits):
        import torch.distributed as dist
        k = min(out.size(0), inp.size(0))
        if k:
            dist.all_to_all_single(out[:k], inp[:k])

    def all_reduce(self, t):
        import torch.distributed as dist
        dist.all_reduce(t)


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, nargs="*", default=[0, 7])
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--fp32", action="store_true")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--comm", choices=("solo", "rccl"), default="solo",
                    help="solo: no-op collectives (compute alone); rccl: RcclVolumeComm on a world-1 RCCL group")
    ap.add_argument("--link-gbs", type=float, default=50.0,
                    help="assumed usable xGMI rate per peer link (GB/s) for the projection (not measured here)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if args.comm == "rccl":
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    make_comm = SoloComm if args.comm == "solo" else RcclVolumeComm
    n, dims, lam = 4, [128, 256, 256, 256], 1e-7
    N, s, d, c = pkg.synth.de_bruijn_edges(n)
    g = pkg.build_propagation_csr(N, s, d, c, device=dev)
    x = torch.randn(N, dims[0], generator=torch.Generator().manual_seed(1234)).to(dev)
    y = _labels(N, n).to(dev)
    dt = torch.float32 if args.fp32 else torch.bfloat16
    el = 4 if args.fp32 else 2
    out = {"config": "config 5: 4-gram B(20,4), dims [128,256,256,256], " + ("fp32" if args.fp32 else "bf16"),
           "world": args.world, "ranks": {}}
    # single-GPU step (train_step + train.Adam), the same model
    m1 = _model(pkg, dims, N, n).to(dev).eval()
    m1.compute_dtype = dt
    opt = train.Adam(m1.parameters(), lr=1e-3)
    data = pkg.Data(x=x, graph=g)
    out["single_gpu_step_ms"] = round(timed(lambda: train.train_step(m1, data, y, opt, l2_lambda=lam), args.reps), 4)
    del m1, opt
    for r in args.ranks:
        mp_ = shard.middle_partition(g, r, args.world)
        m = _model(pkg, dims, N, n).to(dev).eval()
        m.compute_dtype = dt
        t0 = time.time()
        tr = shard.MiddleTrainer(m, mp_, l2_lambda=lam, comm=make_comm())
        setup = time.time() - t0
        yo = y[mp_.own]
        ms = timed(lambda: tr.step(x, yo), args.reps)
        mg = _model(pkg, dims, N, n).to(dev).eval()
        mg.compute_dtype = dt
        trg = shard.MiddleTrainer(mg, mp_, l2_lambda=lam, comm=make_comm(), graphs=True)
        for _ in range(trg.WARM + 1):  # eager warm-up steps, then the capture
            trg.step(x, yo)
        ms_graph = timed(lambda: trg.step(x, yo), args.reps)
        trg.close()
        del trg, mg
        ghost = int(mp_.recv_ids.numel())
        sent = int(mp_.send_pos.numel())
        widths = dims[1:-1]  # layer boundaries: outputs of every layer but the last
        fwd = sum((ghost) * w * el for w in widths)
        bwd = sum((ghost) * w * el for w in widths)
        dense = tr.flat.numel() * 4
        peers = max(1, sum(1 for k in mp_.recv_counts if k))
        xfer_ms = (fwd + bwd) / peers / (args.link_gbs * 1e9) * 1e3 + 2 * dense / (args.link_gbs * 1e9 * 7) * 1e3
        out["ranks"][r] = {"own_rows": mp_.n_own, "ghost_rows": ghost, "rows_sent": sent, "step_ms": round(ms, 4),
                           "step_ms_hip_graph": round(ms_graph, 4),
                           "setup_s": round(setup, 2), "exchange_bytes_per_step": fwd + bwd,
                           "allreduce_bytes": dense, "source_peers": peers,
                           "projected_xfer_ms_at_link": round(xfer_ms, 4)}
        print(f"[probe] rank {r}/{args.world}: own {mp_.n_own} ghost {ghost} step {ms:.3f} ms (graph {ms_graph:.3f}) "
              f"(single GPU {out['single_gpu_step_ms']:.3f} ms)", file=sys.stderr, flush=True)
        del tr, m
    worst = max(min(v["step_ms"], v["step_ms_hip_graph"]) + v["projected_xfer_ms_at_link"]
                for v in out["ranks"].values())
    out["projected_p8_step_ms"] = round(worst, 4)
    out["projected_speedup"] = round(out["single_gpu_step_ms"] / worst, 2)
    out["link_assumption_gbs"] = args.link_gbs
    out["comm"] = args.comm
    out["note"] = (("per-rank compute measured with no-op collectives" if args.comm == "solo" else
                    "per-rank step with the product's collective calls on a world-1 RCCL group (RcclVolumeComm: "
                    "the exchange's rows sent to the rank itself, RCCL per-call costs included, no xGMI transfer)")
                   + "; exchange priced at the assumed link rate, all ghost rows of a rank spread over its source "
                     "peers' links, not overlapped with compute")
    print(json.dumps(out))
    if args.comm == "rccl":
        import gc
        import torch.distributed as dist
        gc.collect()
        torch.cuda.synchronize()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
