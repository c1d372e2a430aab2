"""Diagnostic: is the bf16 ShardedTrainer step deterministic at world 1, and which gradients differ between
collectives off / on (shard.FORCE_COLLECTIVES) after ONE step."""
import os
import sys
import socket
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
import torch
import torch.distributed as dist
from __graft_entry__ import load_package
pkg = load_package()
from protgram_directgcn_amd import shard
from test_gpu_rccl import _model

with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
N, s_, d, c = pkg.synth.de_bruijn_edges(3)
g = pkg.build_propagation_csr(N, s_, d, c, device=dev)
x = torch.randn(N, 128, generator=torch.Generator().manual_seed(1234)).to(dev)
y = (torch.arange(N, device=dev) // 400) % 20
part = shard.partition(g, 0, 1, transpose=True)


def run(force, dt):
    shard.FORCE_COLLECTIVES = force
    m = _model(pkg, N, [128, 128, 128], dev, 3)
    m.compute_dtype = dt
    tr = shard.ShardedTrainer(m, part, lr=1e-3, l2_lambda=1e-3)
    loss = tr.step(x, y)
    torch.cuda.synchronize()
    gr = {}
    for li, dd in enumerate(tr.own):
        for k, leaf in dd.items():
            gr[f"convs.{li}.{k}"] = leaf.grad.detach().float().clone()
    for name, p in m.named_parameters():
        if name not in gr and p.grad is not None:
            gr[name] = p.grad.detach().float().clone()
    return float(loss), gr


for dt in (torch.bfloat16, torch.float32):
    a = run(False, dt)
    b = run(False, dt)
    f = run(True, dt)
    print(dt, "loss", a[0], b[0], f[0])
    for name in a[1]:
        d1 = float((a[1][name] - b[1][name]).abs().max())
        d2 = float((a[1][name] - f[1][name]).abs().max())
        if d1 or d2:
            print(f"  {name}: repeat {d1:.3e}  force {d2:.3e}  scale {float(a[1][name].abs().max()):.3e}")
dist.destroy_process_group()
