"""Node-range partition of the DirectGCN forward over the GPUs of one node.

Rank p owns destination rows [r0, r1) = [p*ceil(N/P), ...). It holds:
  * its CSR rows (global column ids): zero-copy row slices of the full CSR
  * a replica of the layer parameters (per-node gates/constant are read at global row ids)
Layer 1 reads the replicated input X (static across steps: no exchange). Every later layer needs
the previous layer's output for ALL rows (the halo of a de Bruijn-like n-gram graph is ~the whole
graph: in-neighbours c+s[:-1] and out-neighbours s[1:]+c of any id range span every segment), so the
owned output rows are exchanged with one RCCL all-gather over xGMI per layer boundary
(``dist.all_gather_into_tensor``, equal-sized shards padded to ceil(N/P) rows).

Forward only (inference / embedding extraction path, ``models_utils.py:265-273``); the single-GPU
training step runs through ``ProtGramDirectGCN`` with autograd.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .graph import CSRGraph


@dataclass
class NodeRangePartition:
    rank: int
    world: int
    n: int
    per: int
    r0: int
    r1: int
    local: CSRGraph
    rows: torch.Tensor  # int64 [r1-r0] global row ids (gate / constant gather)

    @property
    def n_local(self) -> int:
        return self.r1 - self.r0


def partition(g: CSRGraph, rank: int, world: int) -> NodeRangePartition:
    if not g.shared:
        raise NotImplementedError("node-range partition needs the shared-pattern CSR")
    n = g.n_rows
    per = math.ceil(n / world)
    r0 = min(n, rank * per)
    r1 = min(n, r0 + per)
    rp = g.rowptr
    e0, e1 = int(rp[r0]), int(rp[r1])
    order = None
    if g.row_order is not None:  # keep the global schedule's relative order of the owned rows
        ro = g.row_order.to(torch.int64)
        order = (ro[(ro >= r0) & (ro < r1)] - r0).to(torch.int32)
    local = CSRGraph(n_rows=r1 - r0, shared=True, rowptr=(rp[r0:r1 + 1] - e0).contiguous(), edges3=g.edges3[e0:e1],
                     rowptr_t=None, edges3_t=None, symmetric=False, nnz=e1 - e0, row_order=order)
    rows = torch.arange(r0, r1, dtype=torch.int64, device=rp.device)
    return NodeRangePartition(rank, world, n, per, r0, r1, local, rows)


def _layer_local(conv, part: NodeRangePartition, h_full, res: nn.Module, act=True):
    Z = ops.spmm3(part.local, h_full)
    prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in conv._dense_params())))
    rows = part.rows if conv.use_vector_coeffs else None
    constant = conv.constant.detach() if conv.use_vector_coeffs else None
    res_x = h_full[part.r0:part.r1]
    if isinstance(res, nn.Linear):
        return ops.layer_dense(Z, prm, 0 if conv.use_vector_coeffs else 1, rows=rows, constant=constant, res_x=res_x,
                               W_res=res.weight.detach(), b_res=res.bias.detach(), act=act)
    return ops.layer_dense(Z, prm, 0 if conv.use_vector_coeffs else 1, rows=rows, constant=constant, res_x=res_x,
                           act=act)


@torch.no_grad()
def sharded_forward(model, part: NodeRangePartition, x_full: torch.Tensor, group=None, gather_buf=None):
    """ProtGramDirectGCN.forward restricted to this rank's rows; returns (log_probs, emb) for rows [r0, r1)."""
    h_full = model._apply_pe(x_full)
    L = len(model.convs)
    h_local = None
    for i, (conv, res) in enumerate(zip(model.convs, model.res_projs)):
        h_local = _layer_local(conv, part, h_full, res)
        if i + 1 < L:
            if part.world > 1:
                buf = gather_buf[i] if gather_buf is not None else None
                h_full = all_gather_rows(h_local, part, group, buf)
            else:
                h_full = h_local
    return model.head(h_local)


def all_gather_rows(h_local: torch.Tensor, part: NodeRangePartition, group=None, out=None) -> torch.Tensor:
    """[n_local, F] per rank -> [N, F] on every rank (RCCL all-gather, shards padded to `per` rows)."""
    Fd = h_local.size(1)
    if h_local.size(0) != part.per:
        pad = h_local.new_zeros(part.per, Fd)
        pad[:h_local.size(0)] = h_local
        h_local = pad
    if out is None:
        out = h_local.new_empty(part.per * part.world, Fd)
    if dist.get_backend(group) == "gloo":  # rehearsal backend (CPU tests, one-GPU dry runs)
        dist.all_gather(list(out.view(part.world, part.per, Fd).unbind(0)), h_local.contiguous(), group=group)
    else:
        dist.all_gather_into_tensor(out, h_local.contiguous(), group=group)
    return out[:part.n]
