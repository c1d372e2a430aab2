"""Node-range partition of the DirectGCN forward over the GPUs of one node.

Rank p owns destination rows [r0, r1) = [p*ceil(N/P), ...). It holds:
  * its CSR rows (global column ids): zero-copy row slices of the full CSR
  * a replica of the layer parameters (per-node gates/constant are read at global row ids)
Layer 1 reads the replicated input X (static across steps: no exchange). Every later layer needs
the previous layer's output for ALL rows (the halo of a de Bruijn-like n-gram graph is ~the whole
graph: in-neighbours c+s[:-1] and out-neighbours s[1:]+c of any id range span every segment), so the
owned output rows are exchanged with one RCCL all-gather over xGMI per layer boundary
(``dist.all_gather_into_tensor``, equal-sized shards padded to ceil(N/P) rows).

Training (``sharded_train_step``, the trainer's step protgram_directgcn_trainer.py:91-100 on P GPUs):
  * the all-gather's autograd backward is a reduce-scatter of the partial input gradients: the
    transposed propagation of this rank's rows scatters into ALL source rows, i.e. dX_partial =
    A[:, owned]^T-block = (for the symmetric n-gram matrices) the owned COLUMN block of the global
    CSR, an SpMM over all N rows reading only the owned rows of dZ (``partition(..., transpose=True)``);
    RCCL ``reduce_scatter_tensor`` sums the P partials into their owners (1x the forward bytes);
  * dense weights/biases (replicated): one flat all-reduce (sum) of their gradients per step;
  * per-node parameters (C_*_vec gates, constant) are only ever read at owned rows, so their owned
    rows get complete gradients locally and need no communication; rows owned elsewhere are stale on
    this rank and never read (gather them with ``gather_node_params`` to checkpoint).
"""
from __future__ import annotations

import math
import weakref
from dataclasses import dataclass, field
from typing import List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .graph import CSRGraph, take

# Run the node-range partition's collectives (all-gather, reduce-scatter, all-reduce) even at world size 1, where they
# are identities: lets a one-GPU box execute the RCCL code paths the 8-GPU run takes (tests/test_gpu_rccl.py).
FORCE_COLLECTIVES = False


def _exchanging(world: int) -> bool:
    return world > 1 or FORCE_COLLECTIVES


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
    cache: dict = field(default_factory=dict)

    @property
    def n_local(self) -> int:
        return self.r1 - self.r0


def partition(g: CSRGraph, rank: int, world: int, transpose: bool = False) -> NodeRangePartition:
    """This rank's row block. ``transpose=True`` also builds the transposed column block needed by the
    backward (training)."""
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
                     rowptr_t=None, edges3_t=None, symmetric=False, nnz=e1 - e0, row_order=order, n_cols=n)
    if transpose:
        local.rowptr_t, local.edges3_t = _column_block(g, r0, r1)
    rows = torch.arange(r0, r1, dtype=torch.int64, device=rp.device)
    return NodeRangePartition(rank, world, n, per, r0, r1, local, rows)


def _column_block(g: CSRGraph, c0: int, c1: int):
    """CSR over all N rows of the transposed structure restricted to source columns [c0, c1), columns
    renumbered from 0: the transposed propagation of the row block [c0, c1). Uses the graph's own
    transposed CSR (rowptr_t / edges3_t, which alias the forward CSR for symmetric matrices). Entries
    stay in ascending column order within each row."""
    rp, e = g.rowptr_t, g.edges3_t
    n = rp.numel() - 1
    col = e[:, 0].to(torch.int64)
    keep = (col >= c0) & (col < c1)
    row_of = torch.repeat_interleave(torch.arange(n, device=rp.device), rp[1:] - rp[:-1])
    cnt = torch.bincount(row_of[keep], minlength=n)
    rowptr_t = torch.zeros(n + 1, dtype=torch.int64, device=rp.device)
    rowptr_t[1:] = torch.cumsum(cnt, 0)
    et = e[keep].clone()
    et[:, 0] -= c0
    return rowptr_t, et


def _rows_slice(g: CSRGraph, a: int, b: int, order: Optional[torch.Tensor]) -> CSRGraph:
    """Rows [a, b) of a row-block CSR (zero-copy), keeping the schedule's order among them."""
    rp = g.rowptr
    e0, e1 = int(rp[a]), int(rp[b])
    o = None
    if order is not None:
        ol = order.to(torch.int64)
        o = (ol[(ol >= a) & (ol < b)] - a).to(torch.int32)
    return CSRGraph(n_rows=b - a, shared=True, rowptr=(rp[a:b + 1] - e0).contiguous(), edges3=g.edges3[e0:e1],
                    symmetric=False, nnz=e1 - e0, row_order=o, n_cols=g.n_cols)


@dataclass
class GatherPlan:
    """Layer-boundary exchange in `chunks` pieces (overlap the all-gather with compute).

    The boundary layer is computed in `chunks` row chunks of `cs` rows; as soon as chunk k is done its
    rows are all-gathered (asynchronously: RCCL's own stream) while chunk k+1 computes. The gathered
    buffer is chunk-major -- [chunk k][rank p][cs rows] -- so the next layers read it through `remap`, a
    once-built copy of the local CSR whose column ids point into that buffer. Entry order inside rows is
    unchanged: results are bit-identical to the unchunked exchange."""
    chunks: int
    cs: int
    first: List[CSRGraph]    # layer-1 row chunks (global column ids, reads the replicated input)
    remap: CSRGraph          # local CSR with buffer column ids (layers >= 2)
    remap_chunks: List[CSRGraph]


def gather_plan(part: NodeRangePartition, chunks: int) -> GatherPlan:
    key = ("plan", chunks)
    cached = part.cache.get(key)
    if cached is not None:
        return cached
    chunks = max(1, min(int(chunks), part.per))
    cs = -(-part.per // chunks)
    W = part.world
    col = part.local.edges3[:, 0].to(torch.int64)
    p = col // part.per
    off = col - p * part.per
    k = off // cs
    pos = (k * W + p) * cs + (off - k * cs)
    e = part.local.edges3.clone()
    e[:, 0] = pos.to(torch.int32)
    remap = CSRGraph(n_rows=part.n_local, shared=True, rowptr=part.local.rowptr, edges3=e, symmetric=False,
                     nnz=part.local.nnz, row_order=part.local.row_order, n_cols=chunks * W * cs)
    bounds = [(min(c * cs, part.n_local), min((c + 1) * cs, part.n_local)) for c in range(chunks)]
    first = [_rows_slice(part.local, a, b, part.local.row_order) for a, b in bounds]
    remap_chunks = [_rows_slice(remap, a, b, part.local.row_order) for a, b in bounds]
    plan = GatherPlan(chunks, cs, first, remap, remap_chunks)
    part.cache[key] = plan
    return plan


def _dense_local(conv, part: NodeRangePartition, Z, res: nn.Module, res_x, a: int, b: int, out=None, act=True):
    """The dense layer over owned rows [r0 + a, r0 + b). They are one contiguous id range, so the per-node gates and
    constant are passed as row slices (no row map): the split-bf16 kernels take the call, as on one GPU."""
    prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in conv._dense_params())))
    vec = conv.use_vector_coeffs
    rows, constant = None, None
    if vec:
        lo, hi = part.r0 + a, part.r0 + b
        for k in ("C_in", "C_out", "C_directed", "C_undirected", "C_all"):
            prm[k] = prm[k][lo:hi]
        constant = conv.constant.detach()[lo:hi] if conv.constant is not None else None
    W_res, b_res = ((res.weight.detach(), res.bias.detach()) if isinstance(res, nn.Linear) else (None, None))
    return ops.layer_dense(Z, prm, 0 if vec else 1, rows=rows, constant=constant, res_x=res_x, W_res=W_res,
                           b_res=b_res, act=act, out=out)


def _all_gather_chunk(send: torch.Tensor, dst: torch.Tensor, part: NodeRangePartition, group=None):
    """send [cs, F] from every rank -> dst [world * cs, F] (rank-major), asynchronous (returns the work). The same
    tensor collective on RCCL and on gloo (the CPU rehearsal backend), so the tests run the product's calls."""
    return dist.all_gather_into_tensor(dst, send, group=group, async_op=True)


@torch.no_grad()
def sharded_forward(model, part: NodeRangePartition, x_full: torch.Tensor, group=None, gather_buf=None,
                    chunks: int = 1):
    """ProtGramDirectGCN.forward restricted to this rank's rows; returns (log_probs, emb) for rows [r0, r1).

    Layer 1 reads the replicated input; each later layer reads the previous layer's rows of all ranks,
    exchanged by all-gather in `chunks` pieces overlapped with the compute (GatherPlan). `gather_buf` is
    accepted for compatibility and unused (buffers come from the caching allocator)."""
    h = model._apply_pe(x_full)
    if model.compute_dtype == torch.bfloat16:
        h = h.to(torch.bfloat16)
    L = len(model.convs)
    plan = gather_plan(part, chunks) if (L > 1 and _exchanging(part.world)) else None
    h_local = None
    for i, (conv, res) in enumerate(zip(model.convs, model.res_projs)):
        first = i == 0
        X = h
        res_all = h[part.r0:part.r1] if first else h_local
        F_out = conv.out_channels
        if plan is not None and i + 1 < L:  # this layer's output is exchanged: compute it in chunks
            W, cs = part.world, plan.cs
            send = X.new_empty(plan.chunks * cs, F_out)
            buf = X.new_empty(plan.chunks * W * cs, F_out)
            works = []
            for c in range(plan.chunks):
                a, b = min(c * cs, part.n_local), min((c + 1) * cs, part.n_local)
                if b > a:
                    gk = plan.first[c] if first else plan.remap_chunks[c]
                    Z = ops.spmm3(gk, X)
                    _dense_local(conv, part, Z, res, res_all[a:b], a, b, out=send[a:b])
                works.append(_all_gather_chunk(send[c * cs:(c + 1) * cs], buf[c * W * cs:(c + 1) * W * cs], part,
                                               group))
            for w in works:
                if w is not None:
                    w.wait()
            h_local = send[:part.n_local]
            h = buf
        else:
            g = part.local if (first or plan is None) else plan.remap
            if not first and plan is None and part.world == 1:
                g = part.local
            Z = ops.spmm3(g, X)
            h_local = _dense_local(conv, part, Z, res, res_all, 0, part.n_local)
            h = h_local
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
    dist.all_gather_into_tensor(out, h_local.contiguous(), group=group)  # RCCL / gloo alike
    return out[:part.n]


def reduce_scatter_rows(d_full: torch.Tensor, part: NodeRangePartition, group=None) -> torch.Tensor:
    """[N, F] partial sums on every rank -> this rank's rows [n_local, F] of their sum over ranks
    (RCCL reduce-scatter; the backward of all_gather_rows)."""
    Fd = d_full.size(1)
    # bf16 partials are summed in fp32 (one rounding of the total, as the single-GPU bf16 backward rounds once)
    wide = d_full.dtype == torch.bfloat16
    buf = d_full.new_zeros(part.per * part.world, Fd, dtype=torch.float32 if wide else d_full.dtype)
    buf[:part.n] = d_full
    out = buf.new_empty(part.per, Fd)
    dist.reduce_scatter_tensor(out, buf, group=group)  # RCCL / gloo alike
    out = out[:part.n_local]
    return out.to(d_full.dtype) if wide else out


class _GatherRows(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h_local, part, group):
        ctx.part, ctx.group = part, group
        return all_gather_rows(h_local, part, group).clone()

    @staticmethod
    def backward(ctx, d_full):
        return reduce_scatter_rows(d_full.contiguous(), ctx.part, ctx.group), None, None


_GATE_NAMES = ("C_in_vec", "C_out_vec", "C_directed_vec", "C_undirected_vec", "C_all_vec")


def _layer_local_train(conv, part: NodeRangePartition, h_full, res: nn.Module, act=True, own: Optional[dict] = None):
    """One layer over this rank's rows with autograd. ``own`` (ShardedTrainer): the layer's per-node parameters as
    owned-row leaves ([n_local, ...], sharing storage with the model's full parameters) -- the dense kernels then
    read contiguous row slices (no row map) and the gradients come out [n_local, ...]; without it the full parameters
    are read at the owned global rows (and their gradients are full-size)."""
    if part.local.rowptr_t is None:
        raise ValueError("training needs partition(..., transpose=True)")
    Z = ops.Propagate3.apply(h_full, part.local, False)
    vec = conv.use_vector_coeffs
    res_x = h_full[part.r0:part.r1]
    W_res, b_res = (res.weight, res.bias) if isinstance(res, nn.Linear) else (None, None)
    params = conv._dense_params()
    if vec and own is not None:
        params = params[:10] + tuple(own[k] for k in _GATE_NAMES)
        rows, constant = None, own["constant"]
    else:
        rows = part.rows if vec else None
        constant = conv.constant if vec else None
    return ops.LayerDense.apply(Z, res_x, constant, W_res, b_res, rows, 0 if vec else 1, act, ops.LEAKY_SLOPE, None,
                                *params)


def sharded_forward_train(model, part: NodeRangePartition, x_full: torch.Tensor, group=None,
                          own: Optional[List[dict]] = None):
    """ProtGramDirectGCN.forward on this rank's rows with autograd (dropout as in the model: training mode
    only, per-rank RNG). Honours ``model.compute_dtype``: in bf16 mode the features, aggregates, layer outputs and
    the exchanged rows are bf16 (half the all-gather bytes), sums fp32, the head fp32. ``own``: per layer, the
    owned-row parameter leaves of ShardedTrainer. Returns (log_probs, emb) for rows [r0, r1)."""
    h_full = model._apply_pe(x_full)
    if model.compute_dtype == torch.bfloat16:
        h_full = h_full.to(torch.bfloat16)
    elif model.compute_dtype != torch.float32:
        raise ValueError("compute_dtype must be torch.float32 or torch.bfloat16")
    L = len(model.convs)
    h_local = None
    for i, (conv, res) in enumerate(zip(model.convs, model.res_projs)):
        h_local = _layer_local_train(conv, part, h_full, res, own=None if own is None else own[i])
        h_local = F.dropout(h_local, p=model.dropout, training=model.training)
        if i + 1 < L:
            h_full = _GatherRows.apply(h_local, part, group) if _exchanging(part.world) else h_local
    return model.head(h_local)


def _is_node_param(name: str, p: torch.Tensor, n: int) -> bool:
    leaf = name.split(".")[-1]
    return (leaf == "constant" or (leaf.startswith("C_") and leaf.endswith("_vec"))) and p.dim() >= 1 and p.size(0) == n


def sharded_train_step(model, part: NodeRangePartition, x_full: torch.Tensor, y_local: torch.Tensor, optimizer,
                       l2_lambda: float = 1e-7, group=None) -> float:
    """One step of the reference's full-batch loop (protgram_directgcn_trainer.py:91-100) on P ranks:
    zero_grad -> forward -> nll_loss (mean over all N nodes) + l2_lambda * sum_p ||p||^2 -> backward ->
    all-reduce of the replicated parameters' gradients -> optimizer.step(). Returns the global loss
    (a host sync, as the reference's loss.item())."""
    optimizer.zero_grad()
    lp, _ = sharded_forward_train(model, part, x_full, group)
    loss = F.nll_loss(lp, y_local, reduction="sum") / part.n
    if l2_lambda:
        l2 = 0.0
        for name, p in model.named_parameters():
            if not p.requires_grad:
                continue
            if _is_node_param(name, p, part.n):
                l2 = l2 + p[part.r0:part.r1].norm(2).pow(2)   # owned rows: each row counted once overall
            else:
                l2 = l2 + p.norm(2).pow(2) / part.world     # replicated: summed over ranks below
        loss = loss + l2_lambda * l2
    loss.backward()
    if _exchanging(part.world):
        dense = [p for name, p in model.named_parameters()
                 if p.grad is not None and not _is_node_param(name, p, part.n)]
        flat = torch.cat([p.grad.reshape(-1) for p in dense])
        dist.all_reduce(flat, group=group)
        off = 0
        for p in dense:
            k = p.numel()
            p.grad.copy_(flat[off:off + k].view_as(p.grad))
            off += k
    optimizer.step()
    tot = loss.detach().reshape(1).clone()
    if _exchanging(part.world):
        dist.all_reduce(tot, group=group)
    return float(tot)


class ShardedTrainer:
    """The reference trainer's full-batch step (``protgram_directgcn_trainer.py:91-100``: zero_grad -> forward ->
    ``nll_loss`` (mean over all N nodes) + ``l2_lambda * sum_p ||p||^2`` -> backward -> Adam step) on P ranks, with
    train.train_step's device-side semantics and the per-node state sharded:

    * per-node parameters (``C_*_vec``, ``constant``): this rank owns rows [r0, r1). It trains owned-row leaves
      that share storage with the model's full parameters, so gradients, Adam moments and the update cover ONLY the
      owned rows (1/P of the N x F ``constant`` state per rank; rows owned elsewhere are stale here and never read
      -- ``gather_node_params`` makes them whole for a checkpoint);
    * replicated parameters (weights, biases, residual projections, decoder): their gradients accumulate into views
      of ONE flat buffer, summed over ranks by one all-reduce (no cat / copy-back);
    * the optimizer is ``train.Adam`` (one launch per step) with the L2 gradient folded into its decay, after the
      all-reduce (so it is added once, not P times); any other optimizer gets ``p.grad += 2 l2_lambda p``;
    * the loss (nll over the owned rows / N plus the L2 value: replicated parameters once, owned rows summed over
      ranks) comes back as a device scalar, all-reduced on the device: no host sync per step;
    * ``model.compute_dtype = torch.bfloat16`` trains in bf16 mode (config 5): bf16 features, aggregates and
      exchanged rows, fp32 sums, parameters and optimizer.

    No GradScaler: the bf16 and fp32 modes need none (the reference's scaler serves its fp16 autocast)."""

    def __init__(self, model, part: NodeRangePartition, lr: float = 1e-3, l2_lambda: float = 1e-7, group=None,
                 optimizer_factory=None, **adam_kw):
        from . import train
        self.model, self.part, self.group, self.l2_lambda = model, part, group, float(l2_lambda)
        self.own: List[dict] = []
        node_leaves, dense = [], []
        full_of = {}
        for conv in model.convs:
            d = {}
            for name, p in conv.named_parameters(recurse=False):
                if _is_node_param(name, p, part.n):
                    leaf = nn.Parameter(p.data[part.r0:part.r1], requires_grad=p.requires_grad)
                    d[name] = leaf
                    full_of[id(p)] = leaf
                    node_leaves.append(leaf)
            self.own.append(d)
        for name, p in model.named_parameters():
            if id(p) not in full_of and p.requires_grad:
                dense.append(p)
        self.dense = dense
        self.node = node_leaves
        dev = dense[0].device if dense else part.local.rowptr.device
        self.flat = torch.zeros(sum(p.numel() for p in dense), dtype=torch.float32, device=dev)
        self.params = dense + [p for p in node_leaves if p.requires_grad]
        if optimizer_factory is None:
            self.opt = train.Adam(self.params, lr=lr, **adam_kw)
        else:
            self.opt = optimizer_factory(self.params)
        self._train = train
        # which parameters autograd reached this step (host-side hooks, no sync): with l2_lambda == 0 the others are
        # not stepped, as torch.optim.Adam skips parameters whose grad is None in the reference loop (the flat
        # buffer gives every replicated parameter a zero grad view). The replicated parameters' autograd graph is the
        # same on every rank, so the local record is the global one.
        self._touched: set = set()
        for prm in self.params:
            prm.register_post_accumulate_grad_hook(lambda t: self._touched.add(id(t)))

    def _grads_into_flat(self):
        off = 0
        for p in self.dense:
            k = p.numel()
            p.grad = self.flat[off:off + k].view_as(p)
            off += k

    def step(self, x_full: torch.Tensor, y_local: torch.Tensor) -> torch.Tensor:
        """One step; returns the global loss as a device scalar (call .item() only when the value is needed)."""
        part, lam, train = self.part, self.l2_lambda, self._train
        for p in self.node:
            p.grad = None
        self.flat.zero_()
        self._grads_into_flat()  # autograd accumulates into the flat buffer's views in place
        lp, _ = sharded_forward_train(self.model, part, x_full, self.group, own=self.own)
        nll = -lp.float().gather(1, y_local.view(-1, 1)).sum() / part.n
        self._touched = set()
        nll.backward()
        if lam:  # parameters with no gradient path still get the L2 gradient and are stepped
            for p in self.node:
                if p.requires_grad and p.grad is None:
                    p.grad = torch.zeros_like(p)
        else:  # no L2 term: only the parameters autograd reached are stepped (torch Adam skips grad None)
            for p in self.params:
                if id(p) not in self._touched:
                    p.grad = None
        if lam:
            l2_rep = train.l2_sqsum(self.dense) if self.dense else nll.new_zeros(())
            l2_own = train.l2_sqsum(self.node) if self.node else nll.new_zeros(())
        else:
            l2_rep = l2_own = nll.new_zeros(())
        parts = torch.stack([nll.detach().reshape(()), (lam * l2_own).reshape(())])
        if _exchanging(part.world):
            if self.flat.numel():
                dist.all_reduce(self.flat, group=self.group)  # sum of the ranks' partial gradients
            dist.all_reduce(parts, group=self.group)
        fold = bool(lam) and isinstance(self.opt, train.Adam)
        if lam and not fold:
            ps = [p for p in self.params if p.grad is not None]
            torch._foreach_add_([p.grad for p in ps], [p.detach() for p in ps], alpha=2.0 * lam)
        if fold:
            self.opt._l2_extra = 2.0 * lam
        try:
            self.opt.step()
        finally:
            if fold:
                self.opt._l2_extra = 0.0
        return parts.sum() + lam * l2_rep

    @torch.no_grad()
    def gather(self):
        """All ranks' per-node parameters whole again (checkpointing): see gather_node_params."""
        gather_node_params(self.model, self.part, self.group)


@torch.no_grad()
def gather_node_params(model, part: NodeRangePartition, group=None):
    """Make every rank's per-node parameters (C_*_vec, constant) whole again by all-gathering the owned
    rows (for checkpointing / switching back to single-GPU inference)."""
    for name, p in model.named_parameters():
        if _is_node_param(name, p, part.n) and _exchanging(part.world):
            flat = p.data.reshape(part.n, -1)
            full = all_gather_rows(flat[part.r0:part.r1].contiguous(), part, group)
            flat.copy_(full)



# ------------------------------------------------------------------------------------------------
# Halo-recompute partition: communication-free multi-GPU forward for graphs that fit one GPU's HBM
# ------------------------------------------------------------------------------------------------
# The north star asks for the RCCL halo exchange "only when the n-gram graph outgrows one GPU's 288 GB HBM".
# Below that size every rank can hold the whole graph and input, so instead of exchanging layer outputs it
# recomputes the (L-1)-hop halo of its rows:
#   S_p            = rows owned by rank p (outputs of the last layer)
#   need[L-1]      = S_p,   need[i] = need[i+1] u N(need[i+1])     (N = CSR neighbours)
#   layer i (0-based) computes rows need[i]; layer 0 gathers from the replicated input.
# The rank relabels the nodes so that every need[i] is a prefix of its own node order (S_p first, then the
# 1-hop halo, then the 2-hop halo, ..., then the rest), which makes each layer a plain single-GPU launch over
# the first |need[i]| rows: the same kernels (pg_spmm3_gated_f32 + the W-stationary dense kernel + the head)
# with contiguous per-node parameters, no row map and no collective on the data path. Each row's entries keep
# their CSR order, so every output row is bit-identical to the single-GPU forward.
# Ownership: contiguous chunks of the graph's locality schedule (CSRGraph.row_order) -- for an n-gram graph the
# schedule groups rows sharing the middle (n-2)-gram, whose neighbourhoods overlap, so the halo of a chunk is
# ~(1-(1-1/P)^3) N rows at L=2 instead of the ~N of a node-id range (whose neighbours span every id).
@dataclass
class HaloPartition:
    rank: int
    world: int
    n: int
    perm: torch.Tensor          # int64 [n]: local id -> global id (owned rows first)
    layer_rows: List[int]       # rows computed by layer i (prefix lengths, non-increasing); last = owned
    graphs: List[CSRGraph]      # layer i: CSR of local rows [0, layer_rows[i]) with local column ids
    cache: dict = field(default_factory=dict)

    @property
    def owned(self) -> int:
        return self.layer_rows[-1]

    @property
    def global_rows(self) -> torch.Tensor:
        """Global ids of the rows this rank outputs (in its output order)."""
        return self.perm[:self.owned]


def halo_owner(g: CSRGraph, world: int) -> torch.Tensor:
    """Node -> rank: balanced contiguous chunks of the locality schedule (node ids when there is none)."""
    n = g.n_rows
    dev = g.rowptr.device
    pos = torch.arange(n, dtype=torch.int64, device=dev)
    owner = torch.empty(n, dtype=torch.int64, device=dev)
    if g.row_order is not None:
        owner[g.row_order.to(torch.int64)] = pos * world // max(n, 1)
    else:
        owner.copy_(pos * world // max(n, 1))
    return owner


def halo_partition(g: CSRGraph, rank: int, world: int, layers: int,
                   owner: Optional[torch.Tensor] = None) -> HaloPartition:
    """This rank's halo-recompute layout for an L-layer forward (see the section comment)."""
    if not g.shared:
        raise NotImplementedError("halo partition needs the shared-pattern CSR")
    if layers < 1:
        raise ValueError("layers must be >= 1")
    n = g.n_rows
    dev = g.rowptr.device
    if owner is None:
        owner = halo_owner(g, world)
    # The index work (halo sets, relabelling, the permuted CSR) runs on the host and the result moves to the
    # device once: it is setup, and the host path is the one the CPU tests exercise. (A device version of the same
    # steps returned wrong records at 5-gram in round 1: ROCm torch's index gather was seen to drop the tail of
    # results >= 1 GiB, see graph.take, tools/gather_probe.py and profiles/r03_gather_probe.txt.)
    owner = owner.to(device="cpu", dtype=torch.int64)
    if owner.numel() != n or (n and (int(owner.min()) < 0 or int(owner.max()) >= world)):
        raise ValueError("owner must assign every node a rank in [0, world)")
    host = torch.device("cpu")
    rp = g.rowptr.to(host)
    edges3 = g.edges3.to(host)
    counts = rp[1:] - rp[:-1]
    row_of = torch.repeat_interleave(torch.arange(n), counts)
    col = edges3[:, 0].to(torch.int64)
    # depth: 0 = owned, k = needed first by layer L-1-k, L = never computed (input gather source only)
    depth = torch.full((n,), layers, dtype=torch.int64)
    need = owner == rank
    depth[need] = 0
    for k in range(1, layers):
        nb = torch.zeros(n, dtype=torch.bool)
        nb[col[need[row_of]]] = True
        new = nb & ~need
        depth[new] = k
        need = need | nb
    perm = torch.sort(depth, stable=True).indices  # by depth, node id order inside a depth
    inv = torch.empty(n, dtype=torch.int64)
    inv[perm] = torch.arange(n, dtype=torch.int64)
    dcount = torch.bincount(depth, minlength=layers + 1)
    cum = torch.cumsum(dcount, 0).tolist()
    layer_rows = [int(cum[layers - 1 - i]) for i in range(layers)]  # layer i computes depths <= L-1-i
    # CSR of the largest prefix (layer 0) in local ids; later layers are zero-copy prefixes of it
    R0 = layer_rows[0]
    old = perm[:R0]
    cnt = counts[old]
    lrp = torch.zeros(R0 + 1, dtype=torch.int64)
    lrp[1:] = torch.cumsum(cnt, 0)
    tot = int(lrp[-1])
    src = (torch.arange(tot, dtype=torch.int64) - torch.repeat_interleave(lrp[:-1], cnt)
           + torch.repeat_interleave(rp[old], cnt))
    e = edges3[src]
    e[:, 0] = inv[e[:, 0].to(torch.int64)].to(torch.int32)
    if tot and (int(e[:, 0].min()) < 0 or int(e[:, 0].max()) >= n):
        raise RuntimeError("halo_partition: relabelled column ids out of range")
    gorder = None
    if g.row_order is not None:  # the global schedule's relative order, restricted to each prefix
        gorder = inv[g.row_order.to(host, torch.int64)]
    lrp_d, e_d = lrp.to(dev), e.to(dev)
    graphs = []
    for i, R in enumerate(layer_rows):
        order = None
        if gorder is not None:
            order = gorder[gorder < R].to(torch.int32).to(dev)
        e1 = int(lrp[R])
        graphs.append(CSRGraph(n_rows=R, shared=True, rowptr=lrp_d[:R + 1], edges3=e_d[:e1], symmetric=False,
                               nnz=e1, row_order=order, n_cols=n if i == 0 else layer_rows[i - 1]))
    return HaloPartition(rank, world, n, perm.to(dev), layer_rows, graphs)


@torch.no_grad()
def halo_inputs(model, hp: HaloPartition, x_full: torch.Tensor):
    """The rank's resident inputs in its own node order: the input features (all n rows: layer 0 gathers from
    anywhere) and, per layer, the per-node parameters (gates, constant) of the rows it computes. Built once per
    parameter set, like the parameter shards of the exchange path; rebuild after the parameters change."""
    x_p = take(x_full, hp.perm.to(x_full.device))
    layers = []
    for conv, R in zip(model.convs, hp.layer_rows):
        prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in conv._dense_params())))
        if conv.use_vector_coeffs:
            rows = hp.perm[:R].to(conv.constant.device)
            for k in ("C_in", "C_out", "C_directed", "C_undirected", "C_all"):
                prm[k] = prm[k].index_select(0, rows).contiguous()
            const = conv.constant.detach().index_select(0, rows).contiguous()
        else:
            const = None
        layers.append((prm, const))
    return x_p, layers


@torch.no_grad()
def halo_forward(model, hp: HaloPartition, inputs) -> tuple:
    """ProtGramDirectGCN.forward (eval) for this rank's rows, without communication. Returns (log_probs, emb)
    for the rows hp.global_rows, in that order."""
    x_p, layers = inputs
    if len(layers) != len(model.convs) or len(hp.graphs) != len(model.convs):
        raise ValueError("halo partition / inputs were built for a different number of layers")
    h = model._apply_pe(x_p)
    if model.compute_dtype == torch.bfloat16:
        h = h.to(torch.bfloat16)
    for conv, res, g, (prm, const) in zip(model.convs, model.res_projs, hp.graphs, layers):
        gate_mode = 0 if conv.use_vector_coeffs else 1
        W_res, b_res = ((res.weight.detach(), res.bias.detach()) if isinstance(res, nn.Linear) else (None, None))
        R = g.n_rows
        Z = ops.spmm3_gated(g, h, prm, gate_mode)
        if Z is not None:
            h = ops.layer_dense(Z, prm, gate_mode, constant=const, res_x=h[:R], W_res=W_res, b_res=b_res, act=True,
                                pregated=True)
        else:  # bf16 mode: gates applied in the dense kernel
            Z = ops.spmm3(g, h)
            h = ops.layer_dense(Z, prm, gate_mode, constant=const, res_x=h[:R], W_res=W_res, b_res=b_res, act=True)
    return model.head(h)


# ---------------------------------------------------------------------------------------------------------------
# Middle partition with a ghost-row exchange (complete n-gram graphs: every K^n n-gram a node, the middle plan
# attached). Rank p owns the nodes a.M.b of a contiguous range of middle (n-2)-grams M in [m0, m1): exactly the
# work units of the middle-tile kernel, so each rank runs pg_spmm3_ngram_mid_rows_f32 over its middles -- the same
# kernel and the same per-row sums as one GPU -- and its rows are bit-identical to the single-GPU forward's. A row
# a.M.b reads only M.b.c (out), c.a.M (in) and itself, so the rows a rank's middles read are a fixed set: its own
# rows plus the ghost rows other ranks own. Layer 1 reads the replicated input. After each other layer, every rank
# sends each other rank exactly the rows of its output that rank reads (one RCCL all_to_all_single, the
# personalised all-gather of the halo rows; ~(1-(1-1/P)^3) N rows received in total at P ranks instead of the
# (P-1)/P N of the node-range all-gather) and scatters what it receives into a global-layout buffer.
# ---------------------------------------------------------------------------------------------------------------
@dataclass
class MiddlePartition:
    rank: int
    world: int
    n: int                      # N = K^ngram
    K: int
    ngram: int
    m0: int                     # owned middles [m0, m1)
    m1: int
    own: torch.Tensor           # int64 [n_own]: global ids of the owned rows, middle-major ((M - m0) K^2 + a K + b)
    own_csr: CSRGraph           # the global CSR's rows `own` (global column ids): the CSR-kernel path
    send_pos: torch.Tensor      # int64: positions (owned-row order) of the rows sent, by (chunk, destination)
    send_counts: List[int]      # rows sent to each rank (all chunks)
    recv_ids: torch.Tensor      # int64: global ids of the rows received, by (chunk, source), ascending ids within
    recv_counts: List[int]      # rows received from each rank (all chunks)
    graph: CSRGraph             # the global graph (its middle plan)
    chunks: int = 1             # the owned middles in `chunks` sub-ranges: a layer's exchange per sub-range
    chunk_bounds: List[tuple] = field(default_factory=list)   # owned middle sub-ranges
    chunk_send: List[List[int]] = field(default_factory=list)  # [chunk][destination] rows sent
    chunk_recv: List[List[int]] = field(default_factory=list)  # [chunk][source] rows received
    cache: dict = field(default_factory=dict)
    loopback: bool = False      # world 1: every owned row is "sent" to this rank itself (exchange test mode)

    @property
    def n_own(self) -> int:
        return int(self.own.numel())

    @property
    def global_rows(self) -> torch.Tensor:
        """Global ids of the rows this rank outputs (in its output order)."""
        return self.own


def ngram_shape(g: CSRGraph):
    """(K, n) of a graph over all K^n n-grams (the tile plan's, else K = 20 when n_rows is a power of 20), or None."""
    if g.ngram is not None:
        return g.ngram.K, g.ngram.n
    N, n, v = g.n_rows, 0, 1
    while v < N:
        v *= 20
        n += 1
    return (20, n) if v == N and n >= 1 else None


def middle_bounds(n_middles: int, world: int) -> List[tuple]:
    """Balanced contiguous middle ranges, one per rank."""
    return [(r * n_middles // world, (r + 1) * n_middles // world) for r in range(world)]


def _middle_rows(K: int, n: int, m0: int, m1: int, dev) -> torch.Tensor:
    """Global ids a.M.b for M in [m0, m1), middle-major ((M, a, b) order)."""
    Kn1 = K ** (n - 1)
    M = torch.arange(m0, m1, dtype=torch.int64, device=dev)
    a = torch.arange(K, dtype=torch.int64, device=dev)
    return (a.view(1, K, 1) * Kn1 + M.view(-1, 1, 1) * K + a.view(1, 1, K)).reshape(-1)


def _middle_reads(K: int, n: int, m0: int, m1: int, dev) -> torch.Tensor:
    """Sorted global ids of every row the middles [m0, m1) read: M.b.c, c.a.M and a.M.b."""
    Kn1, Kn2 = K ** (n - 1), K ** (n - 2)
    M = torch.arange(m0, m1, dtype=torch.int64, device=dev)
    t = torch.arange(K * K, dtype=torch.int64, device=dev)
    c = torch.arange(K, dtype=torch.int64, device=dev)
    out_src = (M.view(-1, 1) * (K * K) + t.view(1, -1)).reshape(-1)
    in_src = (c.view(K, 1, 1) * Kn1 + c.view(1, K, 1) * Kn2 + M.view(1, 1, -1)).reshape(-1)
    return torch.unique(torch.cat([out_src, in_src, _middle_rows(K, n, m0, m1, dev)]))


def middle_partition(g: CSRGraph, rank: int, world: int, chunks: int = 1, loopback: bool = False) -> MiddlePartition:
    """This rank's middle partition of a complete n-gram graph (see the section comment). Setup work, once per
    graph: the exchange lists of every rank pair are built from the closed-form read sets (and checked against
    the CSR's own columns), so both ends of each pair agree without communication. With chunks > 1 every rank's
    middles are cut into `chunks` sub-ranges and the lists are grouped by the sender's sub-range, so each sub-range's
    rows can be exchanged as soon as they are computed (MiddleRunner overlaps that exchange with the next one).
    loopback (world 1 only): the lists send every owned row of each sub-range to this rank itself, so a one-GPU run
    executes the exchange path (gather, asynchronous all_to_all_single, scatter) with an identity exchange."""
    if loopback and world != 1:
        raise ValueError("loopback is a world-size-1 test mode")
    shape = ngram_shape(g)
    if shape is None or not g.shared:
        raise NotImplementedError("middle partition needs a shared-pattern graph over all K^n n-grams")
    K, n = shape
    if n < 3:
        raise NotImplementedError("middle partition needs n >= 3 (one middle per (n-2)-gram)")
    Kn1, Kn2 = K ** (n - 1), K ** (n - 2)
    if world > Kn2:
        raise ValueError(f"{world} ranks but only {Kn2} middles")
    dev = g.rowptr.device
    bounds = middle_bounds(Kn2, world)
    chunks = max(1, min(chunks, min(b - a for a, b in bounds)))
    starts = torch.tensor([b[0] for b in bounds], dtype=torch.int64, device=dev)
    m0, m1 = bounds[rank]

    chunk_of = torch.empty(Kn2, dtype=torch.int64)  # middle -> sub-range of its owner's range
    for a, b in bounds:
        for cc in range(chunks):
            chunk_of[a + cc * (b - a) // chunks:a + (cc + 1) * (b - a) // chunks] = cc
    chunk_of = chunk_of.to(dev)

    def owner_pos_chunk(x):
        Mx = (x % Kn1) // K
        q = torch.searchsorted(starts, Mx, right=True) - 1
        pos = (Mx - starts[q]) * (K * K) + (x // Kn1) * K + x % K
        return q, pos, chunk_of[Mx]

    own = _middle_rows(K, n, m0, m1, dev)
    sends = [[None] * world for _ in range(chunks)]
    chunk_send = [[0] * world for _ in range(chunks)]
    chunk_recv = [[0] * world for _ in range(chunks)]
    recv_ids = None
    for p in range(world):
        reads = _middle_reads(K, n, *bounds[p], dev)
        q, pos, c = owner_pos_chunk(reads)
        if p == rank:
            ghost = q != rank
            gq, gc, gid = q[ghost], c[ghost], reads[ghost]
            order = torch.sort(gc * world + gq, stable=True).indices  # by (chunk, source), ascending ids within
            recv_ids = gid[order]
            cnt = torch.bincount(gc * world + gq, minlength=chunks * world).view(chunks, world).tolist()
            chunk_recv = cnt
        else:
            mine = q == rank
            pm, cm = pos[mine], c[mine]
            for cc in range(chunks):
                sel = pm[cm == cc]
                sends[cc][p] = sel
                chunk_send[cc][p] = int(sel.numel())
    empty = torch.zeros(0, dtype=torch.int64, device=dev)
    send_pos = torch.cat([sends[cc][p] if sends[cc][p] is not None else empty
                          for cc in range(chunks) for p in range(world)]) if world > 1 else empty
    send_counts = [sum(chunk_send[cc][p] for cc in range(chunks)) for p in range(world)]
    recv_counts = [sum(chunk_recv[cc][p] for cc in range(chunks)) for p in range(world)]
    if recv_ids is None:
        recv_ids = empty
    L = m1 - m0
    chunk_bounds = [(m0 + cc * L // chunks, m0 + (cc + 1) * L // chunks) for cc in range(chunks)]
    if loopback:  # each sub-range's own rows to itself, in owned-row order (positions = ids' order in `own`)
        K2 = K * K
        pos_c = [torch.arange((a - m0) * K2, (b - m0) * K2, dtype=torch.int64, device=dev) for a, b in chunk_bounds]
        send_pos = torch.cat(pos_c)
        recv_ids = _middle_rows(K, n, m0, m1, dev)[send_pos]
        chunk_send = [[int(pc.numel())] for pc in pos_c]
        chunk_recv = [[int(pc.numel())] for pc in pos_c]
        send_counts = recv_counts = [int(send_pos.numel())]
    # the owned rows' CSR (global column ids), and the check that it reads nothing outside the closed-form set
    rp = g.rowptr
    cnt = rp[own + 1] - rp[own]
    lrp = torch.zeros(own.numel() + 1, dtype=torch.int64, device=dev)
    lrp[1:] = torch.cumsum(cnt, 0)
    tot = int(lrp[-1])
    src = (torch.arange(tot, dtype=torch.int64, device=dev) - torch.repeat_interleave(lrp[:-1], cnt)
           + torch.repeat_interleave(rp[own], cnt))
    e = take(g.edges3, src)
    reads = _middle_reads(K, n, m0, m1, dev)
    if tot and not bool(torch.isin(e[:, 0].to(torch.int64), reads).all()):
        raise ValueError("the graph has entries outside the n-gram out/in/self slots: not a middle-partitionable graph")
    own_csr = CSRGraph(n_rows=own.numel(), shared=True, rowptr=lrp, edges3=e, symmetric=False, nnz=tot,
                       row_order=None, n_cols=g.n_rows)
    return MiddlePartition(rank, world, g.n_rows, K, n, m0, m1, own, own_csr, send_pos, send_counts, recv_ids,
                           recv_counts, g, chunks, chunk_bounds, chunk_send, chunk_recv, loopback=loopback)


@torch.no_grad()
def middle_inputs(model, mp: MiddlePartition):
    """Per layer, the per-node parameters (gates, constant) at the owned rows, in the owned-row order. Built once per
    parameter set (rebuild after the parameters change), like halo_inputs."""
    layers = []
    for conv in model.convs:
        prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in conv._dense_params())))
        if conv.use_vector_coeffs:
            rows = mp.own.to(conv.constant.device)
            for k in ("C_in", "C_out", "C_directed", "C_undirected", "C_all"):
                prm[k] = prm[k].index_select(0, rows).contiguous()
            const = conv.constant.detach().index_select(0, rows).contiguous()
        else:
            const = None
        layers.append((prm, const))
    return layers


@torch.no_grad()
def _full_inputs(conv):
    """A layer's dense parameters and constant over every row (MiddleRunner's replicated layers)."""
    prm = dict(zip(ops._DENSE_KEYS, (p.detach() for p in conv._dense_params())))
    return prm, (conv.constant.detach() if conv.use_vector_coeffs else None)


def _owned_spmm3(mp: MiddlePartition, X: torch.Tensor) -> torch.Tensor:
    """Aggregates of the owned rows (owned-row order) from X in the global row layout: the middle-tile kernel over
    the owned middles where it takes the call (fp32, F % 16 == 0), else the CSR kernels over the owned rows' CSR."""
    if mp.graph.ngram is not None and ops._mid_ok(mp.graph, X, ops.default_flags()):
        return ops.spmm3_middles(mp.graph, X, mp.m0, mp.m1)
    return ops.spmm3(mp.own_csr, X)


def _exchange_rows(mp: MiddlePartition, h_own: torch.Tensor, group=None) -> torch.Tensor:
    """The next layer's input in the global row layout: this rank's rows plus the ghost rows it reads, received
    from their owners by one all_to_all_single (the same tensor collective on RCCL and on gloo). Rows nobody
    reads stay unwritten. (MiddleRunner does the same per chunk, overlapped.)"""
    F_ = h_own.size(1)
    X = h_own.new_empty(mp.n, F_)
    ops.rows_scatter(h_own, mp.own, X, check_idx=False)
    if mp.world > 1 or mp.loopback:
        send = ops.rows_gather(h_own, mp.send_pos, check_idx=False)
        stage = h_own.is_cuda and dist.get_backend(group) == "gloo"  # gloo (CPU rehearsal backend): host buffers
        if stage:
            send = send.cpu()
        recv = send.new_empty(int(mp.recv_ids.numel()), F_)
        # send_pos / recv_ids are grouped by (chunk, rank): one all_to_all per chunk, whose slices are rank-grouped
        # (a single call over all chunks would need the buffers grouped by rank alone)
        s0 = r0 = 0
        for c in range(mp.chunks):
            ns, nr = sum(mp.chunk_send[c]), sum(mp.chunk_recv[c])
            dist.all_to_all_single(recv[r0:r0 + nr], send[s0:s0 + ns], mp.chunk_recv[c], mp.chunk_send[c],
                                   group=group)
            s0, r0 = s0 + ns, r0 + nr
        ops.rows_scatter(recv.to(X.device) if stage else recv, mp.recv_ids, X, check_idx=False)
    return X


@torch.no_grad()
def middle_forward(model, mp: MiddlePartition, x_full: torch.Tensor, inputs=None, group=None) -> tuple:
    """ProtGramDirectGCN.forward (eval) for this rank's rows; returns (log_probs, emb) for the rows mp.global_rows,
    in that order. `inputs` = middle_inputs(model, mp) (built here when None)."""
    layers = inputs if inputs is not None else middle_inputs(model, mp)
    if len(layers) != len(model.convs):
        raise ValueError("middle inputs were built for a different number of layers")
    h = model._apply_pe(x_full)
    if model.compute_dtype == torch.bfloat16:
        h = h.to(torch.bfloat16)
    X, res_x = h, ops.rows_gather(h, mp.own, check_idx=False)
    L = len(model.convs)
    for i, (conv, res, (prm, const)) in enumerate(zip(model.convs, model.res_projs, layers)):
        gate_mode = 0 if conv.use_vector_coeffs else 1
        W_res, b_res = ((res.weight.detach(), res.bias.detach()) if isinstance(res, nn.Linear) else (None, None))
        Z = _owned_spmm3(mp, X)
        h_own = ops.layer_dense(Z, prm, gate_mode, constant=const, res_x=res_x, W_res=W_res, b_res=b_res, act=True)
        if i + 1 < L:
            X = _exchange_rows(mp, h_own, group)
        res_x = h_own
    return model.head(h_own)


class MiddleRunner:
    """The bench's multi-GPU forward on the middle partition, for a fixed input.

    Every layer but the last runs in the partition's `chunks` middle sub-ranges: sub-range c's rows are propagated
    (middle-tile kernel over its middles), transformed (dense kernel on its rows), and the rows other ranks read
    are gathered and handed to an asynchronous all_to_all_single, which runs on the collective's own stream while
    sub-range c + 1 computes. The next layer waits for all of them, scatters its own and the received rows into its
    global-layout input, and so on; the last layer runs whole and ends in the head. Each compute segment is
    captured once as a HIP graph (torch.cuda.CUDAGraph) and replayed, so a rank issues L-1 x chunks + 1 graph
    launches and the collectives per forward; the collectives stay outside the graphs. `graphs=False` (or a CPU
    input) runs the segments eagerly; gloo (the CPU rehearsal backend) exchanges synchronously through host
    buffers. Rebuild the runner after the parameters or the input change. The rows it returns are bit-identical
    to middle_forward's (and to the single-GPU forward's)."""

    def __init__(self, model, mp: MiddlePartition, x_full: torch.Tensor, inputs=None, group=None,
                 graphs: bool = True, replicate: bool = False):
        self.model, self.mp, self.x, self.group = model, mp, x_full, group
        self.layers = inputs if inputs is not None else middle_inputs(model, mp)
        self.L = len(model.convs)
        self.replicate = replicate
        dev = x_full.device
        self.dt = torch.bfloat16 if model.compute_dtype == torch.bfloat16 else x_full.dtype
        self.bufs = [torch.empty(mp.n, conv.in_channels, device=dev, dtype=self.dt) for conv in model.convs[1:]]
        nrecv = 0 if replicate else int(mp.recv_ids.numel())
        self.recv = [torch.empty(nrecv, conv.in_channels, device=dev, dtype=self.dt) for conv in model.convs[1:]]
        # replicate: every layer but the last over all rows, on every rank (the full parameters), into self.bufs
        self.full = [_full_inputs(conv) for conv in model.convs[:-1]] if replicate else None
        self.hout = [torch.empty(mp.n_own, conv.out_channels, device=dev, dtype=self.dt) for conv in model.convs[:-1]]
        K2 = mp.K * mp.K
        self.row_bounds = [((a - mp.m0) * K2, (b - mp.m0) * K2) for a, b in mp.chunk_bounds]
        off, self.send_slices = 0, []
        for c in range(mp.chunks):
            k = sum(mp.chunk_send[c])
            self.send_slices.append((off, off + k))
            off += k
        off, self.recv_slices = 0, []
        for c in range(mp.chunks):
            k = sum(mp.chunk_recv[c])
            self.recv_slices.append((off, off + k))
            off += k
        # the CSR path's row blocks (bf16 / no middle plan), cut before any capture (slicing reads rowptr on the host)
        self.csr_chunks = [_rows_slice(mp.own_csr, r0, r1, None) for r0, r1 in self.row_bounds]
        # mapped: the dense kernel reads the residual rows and writes the output rows of this rank's middles in the
        # global row layout itself (pg_directgcn_dense_ngram_rows_f32): no residual gather, no scatter of the own
        # rows; only the received rows are scattered. fp32 on the GPU, every layer 128 -> 128 with an identity
        # residual (the pipelined split-bf16 kernel's shape); otherwise rows_gather / rows_scatter around the launch
        self.mapped = (x_full.is_cuda and self.dt == torch.float32 and mp.K == 20
                       and all(cv.in_channels == 128 and cv.out_channels == 128 for cv in model.convs)
                       and not any(isinstance(r, nn.Linear) for r in model.res_projs))
        self.Kn1 = mp.K ** (mp.ngram - 1)
        self.xchg = mp.world > 1 or mp.loopback
        self.send_glob = mp.own[mp.send_pos] if self.xchg else None  # the sent rows' global ids
        backend = dist.get_backend(group) if (self.xchg and dist.is_initialized()) else None
        self.sync = (not x_full.is_cuda) or backend == "gloo"
        self.state = {}
        self.works = []
        self.graphs = None
        with torch.no_grad():
            for _ in range(2):  # eager warm-up: kernel attributes, allocator pools, lazy library state
                out = self._run_eager()
        if x_full.is_cuda:
            torch.cuda.synchronize()
        self.out = out
        if graphs and x_full.is_cuda:
            self._capture()

    # ---- segments (graph bodies)
    def _prepare(self, i: int):
        """Layer i's global-layout input and its residual rows (owned-row order; replicated layers: all rows)."""
        mp, model = self.mp, self.model
        if i == 0:
            h = model._apply_pe(self.x)
            if model.compute_dtype == torch.bfloat16:
                h = h.to(torch.bfloat16)
            self.state["X"] = h
            if self.replicate and self.L > 1:
                self.state["res"] = h
            else:  # mapped: the dense kernel reads the residual rows from h itself
                self.state["res"] = None if self.mapped else ops.rows_gather(h, mp.own, check_idx=False)
        elif self.replicate:
            X = self.bufs[i - 1]  # the replicated layer's output, every row
            self.state["X"] = X
            if i + 1 < self.L:
                self.state["res"] = X
            else:
                self.state["res"] = None if self.mapped else ops.rows_gather(X, mp.own, check_idx=False)
        else:
            X, h_prev = self.bufs[i - 1], self.hout[i - 1]
            if not self.mapped:  # mapped: layer i - 1's dense kernel wrote the own rows into X
                ops.rows_scatter(h_prev, mp.own, X, check_idx=False)
            if self.xchg and self.recv[i - 1].size(0):
                ops.rows_scatter(self.recv[i - 1], mp.recv_ids, X, check_idx=False)
            self.state["X"], self.state["res"] = X, None if self.mapped else h_prev

    def _compute_full(self, i: int):
        """A replicated layer: the single-GPU layer over every row, into the next layer's global-layout input."""
        conv, res = self.model.convs[i], self.model.res_projs[i]
        prm, const = self.full[i]
        W_res, b_res = ((res.weight.detach(), res.bias.detach()) if isinstance(res, nn.Linear) else (None, None))
        X = self.state["X"]
        return ops.layer_dense(ops.spmm3(self.mp.graph, X), prm, 0 if conv.use_vector_coeffs else 1, constant=const,
                               res_x=self.state["res"], W_res=W_res, b_res=b_res, act=True, out=self.bufs[i])

    def _compute(self, i: int, c: Optional[int]):
        """Layer i over chunk c's middles (c None: all owned middles); returns the layer output rows."""
        mp, model = self.mp, self.model
        conv, res = model.convs[i], model.res_projs[i]
        prm, const = self.layers[i]
        if c is None:
            (a, b), (r0, r1) = (mp.m0, mp.m1), (0, mp.n_own)
        else:
            (a, b), (r0, r1) = mp.chunk_bounds[c], self.row_bounds[c]
        X = self.state["X"]
        if mp.graph.ngram is not None and ops._mid_ok(mp.graph, X, ops.default_flags()):
            Z = ops.spmm3_middles(mp.graph, X, a, b)
        else:
            Z = ops.spmm3(mp.own_csr if c is None else self.csr_chunks[c], X)
        if conv.use_vector_coeffs:
            prm = dict(prm)
            for k in ("C_in", "C_out", "C_directed", "C_undirected", "C_all"):
                prm[k] = prm[k][r0:r1]
            const = const[r0:r1] if const is not None else None
        gate_mode = 0 if conv.use_vector_coeffs else 1
        if self.mapped:  # residual rows from X, output rows into the next layer's input (global layout)
            last = i + 1 == self.L
            y = ops.layer_dense_ngram_rows(Z, prm, gate_mode, self.Kn1, a, constant=const, res_x=X, map_res=True,
                                           out=None if last else self.bufs[i], map_out=not last, act=True)
            if y is None:
                raise RuntimeError("pg_directgcn_dense_ngram_rows_f32 did not take the layer's shape")
            return y
        res_x = self.state["res"][r0:r1]
        W_res, b_res = ((res.weight.detach(), res.bias.detach()) if isinstance(res, nn.Linear) else (None, None))
        out = self.hout[i][r0:r1] if i + 1 < self.L else None
        return ops.layer_dense(Z, prm, gate_mode, constant=const, res_x=res_x, W_res=W_res, b_res=b_res, act=True,
                               out=out)

    def _segment(self, i: int, c: Optional[int]):
        """One graph body: [layer input (first chunk)], chunk c of layer i, the rows it sends (or the head)."""
        if c is None or c <= 0:
            self._prepare(i)
        if c == -1:
            self._compute_full(i)
            return None
        h = self._compute(i, c)
        if i + 1 < self.L:
            if self.xchg:
                s0, s1 = self.send_slices[c]
                if self.mapped:
                    self.state[("send", i, c)] = ops.rows_gather(self.bufs[i], self.send_glob[s0:s1],
                                                                 check_idx=False)
                else:
                    self.state[("send", i, c)] = ops.rows_gather(self.hout[i], self.mp.send_pos[s0:s1],
                                                                 check_idx=False)
            return None
        return self.model.head(h)

    # ---- exchange (outside the graphs)
    def _exchange(self, i: int, c: int):
        mp = self.mp
        if not self.xchg:
            return
        send = self.state[("send", i, c)]
        r0, r1 = self.recv_slices[c]
        recv = self.recv[i][r0:r1]
        if self.sync:  # gloo / CPU: synchronous, through host buffers for device tensors
            r = recv.new_empty(recv.shape, device="cpu")
            dist.all_to_all_single(r, send.cpu(), mp.chunk_recv[c], mp.chunk_send[c], group=self.group)
            recv.copy_(r)
        else:
            self.works.append(dist.all_to_all_single(recv, send, mp.chunk_recv[c], mp.chunk_send[c],
                                                     group=self.group, async_op=True))

    def _wait(self):
        for w in self.works:
            w.wait()  # RCCL: the current stream waits for the collective's stream (no host block)
        self.works = []

    def _plan(self):
        """The segment sequence: (layer, chunk) pairs; the last layer whole (chunk None); replicated layers -1."""
        if self.replicate:
            return [(i, -1) for i in range(self.L - 1)] + [(self.L - 1, None)]
        seq = [(i, c) for i in range(self.L - 1) for c in range(self.mp.chunks)]
        return seq + [(self.L - 1, None)]

    def _run_eager(self):
        out = None
        for i, c in self._plan():
            if c is None or c == 0:
                self._wait()
            out = self._segment(i, c)
            if c is not None and c >= 0:
                self._exchange(i, c)
        self._wait()
        return out

    def _capture(self):
        """Capture every compute segment once (setup). No collective is in flight while a segment is captured:
        each exchange is drained (host sync) before the next capture begins, and the capture mode is thread-local,
        so the collective library's own threads (progress, watchdog) cannot invalidate it. If the capture fails
        anyway, the runner stays eager (a warning on stderr), with the same results."""
        self.graphs = []
        pool = torch.cuda.graph_pool_handle()
        try:
            for i, c in self._plan():
                gph = torch.cuda.CUDAGraph()
                with torch.no_grad(), torch.cuda.graph(gph, pool=pool, capture_error_mode="thread_local"):
                    out = self._segment(i, c)
                gph.replay()  # this segment's outputs for the next capture's inputs
                if c is not None and c >= 0:
                    self._exchange(i, c)
                self._wait()
                torch.cuda.synchronize()
                self.graphs.append(gph)
        except RuntimeError as e:  # pragma: no cover - depends on the collective library
            import sys
            print(f"[MiddleRunner] HIP graph capture failed ({e}); running the segments eagerly", file=sys.stderr)
            self.graphs = None
            self.works = []
            torch.cuda.synchronize()
            with torch.no_grad():
                out = self._run_eager()
            torch.cuda.synchronize()
        self.out = out

    @torch.no_grad()
    def __call__(self):
        """(log_probs, emb) for mp.global_rows. With graphs, the returned tensors are the graph's static outputs:
        overwritten by the next call."""
        if self.graphs is None:
            return self._run_eager()
        for gph, (i, c) in zip(self.graphs, self._plan()):
            if c is None or c == 0:
                self._wait()
            gph.replay()
            if c is not None and c >= 0:
                self._exchange(i, c)
        self._wait()
        return self.out


# ---------------------------------------------------------------------------------------------------------------
# Middle-partition training (BASELINE config 5: the trainer's full-batch step on P ranks without any N x F collective)
# ---------------------------------------------------------------------------------------------------------------
# Per layer the rank propagates its middles with the middle-tile kernel (spmm3_middles: Z of its rows, middle-major)
# from the layer input in the global row layout, in which only its own rows and the ghost rows its middles read are
# valid (the forward exchange: MiddlePartition's lists, one all_to_all per layer boundary and chunk). Backward:
#   * the propagation's input gradient is A[own, :]^T dZ_own -- nonzero exactly on own + ghost rows -- from the
#     transposed CSR kernel over the rank's COLUMN block (MiddleTranspose: rows = own + ghost, columns = owned-row
#     positions; the n-gram matrices are symmetric, so it is the owned rows' CSR transposed);
#   * the exchange's backward sends each ghost row's gradient back to its owner (the reverse all_to_all over the same
#     lists, F wide like the forward) and the owner adds what it receives to its own rows' gradients, one source
#     rank at a time (each slice holds distinct rows: deterministic sums);
#   * dense weights / biases are replicated (one flat all-reduce of their gradients per step), per-node parameters
#     (gates, constant) are owned-row leaves in middle-major order (no communication; `sync_model` writes them back).
# So a layer boundary costs 2 x (ghost rows x F) per rank over xGMI instead of the node-range trainer's N x F
# all-gather + N x F reduce-scatter. Reference: protgram_directgcn_trainer.py:76-108 (loop), config.py:63 (dims).
class TorchComm:
    """The collectives the middle trainer uses, over torch.distributed (RCCL for CUDA tensors on 'nccl'; gloo stages
    device tensors through host buffers).

    `capturable` (RCCL only): every call is a synchronous-form torch.distributed collective on the caller's current
    stream, so inside a HIP-graph capture (MiddleTrainer(graphs=True)) ProcessGroupNCCL's fork onto its RCCL stream and
    the join back (event record / stream wait) are captured with the RCCL kernels, and each replay re-runs the
    exchange on the same buffers. gloo stages through host memory (`.cpu()` synchronises): not capturable."""

    def __init__(self, group=None):
        self.group = group
        self.capturable = dist.is_initialized() and dist.get_backend(group) == "nccl"

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits):
        if inp.is_cuda and dist.get_backend(self.group) == "gloo":
            o = out.new_empty(out.shape, device="cpu")
            dist.all_to_all_single(o, inp.cpu(), list(out_splits), list(in_splits), group=self.group)
            out.copy_(o)
        else:
            dist.all_to_all_single(out, inp, list(out_splits), list(in_splits), group=self.group)

    def all_reduce(self, t: torch.Tensor):
        if t.is_cuda and dist.get_backend(self.group) == "gloo":
            h = t.cpu()
            dist.all_reduce(h, group=self.group)
            t.copy_(h)
        else:
            dist.all_reduce(t, group=self.group)

    def all_gather(self, out: torch.Tensor, t: torch.Tensor):
        """out [world * rows, ...] <- every rank's t [rows, ...], rank-major."""
        if t.is_cuda and dist.get_backend(self.group) == "gloo":
            o = out.new_empty(out.shape, device="cpu")
            dist.all_gather_into_tensor(o, t.cpu(), group=self.group)
            out.copy_(o)
        else:
            dist.all_gather_into_tensor(out, t, group=self.group)


@dataclass
class MiddleTranspose:
    """The rank's column block of the (symmetric) propagation matrices as a transposed CSR over all N rows: row j
    holds an entry (column = owned-row position of i, the weights of A[i, j]) for every owned row i that reads j.
    `rows` (int32) lists the rows with entries (own + ghost) -- the rows pg_spmm3t_f32 / _bf16 compute."""
    rowptr: torch.Tensor
    edges3: torch.Tensor
    rows: torch.Tensor
    nnz: int


def middle_transpose(mp: MiddlePartition) -> MiddleTranspose:
    hit = mp.cache.get("transpose")
    if hit is not None:
        return hit
    if not mp.graph.symmetric:
        raise NotImplementedError("middle training needs symmetric propagation matrices (n-gram graphs)")
    oc = mp.own_csr
    dev = oc.rowptr.device
    cnt = oc.rowptr[1:] - oc.rowptr[:-1]
    pos = torch.repeat_interleave(torch.arange(mp.n_own, dtype=torch.int64, device=dev), cnt)
    j = oc.edges3[:, 0].to(torch.int64)
    order = torch.sort(j * max(mp.n_own, 1) + pos).indices  # by (row j, owned position): ascending within a row
    e = take(oc.edges3, order).clone()
    e[:, 0] = take(pos, order).to(torch.int32)
    js = take(j, order)
    rowptr = torch.zeros(mp.n + 1, dtype=torch.int64, device=dev)
    rowptr[1:] = torch.cumsum(torch.bincount(js, minlength=mp.n), 0)
    rows = torch.unique(js).to(torch.int32)
    mt = MiddleTranspose(rowptr, e.contiguous(), rows, int(e.size(0)))
    mp.cache["transpose"] = mt
    return mt


class _MidPropagate(torch.autograd.Function):
    """X (global row layout; own + ghost rows valid) -> Z of the owned rows [n_own, 3F] (middle-major)."""

    @staticmethod
    def forward(ctx, X, mp: MiddlePartition):
        ctx.mp = mp
        return _owned_spmm3(mp, X)

    @staticmethod
    def backward(ctx, dZ):
        if not ctx.needs_input_grad[0]:
            return None, None
        mp = ctx.mp
        mt = middle_transpose(mp)
        return ops.spmm3t_rows(mt.rowptr, mt.edges3, mt.rows, dZ.contiguous(), mp.n), None


def reverse_exchange(mp: MiddlePartition, dX: torch.Tensor, comm) -> torch.Tensor:
    """Backward of the forward exchange: the gradients of this rank's ghost rows (dX at mp.recv_ids) go back to their
    owners; returns the [n_own, F] sum of what the other ranks sent for this rank's rows (at least fp32), each source's slice
    added in turn (distinct rows per slice: deterministic)."""
    F_ = dX.size(1)
    send = dX.index_select(0, mp.recv_ids)  # ordered (chunk, source) as received forward
    recv = send.new_empty(int(mp.send_pos.numel()), F_)
    s0 = r0 = 0
    for c in range(mp.chunks):
        ns, nr = sum(mp.chunk_recv[c]), sum(mp.chunk_send[c])
        comm.all_to_all(recv[r0:r0 + nr], send[s0:s0 + ns], mp.chunk_send[c], mp.chunk_recv[c])
        s0, r0 = s0 + ns, r0 + nr
    out = torch.zeros(mp.n_own, F_, dtype=torch.promote_types(dX.dtype, torch.float32), device=dX.device)
    recv = recv.to(out.dtype)  # one widening pass (bf16 mode), then the per-source adds
    off = 0
    for c in range(mp.chunks):
        for q in range(len(mp.chunk_send[c])):
            k = mp.chunk_send[c][q]
            if k:
                out.index_add_(0, mp.send_pos[off:off + k], recv[off:off + k])
            off += k
    return out


def forward_exchange(mp: MiddlePartition, h_own: torch.Tensor, comm) -> torch.Tensor:
    """The next layer's input in the global row layout: own rows + the ghost rows received from their owners (other
    rows unwritten); per chunk one all_to_all (the lists are grouped by (chunk, rank))."""
    F_ = h_own.size(1)
    X = h_own.new_empty(mp.n, F_)
    # on the device the row moves are pg_rows_scatter / pg_rows_gather (16-B pieces; the lists are the partition's
    # closed form, checked when it was built); host tensors (the gloo rehearsals) take torch's index ops
    dev = h_own.is_cuda
    h_own = h_own.contiguous()
    if dev:
        ops.rows_scatter(h_own, mp.own, X, check_idx=False)
    else:
        X.index_copy_(0, mp.own, h_own)
    if mp.world > 1 or mp.loopback:
        send = ops.rows_gather(h_own, mp.send_pos, check_idx=False) if dev else h_own.index_select(0, mp.send_pos)
        recv = send.new_empty(int(mp.recv_ids.numel()), F_)
        s0 = r0 = 0
        for c in range(mp.chunks):
            ns, nr = sum(mp.chunk_send[c]), sum(mp.chunk_recv[c])
            comm.all_to_all(recv[r0:r0 + nr], send[s0:s0 + ns], mp.chunk_recv[c], mp.chunk_send[c])
            s0, r0 = s0 + ns, r0 + nr
        if dev:
            ops.rows_scatter(recv, mp.recv_ids, X, check_idx=False)
        else:
            X.index_copy_(0, mp.recv_ids, recv)
    return X


class _MidExchange(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h_own, mp: MiddlePartition, comm):
        ctx.mp, ctx.comm = mp, comm
        return forward_exchange(mp, h_own, comm)

    @staticmethod
    def backward(ctx, dX):
        mp = ctx.mp
        if mp.loopback:  # the received copies overwrote the own rows: they carry the whole gradient
            d = reverse_exchange(mp, dX, ctx.comm)
        else:
            d = dX.index_select(0, mp.own).float()
            if mp.world > 1:
                d = d + reverse_exchange(mp, dX, ctx.comm)
        return d.to(dX.dtype), None, None


@dataclass
class MiddleScatter:
    """The middle partition's scatter-form backward (pg_spmm3t_ngram_scatter_*): the rank's scatter plan and, over the
    kernel's part rows T (D | P | S, include/pg_directgcn.h), the per-row lists pg_rows_gather_sum sums: the ghost rows
    sent back (recv_ids order) and the owned rows (their own parts, unless loopback, then the rows received for them,
    as -1 - position in the receive buffer)."""
    splan: torch.Tensor
    send_ptr: torch.Tensor
    send_idx: torch.Tensor
    own_ptr: torch.Tensor
    own_idx: torch.Tensor


def _csr_lists(counts: torch.Tensor):
    ptr = torch.zeros(counts.numel() + 1, dtype=torch.int64, device=counts.device)
    ptr[1:] = torch.cumsum(counts, 0)
    return ptr


def middle_scatter(mp: MiddlePartition) -> Optional[MiddleScatter]:
    """Setup of the scatter-form backward, once per partition (cached): the scatter plan of the rank's middles and
    the row lists (scatter_lists); None without a middle plan on the device (K = 20)."""
    if "scatter" in mp.cache:
        return mp.cache["scatter"]
    ng = mp.graph.ngram
    if ng is None or getattr(ng, "mplan", None) is None or mp.K != 20 or not mp.own.is_cuda:
        mp.cache["scatter"] = None
        return None
    sc = MiddleScatter(ops.ngram_scatter_plan(mp.graph, mp.m0, mp.m1), *scatter_lists(mp))
    mp.cache["scatter"] = sc
    return sc


def scatter_lists(mp: MiddlePartition):
    """(send_ptr, send_idx, own_ptr, own_idx) of the scatter-form backward (MiddleScatter), on mp's device. Part row t
    of T (D | P | S, include/pg_directgcn.h) targets one global row; a row's list holds its part rows in T-row order;
    the ghost rows' lists come in recv_ids order (what goes back to each owner), the owned rows' lists hold their own
    parts (none in loopback mode: the received copies replaced the own rows), then -1 - e for each receive-buffer
    entry e of that row, in order."""
    hit = mp.cache.get("scatter_lists")
    if hit is not None:
        return hit
    dev = mp.own.device
    K, n = mp.K, mp.ngram
    Kn1, Kn2 = K ** (n - 1), K ** (n - 2)
    M = torch.arange(mp.m0, mp.m1, dtype=torch.int64, device=dev).view(-1, 1, 1)
    x = torch.arange(K, dtype=torch.int64, device=dev).view(1, -1, 1)
    y = torch.arange(K, dtype=torch.int64, device=dev).view(1, 1, -1)
    tgt = torch.cat([(x * Kn1 + M * K + y).reshape(-1),         # D: (a, b) -> a.M.b
                     (M * (K * K) + x * K + y).reshape(-1),     # P: (b, c) -> M.b.c
                     (x * Kn1 + y * Kn2 + M).reshape(-1)])      # S: (c, a) -> c.a.M
    order = torch.sort(tgt, stable=True).indices                # T rows by global row, ascending T row within
    cnt = torch.bincount(tgt, minlength=mp.n)
    gptr = _csr_lists(cnt)

    def t_rows(rows: torch.Tensor, counts: torch.Tensor):
        p = _csr_lists(counts)
        tot = int(p[-1])
        k = torch.arange(tot, dtype=torch.int64, device=dev) - torch.repeat_interleave(p[:-1], counts)
        return order[torch.repeat_interleave(gptr[rows], counts) + k]

    # ghost rows sent back: their parts (every ghost row is read by an owned middle: at least one part)
    c_send = cnt[mp.recv_ids]
    send_ptr = _csr_lists(c_send)
    send_idx = t_rows(mp.recv_ids, c_send).to(torch.int32)
    # owned rows: own parts (the received copies replace them in loopback mode), then the received rows in order
    c_own = torch.zeros(mp.n_own, dtype=torch.int64, device=dev) if mp.loopback else cnt[mp.own]
    c_rcv = torch.bincount(mp.send_pos, minlength=mp.n_own) if mp.send_pos.numel() else torch.zeros_like(c_own)
    own_ptr = _csr_lists(c_own + c_rcv)
    own_idx = torch.empty(int(own_ptr[-1]), dtype=torch.int64, device=dev)
    if int(c_own.sum()):
        k = torch.arange(int(c_own.sum()), dtype=torch.int64, device=dev) - torch.repeat_interleave(
            _csr_lists(c_own)[:-1], c_own)
        own_idx[torch.repeat_interleave(own_ptr[:-1], c_own) + k] = t_rows(mp.own, c_own)
    if mp.send_pos.numel():
        e = torch.sort(mp.send_pos, stable=True).indices        # receive-buffer entries by owned row, in order
        k = torch.arange(e.numel(), dtype=torch.int64, device=dev) - torch.repeat_interleave(_csr_lists(c_rcv)[:-1], c_rcv)
        own_idx[torch.repeat_interleave(own_ptr[:-1] + c_own, c_rcv) + k] = -1 - e
    if own_idx.numel() >= 2 ** 31 or 3 * mp.n_own >= 2 ** 31:
        raise ValueError("middle_scatter: lists exceed int32")
    lists = (send_ptr, send_idx, own_ptr, own_idx.to(torch.int32))
    mp.cache["scatter_lists"] = lists
    return lists


def _scatter_ok(mp: MiddlePartition, h_own: torch.Tensor) -> bool:
    return h_own.is_cuda and h_own.size(1) % 16 == 0 and middle_scatter(mp) is not None


class _MidExchangePropagate(torch.autograd.Function):
    """h_own (owned rows) -> Z of the owned rows [n_own, 3F]: the ghost-row exchange (forward_exchange), then the
    owned-middle propagation. Backward in scatter form: the owned middles' gradient dZ goes to the rows they read
    (pg_spmm3t_ngram_scatter_*: D / P / S parts, no CSR pass over the rank's column block); the ghost rows' sums go
    back to their owners (one pg_rows_gather_sum, the all_to_all per chunk), and each owned row sums its own parts
    and the rows received for it (one pg_rows_gather_sum, fp32, one rounding to h_own's dtype)."""

    @staticmethod
    def forward(ctx, h_own, mp: MiddlePartition, comm):
        ctx.mp, ctx.comm, ctx.hdtype = mp, comm, h_own.dtype
        return _owned_spmm3(mp, forward_exchange(mp, h_own, comm))

    @staticmethod
    def backward(ctx, dZ):
        mp, comm = ctx.mp, ctx.comm
        sc = middle_scatter(mp)
        T = ops.spmm3t_scatter(sc.splan, dZ.contiguous())
        F_ = T.size(1)
        recv = None
        if mp.world > 1 or mp.loopback:
            send = ops.rows_gather_sum(T, sc.send_ptr, sc.send_idx, int(mp.recv_ids.numel()), F_,
                                       out_dtype=ctx.hdtype)
            recv = send.new_empty(int(mp.send_pos.numel()), F_)
            s0 = r0 = 0
            for c in range(mp.chunks):
                ns, nr = sum(mp.chunk_recv[c]), sum(mp.chunk_send[c])
                comm.all_to_all(recv[r0:r0 + nr], send[s0:s0 + ns], mp.chunk_send[c], mp.chunk_recv[c])
                s0, r0 = s0 + ns, r0 + nr
        d = ops.rows_gather_sum(T, sc.own_ptr, sc.own_idx, mp.n_own, F_, B=recv, out_dtype=ctx.hdtype)
        return d, None, None


class MiddleTrainer:
    """ShardedTrainer's step (the reference's full-batch loop, protgram_directgcn_trainer.py:91-100: zero_grad ->
    forward -> nll_loss (mean over all N nodes) + l2_lambda * sum_p ||p||^2 -> backward -> Adam step) on the middle
    partition (see the section comment): the middle-tile forward over the rank's middles, ghost-row exchanges only.
    Same optimizer semantics as ShardedTrainer (train.Adam with the L2 gradient folded in, device-side loss, no host
    sync per step); `comm` = the collectives (TorchComm(group) by default). Per-node parameters live in owned-row
    leaves in middle-major order (self.own[layer][name]); `sync_model()` writes them into this rank's rows of the
    model's full per-node parameters (rows owned elsewhere stay stale on this rank, as with ShardedTrainer)."""

    def __init__(self, model, mp: MiddlePartition, lr: float = 1e-3, l2_lambda: float = 1e-7, comm=None,
                 optimizer_factory=None, graphs: bool = False, **adam_kw):
        from . import train
        self.model, self.mp, self.l2_lambda = model, mp, float(l2_lambda)
        self.comm = comm if comm is not None else TorchComm()
        # graphs: after WARM eager steps the whole step (forward, backward, collectives, optimizer) is captured once as
        # a HIP graph and replayed: at a rank's share of the graph the eager step is bound by host-side launches, not
        # by the GPU (profiles/r04_middle_train_rank0_breakdown.txt). Needs collectives that can be captured
        # (comm.capturable: no-op / RCCL stream collectives; not gloo, which stages through host memory)
        self.graphs = bool(graphs)
        if self.graphs and not getattr(self.comm, "capturable", False):
            raise ValueError("graphs=True needs a comm whose collectives can be captured (comm.capturable)")
        self._graph = None
        self._eager_steps = 0
        self.xchg = mp.world > 1 or mp.loopback
        self.own: List[dict] = []
        node_ids, dense, node_leaves = set(), [], []
        rows = mp.own
        for conv in model.convs:
            d = {}
            for name, p in conv.named_parameters(recurse=False):
                if _is_node_param(name, p, mp.n):
                    leaf = nn.Parameter(p.detach().index_select(0, rows.to(p.device)).contiguous(),
                                        requires_grad=p.requires_grad)
                    d[name] = leaf
                    node_ids.add(id(p))
                    node_leaves.append(leaf)
            self.own.append(d)
        for name, p in model.named_parameters():
            if id(p) not in node_ids and p.requires_grad:
                dense.append(p)
        self.dense, self.node = dense, node_leaves
        dev = dense[0].device if dense else mp.own.device
        self.flat = torch.zeros(sum(p.numel() for p in dense), dtype=torch.float32, device=dev)
        self.params = dense + [p for p in node_leaves if p.requires_grad]
        # train.Adam over two groups (replicated, per-node): its launches also return each group's L2 value of the
        # pre-update parameters (the loss's two L2 terms, one of them all-reduced), so no separate sums are launched
        node_req = [p for p in node_leaves if p.requires_grad]
        self._sq_groups = None
        if optimizer_factory is None:
            groups = [g for g in ({"params": dense}, {"params": node_req}) if g["params"]]
            self.opt = train.Adam(groups, lr=lr, **adam_kw)
            if len(node_req) == len(node_leaves):
                self._sq_groups = (0 if dense else None, (1 if dense else 0) if node_req else None)
        else:
            self.opt = optimizer_factory(self.params)
        self._train = train
        self._touched: set = set()
        for prm in self.params:
            prm.register_post_accumulate_grad_hook(lambda t: self._touched.add(id(t)))
        middle_transpose(mp)  # setup work, outside the steps
        middle_scatter(mp)

    def forward(self, x_full: torch.Tensor, need_emb: bool = True):
        """(log_probs, emb) of the owned rows (middle-major) with autograd (emb None when need_emb is False: the step's
        loss reads only the log-probs)."""
        return self.model.head(self.body(x_full), need_emb=need_emb)

    def body(self, x_full: torch.Tensor) -> torch.Tensor:
        """The layers over the owned rows (middle-major), with autograd: the input of the prediction head."""
        model, mp = self.model, self.mp
        h = model._apply_pe(x_full)
        if model.compute_dtype == torch.bfloat16:
            h = self._bf16_input(h) if h is x_full and not h.requires_grad else h.to(torch.bfloat16)
        elif model.compute_dtype != torch.float32:
            raise ValueError("compute_dtype must be torch.float32 or torch.bfloat16")
        X, res_x = h, h.index_select(0, mp.own)
        L = len(model.convs)
        h_own = None
        # the layer dropout fused into the dense epilogue (ops.FUSED_DROPOUT, as ProtGramDirectGCN.body): one draw of
        # the layers' seeds per step, salted by the rank's first middle so that ranks (whose launches count their own
        # rows from 0) draw independent masks
        p_drop = float(model.dropout) if model.training else 0.0
        seeds = None
        if ops.FUSED_DROPOUT and 0.0 < p_drop < 1.0 and x_full.is_cuda:
            seeds = torch.randint(0, 1 << 62, (L,), device=x_full.device, dtype=torch.int64)
            seeds ^= ((mp.m0 + 1) * 0x9E3779B97F4A7C15) & ((1 << 62) - 1)  # a 62-bit hash of m0: no int64 overflow
        for i, (conv, res) in enumerate(zip(model.convs, model.res_projs)):
            if i == 0:
                Z = _MidPropagate.apply(X, mp)  # the input carries no gradient
            elif _scatter_ok(mp, h_own):
                Z = _MidExchangePropagate.apply(h_own, mp, self.comm)
            else:
                Z = _MidPropagate.apply(_MidExchange.apply(h_own, mp, self.comm), mp)
            vec = conv.use_vector_coeffs
            params = conv._dense_params()
            own = self.own[i]
            if vec:
                params = params[:10] + tuple(own[k] for k in _GATE_NAMES)
                constant = own["constant"]
            else:
                constant = None
            W_res, b_res = (res.weight, res.bias) if isinstance(res, nn.Linear) else (None, None)
            drop = (p_drop, seeds[i:i + 1]) if seeds is not None else None
            h_own = ops.LayerDense.apply(Z, res_x, constant, W_res, b_res, None, 0 if vec else 1, True,
                                         ops.LEAKY_SLOPE, drop, *params)
            if drop is None:
                h_own = F.dropout(h_own, p=model.dropout, training=model.training)
            res_x = h_own
        return h_own

    def _fused_head(self, h_own: torch.Tensor, y_own: torch.Tensor):
        """The prediction head's forward and backward in one kernel where it takes the shape (train.HEAD_FUSED; bf16
        h at F = 256: ops.head_train_bf16, fp32 at F = 128: ops.head_train): the owned rows' nll summed and divided by
        the global N (weight = own rows / N), the decoder's gradients assigned, h's gradient handed to autograd's
        backward. Returns the nll (device scalar) or None (the caller runs the framework ops)."""
        from . import ops
        train, model, mp = self._train, self.model, self.mp
        head = model.head_train_args() if train.HEAD_FUSED else None
        if head is None or not h_own.is_cuda:
            return None
        W1, b1, W2, b2, p_drop = head
        seed = None
        if p_drop > 0:  # salted by the rank's first middle, as the layers' seeds
            seed = torch.randint(0, 1 << 62, (1,), device=h_own.device, dtype=torch.int64)
            seed ^= ((mp.m0 + 7) * 0xD1B54A32D192ED03) & ((1 << 62) - 1)
        w = float(h_own.size(0)) / float(mp.n)
        if h_own.dtype == torch.bfloat16:
            r = ops.head_train_bf16(h_own, W1, b1, W2, b2, y_own, w, p_drop, seed)
        else:
            r = ops.head_train(h_own, W1, b1, W2, b2, y_own, w, p_drop, seed)
        if r is None:
            return None
        loss, dh, grads = r
        for prm, gr in zip((W1, b1, W2, b2), grads):
            if prm.requires_grad:
                prm.grad = gr
                self._touched.add(id(prm))
        torch.autograd.backward(h_own, grad_tensors=dh)
        return loss

    WARM = 3
    _xb = None

    def _bf16_input(self, x: torch.Tensor) -> torch.Tensor:
        """bf16 copy of a step-invariant input (no PE, no gradient): converted once, and again only when x changes
        (another tensor, or a new version counter: copy_ and in-place writes bump it), in place, so a captured step
        reads the refreshed values at the same address (the whole-N conversion was ~25 us of a config-5 rank step)."""
        c = self._xb
        if c is not None and c[0]() is x and c[1] == x._version:
            return c[2]
        if c is not None and c[2].shape == x.shape and c[2].device == x.device:
            xb = c[2]
            xb.copy_(x)
        else:
            xb = x.to(torch.bfloat16)
        self._xb = (weakref.ref(x), x._version, xb)
        return xb

    def step(self, x_full: torch.Tensor, y_own: torch.Tensor) -> torch.Tensor:
        """One step; y_own = the labels of the owned rows (y[mp.own]). Returns the global loss (device scalar; with
        graphs, the graph's static output, overwritten by the next step)."""
        if not self.graphs:
            return self._step(x_full, y_own)
        if self._graph is None:
            if self._eager_steps < self.WARM:  # allocator pools, Adam state, descriptor lists, index checks
                self._eager_steps += 1
                return self._step(x_full, y_own)
            self._capture(x_full, y_own)  # replays once: this step
            return self._loss
        if x_full is not self._x:
            self._x.copy_(x_full)
        if y_own is not self._y:
            self._y.copy_(y_own)
        if self._xb is not None:
            self._bf16_input(self._x)  # refreshed outside the graph when x changed (no-op otherwise)
        # train.Adam's lr / weight_decay are device scalars refreshed here, outside the graph, so a schedule that
        # changed the learning rate since the last replay (train.fit's ReduceLROnPlateau) takes effect now; another
        # optimizer whose settings changed is captured again
        if not self._train.replay_ready(self.opt, self._snap):
            torch.cuda.synchronize()
            self._graph = self._keep = None
            self._capture(self._x, self._y)
            return self._loss
        self._graph.replay()
        return self._loss

    def close(self):
        """Release the captured step (its graph holds RCCL kernels of this process group's communicator): call before
        destroy_process_group. Later steps run eagerly again until the next capture."""
        torch.cuda.synchronize()
        self._graph = None
        self._keep = None
        self._eager_steps = 0

    CHECK = True  # train.check_deferred before the first replay of every capture

    def _capture(self, x_full, y_own):
        self._x, self._y = x_full, y_own
        if isinstance(self.opt, self._train.Adam):
            self.opt.refresh_hyper()
        self._train.prepare_capture(x_full.device)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            self._loss = self._step(self._x, self._y)
        # everything the captured launches read by address stays alive with the graph: Adam's and the L2 sum's
        # device descriptor lists (and their pinned staging copies, which captured uploads re-read)
        self._keep = (list(getattr(self.opt, "_tl_cache", {}).values()) + list(self._train._LISTS.values()) +
                      self._train.flush_deferred())
        if self.CHECK:  # every table written after the capture reads back, every address in it is a live block
            self._train.check_deferred(self._keep)
        self._graph, self._snap = g, self._train.hyper_snapshot(self.opt)
        g.replay()  # the step the capture recorded

    def _step(self, x_full: torch.Tensor, y_own: torch.Tensor) -> torch.Tensor:
        # bf16 mode with train.Adam: the owned per-node constants' gradients stay the layers' bf16 dpre, read by Adam
        # directly (train.DEFER_CONST_GRAD, as train.train_step: no fp32 copy written by the backward, none copied
        # into a home buffer, half the bytes read by Adam; the same update bits)
        from . import ops
        defer = (self._train.DEFER_CONST_GRAD and isinstance(self.opt, self._train.Adam)
                 and self.model.compute_dtype == torch.bfloat16)
        prev = ops._DEFER_CONST_GRAD
        ops._DEFER_CONST_GRAD = defer
        try:
            return self._step_body(x_full, y_own)
        finally:
            ops._DEFER_CONST_GRAD = prev
            ops._DEFERRED_GRADS.clear()

    def _step_body(self, x_full: torch.Tensor, y_own: torch.Tensor) -> torch.Tensor:
        from .ops import deferred_grad
        mp, lam, train = self.mp, self.l2_lambda, self._train
        # autograd assigns each parameter's gradient (no .grad preset: a preset one costs an add kernel per parameter
        # per step, ~0.3 ms at config 5); then one multi-tensor copy moves them into their fixed homes: the flat
        # buffer of the replicated parameters (one all-reduce) and, with graphs, persistent per-node buffers (fixed
        # addresses: the optimizer's descriptor lists built in the eager warm-up serve the capture and its replays)
        if self.graphs and not hasattr(self, "_node_grads"):
            self._node_grads = [torch.zeros_like(p) for p in self.node]
        if not hasattr(self, "_flat_views"):
            views, off = [], 0
            for p in self.dense:
                k = p.numel()
                views.append(self.flat[off:off + k].view_as(p))
                off += k
            self._flat_views = views
        for p in self.dense + self.node:
            p.grad = None
        self.flat.zero_()
        self._touched = set()
        h_own = self.body(x_full)
        nll = self._fused_head(h_own, y_own)  # the head in one kernel (config 5: bf16, F = 256)
        if nll is None:
            lp, _ = self.model.head(h_own, need_emb=False)
            nll = -lp.float().gather(1, y_own.view(-1, 1)).sum() / mp.n
            nll.backward()
        homes = [(p, h, False) for p, h in zip(self.dense, self._flat_views)]
        if self.graphs:
            homes += [(p, h, True) for p, h in zip(self.node, self._node_grads)]
        have = [(p, h) for p, h, _ in homes if p.grad is not None]
        if have:
            torch._foreach_copy_([h for _, h in have], [p.grad for p, _ in have])
        for p, h, node in homes:
            if node and p.grad is None and deferred_grad(p) is not None:
                continue  # Adam reads the filed bf16 gradient
            if p.grad is None and node:
                h.zero_()  # an unused per-node parameter: its persistent buffer holds zeros (the flat one is zeroed)
            p.grad = h
        fold = bool(lam) and isinstance(self.opt, train.Adam)
        fused = fold and self._sq_groups is not None  # the L2 values come out of the Adam launches
        zero = nll.new_zeros(())
        if lam:
            for p in self.node:
                if p.requires_grad and p.grad is None and deferred_grad(p) is None:
                    p.grad = torch.zeros_like(p)
            if not fused:
                l2_rep = train.l2_sqsum(self.dense) if self.dense else zero
                l2_own = train.l2_sqsum(self.node) if self.node else zero
        else:
            for p in self.params:
                if id(p) not in self._touched:
                    p.grad = None
            l2_rep = l2_own = zero
        if self.xchg and (mp.world > 1 or FORCE_COLLECTIVES) and self.flat.numel():
            self.comm.all_reduce(self.flat)
        if lam and not fold:
            ps = [p for p in self.params if p.grad is not None]
            torch._foreach_add_([p.grad for p in ps], [p.detach() for p in ps], alpha=2.0 * lam)
        if fold:
            self.opt._l2_extra = 2.0 * lam
            self.opt._want_sqsum = "groups" if fused else False
        try:
            self.opt.step()
        finally:
            if fold:
                self.opt._l2_extra = 0.0
                self.opt._want_sqsum = False
        if fused:
            sums = self.opt._last_sqsum_groups
            gd, gn = self._sq_groups
            l2_rep = sums[gd] if gd is not None and sums[gd] is not None else zero
            l2_own = sums[gn] if gn is not None and sums[gn] is not None else zero
        parts = torch.stack([nll.detach().reshape(()), (lam * l2_own).reshape(())])
        if self.xchg and (mp.world > 1 or FORCE_COLLECTIVES):
            self.comm.all_reduce(parts)
        return parts.sum() + lam * l2_rep

    @torch.no_grad()
    def sync_model(self):
        """Write this rank's owned-row leaves into the model's full per-node parameters (rows mp.own)."""
        for conv, d in zip(self.model.convs, self.own):
            for name, leaf in d.items():
                getattr(conv, name).data.index_copy_(0, self.mp.own.to(leaf.device), leaf.data)

    @torch.no_grad()
    def gather(self):
        """Every rank's per-node parameters whole on every rank (checkpointing): the owned rows of all ranks,
        all-gathered (padded to the largest share) and written at their global rows."""
        self.sync_model()
        mp = self.mp
        if mp.world == 1:
            return
        Kn2 = mp.K ** (mp.ngram - 2)
        dev = mp.own.device
        rows = [_middle_rows(mp.K, mp.ngram, a, b, dev) for a, b in middle_bounds(Kn2, mp.world)]
        most = max(r.numel() for r in rows)
        for conv, d in zip(self.model.convs, self.own):
            for name, leaf in d.items():
                full = getattr(conv, name).data
                flat = leaf.data.reshape(leaf.size(0), -1)
                pad = flat.new_zeros(most, flat.size(1))
                pad[:flat.size(0)] = flat
                out = pad.new_empty(mp.world * most, flat.size(1))
                self.comm.all_gather(out, pad)
                fv = full.view(full.size(0), -1)
                for q, r in enumerate(rows):
                    fv.index_copy_(0, r.to(full.device), out[q * most:q * most + r.numel()])
