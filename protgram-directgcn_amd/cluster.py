"""Cluster-GCN path: batched subgraph extraction for the reference's clustered
trainer (``protgram_directgcn_trainer.py:110-198``, used by default for graphs above 10,000 nodes,
config.py:98-104).

The reference partitions the graph with METIS (or Louvain), then for every cluster calls PyG
``subgraph(cluster_nodes, edge_index, edge_attr, relabel_nodes=True)`` on each of the three adjacencies
(:178-197) -- a scan of all E entries per cluster. Here:

* ``cluster_count`` is the reference's cluster-count rule (:154-156);
* ``range_clusters`` replaces METIS/Louvain (neither is installed) with contiguous ranges of a
  node order. With a graph's locality schedule as the order (``CSRGraph.row_order``: rows sorted by
  (min out-neighbour, min in-neighbour)), consecutive nodes share their neighbour sets, so the ranges keep
  many edges inside their clusters;
* ``build_subgraphs`` extracts every cluster's three relabelled COO adjacencies in ONE pass over the edges
  (O(E) instead of O(E * clusters)), with PyG's ``subgraph`` semantics exactly: an entry is kept when both
  endpoints are in the cluster, entries keep their original order, ids are relabelled to positions in the
  cluster's node list. Each ``Data`` has the fields the reference builds (x, y, the six edge tensors,
  original_indices) plus ``graph``: the subgraph's device CSR, cut from one batched CSR build, so the
  model never converts COO per step;
* ``union_graph`` is the block-diagonal union of all clusters over the cluster-major node order: one
  propagation launch covers every subgraph (batched inference / embedding extraction,
  ``clustered_forward``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional

import torch

from .data import Data
from .graph import CSRGraph, _bits, _rowptr, _sort_by, take


def cluster_count(num_nodes: int, target_nodes: int = 500, min_clusters: int = 2, max_clusters: int = 500) -> int:
    """protgram_directgcn_trainer.py:154-156 (GCN_TARGET_NODES_PER_CLUSTER / MIN / MAX, config.py:102-104)."""
    c = math.ceil(num_nodes / target_nodes)
    return min(max(min_clusters, c), max_clusters)


def range_clusters(num_nodes: int, num_clusters: int, order: Optional[torch.Tensor] = None,
                   device="cpu") -> torch.Tensor:
    """Cluster id per node: `order` (default 0..N-1) cut into `num_clusters` contiguous, equal ranges."""
    n = int(num_nodes)
    k = max(1, min(int(num_clusters), max(n, 1)))
    if order is None:
        order = torch.arange(n, device=device)
    order = order.to(torch.int64)
    parts = torch.empty(n, dtype=torch.int64, device=order.device)
    parts[order] = (torch.arange(n, device=order.device) * k) // max(n, 1)
    return parts


@dataclass
class ClusterLayout:
    """Cluster-major node order: cluster c owns nodes[ptr[c]:ptr[c+1]] (ascending ids), in the order in
    which the reference collects clusters (first appearance of the id when nodes are visited in order,
    trainer :172-175)."""
    nodes: torch.Tensor   # int64 [N]
    ptr: torch.Tensor     # int64 [C+1]
    rank: torch.Tensor    # int64 [N]: cluster index (0..C-1) of every node
    pos: torch.Tensor     # int64 [N]: position of every node inside its cluster

    @property
    def num_clusters(self) -> int:
        return self.ptr.numel() - 1


def layout_of(parts: torch.Tensor) -> ClusterLayout:
    parts = parts.to(torch.int64)
    n = parts.numel()
    dev = parts.device
    ids, inv = torch.unique(parts, return_inverse=True)
    first = torch.full((ids.numel(),), n, dtype=torch.int64, device=dev)
    first.scatter_reduce_(0, inv, torch.arange(n, device=dev), reduce="amin")
    rank_of_id = torch.empty_like(first)
    rank_of_id[torch.argsort(first)] = torch.arange(ids.numel(), device=dev)
    rank = rank_of_id[inv]
    nodes = _sort_by(rank)  # stable: ascending node ids inside each cluster
    counts = torch.bincount(rank, minlength=ids.numel())
    ptr = torch.zeros(ids.numel() + 1, dtype=torch.int64, device=dev)
    ptr[1:] = torch.cumsum(counts, 0)
    pos = torch.empty(n, dtype=torch.int64, device=dev)
    pos[nodes] = torch.arange(n, device=dev) - ptr[rank[nodes]]
    return ClusterLayout(nodes, ptr, rank, pos)


def _cut(lay: ClusterLayout, ei: torch.Tensor, ew: Optional[torch.Tensor]):
    """PyG subgraph(relabel_nodes=True) for every cluster at once: (local ei [2, E'], weights [E'] or None,
    edge ptr [C+1]) with the kept entries grouped by cluster in their original order."""
    ei = ei.to(torch.int64)
    s, d = ei[0], ei[1]
    keep = lay.rank[s] == lay.rank[d]
    ks, kd = s[keep], d[keep]
    kc = lay.rank[ks]
    p = _sort_by(kc)
    local = torch.stack([take(lay.pos, take(ks, p)), take(lay.pos, take(kd, p))])
    w = take(ew.reshape(-1)[keep], p) if ew is not None else None
    counts = torch.bincount(kc, minlength=lay.num_clusters)
    eptr = torch.zeros(lay.num_clusters + 1, dtype=torch.int64, device=ei.device)
    eptr[1:] = torch.cumsum(counts, 0)
    return local, w, eptr


def build_subgraphs(num_nodes: int, parts: torch.Tensor, ei_in, ew_in, ei_out, ew_out, ei_und, ew_und,
                    x: torch.Tensor, y: Optional[torch.Tensor] = None, with_graph: bool = True) -> List[Data]:
    """The reference's _create_clustered_subgraphs (trainer :178-197) for a given partition, in one pass.
    `parts`: cluster id per node (any integer ids). Returns one Data per cluster, clusters in the
    reference's order."""
    lay = layout_of(parts.to(ei_in.device))
    cut = [_cut(lay, ei, ew) for ei, ew in ((ei_in, ew_in), (ei_out, ew_out), (ei_und, ew_und))]
    shared = (ei_in.shape == ei_out.shape == ei_und.shape and torch.equal(ei_in, ei_out)
              and torch.equal(ei_in, ei_und))
    ptr = lay.ptr.tolist()
    eps = [c[2].tolist() for c in cut]
    graphs = _batched_csrs(lay, cut, ptr, eps[0]) if (with_graph and shared) else None
    out = []
    for c in range(lay.num_clusters):
        nodes = lay.nodes[ptr[c]:ptr[c + 1]]
        fields = {}
        for (local, w, _), e, (ik, wk) in zip(cut, eps, (("edge_index_in", "edge_weight_in"),
                                                      ("edge_index_out", "edge_weight_out"),
                                                      ("edge_index_undirected_norm", "edge_weight_undirected_norm"))):
            fields[ik] = local[:, e[c]:e[c + 1]].contiguous()
            fields[wk] = w[e[c]:e[c + 1]] if w is not None else None
        d = Data(x=x[nodes], y=(y[nodes] if (y is not None and y.numel() > 0) else torch.empty(0)),
                 original_indices=nodes, **fields)
        if graphs is not None:
            d.graph = graphs[c]
        out.append(d)
    return out


def _batched_csrs(lay: ClusterLayout, cut, ptr, eptr) -> List[CSRGraph]:
    """All clusters' shared-pattern CSRs from one sort: entries ordered by (cluster, local destination),
    stable (so within a row the COO order is kept, as csr_from_coo does), then cut per cluster."""
    local, w_in, _ = cut[0]
    w_out, w_und = cut[1][1], cut[2][1]
    dev = local.device
    E = local.size(1)
    ones = torch.ones(E, dtype=torch.float32, device=dev)
    wi = w_in if w_in is not None else ones
    wo = w_out if w_out is not None else ones
    wu = w_und if w_und is not None else ones
    # global row of every entry in the cluster-major order: cluster offset + local destination
    cl = torch.repeat_interleave(torch.arange(len(ptr) - 1, device=dev), torch.tensor(
        [eptr[c + 1] - eptr[c] for c in range(len(ptr) - 1)], device=dev))
    offs = torch.tensor(ptr[:-1], dtype=torch.int64, device=dev)
    grow = offs[cl] + local[1]
    p = _sort_by(grow)
    rec = torch.stack([take(local[0], p).to(torch.int32), _bits(take(wi, p)), _bits(take(wo, p)), _bits(take(wu, p))],
                      1).contiguous()
    rowptr = _rowptr(grow, ptr[-1])
    pt = _sort_by(offs[cl] + local[0])
    rec_t = torch.stack([take(local[1], pt).to(torch.int32), _bits(take(wi, pt)), _bits(take(wo, pt)),
                        _bits(take(wu, pt))], 1).contiguous()
    rowptr_t = _rowptr(offs[cl] + local[0], ptr[-1])
    out = []
    for c in range(len(ptr) - 1):
        r0, r1 = ptr[c], ptr[c + 1]
        e0, e1 = eptr[c], eptr[c + 1]
        rp = (rowptr[r0:r1 + 1] - e0).contiguous()
        ed = rec[e0:e1]
        rpt = (rowptr_t[r0:r1 + 1] - e0).contiguous()
        edt = rec_t[e0:e1]
        sym = torch.equal(rp, rpt) and torch.equal(ed, edt)
        g = CSRGraph(n_rows=r1 - r0, shared=True, rowptr=rp, edges3=ed, rowptr_t=rp if sym else rpt,
                     edges3_t=ed if sym else edt, symmetric=sym, nnz=e1 - e0)
        out.append(g)
    return out


def union_graph(subgraphs: List[Data]) -> CSRGraph:
    """Block-diagonal union of the clusters' CSRs over the cluster-major node order (one launch for all)."""
    gs = [d.graph for d in subgraphs]
    rps, eds, rpts, edts, off_n, off_e = [], [], [], [], 0, 0
    sym = all(g.symmetric for g in gs)
    for g in gs:
        rps.append(g.rowptr[:-1] + off_e)
        rpts.append(g.rowptr_t[:-1] + off_e)
        e = g.edges3.clone()
        e[:, 0] += off_n
        eds.append(e)
        et = g.edges3_t.clone()
        et[:, 0] += off_n
        edts.append(et)
        off_n += g.n_rows
        off_e += g.nnz
    dev = gs[0].rowptr.device
    end = torch.tensor([off_e], dtype=torch.int64, device=dev)
    rp = torch.cat(rps + [end])
    ed = torch.cat(eds)
    if sym:
        return CSRGraph(n_rows=off_n, shared=True, rowptr=rp, edges3=ed, rowptr_t=rp, edges3_t=ed, symmetric=True,
                        nnz=off_e)
    return CSRGraph(n_rows=off_n, shared=True, rowptr=rp, edges3=ed, rowptr_t=torch.cat(rpts + [end]),
                    edges3_t=torch.cat(edts), symmetric=False, nnz=off_e)


@torch.no_grad()
def clustered_forward(model, subgraphs: List[Data], union: Optional[CSRGraph] = None):
    """Every cluster's forward (model(subgraph) for each, as the clustered trainer would evaluate them) in ONE
    pass over the union graph. Returns (log_probs, emb) per node in the ORIGINAL node order (nodes not in
    any cluster get zeros)."""
    g = union if union is not None else union_graph(subgraphs)
    nodes = torch.cat([d.original_indices for d in subgraphs])
    x = torch.cat([d.x for d in subgraphs])
    lp, emb = model(Data(x=x, graph=g, original_indices=nodes))
    n = int(nodes.max()) + 1 if nodes.numel() else 0
    lp_full = lp.new_zeros(n, lp.size(1))
    emb_full = emb.new_zeros(n, emb.size(1))
    lp_full[nodes] = lp
    emb_full[nodes] = emb
    return lp_full, emb_full
