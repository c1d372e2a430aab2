"""ORACLE (test infrastructure only): CPU restatement of the reference's adjacency construction.

Restates ``DirectedNgramGraph`` (``src/utils/graph_utils.py:140-300``) with torch.sparse on CPU, op for
op, from the raw edge table the reference reads from parquet (unique ``(source, target)`` rows with a
float32 transition count, ``graph_utils.py:109-112``):

* ``A_out_w`` = coalesced COO of counts (:154); ``A_in_w = A_out_w.t()`` (:158)
* ``A_undirected_norm`` = D^-1/2 (unique(sym(E)) ++ arange self-loops) D^-1/2 (:160-196); PyG's
  ``add_self_loops`` APPENDS loops, so a raw self-loop ends with multiplicity 2
* ``mathcal_A`` = sqrt(0.5 * (Ahat^2 + Ahat^T^2) + eps) + I with Ahat = D^-1 A (:198-273), eps=1e-9

Returns each matrix as ``(indices int64 [2, nnz], values float32 [nnz])`` in coalesced (row-major) order.
"""
from __future__ import annotations

import numpy as np
import torch


def _sparse_identity(n: int) -> torch.Tensor:
    # graph_utils.py:290-300
    if n <= 0:
        return torch.sparse_coo_tensor(torch.empty((2, 0), dtype=torch.long), torch.empty(0), (max(0, n),) * 2).coalesce()
    idx = torch.arange(n).unsqueeze(0).repeat(2, 1)
    return torch.sparse_coo_tensor(idx, torch.ones(n, dtype=torch.float32), (n, n)).coalesce()


def _propagation(A: torch.Tensor, n: int, eps: float) -> torch.Tensor:
    # graph_utils.py:198-273
    if n == 0 or A._nnz() == 0:
        return torch.sparse_coo_tensor(torch.empty((2, 0), dtype=torch.long), torch.empty(0, dtype=torch.float32),
                                       (n, n)).coalesce()
    row_sum = torch.sparse.sum(A, dim=1).to_dense()
    d_inv = torch.zeros_like(row_sum, dtype=torch.float32)
    nz = row_sum != 0
    if torch.any(nz):
        d_inv[nz] = 1.0 / row_sum[nz]
    idx, val = A.indices(), A.values()
    An = torch.sparse_coo_tensor(idx, val * d_inv[idx[0]], A.size()).coalesce()
    An_sq = torch.sparse_coo_tensor(An.indices(), An.values().pow(2), An.size()).coalesce()
    S = (An_sq + An_sq.t().coalesce()).coalesce()
    S = torch.sparse_coo_tensor(S.indices(), S.values() * 0.5, S.size()).coalesce()
    base_vals = torch.sqrt(S.values() + torch.tensor(eps, dtype=torch.float32))
    base = torch.sparse_coo_tensor(S.indices(), base_vals, S.size()).coalesce()
    return (base + _sparse_identity(n)).coalesce()


def _undirected(src: np.ndarray, dst: np.ndarray, n: int) -> torch.Tensor:
    # graph_utils.py:160-196
    pairs = np.unique(np.stack([src, dst], axis=1), axis=0)
    sym = np.unique(np.concatenate([pairs, pairs[:, [1, 0]]], axis=0), axis=0)
    ei = torch.from_numpy(sym.T.copy()).long().reshape(2, -1)
    loops = torch.arange(n, dtype=torch.long).view(1, -1).repeat(2, 1)
    ei = torch.cat([ei, loops], dim=1)
    w = torch.ones(ei.size(1), dtype=torch.float32)
    row, col = ei
    deg = torch.zeros(n, dtype=torch.float32).scatter_add_(0, col, torch.ones(col.numel(), dtype=torch.float32))
    dis = deg.pow(-0.5)
    dis[dis == float("inf")] = 0
    vals = dis[row] * w * dis[col]
    return torch.sparse_coo_tensor(ei, vals, (n, n)).coalesce()


def build_matrices(num_nodes: int, src, dst, cnt, eps: float = 1e-9) -> dict:
    """All three propagation matrices of the reference for one n-gram level."""
    n = int(num_nodes)
    src = np.asarray(src, np.int64)
    dst = np.asarray(dst, np.int64)
    cnt = np.asarray(cnt, np.float32)
    out = {}
    if src.size == 0:
        empty = (torch.empty((2, 0), dtype=torch.long), torch.empty(0, dtype=torch.float32))
        A_und = _undirected(src.reshape(0), dst.reshape(0), n) if n > 0 else None
        out["in"] = empty
        out["out"] = empty
        out["und"] = (A_und.indices(), A_und.values()) if A_und is not None else empty
        return out
    ei = torch.stack([torch.from_numpy(src), torch.from_numpy(dst)]).long()
    A_out = torch.sparse_coo_tensor(ei, torch.from_numpy(cnt).float(), (n, n)).coalesce()
    A_in = A_out.t().coalesce()
    A_und = _undirected(src, dst, n)
    P_out = _propagation(A_out, n, eps)
    P_in = _propagation(A_in, n, eps)
    out["in"] = (P_in.indices(), P_in.values())
    out["out"] = (P_out.indices(), P_out.values())
    out["und"] = (A_und.indices(), A_und.values())
    return out
