"""Device-resident CSR for the DirectGCN propagation (HBM layout of SURVEY §8b/§8d).

Two ways in:

* :func:`csr_from_coo` -- the drop-in boundary. Takes the reference's COO inputs exactly as the
  trainer wires them (``edge_index_* = mathcal_A_*.indices()``, ``edge_weight_* = .values()``,
  ``protgram_directgcn_trainer.py:362-367``; or the benchmarker's ``edge_weight=None`` wiring,
  ``gnn_benchmarker.py:297-305``), detects whether the three adjacencies share one pattern, and
  converts once to CSR keyed by destination (``ei[1]``). Results are cached per input tensors.
* :func:`build_propagation_csr` -- builds the three n-gram propagation matrices directly from the raw
  transition table (the reference's edge parquet, ``graph_utils.py:106-119``) in shared-pattern form,
  with the normalisation (``graph_utils.py:160-273``) done on the GPU by ``pg_edges_normalize_f32``
  or fused into the SpMM (``pg_spmm3_fusednorm_f32``).

HBM layout, shared pattern (n-gram graphs):
  rowptr  int64 [n+1]
  edges3  int32 [nnz, 4] = {col, bits(w_in), bits(w_out), bits(w_und)}  -- 16 B per entry, one load
  raw     int32 [nnz, 4] = {col, bits(a_fwd), bits(a_bwd), bits(m_und)}  (fused-norm mode)
  node_norm f32 [n, 4]  = {1/dout, 1/din, deg_und^-1/2, 0}
Non-shared patterns keep one ``{col, bits(w)}`` CSR (8 B per entry) per adjacency.
Backward uses the transposed CSR; when all three matrices are symmetric (always true for the n-gram
matrices) it aliases the forward CSR.
"""
from __future__ import annotations

import math

from dataclasses import dataclass, field
from typing import Optional

import numpy as np
import torch

# (key -> (source tensors, CSRGraph)). Holding the source tensors keeps their storage alive, so a key
# (data_ptr, version, shape, ...) can never match a different tensor that reused freed memory. Sized for
# Cluster-GCN training (one entry per subgraph: the reference's default is up to 500 clusters).
_CACHE: "dict[tuple, tuple]" = {}
_CACHE_MAX = 1024


@dataclass
class ShapedAdjacency:
    """One adjacency in CSR-by-destination form with its transpose (CSR-by-source)."""
    rowptr: torch.Tensor
    edges: torch.Tensor  # int32 [nnz, 2] {col, bits(w)}
    rowptr_t: torch.Tensor
    edges_t: torch.Tensor
    nnz: int


@dataclass
class NgramPlan:
    """Weights of a shared-pattern graph over all K^n n-grams laid out for the n-gram tile kernels
    (pg_ngram_plan_f32 / pg_spmm3_ngram_f32 / pg_spmm3t_ngram_f32): node id = base-K number of the n-gram."""
    K: int
    n: int
    plan: torch.Tensor  # fp32 [pg_ngram_plan_floats(K, n, K^n)]: 4x4-block layout (transposed kernels, block-4 forward)
    mplan: Optional[torch.Tensor] = None  # fp32 [pg_ngram_mplan_floats(K, n, K^n)]: middle layout (middle-tile forward)
    _diag3: Optional[torch.Tensor] = field(default=None, repr=False, compare=False)

    def diag3(self) -> torch.Tensor:
        """The middle plan's diagonal slots as fp32 [K^n, 3] (row i = a.M.b: Wdiag_k[a, b] of middle M, k = in, out,
        undirected) -- the term pg_spmm3t_ngram_mid_offdiag_f32 leaves to its caller. A self-loop that is also an
        out-neighbour (a constant n-gram) sits in its out-slot, not here. Computed once (a view of the plan)."""
        if self._diag3 is None:
            K = self.K
            Kn2 = K ** (self.n - 2)
            d = self.mplan.view(Kn2, MPLAN_FLOATS)[:, MPLAN_DIAG:MPLAN_DIAG + 3 * K * K].view(Kn2, K, K, 3)  # [M][a][b]
            self._diag3 = d.permute(1, 0, 2, 3).reshape(K ** self.n, 3).contiguous()  # row a K^(n-1) + M K + b
        return self._diag3


# middle-plan layout (pg_ngram_mid.hip): floats per middle, offset of the diagonal slots [a][b][k]
MPLAN_FLOATS = 52_400
MPLAN_DIAG = 51_200


# The K = 20 grid of the mapped plan: the standard amino-acid letters (any other character -- the builder's padding
# ' ', X / U / B / Z / O -- puts an n-gram off the grid).
GRID_LETTERS = "ACDEFGHIKLMNPQRSTVWY"


@dataclass
class NgramMap:
    """A builder-produced graph (run_graph_builder.py: node ids = sorted-string ranks of the n-grams PRESENT over an
    alphabet with the padding ' ', data_builder.py:29-35, 164-173) laid out for the middle-tile kernel on the grid of
    the K = 20 standard letters (build_ngram_map): the grid part runs pg_spmm3_ngram_mid_map_f32 (X / Z at node rows
    through gmap), the rest -- rows off the grid and entries with no grid slot -- one residual pass
    (pg_spmm3_resid_f32: overwrite the off-grid rows, add into the grid rows with residual entries)."""
    K: int
    n: int
    mplan: torch.Tensor      # fp32 [K^(n-2) * 52,400]: middle plan of the grid part
    gmap: torch.Tensor       # int32 [K^n]: node row of grid row g, -1 = n-gram not a node
    ginv: torch.Tensor       # int32 [N]: grid row of node i, -1 = off the grid
    res_rowptr: torch.Tensor  # int64 [n_res + 1]: compact CSR of the residual rows (list position -> entries)
    res_rows: torch.Tensor    # int32 [n_res]: node row; bit 31 set = a grid row (the pass adds to the tile output)
    res_edges: torch.Tensor   # int32 [nnz_res, 4]: the residual entries (records as edges3, CSR order kept)
    n_grid: int = 0           # nodes on the grid
    nnz_res: int = 0
    n_off: int = 0            # residual rows off the grid (overwritten)
    n_acc: int = 0            # residual rows on the grid (added to)


@dataclass
class CSRGraph:
    n_rows: int
    shared: bool
    rowptr: Optional[torch.Tensor] = None
    edges3: Optional[torch.Tensor] = None
    rowptr_t: Optional[torch.Tensor] = None
    edges3_t: Optional[torch.Tensor] = None
    symmetric: bool = False
    adj: list = field(default_factory=list)  # non-shared: [in, out, und] ShapedAdjacency
    raw: Optional[torch.Tensor] = None
    node_norm: Optional[torch.Tensor] = None
    eps: float = 1e-9
    nnz: int = 0
    row_order: Optional[torch.Tensor] = None  # int32 processing schedule of destination rows (None = 0..n-1)
    n_cols: Optional[int] = None             # rows of X (= output rows of the transpose); None = n_rows
    ngram: Optional[NgramPlan] = None        # n-gram tile plan (build_ngram_plan), used instead of the CSR kernels
    ngram_map: Optional[NgramMap] = None     # mapped middle plan of a builder-produced graph (build_ngram_map)

    @property
    def device(self):
        t = self.rowptr if self.shared else self.adj[0].rowptr
        return t.device

    def to(self, device) -> "CSRGraph":
        """A copy with every tensor on `device` (self if already there)."""
        device = torch.device(device)
        if self.device == device:
            return self
        mv = lambda t: None if t is None else t.to(device)  # noqa: E731
        g = CSRGraph(n_rows=self.n_rows, shared=self.shared, rowptr=mv(self.rowptr), edges3=mv(self.edges3),
                     symmetric=self.symmetric, raw=mv(self.raw), node_norm=mv(self.node_norm), eps=self.eps,
                     nnz=self.nnz, row_order=mv(self.row_order), n_cols=self.n_cols)
        if self.symmetric and self.rowptr_t is self.rowptr:
            g.rowptr_t, g.edges3_t = g.rowptr, g.edges3
        else:
            g.rowptr_t, g.edges3_t = mv(self.rowptr_t), mv(self.edges3_t)
        g.adj = [ShapedAdjacency(mv(a.rowptr), mv(a.edges), mv(a.rowptr_t), mv(a.edges_t), a.nnz) for a in self.adj]
        if self.ngram is not None:
            g.ngram = NgramPlan(self.ngram.K, self.ngram.n, self.ngram.plan.to(device),
                                None if self.ngram.mplan is None else self.ngram.mplan.to(device))
        if self.ngram_map is not None:
            m = self.ngram_map
            g.ngram_map = NgramMap(m.K, m.n, *(mv(t) for t in (m.mplan, m.gmap, m.ginv, m.res_rowptr, m.res_rows,
                                                                 m.res_edges)), m.n_grid, m.nnz_res, m.n_off, m.n_acc)
        return g

    def tensors(self):
        ts = [self.rowptr, self.edges3, self.rowptr_t, self.edges3_t, self.row_order,
              self.ngram.plan if self.ngram is not None else None,
              self.ngram.mplan if self.ngram is not None else None]
        if self.ngram_map is not None:
            m = self.ngram_map
            ts += [m.mplan, m.gmap, m.ginv, m.res_rowptr, m.res_rows, m.res_edges]
        for a in self.adj:
            ts += [a.rowptr, a.edges, a.rowptr_t, a.edges_t]
        return [t for t in ts if t is not None]

    def nnz_total(self) -> int:
        return 3 * self.nnz if self.shared else sum(a.nnz for a in self.adj)

    def algorithmic_bytes(self, F: int, elem: int = 4) -> int:
        """SURVEY §8d B_agg: rowptr + records + one X-row gather per entry + 3 output rows."""
        n = self.n_rows
        if self.shared:
            return 8 * (n + 1) + self.nnz * (16 + F * elem) + 3 * n * F * elem
        return sum(8 * (n + 1) + a.nnz * (8 + F * elem) + n * F * elem for a in self.adj)

    def compulsory_bytes(self, F: int, elem: int = 4, gated: bool = False) -> int:
        """SURVEY §8d's compulsory model: rowptr + records once, every X row read ONCE (the rows of X the
        graph references: n_cols, or n_rows), 3 output rows; gated launches also read 5 fp32 gates per row.
        With an n-gram plan (the tile kernels run: middle-tile fp32 / bf16 for F % 16 == 0, else 4x4-block fp32 at
        F = 64 / 128 / 256) the plan's weights replace rowptr + records.
        The byte floor a propagation launch cannot go below; the roofline fraction is priced on it."""
        n = self.n_rows
        nx = self.n_cols if self.n_cols is not None else n
        g = 20 * n if gated else 0
        if self.ngram is not None and self.ngram.mplan is not None and F % 16 == 0 and elem in (2, 4):
            return 4 * self.ngram.mplan.numel() + nx * F * elem + 3 * n * F * elem + g  # middle-tile kernel: its plan
        if self.ngram_map is not None and F % 16 == 0 and elem == 4:  # mapped middle-tile kernel + residual CSR pass
            m = self.ngram_map
            nr = m.n_off + m.n_acc  # residual rows: list entry + rowptr + records (+ the added-to Z rows re-read)
            return (4 * m.mplan.numel() + 4 * m.gmap.numel() + nx * F * elem + 3 * n * F * elem + g
                    + 12 * nr + 16 * m.nnz_res + 3 * m.n_acc * F * elem)
        if self.ngram is not None and F in (64, 128, 256) and elem == 4:  # the n-gram tile kernel reads its plan instead
            return 4 * self.ngram.plan.numel() + nx * F * elem + 3 * n * F * elem + g
        if self.shared:
            return 8 * (n + 1) + 16 * self.nnz + nx * F * elem + 3 * n * F * elem + g
        return sum(8 * (n + 1) + 8 * a.nnz + nx * F * elem + n * F * elem for a in self.adj) + g


_TAKE_PIECE_BYTES = 1 << 28  # bytes of result per gather piece


def take(t: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """``t[idx]`` along dim 0. On the GPU, a result of 256 MiB or more is gathered in pieces of at most 256 MiB of
    result (max(1, 2^28 // row bytes) indices each, whatever the row width): ROCm torch's index gather (torch
    2.10+rocm7.0 on MI355X) was seen to leave the tail of results of 1 GiB or more unwritten (round 2: ``edges3[src]``
    with 114.8M indices into the 5-gram [131M, 4] int32 records returned its last 2^26 rows as zeros, which was the
    round-1 device halo_partition fault). tools/gather_probe.py re-measures the raw gather
    (profiles/r03_gather_probe.txt) and tests/test_gpu_parity.py::test_take_large_wide_rows pins take() itself
    against a host gather at > 1 GiB with 512-B rows."""
    row = t.element_size() * (t[0].numel() if t.dim() > 1 and t.size(0) else 1)
    if not t.is_cuda or idx.numel() * row < _TAKE_PIECE_BYTES:
        return t[idx]
    step = max(1, _TAKE_PIECE_BYTES // max(row, 1))
    return torch.cat([t[idx[k:k + step]] for k in range(0, idx.numel(), step)])


def _bits(w: torch.Tensor) -> torch.Tensor:
    return w.contiguous().to(torch.float32).view(torch.int32)


def _sort_by(primary: torch.Tensor) -> torch.Tensor:
    """Stable sort by row only: within a row the entries keep their COO order, which is the order in
    which the reference's scatter_add_ accumulates them (so sums round identically). For a coalesced
    COO this is ascending column order."""
    return torch.sort(primary, stable=True).indices


def _rowptr(rows: torch.Tensor, n: int) -> torch.Tensor:
    counts = torch.bincount(rows, minlength=n) if rows.numel() else torch.zeros(n, dtype=torch.long,
                                                                                   device=rows.device)
    rp = torch.zeros(n + 1, dtype=torch.int64, device=rows.device)
    rp[1:] = torch.cumsum(counts[:n], 0)
    return rp


def _validate(ei: torch.Tensor, n_rows: int, name: str):
    if ei.dim() != 2 or ei.size(0) != 2:
        raise ValueError(f"{name} must have shape [2, nnz], got {tuple(ei.shape)}")
    if ei.numel():
        lo, hi = int(ei.min()), int(ei.max())
        if lo < 0 or hi >= n_rows:
            raise IndexError(f"{name} holds node ids in [{lo}, {hi}] outside [0, {n_rows})")


def _single(ei: torch.Tensor, ew: Optional[torch.Tensor], n: int) -> ShapedAdjacency:
    ei = ei.to(torch.int64)
    src, dst = ei[0], ei[1]
    w = torch.ones(src.numel(), dtype=torch.float32, device=ei.device) if ew is None else ew.reshape(-1)
    if w.numel() != src.numel():
        raise ValueError("edge_weight length does not match edge_index")
    p = _sort_by(dst)
    e = torch.stack([take(src, p).to(torch.int32), _bits(take(w, p))], 1).contiguous()
    pt = _sort_by(src)
    et = torch.stack([take(dst, pt).to(torch.int32), _bits(take(w, pt))], 1).contiguous()
    return ShapedAdjacency(_rowptr(dst, n), e, _rowptr(src, n), et, int(src.numel()))


def _key(*ts, n):
    k = [n]
    for t in ts:
        if t is None:
            k.append(None)
        else:
            k.append((t.data_ptr(), t._version, tuple(t.shape), t.dtype, str(t.device)))
    return tuple(k)


def csr_from_coo(num_rows: int, ei_in, ew_in, ei_out, ew_out, ei_und, ew_und, cache: bool = True,
                 ngram_alphabet: Optional[int] = 20) -> CSRGraph:
    """Convert the reference's three COO adjacencies to the device CSR (cached by tensor identity).

    This is the path the reference trainer's unchanged wiring takes (``Data.edge_index_* = mathcal_A_*.indices()``,
    ``edge_weight_* = .values()``, ``protgram_directgcn_trainer.py:362-367``, read by ``protgram_directgcn.py:196-203``).
    When the three matrices share one pattern and the graph holds all ngram_alphabet^n n-grams in base-K id order (the
    builder's sorted-string ids when every n-gram occurs), the n-gram tile plan (build_ngram_plan) and the middle-major
    locality schedule (ngram_schedule) are attached, so this path runs the same kernels as a graph built by
    build_propagation_csr. The plan kernel rejects (and the graph keeps the CSR kernels for) any pattern with an entry
    that is neither a transition, a reverse transition nor the diagonal. ngram_alphabet=None: no plan."""
    key = _key(ei_in, ew_in, ei_out, ew_out, ei_und, ew_und, n=num_rows) + (ngram_alphabet,)
    if cache:
        hit = _CACHE.get(key)
        if hit is not None:
            _CACHE[key] = _CACHE.pop(key)  # LRU
            return hit[1]
    n = int(num_rows)
    for name, ei in (("edge_index_in", ei_in), ("edge_index_out", ei_out), ("edge_index_undirected", ei_und)):
        _validate(ei, n, name)
    shared = (ei_in.shape == ei_out.shape == ei_und.shape and ei_in.numel() > 0
              and torch.equal(ei_in, ei_out) and torch.equal(ei_in, ei_und))
    if shared:
        ei = ei_in.to(torch.int64)
        src, dst = ei[0], ei[1]
        nnz = src.numel()
        ones = None

        def w(t):
            nonlocal ones
            if t is None:
                if ones is None:
                    ones = torch.ones(nnz, dtype=torch.float32, device=ei.device)
                return ones
            if t.numel() != nnz:
                raise ValueError("edge_weight length does not match edge_index")
            return t.reshape(-1)

        wi, wo, wu = w(ew_in), w(ew_out), w(ew_und)
        p = _sort_by(dst)
        edges3 = torch.stack([take(src, p).to(torch.int32), _bits(take(wi, p)), _bits(take(wo, p)),
                              _bits(take(wu, p))], 1).contiguous()
        rowptr = _rowptr(dst, n)
        pt = _sort_by(src)
        edges3_t = torch.stack([take(dst, pt).to(torch.int32), _bits(take(wi, pt)), _bits(take(wo, pt)),
                                _bits(take(wu, pt))], 1).contiguous()
        rowptr_t = _rowptr(src, n)
        sym = torch.equal(rowptr, rowptr_t) and torch.equal(edges3, edges3_t)
        if sym:
            rowptr_t, edges3_t = rowptr, edges3
        g = CSRGraph(n_rows=n, shared=True, rowptr=rowptr, edges3=edges3, rowptr_t=rowptr_t, edges3_t=edges3_t,
                     symmetric=sym, nnz=nnz)
        if ngram_alphabet and rowptr.is_cuda:
            g.ngram = build_ngram_plan(g, ngram_alphabet)
            if g.ngram is not None:
                g.row_order = ngram_schedule(g.ngram.K, g.ngram.n, rowptr.device)
    else:
        g = CSRGraph(n_rows=n, shared=False,
                     adj=[_single(ei_in, ew_in, n), _single(ei_out, ew_out, n), _single(ei_und, ew_und, n)])
    if cache:
        if len(_CACHE) >= _CACHE_MAX:
            _CACHE.pop(next(iter(_CACHE)))
        _CACHE[key] = ((ei_in, ew_in, ei_out, ew_out, ei_und, ew_und), g)
    return g


def clear_cache():
    _CACHE.clear()


# ------------------------------------------------------------------------------------------------
# n-gram propagation matrices straight from the raw transition table
# ------------------------------------------------------------------------------------------------
@dataclass
class RawNgramCSR:
    n: int
    rowptr: torch.Tensor     # int64 [n+1]
    raw: torch.Tensor        # int32 [nnz, 4] {col, a_fwd, a_bwd, m_und}
    node_norm: torch.Tensor  # f32 [n, 4]
    nnz: int
    row_order: Optional[torch.Tensor] = None


def locality_schedule(n: int, src: torch.Tensor, dst: torch.Tensor) -> torch.Tensor:
    """Row processing order that makes concurrently scheduled rows share neighbour rows in L2.

    Key = (min out-neighbour, min in-neighbour). In an n-gram transition graph the out-neighbours of
    s_1..s_n are s_2..s_n c (a function of the (n-1)-suffix) and the in-neighbours are c s_1..s_{n-1}
    (a function of the prefix), so sorting by the key groups the rows with identical out-neighbour
    sets, and consecutive groups share the middle s_2..s_{n-1}: a run of 400 rows then touches only
    ~800 distinct feature rows (vs ~16,400 gathers). For graphs without that structure it is just a
    deterministic permutation. Changes the schedule only, never the result."""
    dev = src.device
    big = torch.full((n,), n, dtype=torch.int64, device=dev)
    min_out = big.clone().scatter_reduce_(0, src, dst, reduce="amin") if src.numel() else big.clone()
    min_in = big.clone().scatter_reduce_(0, dst, src, reduce="amin") if src.numel() else big.clone()
    key = min_out * (n + 1) + min_in
    return torch.sort(key, stable=True).indices.to(torch.int32)


def ngram_schedule(K: int, n: int, device="cpu") -> torch.Tensor:
    """The locality schedule of a graph over all K^n n-grams in base-K id order, in closed form: rows sorted by
    (middle s_2..s_{n-1}, last letter, first letter). For a complete transition graph this is exactly the order
    locality_schedule computes from the transitions (min out-neighbour M.b.0, then min in-neighbour 0.a.M); it is
    used where only the symmetric propagation pattern is at hand (csr_from_coo). A schedule, never a result change."""
    Kn1, Kn2 = K ** (n - 1), K ** (n - 2)
    mid = torch.arange(Kn2, dtype=torch.int64, device=device).view(-1, 1, 1)
    b = torch.arange(K, dtype=torch.int64, device=device).view(1, -1, 1)
    a = torch.arange(K, dtype=torch.int64, device=device).view(1, 1, -1)
    return (a * Kn1 + mid * K + b).reshape(-1).to(torch.int32)


def ngram_raw_csr(num_nodes: int, src, dst, cnt, device="cpu", schedule: bool = True) -> RawNgramCSR:
    """Shared pattern of (A u A^T u I) with raw counts, plus per-node normalisation terms.

    Integer work (pattern, grouping, sorting) runs with torch on ``device``; the O(n) float terms are
    computed on the host with IEEE float32 ops so they equal the reference's torch CPU values bit for
    bit: 1/rowsum (graph_utils.py:231-235) and deg^-1/2 (graph_utils.py:187-189)."""
    n = int(num_nodes)
    src_np = np.asarray(src, dtype=np.int64)
    dst_np = np.asarray(dst, dtype=np.int64)
    cnt_np = np.asarray(cnt, dtype=np.float32)
    if src_np.size and (src_np.min() < 0 or max(src_np.max(), dst_np.max()) >= n):
        raise IndexError("edge ids outside [0, num_nodes)")
    dev = torch.device(device)
    s = torch.from_numpy(src_np).to(dev)
    d = torch.from_numpy(dst_np).to(dev)
    c = torch.from_numpy(cnt_np).to(dev)
    ar = torch.arange(n, dtype=torch.int64, device=dev)
    zeros_e = torch.zeros_like(c)
    rows = torch.cat([d, s, ar])
    cols = torch.cat([s, d, ar])
    a_fwd = torch.cat([c, zeros_e, torch.zeros(n, device=dev)])
    a_bwd = torch.cat([zeros_e, c, torch.zeros(n, device=dev)])
    key = rows * max(n, 1) + cols
    uk, inv = torch.unique(key, sorted=True, return_inverse=True)
    nnz = uk.numel()
    af = torch.zeros(nnz, dtype=torch.float32, device=dev).index_add_(0, inv, a_fwd)
    ab = torch.zeros(nnz, dtype=torch.float32, device=dev).index_add_(0, inv, a_bwd)
    r_row = uk // max(n, 1)
    r_col = uk % max(n, 1)
    m = torch.where((r_row == r_col) & (af > 0), 2.0, 1.0).to(torch.float32)
    rowptr = _rowptr(r_row, n)
    raw = torch.stack([r_col.to(torch.int32), _bits(af), _bits(ab), _bits(m)], 1).contiguous()
    # per-node terms (host, O(n))
    dout = np.bincount(src_np, weights=cnt_np.astype(np.float64), minlength=n).astype(np.float32)
    din = np.bincount(dst_np, weights=cnt_np.astype(np.float64), minlength=n).astype(np.float32)
    one = np.float32(1.0)
    with np.errstate(divide="ignore"):
        dout_inv = np.where(dout != 0, one / np.where(dout != 0, dout, one), np.float32(0)).astype(np.float32)
        din_inv = np.where(din != 0, one / np.where(din != 0, din, one), np.float32(0)).astype(np.float32)
    # integer degree (multiplicity 1, or 2 on a raw self-loop): exact in float32 below 2^24
    deg = (torch.bincount(r_row, minlength=n) + torch.bincount(r_row[m == 2.0], minlength=n)).cpu().numpy()
    deg = deg.astype(np.float32)
    with np.errstate(divide="ignore"):
        r = (one / np.sqrt(deg)).astype(np.float32)
    r[np.isinf(r)] = 0
    nn_ = np.stack([dout_inv, din_inv, r, np.zeros(n, np.float32)], 1).astype(np.float32)
    node_norm = torch.from_numpy(np.ascontiguousarray(nn_)).to(dev)
    order = locality_schedule(n, s, d) if schedule else None
    return RawNgramCSR(n, rowptr, raw, node_norm, int(nnz), order)


def build_ngram_plan(g: CSRGraph, K: int = 20) -> Optional[NgramPlan]:
    """The n-gram tile plan of a shared-pattern device graph whose node ids are the base-K numbers of ALL K^n
    n-grams (n >= 2; the builder's sorted-string ids when every n-gram occurs), or None when the graph is not
    one (size not a power of K, or an entry that is neither a transition nor the diagonal -- counted by the
    plan kernel and checked here with one host sync, at build time)."""
    from . import ops
    if not g.shared or g.edges3 is None or not g.rowptr.is_cuda or g.n_rows < K * K:
        return None
    n = int(round(math.log(g.n_rows) / math.log(K)))
    if K ** n != g.n_rows:
        return None
    lib = ops.load_library()
    floats = int(lib.pg_ngram_plan_floats(K, n, g.n_rows))
    if floats < 0:
        return None
    plan = torch.empty(floats, dtype=torch.float32, device=g.rowptr.device)
    bad = torch.zeros(2, dtype=torch.int32, device=g.rowptr.device)
    ops.check(lib.pg_ngram_plan_f32(K, n, g.n_rows, ops._p(g.rowptr), ops._p(g.edges3), ops._p(plan), floats,
                                    ops._p(bad), ops._stream(plan)), "pg_ngram_plan_f32")
    mplan = None
    mfloats = int(lib.pg_ngram_mplan_floats(K, n, g.n_rows))
    if mfloats > 0:
        mplan = torch.empty(mfloats, dtype=torch.float32, device=g.rowptr.device)
        ops.check(lib.pg_ngram_mplan_f32(K, n, g.n_rows, ops._p(g.rowptr), ops._p(g.edges3), ops._p(mplan), mfloats,
                                         ops._p(bad[1:]), ops._stream(mplan)), "pg_ngram_mplan_f32")
    if int(bad[0].item()) != 0 or (mplan is not None and int(bad[1].item()) != 0):
        return None
    return NgramPlan(K, n, plan, mplan)


def _grid_rows(node_keys: torch.Tensor, alphabet: str, n: int, letters: str) -> torch.Tensor:
    """Grid row (base-len(letters) number over `letters`) of every node key (base-len(alphabet) number over
    `alphabet`'s code), -1 where a character is not one of `letters`."""
    Ka, Kg = max(len(alphabet), 1), len(letters)
    lut = torch.full((Ka,), -1, dtype=torch.int64)
    for code, ch in enumerate(alphabet):
        pos = letters.find(ch)
        if pos >= 0:
            lut[code] = pos
    lut = lut.to(node_keys.device)
    k = node_keys.to(torch.int64).clone()
    grid = torch.zeros_like(k)
    ok = torch.ones_like(k, dtype=torch.bool)
    scale = 1
    for _ in range(n):  # last character first
        d = lut[k % Ka]
        ok &= d >= 0
        grid += d.clamp(min=0) * scale
        scale *= Kg
        k //= Ka
    return torch.where(ok, grid, torch.full_like(grid, -1))


def build_ngram_map(g: CSRGraph, node_keys: torch.Tensor, alphabet: str, n: int, letters: str = GRID_LETTERS,
                    min_fill: float = 0.5) -> Optional[NgramMap]:
    """The mapped middle plan (NgramMap) of a shared-pattern device graph whose node i is the n-gram with key
    node_keys[i] (base-len(alphabet) digits in `alphabet`'s code, e.g. ngram.NgramTransitions), or None when the
    grid part is too small to pay (fewer than min_fill * 20^n nodes on the grid: the kernel walks the whole grid),
    or the graph is not shared-pattern on the GPU. Every CSR entry goes either to its grid slot or to the
    residual CSR, so the result covers the whole propagation; integer work only (torch sorts and one plan kernel)."""
    from . import ops
    K = len(letters)
    if (K != 20 or len(set(letters)) != K or not g.shared or g.edges3 is None or not g.rowptr.is_cuda or n < 2
            or node_keys.numel() != g.n_rows):
        return None
    grid_n = K ** n
    if grid_n >= 2 ** 31:
        return None
    dev = g.rowptr.device
    ginv = _grid_rows(node_keys.to(dev), alphabet, n, letters)
    on = ginv >= 0
    n_grid = int(on.sum())
    if n_grid < min_fill * grid_n:
        return None
    if n_grid and int(torch.unique(ginv[on]).numel()) != n_grid:
        raise ValueError("two nodes share one n-gram (node keys must be distinct)")
    gmap = torch.full((grid_n,), -1, dtype=torch.int32, device=dev)
    gmap[ginv[on]] = torch.nonzero(on).view(-1).to(torch.int32)
    ginv = ginv.to(torch.int32).contiguous()
    lib = ops.load_library()
    floats = int(lib.pg_ngram_mplan_floats(K, n, grid_n))
    mplan = torch.empty(floats, dtype=torch.float32, device=dev)
    resid = torch.empty(max(g.nnz, 1), dtype=torch.uint8, device=dev)
    ops.check(lib.pg_ngram_mplan_map_f32(K, n, g.n_rows, ops._p(g.rowptr), ops._p(g.edges3), ops._p(ginv),
                                         ops._p(mplan), floats, ops._p(resid), ops._stream(mplan)),
              "pg_ngram_mplan_map_f32")
    rmask = resid[:g.nnz].bool()
    rows = torch.repeat_interleave(torch.arange(g.n_rows, device=dev), g.rowptr[1:] - g.rowptr[:-1])
    res_edges = g.edges3[rmask].contiguous()  # CSR order kept: ascending column within a row
    cnt = torch.bincount(rows[rmask], minlength=g.n_rows)
    # listed rows: every node off the grid (even without entries: its Z row is written as 0), and the grid nodes with
    # residual entries; node order, so the compact CSR is the residual entries in their CSR order
    listed = (~on) | (cnt > 0)
    ids = torch.nonzero(listed).view(-1)
    res_rowptr = torch.zeros(ids.numel() + 1, dtype=torch.int64, device=dev)
    res_rowptr[1:] = torch.cumsum(cnt[ids], 0)
    add = on[ids]
    res_rows = torch.where(add, ids | (1 << 31), ids).to(torch.int64)
    res_rows = (res_rows - (res_rows >= 2 ** 31).to(torch.int64) * 2 ** 32).to(torch.int32)  # bit 31 as int32 sign
    n_acc = int(add.sum())
    return NgramMap(K, n, mplan, gmap, ginv, res_rowptr, res_rows.contiguous(), res_edges, n_grid,
                    int(res_edges.size(0)), int(ids.numel()) - n_acc, n_acc)


def attach_ngram_map(g: CSRGraph, transitions, letters: str = GRID_LETTERS, min_fill: float = 0.5) -> CSRGraph:
    """Attach the mapped middle plan to a graph of a builder-produced level (`transitions`: an
    ngram.NgramTransitions -- ngram_transitions, read_level or transitions_from_table -- whose node ids are the
    graph's rows). For the reference trainer's wiring (csr_from_coo on mathcal_A_*), pass the level the matrices
    were built from. A graph that already runs the complete-grid plan (g.ngram) is left as it is."""
    if g.ngram is None:
        g.ngram_map = build_ngram_map(g, transitions.node_keys, transitions.alphabet, transitions.n, letters,
                                      min_fill)
    return g


def build_propagation_csr(num_nodes: int, src, dst, cnt, device="cuda", eps: float = 1e-9,
                          keep_raw: bool = True, schedule: bool = True,
                          ngram_alphabet: Optional[int] = 20, transitions=None) -> CSRGraph:
    """Shared-pattern device CSR of (mathcal_A_in, mathcal_A_out, A_undirected_norm) from raw counts.

    Weights are materialised on the GPU by ``pg_edges_normalize_f32`` (bit-exact closed form of
    graph_utils.py:198-273 / :160-196). When the node set is all ngram_alphabet^n n-grams (node id = base-K
    number), the n-gram tile plan is attached as well (build_ngram_plan; None to skip). With `transitions` (the
    ngram.NgramTransitions of a builder-produced level these counts come from) a graph that is not the complete grid
    gets the mapped middle plan instead (attach_ngram_map)."""
    from . import ops

    if int(num_nodes) > 0 and np.asarray(src).size == 0:
        raise ValueError("graph without transitions: its mathcal_A_in/out are empty while A_undirected_norm "
                         "holds self-loops (no shared pattern); use csr_from_coo on the reference matrices")
    rc = ngram_raw_csr(num_nodes, src, dst, cnt, device=device, schedule=schedule)
    edges3 = ops.edges_normalize(rc, eps)
    g = CSRGraph(n_rows=rc.n, shared=True, rowptr=rc.rowptr, edges3=edges3, rowptr_t=rc.rowptr,
                 edges3_t=edges3, symmetric=True, raw=rc.raw if keep_raw else None,
                 node_norm=rc.node_norm if keep_raw else None, eps=eps, nnz=rc.nnz, row_order=rc.row_order)
    if ngram_alphabet and g.edges3.is_cuda:
        g.ngram = build_ngram_plan(g, ngram_alphabet)
        if g.ngram is None and transitions is not None:
            attach_ngram_map(g, transitions)
    return g
