"""Torch-facing wrappers of the C-ABI kernels and their autograd rules.

Forward passes run only in the HIP library (``libpgdgcn.so``) on the caller's current HIP stream.
Backward passes use the same library: the sparse transposed propagation (``pg_spmm3t_f32`` /
``pg_spmm1_f32``) and the dense layer backward (``pg_directgcn_dense_bwd_f32``; torch GPU ops only for
shapes it does not take, F_in or F_out not a multiple of 4). CPU tensors are rejected:
there is no CPU implementation of the product path.
"""
from __future__ import annotations

import ctypes
import functools
import weakref
from typing import Optional

import torch

from . import _lib
from ._lib import PG_FLAG_NGRAM_BLOCK4, PG_FLAG_NO_NGRAM, LayerArgs, check, default_flags, load_library
from .graph import CSRGraph, ShapedAdjacency

LEAKY_SLOPE = 0.01  # F.leaky_relu default, protgram_directgcn.py:215

# training-mode dropout after each layer (protgram_directgcn.py:216) fused into the dense epilogue: a counter-based
# draw (pg::drop_hash) instead of a separate dropout pass and its mask; the backward reads the mask off the layer
# output. False: F.dropout (torch's generator stream).
FUSED_DROPOUT = True

# training on complete n-gram graphs: PropagateDense (the span dense backward + the off-diagonal transposed kernel)
# for layers whose input needs its gradient; False: Propagate3 + LayerDense (the 4x4-block transposed kernel)
SPAN_BACKWARD = True
BF16_BACKWARD = True  # bf16 mode trains through pg_directgcn_dense_bwd_bf16 / pg_spmm3t_bf16
# Inference (no autograd) forwards gate the aggregates in the propagation's store (pg_spmm3_gated_f32) and run the
# dense kernel on the pre-gated operand; False = the training-path kernels in inference too.
PREGATED_INFERENCE = True

# Optional live timing of the hot-path kernels: when set to a list, each launch of that class appends one
# (start, end) pair of HIP events recorded on its launch stream around it (bench.py's per-kernel roofline):
SPMM_EVENTS: Optional[list] = None   # propagation (spmm3, spmm3_middles, spmm3_gated)
DENSE_EVENTS: Optional[list] = None  # dense layer (layer_dense, layer_dense_ngram_rows)
HEAD_EVENTS: Optional[list] = None   # fused head (head)


def _ev_start(x, kind: str = "SPMM"):
    if globals()[kind + "_EVENTS"] is None:
        return None
    e0 = torch.cuda.Event(enable_timing=True)
    e0.record(torch.cuda.current_stream(x.device))
    return e0


def _ev_end(x, e0, kind: str = "SPMM"):
    lst = globals()[kind + "_EVENTS"]
    if e0 is not None and lst is not None:
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record(torch.cuda.current_stream(x.device))
        lst.append((e0, e1))


def _require_graph_on(g, x):
    for t in g.tensors():
        if t.device != x.device:
            raise RuntimeError(f"graph tensors on {t.device} but features on {x.device}: move the graph "
                               "(CSRGraph.to) -- the kernels read both")


def _require_gpu(*ts):
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError("protgram_directgcn_amd runs on the MI355X only: got a CPU tensor "
                               "(move the model and data to 'cuda'; there is no CPU fallback)")
        if t.dtype not in (torch.float32, torch.bfloat16, torch.int32, torch.int64):
            raise TypeError(f"unsupported dtype {t.dtype}")


# Deferred bf16 gradients (train.train_step in bf16 mode with train.Adam and no GradScaler). The per-node constant's
# gradient is the layer's dpre (protgram_directgcn.py:130-133: the constant is added to the pre-activation), which
# the bf16 dense backward stores in bf16 for its weight gradient anyway; instead of a widened fp32 copy as
# constant.grad (written by the backward, read by Adam: 6 B per element per step, 0.74 GB at config 5), the layer
# backward leaves the constant's .grad None and files the bf16 dpre here, keyed by the parameter's address, and
# train.Adam reads it directly (pg_adam_desc_t.gtype = 1; exactly widened: the same update bits). train_step
# switches this on around its backward and optimizer step only, and empties the table after.
_DEFER_CONST_GRAD = False
_DEFERRED_GRADS: dict = {}


def deferred_grad(p: torch.Tensor) -> Optional[torch.Tensor]:
    """The bf16 gradient a layer backward filed for parameter p in this train_step (None if none)."""
    return _DEFERRED_GRADS.get(p.data_ptr()) if _DEFERRED_GRADS else None


def _defer_const(constant, need: bool, M: int, rows) -> bool:
    return (_DEFER_CONST_GRAD and need and constant is not None and constant.dtype == torch.float32 and rows is None
            and constant.dim() == 2 and constant.size(0) == M and constant.is_contiguous())


def _file_deferred(constant, dpre) -> bool:
    if not (_is_bf16(dpre) and dpre.is_contiguous() and dpre.shape == constant.shape):
        return False
    if constant.data_ptr() in _DEFERRED_GRADS:
        raise RuntimeError("a deferred gradient was filed twice for one parameter")
    _DEFERRED_GRADS[constant.data_ptr()] = dpre
    return True


def _p(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(t: torch.Tensor):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _f32c(t: torch.Tensor) -> torch.Tensor:
    return t.contiguous() if t.dtype == torch.float32 else t.float().contiguous()


def _bf16c(t: torch.Tensor) -> torch.Tensor:
    return t.contiguous() if t.dtype == torch.bfloat16 else t.to(torch.bfloat16).contiguous()


def _is_bf16(t) -> bool:
    return t is not None and t.dtype == torch.bfloat16


# ------------------------------------------------------------------------------------------------
# raw kernel calls
# ------------------------------------------------------------------------------------------------
def _ngram_ok(g: CSRGraph, x: torch.Tensor, fl: int, widths=(64, 128), dtype=torch.float32) -> bool:
    """The n-gram tile kernels take this call: the graph has a plan, x has the kernel's dtype, a supported width
    and exactly the graph's rows, and PG_FLAG_NO_NGRAM is not set."""
    return (g.ngram is not None and not (fl & PG_FLAG_NO_NGRAM) and x.dtype == dtype
            and x.size(0) == g.n_rows and x.size(1) in widths)


def _mid_ok(g: CSRGraph, x: torch.Tensor, fl: int) -> bool:
    """The middle-tile forward (pg_spmm3_ngram_mid_f32 / _bf16) takes this call: fp32 or bf16 x with the graph's rows,
    F a multiple of 16, a middle plan, and neither PG_FLAG_NO_NGRAM nor PG_FLAG_NGRAM_BLOCK4."""
    return (g.ngram is not None and g.ngram.mplan is not None and not (fl & (PG_FLAG_NO_NGRAM | PG_FLAG_NGRAM_BLOCK4))
            and x.dtype in (torch.float32, torch.bfloat16) and x.size(0) == g.n_rows and x.size(1) % 16 == 0)


def _ngram_fwd(lib, g, x, a, Z, fl, s):
    """Launch the n-gram forward (middle-tile kernel by default, 4x4-block kernel under PG_FLAG_NGRAM_BLOCK4 or where
    the middle kernel does not take the shape); returns the library's return code."""
    ng, N, F = g.ngram, g.n_rows, x.size(1)
    if _mid_ok(g, x, fl):
        rc = lib.pg_spmm3_ngram_mid_f32(ng.K, ng.n, N, _p(ng.mplan), _p(x), x.stride(0), F, a, _p(Z), Z.stride(0), fl, s)
        if rc != _lib.PG_ERR_UNSUPPORTED:
            return rc
    if _ngram_ok(g, x, fl, (64, 128, 256)):
        return lib.pg_spmm3_ngram_f32(ng.K, ng.n, N, _p(ng.plan), _p(x), x.stride(0), F, a, _p(Z), Z.stride(0), fl, s)
    return _lib.PG_ERR_UNSUPPORTED


def _map_ok(g: CSRGraph, x: torch.Tensor, fl: int) -> bool:
    """The mapped middle-tile forward (builder-produced graphs, g.ngram_map) takes this call: fp32 x with the graph's
    rows, F a multiple of 16, and PG_FLAG_NO_NGRAM not set."""
    return (g.ngram_map is not None and not (fl & PG_FLAG_NO_NGRAM) and x.dtype == torch.float32
            and x.size(0) == g.n_rows and x.size(1) % 16 == 0)


def _map_fwd(lib, g, x, Z, fl, s):
    """Mapped n-gram forward: the grid part by pg_spmm3_ngram_mid_map_f32, then one residual pass
    (pg_spmm3_resid_f32) over the off-grid rows (overwritten) and the grid rows with residual entries (added to).
    Returns the first non-zero return code (PG_ERR_UNSUPPORTED before anything launched: the caller falls back)."""
    m, F = g.ngram_map, x.size(1)
    rc = lib.pg_spmm3_ngram_mid_map_f32(m.K, m.n, _p(m.mplan), _p(m.gmap), _p(x), x.stride(0), F, _p(Z), Z.stride(0),
                                        fl, s)
    if rc:
        return rc
    if m.res_rows.numel():
        check(lib.pg_spmm3_resid_f32(m.res_rows.numel(), _p(m.res_rowptr), _p(m.res_rows), _p(m.res_edges), _p(x),
                                     x.stride(0), F, _p(Z), Z.stride(0), fl, s), "pg_spmm3_resid_f32")
    return 0


def spmm3(g: CSRGraph, x: torch.Tensor, out: Optional[torch.Tensor] = None, fused: bool = False,
          flags: Optional[int] = None) -> torch.Tensor:
    """Z = [A_in x | A_out x | A_und x] ([n_rows, 3F]) through the HIP kernels. bf16 x -> bf16 Z
    (pg_spmm3_bf16: fp32 sums, one rounding).

    Numerics: on a graph with an n-gram tile plan (g.ngram: every K^n n-gram present, attached by
    build_propagation_csr and csr_from_coo) the default is the tile kernel, which sums the same w*x terms in another
    order with FMAs: within |d| <= 1e-5 + 1e-5|ref| of the reference's propagate(), not bit-exact, and it applies
    0 * x for missing transitions, so x must be finite (an inf in a grid-adjacent row becomes NaN). Pass
    flags=default_flags() | PG_FLAG_NO_NGRAM for the CSR kernels: bit-exact to the reference and tolerant of
    non-finite inputs. Graphs without a plan (any other node set) always run the CSR kernels."""
    lib = load_library()
    if _is_bf16(x):
        return _spmm3_bf16(lib, g, x, out, fused, flags)
    x = _f32c(x)
    _require_gpu(x)
    _require_graph_on(g, x)
    N, F = g.n_rows, x.size(1)
    if x.size(0) < N:
        raise ValueError("x has fewer rows than the graph")
    Z = out if out is not None else torch.empty(N, 3 * F, device=x.device, dtype=torch.float32)
    fl = default_flags() if flags is None else flags
    s = _stream(x)
    ev = _ev_start(x)
    if g.shared and not fused and g.ngram is not None:
        rc = _ngram_fwd(lib, g, x, None, Z, fl, s)
        if rc != _lib.PG_ERR_UNSUPPORTED:  # unaligned operands / other widths: the CSR kernel below
            check(rc, "pg_spmm3_ngram_(mid_)f32")
            _ev_end(x, ev)
            return Z
    if g.shared and not fused and _map_ok(g, x, fl):  # builder-produced graphs: mapped middle-tile + residual
        rc = _map_fwd(lib, g, x, Z, fl, s)
        if rc != _lib.PG_ERR_UNSUPPORTED:
            check(rc, "pg_spmm3_ngram_mid_map_f32")
            _ev_end(x, ev)
            return Z
    if g.shared:
        if fused:
            if g.raw is None:
                raise ValueError("graph has no raw-count records (build it with build_propagation_csr)")
            check(lib.pg_spmm3_fusednorm_f32(N, _p(g.rowptr), _p(g.row_order), _p(g.raw), _p(g.node_norm), g.eps, _p(x),
                                             x.stride(0), F, _p(Z), Z.stride(0), fl, s), "pg_spmm3_fusednorm_f32")
        else:
            check(lib.pg_spmm3_f32(N, _p(g.rowptr), _p(g.row_order), _p(g.edges3), _p(x), x.stride(0), F, _p(Z),
                                   Z.stride(0), fl, s), "pg_spmm3_f32")
    else:
        for k, a in enumerate(g.adj):
            check(lib.pg_spmm1_f32(N, _p(a.rowptr), None, _p(a.edges), _p(x), x.stride(0), F, _p(Z[:, k * F:]),
                                   Z.stride(0), 0, fl, s), "pg_spmm1_f32")
    _ev_end(x, ev)
    return Z


def spmm3_middles(g: CSRGraph, x: torch.Tensor, m_begin: int, m_end: int, flags: Optional[int] = None,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """pg_spmm3_ngram_mid_rows_f32: Z = [A_in x | A_out x | A_und x] for the nodes a.M.b of the middles
    M in [m_begin, m_end) only, in middle-major order (row (M - m_begin) K^2 + a K + b), x in the global row layout
    (only the rows those middles read need be valid). The middle partition's per-rank propagation (shard.py).
    Needs g.ngram with a middle plan and fp32 or bf16 x (bf16 Z: pg_spmm3_ngram_mid_rows_bf16) with F % 16 == 0:
    raises otherwise (callers check `_mid_ok`)."""
    lib = load_library()
    bf = _is_bf16(x)
    x = _bf16c(x) if bf else _f32c(x)
    _require_gpu(x)
    _require_graph_on(g, x)
    fl = default_flags() if flags is None else flags
    if not _mid_ok(g, x, fl):
        raise ValueError("spmm3_middles needs a graph with a middle plan and fp32 x with F % 16 == 0")
    ng, N, F = g.ngram, g.n_rows, x.size(1)
    K2 = ng.K * ng.K
    rows = (m_end - m_begin) * K2
    Z = out if out is not None else torch.empty(rows, 3 * F, device=x.device, dtype=x.dtype)
    if Z.shape != (rows, 3 * F) or Z.stride(1) != 1 or Z.dtype != x.dtype:
        raise ValueError("out must be [(m_end - m_begin) K^2, 3F] of x's dtype with unit column stride")
    ev = _ev_start(x)
    fn = lib.pg_spmm3_ngram_mid_rows_bf16 if bf else lib.pg_spmm3_ngram_mid_rows_f32
    check(fn(ng.K, ng.n, N, _p(ng.mplan), _p(x), x.stride(0), F, m_begin, m_end, _p(Z), Z.stride(0), fl, _stream(x)),
          "pg_spmm3_ngram_mid_rows_" + ("bf16" if bf else "f32"))
    _ev_end(x, ev)
    return Z


_IDX_OK: dict = {}


def _check_index(idx: torch.Tensor, n: int, distinct: bool, what: str):
    """Range (and, for scatters, distinctness) check of a row-index tensor, once per tensor: the entry holds a weak
    reference, so a new tensor at a reused address never hits it. One host sync on a miss: callers that capture HIP
    graphs (shard.MiddleRunner) pass indices built and checked at setup with check=False instead."""
    k = (idx.data_ptr(), idx._version, idx.numel(), str(idx.device), int(n), bool(distinct))
    hit = _IDX_OK.get(k)
    if hit is not None and hit() is idx:
        return
    if idx.numel():
        lo, hi = int(idx.min()), int(idx.max())
        if lo < 0 or hi >= n:
            raise IndexError(f"{what}: row indices in [{lo}, {hi}] outside [0, {n})")
        if distinct and int(torch.unique(idx).numel()) != idx.numel():
            raise ValueError(f"{what}: indices must be distinct (each destination row written once)")
    if len(_IDX_OK) > 256:
        _IDX_OK.clear()
    _IDX_OK[k] = weakref.ref(idx)


def rows_gather(src: torch.Tensor, idx: torch.Tensor, out: Optional[torch.Tensor] = None,
                check_idx: bool = True) -> torch.Tensor:
    """out[i] = src[idx[i]] (pg_rows_gather; rows of any dtype, unit column stride). The indices are range-checked
    once per index tensor (IndexError); check_idx=False skips that (indices known valid, e.g. inside a capture)."""
    lib = load_library()
    _require_gpu(src)
    if src.dim() != 2 or src.stride(1) != 1:
        raise ValueError("rows_gather needs a 2-D source with unit column stride")
    idx = idx.to(device=src.device, dtype=torch.int64).contiguous()
    if check_idx:
        _check_index(idx, src.size(0), False, "rows_gather")
    out = out if out is not None else torch.empty(idx.numel(), src.size(1), device=src.device, dtype=src.dtype)
    if out.shape != (idx.numel(), src.size(1)) or out.dtype != src.dtype or out.stride(1) != 1:
        raise ValueError("rows_gather: out must be [len(idx), src.size(1)] of src's dtype")
    es = src.element_size()
    check(lib.pg_rows_gather(_p(src), src.stride(0) * es, _p(idx), idx.numel(), src.size(1) * es, _p(out),
                             out.stride(0) * es, _stream(src)), "pg_rows_gather")
    return out


def rows_scatter(src: torch.Tensor, idx: torch.Tensor, dst: torch.Tensor, check_idx: bool = True) -> torch.Tensor:
    """dst[idx[i]] = src[i] (pg_rows_scatter; distinct indices; rows of any dtype, unit column stride). The indices
    are checked once per index tensor for range (IndexError) and distinctness (ValueError); check_idx=False skips
    that (indices known valid, e.g. inside a capture)."""
    lib = load_library()
    _require_gpu(src)
    if src.dim() != 2 or dst.dim() != 2 or src.size(1) != dst.size(1) or src.dtype != dst.dtype:
        raise ValueError("rows_scatter: src and dst must be 2-D of the same width and dtype")
    if src.stride(1) != 1 or dst.stride(1) != 1 or idx.numel() != src.size(0):
        raise ValueError("rows_scatter: unit column strides and one index per source row")
    idx = idx.to(device=src.device, dtype=torch.int64).contiguous()
    if check_idx:
        _check_index(idx, dst.size(0), True, "rows_scatter")
    es = src.element_size()
    check(lib.pg_rows_scatter(_p(src), src.stride(0) * es, _p(idx), idx.numel(), src.size(1) * es, _p(dst),
                              dst.stride(0) * es, _stream(src)), "pg_rows_scatter")
    return dst


def rows_gather_sum(A: Optional[torch.Tensor], rowptr: torch.Tensor, idx: torch.Tensor, n_out: int, F: int,
                    B: Optional[torch.Tensor] = None, out_dtype=torch.float32) -> torch.Tensor:
    """pg_rows_gather_sum: out[i] = sum over e in [rowptr[i], rowptr[i+1]) of (A[idx[e]] if idx[e] >= 0 else
    B[-1 - idx[e]]), in entry order, in fp32; A fp32, B fp32 or bf16, out fp32 or bf16 (one rounding). rowptr int64
    [n_out + 1], idx int32 -- lists built and range-checked by their owner (shard.middle_scatter)."""
    lib = load_library()
    ref = A if A is not None else B
    _require_gpu(ref)
    for t in (A, B):
        if t is not None and (t.dim() != 2 or t.stride(1) != 1 or t.size(1) < F):
            raise ValueError("rows_gather_sum: 2-D sources with unit column stride and >= F columns")
    if A is not None and A.dtype != torch.float32:
        raise ValueError("rows_gather_sum: A must be fp32")
    b_bf = B is not None and _is_bf16(B)
    if B is not None and not b_bf and B.dtype != torch.float32:
        raise ValueError("rows_gather_sum: B must be fp32 or bf16")
    if rowptr.dtype != torch.int64 or idx.dtype != torch.int32 or rowptr.numel() != n_out + 1:
        raise ValueError("rows_gather_sum: int64 rowptr of n_out + 1 entries and int32 idx")
    o_bf = out_dtype == torch.bfloat16
    if not o_bf and out_dtype != torch.float32:
        raise ValueError("rows_gather_sum: out_dtype fp32 or bf16")
    out = torch.empty(n_out, F, device=ref.device, dtype=out_dtype)
    check(lib.pg_rows_gather_sum(_p(A), A.stride(0) if A is not None else F, _p(B),
                                 B.stride(0) if B is not None else F, int(b_bf), _p(rowptr), _p(idx), n_out, F,
                                 _p(out), out.stride(0), int(o_bf), _stream(ref)), "pg_rows_gather_sum")
    return out


def ngram_scatter_plan(g: CSRGraph, m_begin: int, m_end: int) -> torch.Tensor:
    """pg_ngram_scatter_plan: the transposed-fragment plan [m_end - m_begin, 78,000] fp32 of the middles
    [m_begin, m_end) (from g.ngram's middle plan; setup work, once per partition)."""
    lib = load_library()
    ng = g.ngram
    if ng is None or ng.mplan is None:
        raise ValueError("ngram_scatter_plan needs a graph with a middle plan")
    _require_gpu(ng.mplan)
    sp = torch.empty(m_end - m_begin, SCATTER_PLAN_FLOATS, device=ng.mplan.device, dtype=torch.float32)
    check(lib.pg_ngram_scatter_plan(ng.K, ng.n, _p(ng.mplan), m_begin, m_end - m_begin, _p(sp), _stream(sp)),
          "pg_ngram_scatter_plan")
    return sp


SCATTER_PLAN_FLOATS = 78_000


def spmm3t_scatter(splan: torch.Tensor, G: torch.Tensor, flags: Optional[int] = None) -> torch.Tensor:
    """pg_spmm3t_ngram_scatter_f32 / _bf16: T [3 n_own, F] fp32 = the D / P / S parts of sum_k A_k^T G_k that a
    middle-partition rank's owned rows send (include/pg_directgcn.h); G [n_own, 3F] (fp32 or bf16, owned rows in
    middle-major order), n_own = 400 * splan.size(0), F % 16 == 0."""
    lib = load_library()
    bf = _is_bf16(G)
    G = _bf16c(G) if bf else _f32c(G)
    _require_gpu(G, splan)
    n_mid = splan.size(0)
    if splan.dim() != 2 or splan.size(1) != SCATTER_PLAN_FLOATS or splan.dtype != torch.float32:
        raise ValueError("spmm3t_scatter: splan must be [n_mid, 78000] fp32 (ngram_scatter_plan)")
    n_own = 400 * n_mid
    if G.dim() != 2 or G.size(0) != n_own or G.size(1) % 48:
        raise ValueError("spmm3t_scatter: G must be [400 n_mid, 3F] with F % 16 == 0")
    F = G.size(1) // 3
    T = torch.empty(3 * n_own, F, device=G.device, dtype=torch.float32)
    fl = default_flags() if flags is None else flags
    fn = lib.pg_spmm3t_ngram_scatter_bf16 if bf else lib.pg_spmm3t_ngram_scatter_f32
    check(fn(_p(splan), n_mid, _p(G), G.stride(0), F, _p(T), T.stride(0), fl, _stream(G)),
          "pg_spmm3t_ngram_scatter_" + ("bf16" if bf else "f32"))
    return T


def _spmm3_bf16(lib, g: CSRGraph, x, out, fused, flags):
    x = _bf16c(x)
    _require_gpu(x)
    _require_graph_on(g, x)
    N, F = g.n_rows, x.size(1)
    if x.size(0) < N:
        raise ValueError("x has fewer rows than the graph")
    if g.shared and not fused:
        Z = out if out is not None else torch.empty(N, 3 * F, device=x.device, dtype=torch.bfloat16)
        fl = default_flags() if flags is None else flags
        ev = _ev_start(x)
        if _mid_ok(g, x, fl):  # complete n-gram graphs: the middle-tile kernel on bf16 rows
            ng = g.ngram
            rc = lib.pg_spmm3_ngram_mid_bf16(ng.K, ng.n, N, _p(ng.mplan), _p(x), x.stride(0), F, _p(Z), Z.stride(0),
                                             fl, _stream(x))
            if rc != _lib.PG_ERR_UNSUPPORTED:
                check(rc, "pg_spmm3_ngram_mid_bf16")
                _ev_end(x, ev)
                return Z
        rc = lib.pg_spmm3_bf16(N, _p(g.rowptr), _p(g.row_order), _p(g.edges3), _p(x), x.stride(0), F, _p(Z),
                               Z.stride(0), fl, _stream(x))
        if rc != _lib.PG_ERR_UNSUPPORTED:
            check(rc, "pg_spmm3_bf16")
            _ev_end(x, ev)
            return Z
    # shapes / graph kinds without a bf16 kernel: the fp32 kernels on the widened input, one rounding
    Z = spmm3(g, x.float(), fused=fused, flags=flags).to(torch.bfloat16)
    if out is not None:
        out.copy_(Z)
        return out
    return Z


def spmm3_gated(g: CSRGraph, x: torch.Tensor, prm: dict, gate_mode: int, flags: Optional[int] = None,
                out: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """pg_spmm3_gated_f32: Z_q = s_q * (A_q x) with the layer's gates applied at the store -- the operand of
    layer_dense(..., pregated=True). fp32, shared pattern, precomputed weights only; None otherwise (callers
    then gate inside the dense kernel)."""
    if _is_bf16(x) or not g.shared or g.edges3 is None:
        return None
    fl = default_flags() if flags is None else flags
    if _mid_ok(g, x, fl) or _map_ok(g, x, fl):  # the middle-tile kernels have no gated store: the dense kernel gates
        return None
    lib = load_library()
    x = _f32c(x)
    _require_gpu(x)
    _require_graph_on(g, x)
    N, F = g.n_rows, x.size(1)
    if x.size(0) < N:
        raise ValueError("x has fewer rows than the graph")
    Z = out if out is not None else torch.empty(N, 3 * F, device=x.device, dtype=torch.float32)
    a, keep = _layer_args(None, prm, gate_mode, M=N)
    ev = _ev_start(x)
    if g.ngram is not None:
        rc = _ngram_fwd(lib, g, x, ctypes.byref(a), Z, fl, _stream(x))
        if rc != _lib.PG_ERR_UNSUPPORTED:
            check(rc, "pg_spmm3_ngram_(mid_)f32")
            _ev_end(x, ev)
            del keep
            return Z
    check(lib.pg_spmm3_gated_f32(N, _p(g.rowptr), _p(g.row_order), _p(g.edges3), _p(x), x.stride(0), F,
                                 ctypes.byref(a), _p(Z), Z.stride(0), fl, _stream(x)), "pg_spmm3_gated_f32")
    _ev_end(x, ev)
    del keep
    return Z


def spmm3t_ngram_acc_bf16(g: CSRGraph, G: torch.Tensor, dX: torch.Tensor, flags: Optional[int] = None,
                          src: Optional[torch.Tensor] = None):
    """dX += sum_k A_k^T G[:, kF:(k+1)F] in place for bf16 G and dX on the 4x4-block transposed n-gram kernel
    (pg_spmm3t_ngram_bf16 with accumulate: the sum in fp32, dX rounded once), or None when that kernel does not take
    the call (the caller adds instead). Used by PropagateDense in bf16 mode: dX = the identity residual's dpre + the
    transposed propagation, one launch and one rounding where autograd ran the kernel and a bf16 add. src: the
    addend read from its own rows instead (dX = src + ..., pg_spmm3t_ngram_add_bf16; src is left as it was)."""
    fl = default_flags() if flags is None else flags
    if not (_is_bf16(G) and _is_bf16(dX) and G.is_contiguous() and dX.is_contiguous() and g.shared and g.symmetric
            and G.size(0) == g.n_rows and dX.size(1) * 3 == G.size(1)
            and _ngram_ok(g, dX, fl, (64, 128, 256), torch.bfloat16)):
        return None
    if src is not None and not (_is_bf16(src) and src.is_contiguous() and src.shape == dX.shape):
        return None
    _require_gpu(G, dX)
    _require_graph_on(g, G)
    lib, ng, F = load_library(), g.ngram, dX.size(1)
    if src is not None:
        rc = lib.pg_spmm3t_ngram_add_bf16(ng.K, ng.n, g.n_rows, _p(ng.plan), _p(G), G.stride(0), F, _p(src),
                                          src.stride(0), _p(dX), dX.stride(0), fl, _stream(G))
        name = "pg_spmm3t_ngram_add_bf16"
    else:
        rc = lib.pg_spmm3t_ngram_bf16(ng.K, ng.n, g.n_rows, _p(ng.plan), _p(G), G.stride(0), F, _p(dX), dX.stride(0),
                                      1, fl, _stream(G))
        name = "pg_spmm3t_ngram_bf16"
    if rc == _lib.PG_ERR_UNSUPPORTED:
        return None
    check(rc, name)
    return dX


def spmm3_t(g: CSRGraph, G: torch.Tensor, flags: Optional[int] = None) -> torch.Tensor:
    """dX = sum_k A_k^T G[:, kF:(k+1)F] (transposed propagation, backward of spmm3). bf16 G -> bf16 dX.
    Same numerics note as spmm3: the n-gram tile kernels (symmetric graphs with a plan: the off-diagonal transposed
    middle-tile kernel + the diagonal term under PG_FLAG_MID_TRANSPOSED, else the 4x4-block one for F in
    {64, 128, 256}) need finite G and match the CSR kernel within fp32 rounding; PG_FLAG_NO_NGRAM selects the CSR kernel (under AMP, GradScaler's scaled
    gradients can overflow to inf: the step is skipped either way, but the skipped values differ)."""
    lib = load_library()
    if _is_bf16(G):
        G = _bf16c(G)
        _require_gpu(G)
        _require_graph_on(g, G)
        N, F = (g.n_cols if g.n_cols is not None else g.n_rows), G.size(1) // 3
        if g.shared:
            dX = torch.empty(N, F, device=G.device, dtype=torch.bfloat16)
            ro = g.row_order if g.symmetric else None
            fl = default_flags() if flags is None else flags
            if g.symmetric and G.size(0) == g.n_rows and (fl & _lib.PG_FLAG_MID_TRANSPOSED) and _mid_ok(g, dX, fl):
                # the transposed middle-tile kernel, diagonal included (bf16 rows leave it room); opt-in: slower than the
                # 4x4-block bf16 kernel (0.164 vs 0.112 ms at B(20,4), F = 128)
                ng = g.ngram
                rc = lib.pg_spmm3t_ngram_mid_bf16(ng.K, ng.n, N, _p(ng.mplan), _p(G), G.stride(0), F, _p(dX),
                                                  dX.stride(0), 0, fl, _stream(G))
                if rc != _lib.PG_ERR_UNSUPPORTED:
                    check(rc, "pg_spmm3t_ngram_mid_bf16")
                    return dX
            if g.symmetric and G.size(0) == g.n_rows and _ngram_ok(g, dX, fl, (64, 128, 256), torch.bfloat16):
                ng = g.ngram
                rc = lib.pg_spmm3t_ngram_bf16(ng.K, ng.n, N, _p(ng.plan), _p(G), G.stride(0), F, _p(dX), dX.stride(0), 0,
                                              fl, _stream(G))
                if rc != _lib.PG_ERR_UNSUPPORTED:
                    check(rc, "pg_spmm3t_ngram_bf16")
                    return dX
            rc = lib.pg_spmm3t_bf16(N, _p(g.rowptr_t), _p(ro), _p(g.edges3_t), _p(G), G.stride(0), F, _p(dX),
                                    dX.stride(0), fl, _stream(G))
            if rc != _lib.PG_ERR_UNSUPPORTED:
                check(rc, "pg_spmm3t_bf16")
                return dX
        return spmm3_t(g, G.float(), flags).to(torch.bfloat16)
    G = _f32c(G)
    _require_gpu(G)
    _require_graph_on(g, G)
    N, F = (g.n_cols if g.n_cols is not None else g.n_rows), G.size(1) // 3
    dX = torch.empty(N, F, device=G.device, dtype=torch.float32)
    fl = default_flags() if flags is None else flags
    s = _stream(G)
    if g.shared and g.symmetric and G.size(0) == g.n_rows and (fl & _lib.PG_FLAG_MID_TRANSPOSED) and _mid_ok(g, dX, fl):
        # the off-diagonal middle-tile kernel + the diagonal term here (opt-in: the extra pass over G costs more than
        # the kernel saves against the 4x4-block kernel)
        rc = _offdiag(lib, g, G, dX, False, fl, s)
        if rc != _lib.PG_ERR_UNSUPPORTED:
            check(rc, "pg_spmm3t_ngram_mid_offdiag_f32")
            d3 = g.ngram.diag3()
            dX += (G[:, :3 * F].view(N, 3, F) * d3.unsqueeze(2)).sum(1)
            return dX
    if g.shared and g.symmetric and G.size(0) == g.n_rows and _ngram_ok(g, dX, fl, (64, 128, 256)):
        ng = g.ngram
        rc = lib.pg_spmm3t_ngram_f32(ng.K, ng.n, N, _p(ng.plan), _p(G), G.stride(0), F, _p(dX), dX.stride(0), 0, fl, s)
        if rc != _lib.PG_ERR_UNSUPPORTED:
            check(rc, "pg_spmm3t_ngram_f32")
            return dX
    if g.shared:
        ro = g.row_order if g.symmetric else None
        check(lib.pg_spmm3t_f32(N, _p(g.rowptr_t), _p(ro), _p(g.edges3_t), _p(G), G.stride(0), F, _p(dX), dX.stride(0), 0,
                                fl, s), "pg_spmm3t_f32")
    else:
        for k, a in enumerate(g.adj):
            check(lib.pg_spmm1_f32(N, _p(a.rowptr_t), None, _p(a.edges_t), _p(G[:, k * F:]), G.stride(0), F, _p(dX),
                                   dX.stride(0), 1 if k else 0, fl, s), "pg_spmm1_f32")
    return dX


def _offdiag(lib, g: CSRGraph, G, dX, accumulate: bool, fl: int, s) -> int:
    ng = g.ngram
    return lib.pg_spmm3t_ngram_mid_offdiag_f32(ng.K, ng.n, g.n_rows, _p(ng.mplan), _p(G), G.stride(0), G.size(1) // 3,
                                               _p(dX), dX.stride(0), 1 if accumulate else 0, fl, s)


def spmm3t_offdiag(g: CSRGraph, G: torch.Tensor, out: Optional[torch.Tensor] = None, flags: Optional[int] = None):
    """dX = sum_k (A_k - Diag_k) G_k (+ out when given: accumulated into it) by the off-diagonal transposed middle-tile
    kernel (pg_spmm3t_ngram_mid_offdiag_f32; fp32, a complete n-gram graph with a middle plan, F % 16 == 0);
    Diag_k = g.ngram.diag3()[:, k]. None when the kernel does not take the call (the caller then runs spmm3_t)."""
    lib = load_library()
    if _is_bf16(G) or not (g.shared and g.symmetric and g.ngram is not None and g.ngram.mplan is not None):
        return None
    G = _f32c(G)
    _require_gpu(G)
    _require_graph_on(g, G)
    N, F = g.n_rows, G.size(1) // 3
    if G.size(0) != N or F % 16:
        return None
    acc = out is not None
    dX = out if acc else torch.empty(N, F, device=G.device, dtype=torch.float32)
    if dX.dtype != torch.float32 or dX.shape != (N, F) or dX.stride(1) != 1:
        raise ValueError("spmm3t_offdiag: out must be fp32 [N, F] with unit column stride")
    fl = default_flags() if flags is None else flags
    rc = _offdiag(lib, g, G, dX, acc, fl, _stream(G))
    if rc == _lib.PG_ERR_UNSUPPORTED:
        return None
    check(rc, "pg_spmm3t_ngram_mid_offdiag_f32")
    return dX


def spmm3t_rows(rowptr_t: torch.Tensor, edges3_t: torch.Tensor, rows: torch.Tensor, G: torch.Tensor, n_out: int,
                flags: Optional[int] = None) -> torch.Tensor:
    """dX[r] = sum_e (w_in G[col, 0:F] + w_out G[col, F:2F] + w_und G[col, 2F:3F]) for the rows r in `rows` (int32)
    of a transposed CSR over n_out rows (pg_spmm3t_f32 / pg_spmm3t_bf16 with `rows` as the row order); the other rows
    of the [n_out, F] result are left unwritten. The middle trainer's propagation backward (shard.MiddleTranspose)."""
    lib = load_library()
    bf = _is_bf16(G)
    G = _bf16c(G) if bf else _f32c(G)
    _require_gpu(G, rowptr_t, edges3_t, rows)
    if rows.dtype != torch.int32 or rowptr_t.numel() != n_out + 1:
        raise ValueError("spmm3t_rows: int32 rows and a rowptr of n_out + 1 entries")
    F = G.size(1) // 3
    dX = torch.empty(n_out, F, device=G.device, dtype=G.dtype)
    fl = default_flags() if flags is None else flags
    if bf:
        check(lib.pg_spmm3t_bf16(rows.numel(), _p(rowptr_t), _p(rows), _p(edges3_t), _p(G), G.stride(0), F, _p(dX),
                                 dX.stride(0), fl, _stream(G)), "pg_spmm3t_bf16")
    else:
        check(lib.pg_spmm3t_f32(rows.numel(), _p(rowptr_t), _p(rows), _p(edges3_t), _p(G), G.stride(0), F, _p(dX),
                                dX.stride(0), 0, fl, _stream(G)), "pg_spmm3t_f32")
    return dX


def spmm1(a: ShapedAdjacency, x: torch.Tensor, transpose: bool = False, flags: Optional[int] = None) -> torch.Tensor:
    lib = load_library()
    x = _f32c(x)
    _require_gpu(x)
    if a.rowptr.device != x.device:
        raise RuntimeError(f"adjacency on {a.rowptr.device} but features on {x.device}")
    N = a.rowptr.numel() - 1
    Y = torch.empty(N, x.size(1), device=x.device, dtype=torch.float32)
    rp, e = (a.rowptr_t, a.edges_t) if transpose else (a.rowptr, a.edges)
    fl = default_flags() if flags is None else flags
    check(lib.pg_spmm1_f32(N, _p(rp), None, _p(e), _p(x), x.stride(0), x.size(1), _p(Y), Y.stride(0), 0, fl,
                           _stream(x)), "pg_spmm1_f32")
    return Y


def edges_normalize(rc, eps: float) -> torch.Tensor:
    """Precomputed {col, w_in, w_out, w_und} records from raw-count records, on the GPU."""
    lib = load_library()
    _require_gpu(rc.raw)
    out = torch.empty_like(rc.raw)
    check(lib.pg_edges_normalize_f32(rc.n, _p(rc.rowptr), _p(rc.raw), _p(rc.node_norm), eps, _p(out),
                                     _stream(rc.raw)), "pg_edges_normalize_f32")
    return out


def pack_weights(prm: dict, W_res=None, b_res=None) -> torch.Tensor:
    """pg_directgcn_pack_f32: [W_mi+W_s | W_mo+W_s | W_u+W_s (| W_res)] + bias sums, packed on every call
    (~5 us). Deliberately not cached: parameters updated by fused optimizers (torch's fused Adam, raw
    kernels) keep their version counter, so a version-keyed cache would serve stale weights."""
    srcs = [prm[k] for k in _PACK_KEYS] + [W_res, b_res]
    lib = load_library()
    F_out, F_in = prm["W_main_in"].shape
    n = lib.pg_directgcn_packed_floats(F_in, F_out, 1 if W_res is not None else 0)
    out = torch.empty(n, device=prm["W_main_in"].device, dtype=torch.float32)
    keep = [_f32c(t.detach()) if t is not None else None for t in srcs]
    a = LayerArgs()
    a.F_in, a.F_out = F_in, F_out
    (a.W_main_in, a.W_main_out, a.W_undirected, a.W_shared, a.b_main_in, a.b_dir_shared_in, a.b_main_out,
     a.b_dir_shared_out, a.b_undirected, a.b_undirected_shared, a.W_res, a.b_res) = [_p(t) for t in keep]
    check(lib.pg_directgcn_pack_f32(ctypes.byref(a), _p(out), _stream(out)), "pg_directgcn_pack_f32")
    return out


def pack_weights_bf16(prm: dict, W_res=None, b_res=None):
    """(fp32 packed operand, its bf16 copy [F_out*K]) for pg_directgcn_dense_bf16 (packed per call, as
    pack_weights)."""
    packed = pack_weights(prm, W_res, b_res)
    lib = load_library()
    F_out, F_in = prm["W_main_in"].shape
    n = F_out * (4 if W_res is not None else 3) * F_in
    out = torch.empty(n, device=packed.device, dtype=torch.bfloat16)
    check(lib.pg_f32_to_bf16(n, _p(packed), _p(out), _stream(packed)), "pg_f32_to_bf16")
    return packed, out


def clear_caches():
    """Drop the COO->CSR cache (graphs are cached by the identity + version of their COO tensors)."""
    from .graph import clear_cache
    clear_cache()


_PACK_KEYS = ("W_main_in", "W_main_out", "W_undirected", "W_shared", "b_main_in", "b_dir_shared_in",
              "b_main_out", "b_dir_shared_out", "b_undirected", "b_undirected_shared")


def _layer_args(Z, prm: dict, gate_mode: int, rows=None, constant=None, res_x=None, W_res=None,
                act: bool = False, slope: float = LEAKY_SLOPE, Y=None, M: Optional[int] = None, drop=None):
    """pg_layer_args_t for the forward block; returns (args, keep-alive list). Z=None (gate-only uses) takes the
    row count from M. drop = (p, seed): the fused layer dropout (seed: device int64 [1]; None in the backward)."""
    if Z is None:
        M, F_in = int(M), prm["W_main_in"].size(1)
    else:
        M, F_in = Z.size(0), Z.size(1) // 3
    F_out = prm["W_main_in"].size(0)
    keep = []

    def c(t):
        if t is None:
            return None
        t = _f32c(t.detach()) if t.dtype != torch.int64 else t.contiguous()
        keep.append(t)
        return _p(t)

    a = LayerArgs()
    a.M, a.F_in, a.F_out = M, F_in, F_out
    b16 = Z is not None and _is_bf16(Z)
    if Z is not None:
        Zc = _bf16c(Z.detach()) if b16 else _f32c(Z.detach())
        keep.append(Zc)
        a.Z, a.ldz = _p(Zc), Zc.stride(0)
    a.gate_mode = gate_mode
    a.C_in, a.C_out, a.C_directed = c(prm["C_in"]), c(prm["C_out"]), c(prm["C_directed"])
    a.C_undirected, a.C_all = c(prm["C_undirected"]), c(prm["C_all"])
    a.rows = c(rows)
    if constant is not None:
        a.constant, a.ld_const = c(constant), constant.size(1)
    if res_x is not None:
        rx = _bf16c(res_x.detach()) if b16 else _f32c(res_x.detach())
        keep.append(rx)
        a.res_x, a.ld_res = _p(rx), rx.stride(0)
    a.W_res = c(W_res)
    a.act, a.slope = int(bool(act)), float(slope)
    if drop is not None and drop[0] > 0:
        a.drop_p = float(drop[0])
        if drop[1] is not None:
            if drop[1].dtype != torch.int64 or not drop[1].is_cuda or drop[1].numel() < 1:
                raise ValueError("the dropout seed must be a device int64 tensor")
            keep.append(drop[1])
            a.drop_seed = _p(drop[1])
    if Y is not None:
        Yc = Y.detach().contiguous()
        keep.append(Yc)
        a.Y, a.ldy = _p(Yc), Yc.stride(0)
    return a, keep


def layer_dense(Z, prm: dict, gate_mode: int, rows=None, constant=None, res_x=None, W_res=None, b_res=None,
                act: bool = False, slope: float = LEAKY_SLOPE, flags: Optional[int] = None,
                out: Optional[torch.Tensor] = None, pregated: bool = False, packs: Optional[list] = None,
                drop=None) -> torch.Tensor:
    """pg_directgcn_dense_f32: gated contraction of the aggregates + epilogue (see the header). bf16 Z ->
    pg_directgcn_dense_bf16 (bf16 output; `packs`, when given, receives its packed weights (fp32, bf16) so that the
    backward of the same step reuses them). drop = (p, seed [1] int64 on the device): the layer's dropout after the
    activation, fused into the epilogue (pg::drop_hash; act required)."""
    lib = load_library()
    _require_gpu(Z)
    if _is_bf16(Z):
        Y = _layer_dense_bf16(Z, prm, gate_mode, rows, constant, res_x, W_res, b_res, act, slope, flags, packs, drop)
        if Y is None:
            Y = layer_dense(Z.float(), prm, gate_mode, rows, constant, None if res_x is None else res_x.float(),
                            W_res, b_res, act, slope, flags, drop=drop).to(torch.bfloat16)
        if out is not None:
            out.copy_(Y)
            return out
        return Y
    M = Z.size(0)
    F_out = prm["W_main_in"].size(0)
    if out is not None:
        if out.shape != (M, F_out) or out.dtype != torch.float32 or out.stride(1) != 1 or out.device != Z.device:
            raise ValueError("out must be a row-major fp32 [M, F_out] tensor on Z's device")
        Y = out
    else:
        Y = torch.empty(M, F_out, device=Z.device, dtype=torch.float32)
    a, keep = _layer_args(Z, prm, gate_mode, rows, constant, res_x, W_res, act, slope, drop=drop)
    a.Y, a.ldy = _p(Y), Y.stride(0)
    fl = default_flags() if flags is None else flags
    if pregated:
        fl |= _lib.PG_FLAG_DENSE_PREGATED
    if W_res is None and rows is None:
        # unpacked weights: the pipelined split-bf16 kernel sums W_q + W_shared itself (no pack launch); any other
        # kernel choice answers PG_ERR_UNSUPPORTED without launching, and the packed call below runs instead
        raw = [_f32c(prm[k].detach()) for k in _PACK_KEYS]
        (a.W_main_in, a.W_main_out, a.W_undirected, a.W_shared, a.b_main_in, a.b_dir_shared_in, a.b_main_out,
         a.b_dir_shared_out, a.b_undirected, a.b_undirected_shared) = [_p(t) for t in raw]
        ev = _ev_start(Z, "DENSE")
        rc = lib.pg_directgcn_dense_f32(ctypes.byref(a), None, fl, _stream(Z))
        if rc != _lib.PG_ERR_UNSUPPORTED:
            check(rc, "pg_directgcn_dense_f32")
            _ev_end(Z, ev, "DENSE")
            del keep, raw
            return Y
    packed = pack_weights(prm, W_res, b_res)
    ev = _ev_start(Z, "DENSE")
    check(lib.pg_directgcn_dense_f32(ctypes.byref(a), _p(packed), fl, _stream(Z)), "pg_directgcn_dense_f32")
    _ev_end(Z, ev, "DENSE")
    del keep
    return Y


def layer_dense_ngram_rows(Z, prm: dict, gate_mode: int, Kn1: int, m0: int, constant=None, res_x=None,
                           map_res: bool = False, out: Optional[torch.Tensor] = None, map_out: bool = False,
                           act: bool = False, slope: float = LEAKY_SLOPE, flags: Optional[int] = None):
    """pg_directgcn_dense_ngram_rows_f32: layer_dense over the middle-major rows of the middles m0, m0 + 1, ...
    (spmm3_middles' rows), with the residual rows read (map_res) and / or the output rows written (map_out) at their
    global n-gram rows of res_x / out (Kn1 = K^(n-1)). Returns the output tensor (out when map_out), or None when
    the shape is not the pipelined split-bf16 kernel's (fp32, F_in = F_out = 128, identity residual): the caller
    then runs layer_dense on gathered rows."""
    lib = load_library()
    _require_gpu(Z)
    if _is_bf16(Z) or Z.dtype != torch.float32:
        return None
    M = Z.size(0)
    F_out = prm["W_main_in"].size(0)
    if map_out:
        if out is None or out.dtype != torch.float32 or out.stride(1) != 1 or out.size(1) != F_out:
            raise ValueError("map_out needs a row-major fp32 out [n_rows, F_out] in the global row layout")
        Y = out
    elif out is not None:
        if out.shape != (M, F_out) or out.dtype != torch.float32 or out.stride(1) != 1 or out.device != Z.device:
            raise ValueError("out must be a row-major fp32 [M, F_out] tensor on Z's device")
        Y = out
    else:
        Y = torch.empty(M, F_out, device=Z.device, dtype=torch.float32)
    if map_res and (res_x is None or res_x.dtype != torch.float32):
        return None
    a, keep = _layer_args(Z, prm, gate_mode, None, constant, res_x, None, act, slope)
    a.Y, a.ldy = _p(Y), Y.stride(0)
    raw = [_f32c(prm[k].detach()) for k in _PACK_KEYS]
    (a.W_main_in, a.W_main_out, a.W_undirected, a.W_shared, a.b_main_in, a.b_dir_shared_in, a.b_main_out,
     a.b_dir_shared_out, a.b_undirected, a.b_undirected_shared) = [_p(t) for t in raw]
    fl = default_flags() if flags is None else flags
    ev = _ev_start(Z, "DENSE")
    rc = lib.pg_directgcn_dense_ngram_rows_f32(ctypes.byref(a), None, int(Kn1), int(m0), int(bool(map_res)),
                                               int(bool(map_out)), fl, _stream(Z))
    del keep, raw
    if rc == _lib.PG_ERR_UNSUPPORTED:
        return None
    check(rc, "pg_directgcn_dense_ngram_rows_f32")
    _ev_end(Z, ev, "DENSE")
    return Y


def _layer_dense_bf16(Z, prm, gate_mode, rows, constant, res_x, W_res, b_res, act, slope, flags, packs=None,
                      drop=None):
    lib = load_library()
    packed, p16 = pack_weights_bf16(prm, W_res, b_res)
    if packs is not None:
        packs[:] = [packed, p16]
    M = Z.size(0)
    F_out = prm["W_main_in"].size(0)
    Y = torch.empty(M, F_out, device=Z.device, dtype=torch.bfloat16)
    a, keep = _layer_args(Z, prm, gate_mode, rows, constant, res_x, W_res, act, slope, drop=drop)
    a.Y, a.ldy = _p(Y), Y.stride(0)
    fl = default_flags() if flags is None else flags
    ev = _ev_start(Z, "DENSE")
    rc = lib.pg_directgcn_dense_bf16(ctypes.byref(a), _p(packed), _p(p16), fl, _stream(Z))
    del keep
    if rc == _lib.PG_ERR_UNSUPPORTED:
        return None
    check(rc, "pg_directgcn_dense_bf16")
    _ev_end(Z, ev, "DENSE")
    return Y


def layer_dense_backward(dY, Z, Y, prm: dict, gate_mode: int, rows=None, res_x=None, W_res=None, b_res=None,
                         act: bool = False, slope: float = LEAKY_SLOPE, flags: Optional[int] = None,
                         need_dZ: bool = True, packs: Optional[list] = None, span: Optional[tuple] = None,
                         drop_p: float = 0.0, dpre_f32: bool = False):
    """pg_directgcn_dense_bwd_f32 (any shape; bf16 operands: pg_directgcn_dense_bwd_bf16, None when F_in / F_out
    are not multiples of 8 -- the caller then runs the fp32 kernels on widened copies). Returns a dict with
      dpre [M, F_out], dZ [M, 3F_in], dres [M, F_in] (projected residual) or None,
      dgate [5, M] (per-row grads of c_in, c_out, c_directed, c_undirected, c_all),
      dB [F_out, K] (grad of the packed segment weights W_main_q + W_shared, W_res), dbsum [4, F_out].
    packs: the bf16 forward's packed weights of the same parameters (LayerDense: saved by its forward), else packed
    here. span = (wdiag [M, 3], e_res): pg_directgcn_dense_bwd_span_f32 (fp32 only), which also returns
    E [M, F_in] = sum_q wdiag[:, q] dZ_q (+ dpre when e_res); None when it does not take the shape.
    drop_p: the forward's fused dropout (Y is its output; the mask is read off Y, pg::act_grad). dpre_f32 (bf16 only):
    also return dpre as fp32 ("dpre_f32": the same rounded values, written by the dgrad kernel)."""
    lib = load_library()
    _require_gpu(dY, Z, Y)
    M, F_in = Z.size(0), Z.size(1) // 3
    F_out = prm["W_main_in"].size(0)
    bf = _is_bf16(Z)
    if bf and (F_in % 8 or F_out % 8):
        return None
    if bf:
        packed, p16 = packs if packs else pack_weights_bf16(prm, W_res, b_res)
        Y = _bf16c(Y)
    else:
        packed = pack_weights(prm, W_res, b_res)
    a, keep = _layer_args(Z, prm, gate_mode, rows, None, res_x, W_res, act, slope, Y=Y,
                          drop=(drop_p, None) if drop_p else None)
    dev = Z.device
    K = (4 if W_res is not None else 3) * F_in
    act_dt = torch.bfloat16 if bf else torch.float32
    dYc = _bf16c(dY) if bf else _f32c(dY)
    dpre = torch.empty(M, F_out, device=dev, dtype=act_dt)
    dZ = torch.empty(M, 3 * F_in, device=dev, dtype=act_dt) if need_dZ else None
    dres = torch.empty(M, F_in, device=dev, dtype=act_dt) if W_res is not None else None
    dgate = torch.empty(5, M, device=dev)
    gates = torch.empty(M, 4, device=dev)
    dW = torch.empty(F_out * K + 4 * F_out, device=dev)
    nwork = lib.pg_directgcn_dense_bwd_workspace(ctypes.byref(a))
    if nwork < 0:
        raise RuntimeError("pg_directgcn_dense_bwd_workspace: bad arguments")
    work = torch.empty(max(int(nwork), 4), device=dev)
    g = _lib.LayerGradArgs()
    g.dY, g.lddy = _p(dYc), dYc.stride(0)
    g.dpre, g.ldp = _p(dpre), dpre.stride(0)
    if dZ is not None:
        g.dZ, g.lddz = _p(dZ), dZ.stride(0)
    if dres is not None:
        g.dres, g.lddres = _p(dres), dres.stride(0)
    g.dgate, g.gates, g.dW = _p(dgate), _p(gates), _p(dW)
    g.work, g.work_floats = _p(work), work.numel()
    dpre32 = None
    if bf and dpre_f32:
        dpre32 = torch.empty(M, F_out, device=dev, dtype=torch.float32)
        g.dpre_f32, g.ldp_f32 = _p(dpre32), dpre32.stride(0)
    fl = default_flags() if flags is None else flags
    E = None
    if span is not None:
        if bf or dZ is None:
            return None
        wdiag, e_res = span
        wdiag = _f32c(wdiag)
        E = torch.empty(M, F_in, device=dev, dtype=torch.float32)
        rc = lib.pg_directgcn_dense_bwd_span_f32(ctypes.byref(a), _p(packed), ctypes.byref(g), _p(wdiag), _p(E),
                                                 E.stride(0), int(bool(e_res)), fl, _stream(Z))
        name = "pg_directgcn_dense_bwd_span_f32"
    elif bf:
        rc = lib.pg_directgcn_dense_bwd_bf16(ctypes.byref(a), _p(packed), _p(p16), ctypes.byref(g), fl, _stream(Z))
        name = "pg_directgcn_dense_bwd_bf16"
    else:
        rc = lib.pg_directgcn_dense_bwd_f32(ctypes.byref(a), _p(packed), ctypes.byref(g), fl, _stream(Z))
        name = "pg_directgcn_dense_bwd_f32"
    if rc == _lib.PG_ERR_UNSUPPORTED:
        return None
    check(rc, name)
    del keep
    return {"dpre": dpre, "dZ": dZ, "dres": dres, "dgate": dgate, "E": E, "dpre_f32": dpre32,
            "dB": dW[:F_out * K].view(F_out, K), "dbsum": dW[F_out * K:].view(4, F_out)}


def head(h: torch.Tensor, W1, b1, W2, b2, eps: float):
    """Fused decoder + log_softmax + L2-normalised embedding (eval-mode forward, no autograd). A bf16 h
    (bf16 mode) is read as bf16 (pg_directgcn_head_bf16); outputs are fp32."""
    lib = load_library()
    _require_gpu(h)
    M, F = h.shape
    H, C = W1.size(0), W2.size(0)
    W1, b1, W2, b2 = (_f32c(t.detach()) for t in (W1, b1, W2, b2))
    logp = torch.empty(M, C, device=h.device, dtype=torch.float32)
    emb = torch.empty(M, F, device=h.device, dtype=torch.float32)
    if _is_bf16(h):
        hb = _bf16c(h.detach())
        ev = _ev_start(hb, "HEAD")
        rc = lib.pg_directgcn_head_bf16(M, F, H, C, _p(hb), hb.stride(0), _p(W1), _p(b1), _p(W2), _p(b2), float(eps),
                                        _p(logp), logp.stride(0), _p(emb), emb.stride(0), _stream(hb))
        if rc != _lib.PG_ERR_UNSUPPORTED:
            check(rc, "pg_directgcn_head_bf16")
            _ev_end(hb, ev, "HEAD")
            return logp, emb
    h = _f32c(h.detach())
    ev = _ev_start(h, "HEAD")
    check(lib.pg_directgcn_head_f32(M, F, H, C, _p(h), h.stride(0), _p(W1), _p(b1), _p(W2), _p(b2), float(eps),
                                    _p(logp), logp.stride(0), _p(emb), emb.stride(0), _stream(h)),
          "pg_directgcn_head_f32")
    _ev_end(h, ev, "HEAD")
    return logp, emb


_LABELS_OK: dict = {}  # (data_ptr, numel, _version, C) of label tensors already checked


def _check_labels(y: torch.Tensor, C: int):
    """Raise like F.nll_loss on a label outside [0, C) (protgram_directgcn_trainer.py:95). One host sync per label
    tensor (cached by address, size and version; the trainer's labels are fixed), none inside a HIP-graph capture,
    where the kernel's NaN loss is the signal."""
    key = (y.data_ptr(), y.numel(), y._version, C)
    if key in _LABELS_OK or y.numel() == 0 or torch.cuda.is_current_stream_capturing():
        return
    lo, hi = torch.aminmax(y)
    if int(lo) < 0 or int(hi) >= C:
        raise IndexError(f"head_train: label out of range [0, {C}): min {int(lo)}, max {int(hi)}")
    if len(_LABELS_OK) > 64:
        _LABELS_OK.clear()
    _LABELS_OK[key] = True


def head_train(h: torch.Tensor, W1, b1, W2, b2, y: torch.Tensor, weight: float = 1.0, drop_p: float = 0.0,
               seed: Optional[torch.Tensor] = None, scale: Optional[torch.Tensor] = None):
    """pg_head_train_f32: the prediction head's training step (decoder Linear -> ReLU -> Dropout -> Linear,
    log_softmax, nll_loss mean * weight; protgram_directgcn.py:218-222, protgram_directgcn_trainer.py:91-100) forward
    and backward in one pass over h. Returns (loss [device scalar, unscaled], dh [M, F] = d(scale * loss)/dh,
    grads (dW1, db1, dW2, db2) of scale * loss), or None when the shape is not taken (F = 128, H = 64, C <= 32 only).
    seed: device int64 [1] for the dropout draw (drop_p > 0); scale: device fp32 scalar (GradScaler) or None."""
    lib = load_library()
    _require_gpu(h, y)
    M, Fd = h.shape
    H, C = W1.size(0), W2.size(0)
    nwork = int(lib.pg_head_train_workspace(M, Fd, H, C))
    if nwork < 0:
        return None
    h = _f32c(h)
    W1, b1, W2, b2 = (_f32c(t.detach()) for t in (W1, b1, W2, b2))
    y = y.contiguous().to(torch.int64)
    dev = h.device
    dh = torch.empty(M, Fd, device=dev, dtype=torch.float32)
    grads = torch.empty(H * Fd + H + C * H + C, device=dev, dtype=torch.float32)
    loss = torch.empty((), device=dev, dtype=torch.float32)
    work = torch.empty(max(nwork, 4), device=dev, dtype=torch.float32)
    if drop_p > 0 and seed is None:
        raise ValueError("head_train: dropout needs a seed tensor")
    _check_labels(y, C)
    rc = lib.pg_head_train_f32(M, Fd, H, C, _p(h), h.stride(0), _p(W1), _p(b1), _p(W2), _p(b2), _p(y),
                               float(weight) / max(M, 1), float(drop_p), _p(seed), _p(scale), _p(dh), dh.stride(0),
                               _p(grads), _p(loss), _p(work), work.numel(), _stream(h))
    if rc == _lib.PG_ERR_UNSUPPORTED:
        return None
    check(rc, "pg_head_train_f32")
    o1, o2, o3 = H * Fd, H * Fd + H, H * Fd + H + C * H
    return loss, dh, (grads[:o1].view(H, Fd), grads[o1:o2], grads[o2:o3].view(C, H), grads[o3:])


def head_train_bf16(h: torch.Tensor, W1, b1, W2, b2, y: torch.Tensor, weight: float = 1.0, drop_p: float = 0.0,
                    seed: Optional[torch.Tensor] = None, scale: Optional[torch.Tensor] = None):
    """pg_head_train_bf16: head_train for the model's bf16 mode at F = 256 (config 5): h bf16 [M, 256], W1 [128, 256],
    C <= 32 classes. Returns (loss, dh bf16 [M, 256] = d(scale * loss)/dh rounded once, grads (dW1, db1, dW2, db2))
    or None when the shape is not taken (the caller runs the framework ops on h.float())."""
    lib = load_library()
    _require_gpu(h, y)
    if not _is_bf16(h) or h.dim() != 2:
        return None
    M, Fd = h.shape
    H, C = W1.size(0), W2.size(0)
    nwork = int(lib.pg_head_train_bf16_workspace(M, Fd, H, C))
    if nwork < 0:
        return None
    h = _bf16c(h)
    W1, b1, W2, b2 = (_f32c(t.detach()) for t in (W1, b1, W2, b2))
    y = y.contiguous().to(torch.int64)
    dev = h.device
    dh = torch.empty(M, Fd, device=dev, dtype=torch.bfloat16)
    grads = torch.empty(H * Fd + H + C * H + C, device=dev, dtype=torch.float32)
    loss = torch.empty((), device=dev, dtype=torch.float32)
    work = torch.empty(max(nwork, 4), device=dev, dtype=torch.float32)
    if drop_p > 0 and seed is None:
        raise ValueError("head_train_bf16: dropout needs a seed tensor")
    _check_labels(y, C)
    rc = lib.pg_head_train_bf16(M, Fd, H, C, _p(h), h.stride(0), _p(W1), _p(b1), _p(W2), _p(b2), _p(y),
                                float(weight) / max(M, 1), float(drop_p), _p(seed), _p(scale), _p(dh), dh.stride(0),
                                _p(grads), _p(loss), _p(work), work.numel(), _stream(h))
    if rc == _lib.PG_ERR_UNSUPPORTED:
        return None
    check(rc, "pg_head_train_bf16")
    o1, o2, o3 = H * Fd, H * Fd + H, H * Fd + H + C * H
    return loss, dh, (grads[:o1].view(H, Fd), grads[o1:o2], grads[o2:o3].view(C, H), grads[o3:])


def gemm_at_b(A: torch.Tensor, B: torch.Tensor):
    """pg_gemm_at_b_f32: (A^T B [P, N], column sums of A [P]) over the M rows, or None when the shape is not
    taken (P or N not a multiple of 4)."""
    lib = load_library()
    _require_gpu(A, B)
    A, B = _f32c(A), _f32c(B)
    M, P = A.shape
    N = B.size(1)
    if P % 4 or N % 4:
        return None
    out = torch.empty(P * N + P, device=A.device, dtype=torch.float32)
    nwork = int(lib.pg_gemm_at_b_workspace(M, P, N))
    work = torch.empty(max(nwork, 4), device=A.device, dtype=torch.float32)
    rc = lib.pg_gemm_at_b_f32(M, P, N, _p(A), A.stride(0), _p(B), B.stride(0), _p(out), _p(work), work.numel(),
                              _stream(A))
    if rc == _lib.PG_ERR_UNSUPPORTED:
        return None
    check(rc, "pg_gemm_at_b_f32")
    return out[:P * N].view(P, N), out[P * N:]


# ------------------------------------------------------------------------------------------------
# autograd
# ------------------------------------------------------------------------------------------------
# The reference trainer runs the model under torch.amp.autocast (protgram_directgcn_trainer.py:93):
# the Functions below compute in the model's own dtype inside autocast regions (fp32, or bf16 in the
# explicit bf16 mode) -- at least the reference's fp16-GEMM precision.
# bf16 inputs (the model's bf16 mode) are kept as they are; fp16 (autocast's default dtype) is widened.


def _fwd32(fn):
    @functools.wraps(fn)
    def forward(ctx, *args):
        if torch.is_autocast_enabled("cuda"):
            args = tuple(a.float() if torch.is_tensor(a) and a.dtype == torch.float16 else a for a in args)
            with torch.autocast("cuda", enabled=False):
                return fn(ctx, *args)
        return fn(ctx, *args)
    return forward


def _bwd32(fn):
    @functools.wraps(fn)
    def backward(ctx, *grads):
        with torch.autocast("cuda", enabled=False):
            return fn(ctx, *grads)
    return backward


class Propagate3(torch.autograd.Function):
    """x [N, F] -> Z [N, 3F] = [A_in x | A_out x | A_und x]; backward = transposed propagation."""

    @staticmethod
    @_fwd32
    def forward(ctx, x, g: CSRGraph, fused: bool = False):
        ctx.g = g
        return spmm3(g, x, fused=fused)

    @staticmethod
    @_bwd32
    def backward(ctx, dZ):
        if not ctx.needs_input_grad[0]:
            return None, None, None
        return spmm3_t(ctx.g, dZ), None, None


class Propagate1(torch.autograd.Function):
    @staticmethod
    @_fwd32
    def forward(ctx, x, a: ShapedAdjacency):
        ctx.a = a
        return spmm1(a, x)

    @staticmethod
    @_bwd32
    def backward(ctx, dY):
        return spmm1(ctx.a, dY, transpose=True), None


_DENSE_KEYS = ("W_main_in", "W_main_out", "W_undirected", "W_shared", "b_main_in", "b_dir_shared_in",
               "b_main_out", "b_dir_shared_out", "b_undirected", "b_undirected_shared",
               "C_in", "C_out", "C_directed", "C_undirected", "C_all")


class LayerDense(torch.autograd.Function):
    """Y = act(sum_k s_k (Z_k W_k'^T + b_k') + constant[rows] + residual) (pg_directgcn_dense_f32).

    Backward: pg_directgcn_dense_bwd_f32 (dX of the propagation is handled by Propagate3):
      G = dpre [W_in' | W_out' | W_und']  ->  dZ_k = s_k G_k,  ds_k = <G_k, Z_k> + <dpre, b_k'>
      dW_k' = (s_k dpre)^T Z_k,  db_k' = sum_m s_k dpre,  and the chain rule through s_k(c)."""

    @staticmethod
    @_fwd32
    def forward(ctx, Z, res_x, constant, W_res, b_res, rows, gate_mode, act, slope, drop, *params):
        prm = dict(zip(_DENSE_KEYS, params))
        # the bf16 kernels' packed weights are kept for the backward (the parameters are saved tensors: autograd
        # refuses a backward after an in-place change to them, so the packed copies cannot go stale before it)
        ctx.packs = []
        Y = layer_dense(Z, prm, gate_mode, rows=rows, constant=constant, res_x=res_x, W_res=W_res, b_res=b_res,
                        act=act, slope=slope, packs=ctx.packs, drop=drop)
        ctx.gate_mode, ctx.act, ctx.slope = gate_mode, act, slope
        ctx.drop_p = drop[0] if drop is not None else 0.0
        ctx.has_res, ctx.has_const = res_x is not None, constant is not None
        ctx.save_for_backward(Z, res_x if res_x is not None else Z.new_empty(0),
                              constant if constant is not None else Z.new_empty(0),
                              W_res if W_res is not None else Z.new_empty(0),
                              rows if rows is not None else Z.new_empty(0, dtype=torch.int64), Y, *params)
        ctx.has_wres, ctx.has_rows = W_res is not None, rows is not None
        return Y

    @staticmethod
    @_bwd32
    def backward(ctx, dY):
        Z, res_x, constant, W_res, rows, Y, *params = ctx.saved_tensors
        prm = dict(zip(_DENSE_KEYS, params))
        res_x = res_x if ctx.has_res else None
        constant = constant if ctx.has_const else None
        W_res = W_res if ctx.has_wres else None
        rows = rows if ctx.has_rows else None
        packs, ctx.packs = ctx.packs, None
        defer = _is_bf16(dY) and _defer_const(constant, ctx.needs_input_grad[2], Z.size(0), rows)
        out = layer_dense_backward(dY, Z, Y, prm, ctx.gate_mode, rows=rows, res_x=res_x, W_res=W_res,
                                   act=ctx.act, slope=ctx.slope, need_dZ=ctx.needs_input_grad[0], packs=packs,
                                   drop_p=ctx.drop_p,
                                   dpre_f32=constant is not None and ctx.needs_input_grad[2]
                                   and constant.dtype == torch.float32 and not defer)
        need_const = ctx.needs_input_grad[2]
        if out is not None and defer and _file_deferred(constant, out["dpre"]):
            need_const = False
        if out is None:  # bf16 shapes the bf16 kernels do not take: the fp32 kernels on widened copies
            out = layer_dense_backward(dY.float(), Z.float(), Y.float(), prm, ctx.gate_mode, rows=rows,
                                       res_x=None if res_x is None else res_x.float(), W_res=W_res, act=ctx.act,
                                       slope=ctx.slope, need_dZ=ctx.needs_input_grad[0], drop_p=ctx.drop_p)
            for k in ("dpre", "dZ", "dres"):
                if out[k] is not None:
                    out[k] = out[k].to(torch.bfloat16)
        grads, d_const, d_res, d_wres, d_bres = _dense_grads(out, prm, ctx.gate_mode, rows, Z, constant, res_x, W_res,
                                                             lambda i: ctx.needs_input_grad[10 + i], need_const)
        return (out["dZ"], d_res, d_const, d_wres, d_bres, None, None, None, None, None, *grads)


def dense_grads_layout(dB: torch.Tensor, dbsum: torch.Tensor, F_in: int):
    """(Wg [S, F_out, F_in] segment-major weight gradients, W_shared's (Wg0 + Wg1) + Wg2 [F_out, F_in], the bias pairs
    [2, 3, F_out]) from the dense backward's dB [F_out, S F_in] and dbsum: one pg_dense_grads_layout_f32 launch on
    the GPU (views of one buffer), the same values as the torch ops it replaces (which CPU tensors still take)."""
    F_out, S = dB.size(0), dB.size(1) // F_in
    if dB.is_cuda and dB.dtype == torch.float32 and dB.is_contiguous() and dbsum.is_contiguous() and F_in % 4 == 0:
        buf = torch.empty((S + 1) * F_out * F_in + 6 * F_out, device=dB.device, dtype=torch.float32)
        rc = load_library().pg_dense_grads_layout_f32(F_out, F_in, S, _p(dB), _p(dbsum), _p(buf), _stream(dB))
        if rc != _lib.PG_ERR_UNSUPPORTED:
            check(rc, "pg_dense_grads_layout_f32")
            plane = F_out * F_in
            return (buf[:S * plane].view(S, F_out, F_in), buf[S * plane:(S + 1) * plane].view(F_out, F_in),
                    buf[(S + 1) * plane:].view(2, 3, F_out))
    Wg = dB.view(F_out, S, F_in).transpose(0, 1).contiguous()
    ws = Wg[0] + Wg[1]
    ws += Wg[2]
    return Wg, ws, dbsum[:3].unsqueeze(0).expand(2, 3, F_out).contiguous()


def _dense_grads(out, prm, gate_mode, rows, Z, constant, res_x, W_res, need, need_const):
    """The parameter gradients of LayerDense / PropagateDense from the dense backward's outputs: (grads in _DENSE_KEYS
    order, d_constant, d_res, d_W_res, d_b_res); need(i) says whether parameter i of _DENSE_KEYS needs its gradient."""
    dpre, dB, dbsum, dgate = out["dpre"], out["dB"], out["dbsum"], out["dgate"]
    M, F_in = Z.size(0), Z.size(1) // 3
    F_out = dB.size(0)
    # Every weight and bias gradient is handed to autograd as its own contiguous tensor, so AccumulateGrad keeps it
    # instead of copying it: column slices of dB break the parameters' layout contract (one strided copy each), and
    # a bias sum shared by two parameters is copied for one of them. One copy lays dB out by segment
    # ([segments, F_out, F_in]); W_shared = (W_in' + W_out') + W_und' as before; one copy doubles the bias sums.
    Wg, ws, bb = dense_grads_layout(dB, dbsum, F_in)
    g = {"W_main_in": Wg[0], "W_main_out": Wg[1], "W_undirected": Wg[2]}
    g["W_shared"] = ws
    g["b_main_in"], g["b_dir_shared_in"] = bb[0, 0], bb[1, 0]
    g["b_main_out"], g["b_dir_shared_out"] = bb[0, 1], bb[1, 1]
    g["b_undirected"], g["b_undirected_shared"] = bb[0, 2], bb[1, 2]
    for q, name in enumerate(("C_in", "C_out", "C_directed", "C_undirected", "C_all")):
        v = prm[name]
        if not need(_DENSE_KEYS.index(name)):
            continue
        if gate_mode == 1:
            g[name] = dgate[q].sum().reshape(v.shape)
        elif rows is not None:
            g[name] = torch.zeros_like(v).index_add_(0, rows, dgate[q].reshape(-1, *v.shape[1:]))
        elif v.size(0) == M:
            g[name] = dgate[q].reshape(v.shape)
        else:
            full = torch.zeros_like(v)
            full[:M] = dgate[q].reshape(M, *v.shape[1:])
            g[name] = full
    d_const = None
    if constant is not None and need_const:
        dp = out.get("dpre_f32")  # the bf16 backward's own fp32 copy (the same values as the conversion below)
        if dp is None or dp.dtype != constant.dtype:
            dp = dpre.to(constant.dtype)
        if rows is None and constant.size(0) == M:
            d_const = dp  # every row of the constant receives exactly its dpre row (no zero-fill + add pass)
        else:
            d_const = torch.zeros_like(constant)
            if rows is not None:
                d_const.index_add_(0, rows, dp)
            else:
                d_const[:M] += dp
    d_res = d_wres = d_bres = None
    if res_x is not None:
        if W_res is None:
            d_res = dpre
        else:
            d_res = out["dres"]
            d_wres = Wg[3]
            d_bres = dbsum[3]
    grads = [g[k] if need(i) else None for i, k in enumerate(_DENSE_KEYS)]
    return grads, d_const, d_res, d_wres, d_bres


class PropagateDense(torch.autograd.Function):
    """Propagate3 + LayerDense in one Function for a layer whose input needs its gradient, on a complete n-gram graph
    (round 5; the autograd of protgram_directgcn.py:101-133 and the residual of :213-215). Forward: the same two
    kernels. Backward: pg_directgcn_dense_bwd_span_f32 writes, next to dZ, E = the transposed propagation's diagonal
    term (+ the identity residual's dpre) from its accumulators, and the off-diagonal transposed middle-tile kernel
    (pg_spmm3t_ngram_mid_offdiag_f32, 657 MB at B(20,4) F = 128) accumulates into E: the input's whole gradient in
    two launches, where Propagate3 + LayerDense run the 4x4-block transposed kernel (1,050 MB) and autograd adds the
    residual's gradient in a third pass. Inputs: (x, g, res, constant, gate_mode, act, slope, drop, *params) with
    res = the layer's residual is x itself (identity), drop = the fused layer dropout (p, seed) or None."""

    @staticmethod
    @_fwd32
    def forward(ctx, x, g: CSRGraph, res: bool, constant, gate_mode, act, slope, drop, *params):
        prm = dict(zip(_DENSE_KEYS, params))
        ctx.bf16 = _is_bf16(x)
        ctx.packs = [] if ctx.bf16 else None  # the bf16 kernels' packed weights, reused by the backward
        Z = spmm3(g, x)
        Y = layer_dense(Z, prm, gate_mode, constant=constant, res_x=x if res else None, act=act, slope=slope,
                        drop=drop, packs=ctx.packs)
        ctx.g, ctx.res, ctx.gate_mode, ctx.act, ctx.slope = g, res, gate_mode, act, slope
        ctx.drop_p = drop[0] if drop is not None else 0.0
        ctx.has_const = constant is not None
        ctx.save_for_backward(Z, Y, constant if constant is not None else Z.new_empty(0), *params)
        return Y

    @staticmethod
    @_bwd32
    def backward(ctx, dY):
        Z, Y, constant, *params = ctx.saved_tensors
        prm = dict(zip(_DENSE_KEYS, params))
        constant = constant if ctx.has_const else None
        g = ctx.g
        if ctx.bf16:
            return PropagateDense._backward_bf16(ctx, dY, Z, Y, constant, prm)
        out = layer_dense_backward(dY, Z, Y, prm, ctx.gate_mode, act=ctx.act, slope=ctx.slope,
                                   span=(g.ngram.diag3(), ctx.res), drop_p=ctx.drop_p)
        if out is None:
            raise RuntimeError("PropagateDense: pg_directgcn_dense_bwd_span_f32 refused a shape supports_span accepted")
        dX = spmm3t_offdiag(g, out["dZ"], out=out["E"])
        if dX is None:
            raise RuntimeError("PropagateDense: the off-diagonal transposed kernel refused a shape supports_span accepted")
        grads, d_const, _, _, _ = _dense_grads(out, prm, ctx.gate_mode, None, Z, constant, None, None,
                                               lambda i: ctx.needs_input_grad[8 + i], ctx.needs_input_grad[3])
        return (dX if ctx.needs_input_grad[0] else None, None, None, d_const, None, None, None, None, *grads)

    @staticmethod
    def _backward_bf16(ctx, dY, Z, Y, constant, prm):
        """bf16 mode: the bf16 dense backward, then the transposed propagation accumulated into the identity
        residual's dpre (spmm3t_ngram_acc_bf16: dX = dpre + sum_k A_k^T dZ_k in fp32, rounded once) -- the autograd
        path (Propagate3 + LayerDense) ran the same kernel into a fresh buffer and added dpre in a separate bf16 pass."""
        packs, ctx.packs = ctx.packs, None
        defer = _defer_const(constant, ctx.needs_input_grad[3], Z.size(0), None)
        dpre_f32 = constant is not None and ctx.needs_input_grad[3] and constant.dtype == torch.float32 and not defer
        out = layer_dense_backward(dY, Z, Y, prm, ctx.gate_mode, act=ctx.act, slope=ctx.slope, packs=packs,
                                   drop_p=ctx.drop_p, dpre_f32=dpre_f32)
        if out is None:
            raise RuntimeError("PropagateDense: the bf16 dense backward refused a shape supports accepted")
        need_const = ctx.needs_input_grad[3]
        deferred = defer and _file_deferred(constant, out["dpre"])
        if deferred:
            need_const = False
        grads, d_const, d_res, _, _ = _dense_grads(out, prm, ctx.gate_mode, None, Z, constant,
                                                   Z.new_empty(0) if ctx.res else None, None,
                                                   lambda i: ctx.needs_input_grad[8 + i], need_const)
        dX = None
        if ctx.needs_input_grad[0]:
            if ctx.res and deferred:  # dpre stays the constant's gradient: dX = dpre + A^T dZ into a new buffer
                dX = spmm3t_ngram_acc_bf16(ctx.g, out["dZ"], torch.empty_like(d_res), src=d_res)
                if dX is None:
                    dX = spmm3_t(ctx.g, out["dZ"]) + d_res
            elif ctx.res:
                # d_res is dpre itself; the constant's gradient (d_const) is its fp32 copy or a conversion made above
                if d_const is not None and d_const.data_ptr() == d_res.data_ptr():
                    d_res = d_res.clone()
                dX = spmm3t_ngram_acc_bf16(ctx.g, out["dZ"], d_res)
                if dX is None:
                    dX = spmm3_t(ctx.g, out["dZ"]) + d_res
            else:
                dX = spmm3_t(ctx.g, out["dZ"])
        return (dX, None, None, d_const, None, None, None, None, *grads)

    @staticmethod
    def supports(g: CSRGraph, x: torch.Tensor, F_out: int, res_x, W_res, rows, fused_norm: bool,
                 flags: Optional[int] = None) -> bool:
        """Whether a layer call takes this path: fp32, a symmetric shared-pattern graph with a middle plan (the
        off-diagonal kernel's domain), F_in % 64 == 0, F_out % 32 == 0, an identity residual (res_x is x) or none,
        no row map, no fused normalisation."""
        fl = default_flags() if flags is None else flags
        common = (x.is_cuda and not fused_norm and rows is None and W_res is None and (res_x is None or res_x is x)
                  and g.shared and g.symmetric and g.ngram is not None and g.n_rows == x.size(0)
                  and (res_x is None or x.size(1) == F_out) and not (fl & _lib.PG_FLAG_NO_NGRAM))
        if _is_bf16(x):  # bf16: the 4x4-block transposed kernel's widths, the bf16 dense backward's (multiples of 8)
            return common and x.size(1) in (64, 128, 256) and F_out % 8 == 0
        return (common and x.dtype == torch.float32 and g.ngram.mplan is not None and x.size(1) % 64 == 0
                and F_out % 32 == 0)


class RowLinear(torch.autograd.Function):
    """y = x W^T + b over many rows (the decoder nn.Linear layers, protgram_directgcn.py:173-177, in
    training). Forward and dx = dy W are plain library GEMMs (hipBLASLt through torch); (dW, db) -- a reduction
    over all M rows, which the library GEMMs tile badly -- run in pg_gemm_at_b_f32 (shapes it does not take:
    the library GEMM)."""

    @staticmethod
    @_fwd32
    def forward(ctx, x, W, b):
        ctx.save_for_backward(x, W)
        ctx.has_b = b is not None
        return torch.nn.functional.linear(x, W, b)

    @staticmethod
    @_bwd32
    def backward(ctx, dy):
        x, W = ctx.saved_tensors
        dx = dy @ W if ctx.needs_input_grad[0] else None
        dW = db = None
        if ctx.needs_input_grad[1] or (ctx.has_b and ctx.needs_input_grad[2]):
            r = gemm_at_b(dy, x) if x.dim() == 2 else None
            if r is None:
                dW, db = dy.reshape(-1, dy.size(-1)).t() @ x.reshape(-1, x.size(-1)), dy.reshape(-1, dy.size(-1)).sum(0)
            else:
                dW, db = r
        return dx, dW, (db if ctx.has_b else None)


def row_linear(x, W, b=None):
    return RowLinear.apply(x, W, b)

