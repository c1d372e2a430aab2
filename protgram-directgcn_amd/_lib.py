"""ctypes binding of the in-tree C-ABI library ``libpgdgcn.so`` (include/pg_directgcn.h).

There is no fallback: if the library is missing or fails to load, every op raises
:class:`NativeLibraryError`. ``load_library()`` needs no GPU (dlopen + symbol check only).
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.environ.get("PG_DIRECTGCN_LIB", os.path.join(_HERE, "libpgdgcn.so"))

PG_OK = 0
PG_FLAG_NO_XCD_REMAP = 1 << 0
PG_FLAG_EDGE_LDS = 1 << 1
PG_FLAG_UNROLL4 = 1 << 2
PG_FLAG_BCAST_RECORDS = 1 << 7
PG_FLAG_NGRAMT_WIDE = 1 << 8
PG_FLAG_NGRAMT_NARROW = 1 << 3
PG_FLAG_NGRAMT_HALVES = 1 << 4
PG_FLAG_DENSE_PREGATED = 1 << 14
PG_FLAG_DENSE_TILED = 1 << 15
PG_FLAG_DENSE_X3 = 1 << 16
PG_FLAG_WGRAD_F32MFMA = 1 << 18
PG_FLAG_WGRAD_BF16_TILED = 1 << 11
PG_FLAG_DGRAD_BF16_TILED = 1 << 10
PG_FLAG_DGRAD_BF16_RESIDENT = 1 << 9
PG_FLAG_DGRAD_F32MFMA = 1 << 17
PG_FLAG_NO_NGRAM = 1 << 20
PG_FLAG_NGRAM_BLOCK4 = 1 << 21
PG_FLAG_MID_NO_PAIRS = 1 << 22
PG_FLAG_MID_LOADER_SYNC = 1 << 19
PG_FLAG_MID_TRANSPOSED = 1 << 23
PG_FLAG_SCATTER_CPW_SHIFT = 24
PG_FLAG_DENSE_A_CACHED = 1 << 12
PG_FLAG_DENSE_NO_IL = 1 << 13

c_i64, c_i32, c_u32, c_f32, c_vp = ctypes.c_int64, ctypes.c_int32, ctypes.c_uint32, ctypes.c_float, ctypes.c_void_p


PG_OK, PG_ERR_ARG, PG_ERR_HIP, PG_ERR_UNSUPPORTED = 0, -1, -2, -3


class NativeLibraryError(RuntimeError):
    pass


class LayerArgs(ctypes.Structure):
    """pg_layer_args_t"""
    _fields_ = [("M", c_i64), ("F_in", c_i64), ("F_out", c_i64),
                ("Z", c_vp), ("ldz", c_i64),
                ("W_main_in", c_vp), ("W_main_out", c_vp), ("W_undirected", c_vp), ("W_shared", c_vp),
                ("b_main_in", c_vp), ("b_dir_shared_in", c_vp),
                ("b_main_out", c_vp), ("b_dir_shared_out", c_vp),
                ("b_undirected", c_vp), ("b_undirected_shared", c_vp),
                ("gate_mode", c_i32),
                ("C_in", c_vp), ("C_out", c_vp), ("C_directed", c_vp), ("C_undirected", c_vp), ("C_all", c_vp),
                ("rows", c_vp),
                ("constant", c_vp), ("ld_const", c_i64),
                ("res_x", c_vp), ("ld_res", c_i64),
                ("W_res", c_vp), ("b_res", c_vp),
                ("act", c_i32), ("slope", c_f32),
                ("Y", c_vp), ("ldy", c_i64),
                ("drop_p", c_f32), ("drop_seed", c_vp)]


class LayerGradArgs(ctypes.Structure):
    """pg_layer_grad_args_t"""
    _fields_ = [("dY", c_vp), ("lddy", c_i64), ("dpre", c_vp), ("ldp", c_i64), ("dZ", c_vp), ("lddz", c_i64),
                ("dres", c_vp), ("lddres", c_i64), ("dgate", c_vp), ("gates", c_vp), ("dW", c_vp),
                ("work", c_vp), ("work_floats", c_i64), ("dpre_f32", c_vp), ("ldp_f32", c_i64)]


# symbol -> (restype, argtypes); every symbol declared in include/pg_directgcn.h
SIGNATURES = {
    "pg_last_error": (ctypes.c_char_p, []),
    "pg_abi_version": (ctypes.c_int, []),
    "pg_spmm3_f32": (ctypes.c_int, [c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_u32, c_vp]),
    "pg_spmm3_gated_f32": (ctypes.c_int, [c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, ctypes.POINTER(LayerArgs), c_vp,
                                          c_i64, c_u32, c_vp]),
    "pg_spmm3_fusednorm_f32": (ctypes.c_int, [c_i64, c_vp, c_vp, c_vp, c_vp, c_f32, c_vp, c_i64, c_i64, c_vp, c_i64,
                                              c_u32, c_vp]),
    "pg_edges_normalize_f32": (ctypes.c_int, [c_i64, c_vp, c_vp, c_vp, c_f32, c_vp, c_vp]),
    "pg_ngram_plan_floats": (c_i64, [ctypes.c_int, ctypes.c_int, c_i64]),
    "pg_ngram_plan_f32": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "pg_spmm3_ngram_f32": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_i64, c_vp, c_vp, c_i64, c_i64,
                                          ctypes.POINTER(LayerArgs), c_vp, c_i64, c_u32, c_vp]),
    "pg_ngram_mplan_floats": (c_i64, [ctypes.c_int, ctypes.c_int, c_i64]),
    "pg_ngram_mplan_f32": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "pg_spmm3_ngram_mid_f32": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_i64, c_vp, c_vp, c_i64, c_i64,
                                              ctypes.POINTER(LayerArgs), c_vp, c_i64, c_u32, c_vp]),
    "pg_spmm3_ngram_mid_rows_f32": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_i64, c_vp, c_vp, c_i64, c_i64, c_i64,
                                                   c_i64, c_vp, c_i64, c_u32, c_vp]),
    "pg_spmm3_ngram_mid_bf16": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_i64, c_vp, c_vp, c_i64, c_i64, c_vp,
                                               c_i64, c_u32, c_vp]),
    "pg_spmm3_ngram_mid_rows_bf16": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_i64, c_vp, c_vp, c_i64, c_i64, c_i64,
                                                    c_i64, c_vp, c_i64, c_u32, c_vp]),
    "pg_ngram_mplan_map_f32": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp,
                                              c_vp]),
    "pg_spmm3_ngram_mid_map_f32": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp,
                                                  c_i64, c_u32, c_vp]),
    "pg_spmm3_resid_f32": (ctypes.c_int, [c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_u32, c_vp]),
    "pg_rows_gather": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp]),
    "pg_rows_scatter": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp]),
    "pg_rows_gather_sum": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, ctypes.c_int, c_vp, c_vp, c_i64, c_i64, c_vp,
                                          c_i64, ctypes.c_int, c_vp]),
    "pg_ngram_scatter_plan": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_vp, c_i64, c_i64, c_vp, c_vp]),
    "pg_spmm3t_ngram_scatter_f32": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_u32, c_vp]),
    "pg_spmm3t_ngram_scatter_bf16": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_u32, c_vp]),
    "pg_spmm3t_ngram_f32": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_i64, c_vp, c_vp, c_i64, c_i64, c_vp, c_i64,
                                           ctypes.c_int, c_u32, c_vp]),
    "pg_spmm3t_ngram_mid_offdiag_f32": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_i64, c_vp, c_vp, c_i64, c_i64,
                                                       c_vp, c_i64, ctypes.c_int, c_u32, c_vp]),
    "pg_spmm3t_ngram_mid_bf16": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_i64, c_vp, c_vp, c_i64, c_i64, c_vp, c_i64,
                                                ctypes.c_int, c_u32, c_vp]),
    "pg_spmm3t_ngram_bf16": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_i64, c_vp, c_vp, c_i64, c_i64, c_vp, c_i64,
                                            ctypes.c_int, c_u32, c_vp]),
    "pg_spmm3t_ngram_add_bf16": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_i64, c_vp, c_vp, c_i64, c_i64, c_vp,
                                                c_i64, c_vp, c_i64, c_u32, c_vp]),
    "pg_spmm3t_f32": (ctypes.c_int, [c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, ctypes.c_int, c_u32,
                                     c_vp]),
    "pg_spmm1_f32": (ctypes.c_int, [c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, ctypes.c_int, c_u32,
                                    c_vp]),
    "pg_directgcn_packed_floats": (c_i64, [c_i64, c_i64, ctypes.c_int]),
    "pg_directgcn_pack_f32": (ctypes.c_int, [ctypes.POINTER(LayerArgs), c_vp, c_vp]),
    "pg_directgcn_dense_f32": (ctypes.c_int, [ctypes.POINTER(LayerArgs), c_vp, c_u32, c_vp]),
    "pg_directgcn_dense_ngram_rows_f32": (ctypes.c_int, [ctypes.POINTER(LayerArgs), c_vp, c_i64, c_i64, c_i32, c_i32,
                                                         c_u32, c_vp]),
    "pg_directgcn_dense_bwd_workspace": (c_i64, [ctypes.POINTER(LayerArgs)]),
    "pg_directgcn_dense_bwd_f32": (ctypes.c_int, [ctypes.POINTER(LayerArgs), c_vp, ctypes.POINTER(LayerGradArgs),
                                                  c_u32, c_vp]),
    "pg_directgcn_dense_bwd_span_f32": (ctypes.c_int, [ctypes.POINTER(LayerArgs), c_vp, ctypes.POINTER(LayerGradArgs),
                                                       c_vp, c_vp, c_i64, c_i32, c_u32, c_vp]),
    "pg_f32_to_bf16": (ctypes.c_int, [c_i64, c_vp, c_vp, c_vp]),
    "pg_spmm3_bf16": (ctypes.c_int, [c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_u32, c_vp]),
    "pg_spmm3t_bf16": (ctypes.c_int, [c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_u32, c_vp]),
    "pg_directgcn_dense_bf16": (ctypes.c_int, [ctypes.POINTER(LayerArgs), c_vp, c_vp, c_u32, c_vp]),
    "pg_directgcn_dense_bwd_bf16": (ctypes.c_int, [ctypes.POINTER(LayerArgs), c_vp, c_vp, ctypes.POINTER(LayerGradArgs),
                                                   c_u32, c_vp]),
    "pg_directgcn_head_bf16": (ctypes.c_int, [c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_f32,
                                              c_vp, c_i64, c_vp, c_i64, c_vp]),
    "pg_ngram_keys": (ctypes.c_int, [c_i64, c_vp, c_vp, c_vp, ctypes.c_int, c_i64, c_vp, c_vp, c_vp]),
    "pg_multi_chunks": (c_i64, [c_i64]),
    "pg_multi_sqsum_f32": (ctypes.c_int, [ctypes.c_int, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "pg_multi_axpy_f32": (ctypes.c_int, [ctypes.c_int, c_vp, c_vp, c_i64, c_f32, c_vp, c_vp]),
    "pg_adam_f32": (ctypes.c_int, [ctypes.c_int, c_vp, c_vp, c_i64, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                   ctypes.c_double, ctypes.c_double, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "pg_multi_sum_f32": (ctypes.c_int, [c_i64, c_vp, c_vp, c_vp]),
    "pg_dense_grads_layout_f32": (ctypes.c_int, [c_i64, c_i64, ctypes.c_int32, c_vp, c_vp, c_vp, c_vp]),
    "pg_gemm_at_b_workspace": (c_i64, [c_i64, c_i64, c_i64]),
    "pg_gemm_at_b_f32": (ctypes.c_int, [c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp]),
    "pg_directgcn_head_f32": (ctypes.c_int, [c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_f32,
                                             c_vp, c_i64, c_vp, c_i64, c_vp]),
    "pg_head_train_workspace": (c_i64, [c_i64, c_i64, c_i64, c_i64]),
    "pg_head_train_f32": (ctypes.c_int, [c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32,
                                         c_f32, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "pg_head_train_bf16_workspace": (c_i64, [c_i64, c_i64, c_i64, c_i64]),
    "pg_head_train_bf16": (ctypes.c_int, [c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32,
                                          c_f32, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp]),
}

_lib = None


def library_path() -> str:
    return _LIB_PATH


def load_library():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        raise NativeLibraryError(
            f"HIP library not found at {_LIB_PATH}; build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (there is no CPU fallback)")
    try:
        lib = ctypes.CDLL(_LIB_PATH)
    except OSError as e:
        raise NativeLibraryError(f"failed to load {_LIB_PATH}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            raise NativeLibraryError(f"{_LIB_PATH} does not export {name}")
        fn.restype, fn.argtypes = res, args
    if lib.pg_abi_version() != 4:
        raise NativeLibraryError("ABI version mismatch")
    _lib = lib
    return lib


def check(rc: int, what: str):
    if rc != PG_OK:
        msg = load_library().pg_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")


def default_flags() -> int:
    """Kernel-variant flags (tuning knob; PG_SPMM_FLAGS env overrides)."""
    v = os.environ.get("PG_SPMM_FLAGS")
    return int(v, 0) if v else 0
