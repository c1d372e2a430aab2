// Fused three-adjacency CSR SpMM for gfx950 (the DirectGCN propagation hot path).
//
// Reference semantics (what one call replaces): per adjacency k, PyG propagate with aggr='add'
//   out[ei[1]] += w_k * x[ei[0]]          (src/models/protgram_directgcn.py:101-112, :137-140)
// The three n-gram adjacencies share one sparsity pattern, so one pass over the
// CSR gathers each source row ONCE and feeds three accumulators (A_in X, A_out X, A_und X).
//
// Work mapping: a "row group" of LPR lanes owns one destination row; lane t holds feature float4s
// t, t+LPR, ... (NV of them), so one gather is LPR*16 B contiguous (512 B at F=128: a half-wave).
// Each lane keeps U gathers in flight (memory-level parallelism for the ~41-entry rows). Rows are
// visited in XCD-contiguous order (pg::xcd_logical_block). No atomics: each output row is written
// by exactly one row group, so results are deterministic.
//
// Numerics: products and sums are issued as separate, correctly rounded operations
// (__fmul_rn/__fadd_rn, no FMA contraction), in ascending source order within a row: the same
// operation sequence as the reference's index_select -> mul -> scatter_add_ on its coalesced COO,
// so each aggregate is bit-identical to the reference's propagate() of the same input.
#include "pg_common.h"

namespace {

enum : int { M3 = 0, M3RAW = 1, M3T = 2, M1 = 3 };

struct SpmmParams {
    int64_t n_rows;
    const int64_t* rowptr;
    const int32_t* row_order;  // processing position -> row (NULL = identity)
    const void* edges;
    const float* X;
    int64_t ldx;
    float* Z;
    int64_t ldz;
    const float4* node_norm;
    float eps;
    int F;
    int accumulate;
    int remap;
    // optional output gates (pg_spmm3_gated_f32): Z_q[i] *= s_q(i) at the store, s = the DirectGCN gates
    // s_in = c_all*c_dir*c_in, s_out = c_all*c_dir*c_out, s_und = c_all*c_und (protgram_directgcn.py:116-133)
    const float *g_in, *g_out, *g_dir, *g_und, *g_all;
    int gate_scalar;
};

// Gate inputs of row `row`, loaded when the row starts (so their latency hides behind the row's gathers) and
// turned into the three gates at the store (1, 1, 1 when the call is not gated). Same products as pg_dense.hip.
struct GateIn {
    float ci, co, cd, cu, ca;
};
__device__ __forceinline__ GateIn gate_in(const SpmmParams& p, int64_t row, bool live) {
    GateIn g{1.f, 1.f, 1.f, 1.f, 1.f};
    if (p.g_all && live) {
        const int64_t r = p.gate_scalar ? 0 : row;
        g = GateIn{p.g_in[r], p.g_out[r], p.g_dir[r], p.g_und[r], p.g_all[r]};
    }
    return g;
}
__device__ __forceinline__ void row_gates(const GateIn& g, float s[3]) {
    const float cad = __fmul_rn(g.ca, g.cd);
    s[0] = __fmul_rn(cad, g.ci);
    s[1] = __fmul_rn(cad, g.co);
    s[2] = __fmul_rn(g.ca, g.cu);
}

__device__ __forceinline__ float fb(int v) { return __int_as_float(v); }
__device__ __forceinline__ float mul(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float add(float a, float b) { return __fadd_rn(a, b); }

__device__ __forceinline__ float4 axpy4(float4 acc, float w, float4 x) {
    acc.x = add(acc.x, mul(w, x.x));
    acc.y = add(acc.y, mul(w, x.y));
    acc.z = add(acc.z, mul(w, x.z));
    acc.w = add(acc.w, mul(w, x.w));
    return acc;
}

// Closed form of the reference's propagation weights for entry (source j -> destination i)
// (graph_utils.py:198-273 for mathcal_A_out / mathcal_A_in, :160-196 for A_undirected_norm):
//   w_out = sqrt(0.5*((a_ji*dout_inv_j)^2 + (a_ij*dout_inv_i)^2) + eps) + [i==j]
//   w_in  = sqrt(0.5*((a_ij*din_inv_j)^2  + (a_ji*din_inv_i)^2)  + eps) + [i==j]
//   w_und = m_ij * (r_j * r_i)
// An identity-only diagonal (no raw count either way) is exactly 1.0 (graph_utils.py:268-269).
struct W3 {
    float in, out, und;
};

__device__ __forceinline__ W3 fused_weights(float a_fwd, float a_bwd, float m, float4 nj, float4 ni, bool diag,
                                            float eps) {
    W3 w;
    if (a_fwd == 0.0f && a_bwd == 0.0f) {
        w.in = 1.0f;
        w.out = 1.0f;
    } else {
        const float d = diag ? 1.0f : 0.0f;
        const float p1 = mul(a_fwd, nj.x), p2 = mul(a_bwd, ni.x);
        const float so = mul(add(mul(p1, p1), mul(p2, p2)), 0.5f);
        w.out = add(pg::sqrt_rn(add(so, eps)), d);
        const float q1 = mul(a_bwd, nj.y), q2 = mul(a_fwd, ni.y);
        const float si = mul(add(mul(q1, q1), mul(q2, q2)), 0.5f);
        w.in = add(pg::sqrt_rn(add(si, eps)), d);
    }
    w.und = mul(m, mul(nj.z, ni.z));
    return w;
}

template <int MODE>
struct Rec {
    using T = int4;
};
template <>
struct Rec<M1> {
    using T = int2;
};

// Number of output accumulators and gathered slices per edge.
template <int MODE>
struct Shape {
    static constexpr int NACC = (MODE == M3 || MODE == M3RAW) ? 3 : 1;
    static constexpr int NSLICE = (MODE == M3T) ? 3 : 1;
};

template <int LPR, int NV, int U, int MODE, bool EDGE_LDS>
__global__ __launch_bounds__(256) void spmm_vec_kernel(SpmmParams p) {
    using R = typename Rec<MODE>::T;
    constexpr int RPB = 256 / LPR;  // rows per block
    constexpr int NACC = Shape<MODE>::NACC;
    constexpr int NSLICE = Shape<MODE>::NSLICE;
    constexpr int CHUNK = 256;  // edge records staged per LDS round (variant B)

    const int64_t lb = pg::xcd_logical_block(blockIdx.x, gridDim.x, p.remap != 0);
    const int64_t row0 = lb * RPB;
    const int grp = threadIdx.x / LPR;
    const int t = threadIdx.x % LPR;
    const int64_t pos = row0 + grp;
    const bool live = pos < p.n_rows;
    const int64_t row = (live && p.row_order) ? (int64_t)p.row_order[pos] : pos;

    const R* __restrict__ E = reinterpret_cast<const R*>(p.edges);
    const float4* __restrict__ X4 = reinterpret_cast<const float4*>(p.X);
    const int64_t ldx4 = p.ldx >> 2;
    const int F4 = p.F >> 2;

    int64_t beg = 0, end = 0;
    if (live) {
        beg = p.rowptr[row];
        end = p.rowptr[row + 1];
    }
    float4 ni = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (MODE == M3RAW) {
        if (live) ni = p.node_norm[row];
    }
    GateIn gin{1.f, 1.f, 1.f, 1.f, 1.f};
    if constexpr (Shape<MODE>::NACC == 3) gin = gate_in(p, row, live);

    float4 acc[NACC][NV];
#pragma unroll
    for (int a = 0; a < NACC; ++a)
#pragma unroll
        for (int v = 0; v < NV; ++v) acc[a][v] = make_float4(0.f, 0.f, 0.f, 0.f);

    auto consume = [&](const R& r, const float4 (&xv)[NSLICE][NV], float4 nj) {
        if constexpr (MODE == M3) {
            const float w0 = fb(r.y), w1 = fb(r.z), w2 = fb(r.w);
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                acc[0][v] = axpy4(acc[0][v], w0, xv[0][v]);
                acc[1][v] = axpy4(acc[1][v], w1, xv[0][v]);
                acc[2][v] = axpy4(acc[2][v], w2, xv[0][v]);
            }
        } else if constexpr (MODE == M3RAW) {
            const W3 w = fused_weights(fb(r.y), fb(r.z), fb(r.w), nj, ni, (int64_t)r.x == row, p.eps);
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                acc[0][v] = axpy4(acc[0][v], w.in, xv[0][v]);
                acc[1][v] = axpy4(acc[1][v], w.out, xv[0][v]);
                acc[2][v] = axpy4(acc[2][v], w.und, xv[0][v]);
            }
        } else if constexpr (MODE == M3T) {
            const float w0 = fb(r.y), w1 = fb(r.z), w2 = fb(r.w);
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                float4 a = acc[0][v];
                a = axpy4(a, w0, xv[0][v]);
                a = axpy4(a, w1, xv[1][v]);
                a = axpy4(a, w2, xv[2][v]);
                acc[0][v] = a;
            }
        } else {
            const float w0 = fb(r.y);
#pragma unroll
            for (int v = 0; v < NV; ++v) acc[0][v] = axpy4(acc[0][v], w0, xv[0][v]);
        }
    };

    auto gather = [&](int col, float4 (&xv)[NSLICE][NV]) {
        const float4* src = X4 + (int64_t)col * ldx4 + t;
#pragma unroll
        for (int s = 0; s < NSLICE; ++s)
#pragma unroll
            for (int v = 0; v < NV; ++v) xv[s][v] = src[s * F4 + v * LPR];
    };

    auto run_range = [&](auto&& rec_at, int64_t e0, int64_t e1) {
        int64_t e = e0;
        for (; e + U <= e1; e += U) {
            R r[U];
#pragma unroll
            for (int u = 0; u < U; ++u) r[u] = rec_at(e + u);
            float4 xv[U][NSLICE][NV];
#pragma unroll
            for (int u = 0; u < U; ++u) gather(r[u].x, xv[u]);
            float4 nj[U];
            if constexpr (MODE == M3RAW) {
#pragma unroll
                for (int u = 0; u < U; ++u) nj[u] = p.node_norm[r[u].x];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) consume(r[u], xv[u], MODE == M3RAW ? nj[u] : ni);
        }
        for (; e < e1; ++e) {
            const R r = rec_at(e);
            float4 xv[NSLICE][NV];
            gather(r.x, xv);
            float4 nj = ni;
            if constexpr (MODE == M3RAW) nj = p.node_norm[r.x];
            consume(r, xv, nj);
        }
    };

    if constexpr (!EDGE_LDS) {
        run_range([&](int64_t e) { return E[e]; }, beg, end);
    } else {
        // Variant B: the block's contiguous edge range is staged CHUNK records at a time in LDS
        // (one coalesced 16-B load per thread), then every row group reads its records from LDS
        // (same address across the group: broadcast, conflict-free).
        __shared__ R tile[CHUNK];
        const int64_t rlast = (row0 + RPB < p.n_rows ? row0 + RPB : p.n_rows);
        const int64_t bbeg = p.rowptr[row0 < p.n_rows ? row0 : p.n_rows];
        const int64_t bend = p.rowptr[rlast];
        for (int64_t c0 = bbeg; c0 < bend; c0 += CHUNK) {
            const int64_t c1 = (c0 + CHUNK < bend) ? c0 + CHUNK : bend;
            __syncthreads();
            if (c0 + threadIdx.x < c1) tile[threadIdx.x] = E[c0 + threadIdx.x];
            __syncthreads();
            const int64_t lo = beg > c0 ? beg : c0;
            const int64_t hi = end < c1 ? end : c1;
            if (lo < hi) run_range([&](int64_t e) { return tile[e - c0]; }, lo, hi);
        }
    }

    if (!live) return;
    float gs[3] = {1.f, 1.f, 1.f};
    if constexpr (NACC == 3) row_gates(gin, gs);
    float4* Z4 = reinterpret_cast<float4*>(p.Z) + row * (p.ldz >> 2) + t;
#pragma unroll
    for (int a = 0; a < NACC; ++a)
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            float4* dst = Z4 + a * F4 + v * LPR;
            float4 val = acc[a][v];
            if (NACC == 3 && p.g_all)
                val = make_float4(mul(val.x, gs[a]), mul(val.y, gs[a]), mul(val.z, gs[a]), mul(val.w, gs[a]));
            if (p.accumulate) {
                const float4 old = *dst;
                val = make_float4(add(old.x, val.x), add(old.y, val.y), add(old.z, val.z), add(old.w, val.w));
            }
            *dst = val;
        }
}

// Variant C (default for F = 4*LPR, LPR in {8,16,32,64}): records through a per-row-group LDS window.
// Counters on gfx950 (tools/pmc_passes.sh) show the broadcast record load of variants A/B costing as much
// L1->VGPR (TD) bandwidth as the feature gathers themselves: every lane of a row group loads the same 16-B
// record, i.e. a 1 KiB wave-instruction for LPR-fold duplicated data, and TD is busy ~94% of the kernel.
// Here the LPR lanes of a group load LPR *consecutive* records (one each, coalesced), park them in the
// group's own LDS window, and read them back as LDS broadcasts: the TD only carries the feature gathers.
// A window is private to one row group inside one wave, so wave-local ordering (the compiler's
// lgkmcnt waits + a wave barrier) replaces block barriers. Same accumulation order: still bit-exact.
template <int LPR, int NV, int U, int MODE, bool GATED>
__device__ __forceinline__ void win_row(const SpmmParams& p, int64_t pos, bool live,
                                        typename Rec<MODE>::T* __restrict__ mywin) {
    using R = typename Rec<MODE>::T;
    constexpr int NACC = Shape<MODE>::NACC;
    constexpr int NSLICE = Shape<MODE>::NSLICE;
    constexpr int WIN = LPR;  // records per window (one per lane)
    const int t = threadIdx.x % LPR;
    const int64_t row = (live && p.row_order) ? (int64_t)p.row_order[pos] : pos;
    const R* __restrict__ E = reinterpret_cast<const R*>(p.edges);
    const float4* __restrict__ X4 = reinterpret_cast<const float4*>(p.X);
    const int64_t ldx4 = p.ldx >> 2;
    const int F4 = p.F >> 2;
    int64_t beg = 0, end = 0;
    if (live) {
        beg = p.rowptr[row];
        end = p.rowptr[row + 1];
    }
    float4 ni = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (MODE == M3RAW) {
        if (live) ni = p.node_norm[row];
    }
    GateIn gin{1.f, 1.f, 1.f, 1.f, 1.f};
    if constexpr (GATED && Shape<MODE>::NACC == 3) gin = gate_in(p, row, live);
    float4 acc[NACC][NV];
#pragma unroll
    for (int a = 0; a < NACC; ++a)
#pragma unroll
        for (int v = 0; v < NV; ++v) acc[a][v] = make_float4(0.f, 0.f, 0.f, 0.f);

    // prefetch the first window into registers
    R nxt = (beg + t < end) ? E[beg + t] : R{};
    for (int64_t w0 = beg; w0 < end; w0 += WIN) {
        __builtin_amdgcn_wave_barrier();  // previous window fully consumed by this group's lanes
        mywin[t] = nxt;
        __builtin_amdgcn_wave_barrier();
        const int64_t wn = w0 + WIN;
        if (wn + t < end) nxt = E[wn + t];  // next window in flight while this one is consumed
        const int n = (int)((end - w0) < WIN ? (end - w0) : WIN);
        int j = 0;
        for (; j + U <= n; j += U) {
            R r[U];
#pragma unroll
            for (int u = 0; u < U; ++u) r[u] = mywin[j + u];
            float4 xv[U][NSLICE][NV];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const float4* src = X4 + (int64_t)r[u].x * ldx4 + t;
#pragma unroll
                for (int s = 0; s < NSLICE; ++s)
#pragma unroll
                    for (int v = 0; v < NV; ++v) xv[u][s][v] = src[s * F4 + v * LPR];
            }
            float4 nj[U];
            if constexpr (MODE == M3RAW) {
#pragma unroll
                for (int u = 0; u < U; ++u) nj[u] = p.node_norm[r[u].x];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if constexpr (MODE == M3) {
#pragma unroll
                    for (int v = 0; v < NV; ++v) {
                        acc[0][v] = axpy4(acc[0][v], fb(r[u].y), xv[u][0][v]);
                        acc[1][v] = axpy4(acc[1][v], fb(r[u].z), xv[u][0][v]);
                        acc[2][v] = axpy4(acc[2][v], fb(r[u].w), xv[u][0][v]);
                    }
                } else if constexpr (MODE == M3RAW) {
                    const W3 w = fused_weights(fb(r[u].y), fb(r[u].z), fb(r[u].w), nj[u], ni, (int64_t)r[u].x == row,
                                               p.eps);
#pragma unroll
                    for (int v = 0; v < NV; ++v) {
                        acc[0][v] = axpy4(acc[0][v], w.in, xv[u][0][v]);
                        acc[1][v] = axpy4(acc[1][v], w.out, xv[u][0][v]);
                        acc[2][v] = axpy4(acc[2][v], w.und, xv[u][0][v]);
                    }
                } else if constexpr (MODE == M3T) {
#pragma unroll
                    for (int v = 0; v < NV; ++v) {
                        float4 a = acc[0][v];
                        a = axpy4(a, fb(r[u].y), xv[u][0][v]);
                        a = axpy4(a, fb(r[u].z), xv[u][1][v]);
                        a = axpy4(a, fb(r[u].w), xv[u][2][v]);
                        acc[0][v] = a;
                    }
                } else {
#pragma unroll
                    for (int v = 0; v < NV; ++v) acc[0][v] = axpy4(acc[0][v], fb(r[u].y), xv[u][0][v]);
                }
            }
        }
        for (; j < n; ++j) {
            const R r = mywin[j];
            const float4* src = X4 + (int64_t)r.x * ldx4 + t;
            float4 xv[NSLICE][NV];
#pragma unroll
            for (int s = 0; s < NSLICE; ++s)
#pragma unroll
                for (int v = 0; v < NV; ++v) xv[s][v] = src[s * F4 + v * LPR];
            if constexpr (MODE == M3) {
#pragma unroll
                for (int v = 0; v < NV; ++v) {
                    acc[0][v] = axpy4(acc[0][v], fb(r.y), xv[0][v]);
                    acc[1][v] = axpy4(acc[1][v], fb(r.z), xv[0][v]);
                    acc[2][v] = axpy4(acc[2][v], fb(r.w), xv[0][v]);
                }
            } else if constexpr (MODE == M3RAW) {
                const W3 w = fused_weights(fb(r.y), fb(r.z), fb(r.w), p.node_norm[r.x], ni, (int64_t)r.x == row, p.eps);
#pragma unroll
                for (int v = 0; v < NV; ++v) {
                    acc[0][v] = axpy4(acc[0][v], w.in, xv[0][v]);
                    acc[1][v] = axpy4(acc[1][v], w.out, xv[0][v]);
                    acc[2][v] = axpy4(acc[2][v], w.und, xv[0][v]);
                }
            } else if constexpr (MODE == M3T) {
#pragma unroll
                for (int v = 0; v < NV; ++v) {
                    float4 a = acc[0][v];
                    a = axpy4(a, fb(r.y), xv[0][v]);
                    a = axpy4(a, fb(r.z), xv[1][v]);
                    a = axpy4(a, fb(r.w), xv[2][v]);
                    acc[0][v] = a;
                }
            } else {
#pragma unroll
                for (int v = 0; v < NV; ++v) acc[0][v] = axpy4(acc[0][v], fb(r.y), xv[0][v]);
            }
        }
    }
    if (!live) return;
    float gs[3] = {1.f, 1.f, 1.f};
    if constexpr (GATED && NACC == 3) row_gates(gin, gs);
    float4* Z4 = reinterpret_cast<float4*>(p.Z) + row * (p.ldz >> 2) + t;
#pragma unroll
    for (int a = 0; a < NACC; ++a)
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            float4* dst = Z4 + a * F4 + v * LPR;
            float4 val = acc[a][v];
            if (GATED && NACC == 3)
                val = make_float4(mul(val.x, gs[a]), mul(val.y, gs[a]), mul(val.z, gs[a]), mul(val.w, gs[a]));
            if (p.accumulate) {
                const float4 old = *dst;
                val = make_float4(add(old.x, val.x), add(old.y, val.y), add(old.z, val.z), add(old.w, val.w));
            }
            *dst = val;
        }
}

template <int LPR, int NV, int U, int MODE, int NT = 256, bool GATED = false>
__global__ __launch_bounds__(NT) void spmm_win_kernel(SpmmParams p) {
    using R = typename Rec<MODE>::T;
    constexpr int RPB = NT / LPR;
    __shared__ __attribute__((aligned(16))) R win[RPB][LPR];
    const int64_t lb = pg::xcd_logical_block(blockIdx.x, gridDim.x, p.remap != 0);
    const int grp = threadIdx.x / LPR;
    const int64_t pos = lb * RPB + grp;
    win_row<LPR, NV, U, MODE, GATED>(p, pos, pos < p.n_rows, win[grp]);
}

// Fallback for feature widths that are not a multiple of 4 (or too wide for the vector path):
// one wave per row, features in chunks of 64 (one per lane), records re-read per chunk.
template <int MODE>
__global__ __launch_bounds__(256) void spmm_scalar_kernel(SpmmParams p) {
    using R = typename Rec<MODE>::T;
    constexpr int NACC = Shape<MODE>::NACC;
    constexpr int NSLICE = Shape<MODE>::NSLICE;
    const int64_t lb = pg::xcd_logical_block(blockIdx.x, gridDim.x, p.remap != 0);
    const int64_t pos = lb * 4 + threadIdx.x / 64;
    const int lane = threadIdx.x % 64;
    if (pos >= p.n_rows) return;
    const int64_t row = p.row_order ? (int64_t)p.row_order[pos] : pos;
    const R* __restrict__ E = reinterpret_cast<const R*>(p.edges);
    const int64_t beg = p.rowptr[row], end = p.rowptr[row + 1];
    float4 ni = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (MODE == M3RAW) ni = p.node_norm[row];
    GateIn gin{1.f, 1.f, 1.f, 1.f, 1.f};
    if constexpr (NACC == 3) gin = gate_in(p, row, true);
    for (int f0 = 0; f0 < p.F; f0 += 64) {
        const int f = f0 + lane;
        const bool on = f < p.F;
        float acc[NACC];
#pragma unroll
        for (int a = 0; a < NACC; ++a) acc[a] = 0.f;
        for (int64_t e = beg; e < end; ++e) {
            const R r = E[e];
            float xv[NSLICE];
#pragma unroll
            for (int s = 0; s < NSLICE; ++s) xv[s] = on ? p.X[(int64_t)r.x * p.ldx + s * p.F + f] : 0.f;
            if constexpr (MODE == M3) {
                acc[0] = add(acc[0], mul(fb(r.y), xv[0]));
                acc[1] = add(acc[1], mul(fb(r.z), xv[0]));
                acc[2] = add(acc[2], mul(fb(r.w), xv[0]));
            } else if constexpr (MODE == M3RAW) {
                const W3 w = fused_weights(fb(r.y), fb(r.z), fb(r.w), p.node_norm[r.x], ni, (int64_t)r.x == row, p.eps);
                acc[0] = add(acc[0], mul(w.in, xv[0]));
                acc[1] = add(acc[1], mul(w.out, xv[0]));
                acc[2] = add(acc[2], mul(w.und, xv[0]));
            } else if constexpr (MODE == M3T) {
                acc[0] = add(acc[0], mul(fb(r.y), xv[0]));
                acc[0] = add(acc[0], mul(fb(r.z), xv[1]));
                acc[0] = add(acc[0], mul(fb(r.w), xv[2]));
            } else {
                acc[0] = add(acc[0], mul(fb(r.y), xv[0]));
            }
        }
        if (on) {
            float gs[3] = {1.f, 1.f, 1.f};
            if constexpr (NACC == 3) row_gates(gin, gs);
#pragma unroll
            for (int a = 0; a < NACC; ++a) {
                float* dst = p.Z + row * p.ldz + a * p.F + f;
                if (NACC == 3 && p.g_all) acc[a] = mul(acc[a], gs[a]);
                *dst = p.accumulate ? add(*dst, acc[a]) : acc[a];
            }
        }
    }
}

// Materialise precomputed weights from raw records (pg_edges_normalize_f32): one thread per entry.
__global__ __launch_bounds__(256) void normalize_kernel(int64_t n_rows, const int64_t* rowptr, const int4* raw,
                                                        const float4* node_norm, float eps, int4* out) {
    const int64_t row = (int64_t)blockIdx.x * 4 + threadIdx.x / 64;  // CSR order (no schedule needed)
    if (row >= n_rows) return;
    const float4 ni = node_norm[row];
    for (int64_t e = rowptr[row] + (threadIdx.x % 64); e < rowptr[row + 1]; e += 64) {
        const int4 r = raw[e];
        const W3 w = fused_weights(fb(r.y), fb(r.z), fb(r.w), node_norm[r.x], ni, (int64_t)r.x == row, eps);
        out[e] = make_int4(r.x, __float_as_int(w.in), __float_as_int(w.out), __float_as_int(w.und));
    }
}

template <int MODE, int LPR, int NV, int U, bool LDS>
void launch_vec(const SpmmParams& p, hipStream_t s) {
    constexpr int RPB = 256 / LPR;
    const int64_t nb = (p.n_rows + RPB - 1) / RPB;
    hipLaunchKernelGGL((spmm_vec_kernel<LPR, NV, U, MODE, LDS>), dim3((unsigned)nb), dim3(256), 0, s, p);
}

template <int MODE, int LPR, int NV>
void launch_vec_u(const SpmmParams& p, uint32_t flags, hipStream_t s) {
    // Default: variant C (record window) with 4 gathers in flight; PG_FLAG_UNROLL4 toggles it to 8.
    // PG_FLAG_BCAST_RECORDS / PG_FLAG_EDGE_LDS select variants A / B (measurement only).
    const bool win = !(flags & (PG_FLAG_EDGE_LDS | PG_FLAG_BCAST_RECORDS));
    if (win && LPR >= 8) {
        const int64_t rpb = 256 / LPR;
        const int64_t nb = (p.n_rows + rpb - 1) / rpb;
        const bool u8 = flags & PG_FLAG_UNROLL4;
        if (p.g_all) {  // gated store (pg_spmm3_gated_f32): the default configuration only
            if constexpr (Shape<MODE>::NACC == 3)
                hipLaunchKernelGGL((spmm_win_kernel<LPR, NV, 4, MODE, 256, true>), dim3((unsigned)nb), dim3(256), 0, s, p);
            return;
        }
if (u8) hipLaunchKernelGGL((spmm_win_kernel<LPR, NV, 8, MODE, 256>), dim3((unsigned)nb), dim3(256), 0, s, p);
        else hipLaunchKernelGGL((spmm_win_kernel<LPR, NV, 4, MODE, 256>), dim3((unsigned)nb), dim3(256), 0, s, p);
        return;
    }
    const bool lds = (flags & PG_FLAG_EDGE_LDS) && p.row_order == nullptr;  // staging needs contiguous rows
    const bool u4 = flags & PG_FLAG_UNROLL4;
    if (lds) {
        if (u4) launch_vec<MODE, LPR, NV, 4, true>(p, s);
        else launch_vec<MODE, LPR, NV, 8, true>(p, s);
    } else {
        if (u4) launch_vec<MODE, LPR, NV, 4, false>(p, s);
        else launch_vec<MODE, LPR, NV, 8, false>(p, s);
    }
}

template <int MODE>
int dispatch(SpmmParams p, uint32_t flags, hipStream_t s, const char* name) {
    if (p.n_rows == 0) return PG_OK;
    p.remap = (flags & PG_FLAG_NO_XCD_REMAP) ? 0 : 1;
    const bool vec_ok = (p.F % 4 == 0) && (p.ldx % 4 == 0) && (p.ldz % 4 == 0) && pg::aligned16(p.X) &&
                        pg::aligned16(p.Z);
    const int F = p.F;
    if (vec_ok) {
        switch (F) {
            case 16: launch_vec_u<MODE, 4, 1>(p, flags, s); return pg::check_launch(name);
            case 32: launch_vec_u<MODE, 8, 1>(p, flags, s); return pg::check_launch(name);
            case 64: launch_vec_u<MODE, 16, 1>(p, flags, s); return pg::check_launch(name);
            case 128: launch_vec_u<MODE, 32, 1>(p, flags, s); return pg::check_launch(name);
            case 256: launch_vec_u<MODE, 64, 1>(p, flags, s); return pg::check_launch(name);
            case 512: launch_vec_u<MODE, 64, 2>(p, flags, s); return pg::check_launch(name);
            default: break;
        }
    }
    const int64_t nb = (p.n_rows + 3) / 4;
    hipLaunchKernelGGL((spmm_scalar_kernel<MODE>), dim3((unsigned)nb), dim3(256), 0, s, p);
    return pg::check_launch(name);
}

int common_checks(int64_t n_rows, const int64_t* rowptr, const void* edges, const float* X, int64_t ldx, int64_t F,
                  float* Z, int64_t ldz, int64_t zwidth, int64_t xwidth) {
    PG_REQUIRE(n_rows >= 0, "n_rows < 0");
    PG_REQUIRE(n_rows < (int64_t(1) << 31) * 64, "n_rows too large");
    PG_REQUIRE(F > 0 && F < (1 << 20), "bad feature width %lld", (long long)F);
    PG_REQUIRE(n_rows == 0 || (rowptr && Z), "null rowptr/output");
    PG_REQUIRE(ldx >= xwidth, "ldx %lld < %lld", (long long)ldx, (long long)xwidth);
    PG_REQUIRE(ldz >= zwidth, "ldz %lld < %lld", (long long)ldz, (long long)zwidth);
    (void)edges;
    (void)X;
    return PG_OK;
}

}  // namespace

extern "C" {

int pg_spmm3_f32(int64_t n_rows, const int64_t* rowptr, const int32_t* row_order, const pg_edge3_t* edges,
                 const float* X, int64_t ldx, int64_t F, float* Z, int64_t ldz, uint32_t flags, void* stream) {
    int rc = common_checks(n_rows, rowptr, edges, X, ldx, F, Z, ldz, 3 * F, F);
    if (rc) return rc;
    SpmmParams p{n_rows, rowptr, row_order, edges, X, ldx, Z, ldz, nullptr, 0.f, (int)F, 0, 1};
    return dispatch<M3>(p, flags, (hipStream_t)stream, "pg_spmm3_f32");
}

int pg_spmm3_gated_f32(int64_t n_rows, const int64_t* rowptr, const int32_t* row_order, const pg_edge3_t* edges,
                       const float* X, int64_t ldx, int64_t F, const pg_layer_args_t* gates, float* Z, int64_t ldz,
                       uint32_t flags, void* stream) {
    int rc = common_checks(n_rows, rowptr, edges, X, ldx, F, Z, ldz, 3 * F, F);
    if (rc) return rc;
    PG_REQUIRE(gates && gates->C_in && gates->C_out && gates->C_directed && gates->C_undirected && gates->C_all,
               "null gate");
    PG_REQUIRE(gates->gate_mode == PG_GATES_VECTOR || gates->gate_mode == PG_GATES_SCALAR, "bad gate_mode");
    PG_REQUIRE(gates->rows == nullptr, "gated propagation takes no original_indices (gate rows = graph rows)");
    SpmmParams p{n_rows, rowptr, row_order, edges, X, ldx, Z, ldz, nullptr, 0.f, (int)F, 0, 1};
    p.g_in = gates->C_in;
    p.g_out = gates->C_out;
    p.g_dir = gates->C_directed;
    p.g_und = gates->C_undirected;
    p.g_all = gates->C_all;
    p.gate_scalar = gates->gate_mode == PG_GATES_SCALAR;
    return dispatch<M3>(p, flags, (hipStream_t)stream, "pg_spmm3_gated_f32");
}

int pg_spmm3_fusednorm_f32(int64_t n_rows, const int64_t* rowptr, const int32_t* row_order, const pg_edgeraw_t* edges,
                           const float* node_norm, float eps, const float* X, int64_t ldx, int64_t F, float* Z,
                           int64_t ldz, uint32_t flags, void* stream) {
    int rc = common_checks(n_rows, rowptr, edges, X, ldx, F, Z, ldz, 3 * F, F);
    if (rc) return rc;
    PG_REQUIRE(n_rows == 0 || (node_norm && pg::aligned16(node_norm)), "node_norm must be 16-byte aligned [n,4]");
    SpmmParams p{n_rows, rowptr, row_order, edges, X, ldx, Z, ldz, reinterpret_cast<const float4*>(node_norm), eps,
                 (int)F, 0, 1};
    return dispatch<M3RAW>(p, flags, (hipStream_t)stream, "pg_spmm3_fusednorm_f32");
}

int pg_spmm3t_f32(int64_t n_rows, const int64_t* rowptr, const int32_t* row_order, const pg_edge3_t* edges,
                  const float* G, int64_t ldg, int64_t F, float* dX, int64_t lddx, int accumulate, uint32_t flags,
                  void* stream) {
    int rc = common_checks(n_rows, rowptr, edges, G, ldg, F, dX, lddx, F, 3 * F);
    if (rc) return rc;
    SpmmParams p{n_rows, rowptr, row_order, edges, G, ldg, dX, lddx, nullptr, 0.f, (int)F, accumulate ? 1 : 0, 1};
    return dispatch<M3T>(p, flags, (hipStream_t)stream, "pg_spmm3t_f32");
}

int pg_spmm1_f32(int64_t n_rows, const int64_t* rowptr, const int32_t* row_order, const pg_edge1_t* edges,
                 const float* X, int64_t ldx, int64_t F, float* Y, int64_t ldy, int accumulate, uint32_t flags,
                 void* stream) {
    int rc = common_checks(n_rows, rowptr, edges, X, ldx, F, Y, ldy, F, F);
    if (rc) return rc;
    SpmmParams p{n_rows, rowptr, row_order, edges, X, ldx, Y, ldy, nullptr, 0.f, (int)F, accumulate ? 1 : 0, 1};
    return dispatch<M1>(p, flags, (hipStream_t)stream, "pg_spmm1_f32");
}

int pg_edges_normalize_f32(int64_t n_rows, const int64_t* rowptr, const pg_edgeraw_t* raw, const float* node_norm,
                           float eps, pg_edge3_t* out, void* stream) {
    PG_REQUIRE(n_rows >= 0, "n_rows < 0");
    if (n_rows == 0) return PG_OK;
    PG_REQUIRE(rowptr && raw && node_norm && out, "null pointer");
    PG_REQUIRE(pg::aligned16(node_norm) && pg::aligned16(raw) && pg::aligned16(out), "16-byte alignment required");
    const int64_t nb = (n_rows + 3) / 4;
    hipLaunchKernelGGL(normalize_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, n_rows, rowptr,
                       reinterpret_cast<const int4*>(raw), reinterpret_cast<const float4*>(node_norm), eps,
                       reinterpret_cast<int4*>(out));
    return pg::check_launch("pg_edges_normalize_f32");
}

}  // extern "C"
