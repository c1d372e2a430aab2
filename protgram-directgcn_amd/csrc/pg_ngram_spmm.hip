// N-gram tile propagation for gfx950: the three DirectGCN aggregates of an n-gram transition graph as dense
// register-blocked products instead of per-entry row gathers.
//
// Structure used (the three matrices share the pattern A u A^T u I): node i of a graph over all
// K^n n-grams is the base-K number s_1..s_n. Its out-neighbours are s_2..s_n c and its in-neighbours c s_1..s_{n-1}
// (c in 0..K-1). Write i = a.M.b (a = s_1, b = s_n, M = the middle n-2 digits): then
//   out-source(i, c) = (M.b).c        -- the same K sources for every row a'.M.b (fixed b)
//   in-source(i, c)  = c.(a.M)         -- the same K sources for every row a.M.b' (fixed a)
// so the rows of one middle M form a K x K grid (a, b) whose out-part is a dense K x K block per column b and
// whose in-part is a dense K x K block per row a. A PA x PB sub-block of that grid is worked by one wave (the
// transposed kernel) or two (the forward, AH = PA/2 a-rows each): a wave loads its sub-block's out- and
// in-sources ONCE per step and applies each to every row of its sub-block that shares it, from registers. Per
// output row that is K(PA+PB)/(PA*PB) + 1 source rows (11 at 4x4, K=20; 16 in the forward's two-wave split)
// instead of the ~2K+1 the per-row CSR kernel gathers (41).
//
// The weights come from the CSR (pg_ngram_plan_f32 scatters every entry into its slot): entry (i, j) goes to
// out-slot c = j mod K if j = out-source(i, c), else to in-slot c = j div K^(n-1) if j = in-source(i, c), else to
// the diagonal slot if j = i; a missing transition leaves a zero weight, and an entry that fits no slot marks the
// plan invalid (the caller then keeps the CSR kernel). An entry that is both an out- and an in-neighbour (a
// mutual pair) or an out-neighbour and the node itself (a constant string) is stored once, in its out-slot, so
// every CSR entry is applied exactly once.
//
// Numerics: each aggregate is the same sum of w*x terms as the reference's propagate(), accumulated with fp32
// FMAs in (out-slots, in-slots, diagonal) order instead of the CSR's ascending-column order: within fp32 rounding
// of the reference (tests: |d| <= 1e-5 + 1e-5|ref|), not bit-exact like pg_spmm3_f32. Zero-weight slots add
// 0 * x, so the inputs must be finite (an inf in a row adjacent in the grid would turn into NaN).
#include "pg_bf16_util.h"
#include "pg_common.h"

namespace {

struct NgramP {
    int K, n;
    int64_t Kn1, Kn2;  // K^(n-1), K^(n-2)
    int64_t n_rows;    // K^n
    const float* plan;
    int64_t blk;       // floats per wave block
    const float* X;
    int64_t ldx;
    float* Z;
    int64_t ldz;
    int F;
    int remap;
    int accumulate;
    const float *g_in, *g_out, *g_dir, *g_und, *g_all;
    int gate_scalar;
    const uint16_t* Xb;  // bf16 mode (BF kernels): X / G and Z / dX as bf16 rows; sums stay fp32, one rounding
    uint16_t* Zb;
    int zk;              // forward: floats between the three output slices (= F, or the full width of a column half)
    int pieces;          // transposed: column pieces of 64 * VEC features per plan block, one wave each (0 = 1)
    const float* C;      // transposed, accumulate: the addend rows (null: Z itself, in place)
    const uint16_t* Cb;
    int64_t ldc;
};

template <int VEC>
struct VT;
template <>
struct VT<1> {
    using T = float;
};
template <>
struct VT<2> {
    using T = float2;
};
template <>
struct VT<4> {
    using T = float4;
};

template <int VEC>
__device__ __forceinline__ void fma_v(typename VT<VEC>::T& acc, float w, const typename VT<VEC>::T& x) {
    if constexpr (VEC == 1) {
        acc = __builtin_fmaf(w, x, acc);
    } else if constexpr (VEC == 2) {
        acc.x = __builtin_fmaf(w, x.x, acc.x);
        acc.y = __builtin_fmaf(w, x.y, acc.y);
    } else {
        acc.x = __builtin_fmaf(w, x.x, acc.x);
        acc.y = __builtin_fmaf(w, x.y, acc.y);
        acc.z = __builtin_fmaf(w, x.z, acc.z);
        acc.w = __builtin_fmaf(w, x.w, acc.w);
    }
}

template <int VEC>
__device__ __forceinline__ typename VT<VEC>::T zero_v() {
    typename VT<VEC>::T z;
    if constexpr (VEC == 1) {
        z = 0.f;
    } else if constexpr (VEC == 2) {
        z = make_float2(0.f, 0.f);
    } else {
        z = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    return z;
}

template <int VEC>
__device__ __forceinline__ typename VT<VEC>::T scale_v(typename VT<VEC>::T v, float s) {
    if constexpr (VEC == 1) {
        return v * s;
    } else if constexpr (VEC == 2) {
        return make_float2(v.x * s, v.y * s);
    } else {
        return make_float4(v.x * s, v.y * s, v.z * s, v.w * s);
    }
}

template <int VEC>
__device__ __forceinline__ typename VT<VEC>::T add_v(typename VT<VEC>::T a, typename VT<VEC>::T b) {
    if constexpr (VEC == 1) {
        return a + b;
    } else if constexpr (VEC == 2) {
        return make_float2(a.x + b.x, a.y + b.y);
    } else {
        return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
    }
}

__device__ __forceinline__ float first_of(float v) { return v; }
__device__ __forceinline__ float first_of(float2 v) { return v.x; }
__device__ __forceinline__ float first_of(float4 v) { return v.x; }

// Row order inside a PA x PB plan block: slot(i, jb) = i*PB + jb (i = a - a0, jb = b - b0), so the rows of a-rows
// i0..i1 are one contiguous run of slots.
__device__ __forceinline__ int plan_slot(int i, int jb, int PB) { return i * PB + jb; }

// VEC consecutive bf16 of a row as fp32 / fp32 rounded to VEC bf16 (round to nearest even, as torch)
template <int VEC>
__device__ __forceinline__ typename VT<VEC>::T ld_bf(const uint16_t* q) {
    if constexpr (VEC == 1) {
        return __uint_as_float((uint32_t)*q << 16);
    } else if constexpr (VEC == 2) {
        const uint32_t w = *reinterpret_cast<const uint32_t*>(q);
        return make_float2(pgbf::lo(w), pgbf::hi(w));
    } else {
        return pgbf::unpack4(*reinterpret_cast<const uint2*>(q));
    }
}
template <int VEC>
__device__ __forceinline__ void st_bf(uint16_t* q, const typename VT<VEC>::T& v) {
    if constexpr (VEC == 1) {
        *q = (uint16_t)pgbf::f2bf(v);
    } else if constexpr (VEC == 2) {
        *reinterpret_cast<uint32_t*>(q) = pgbf::pack2(v.x, v.y);
    } else {
        *reinterpret_cast<uint2*>(q) = pgbf::pack4(v);
    }
}

// Forward: Z[i] = [A_in X | A_out X | A_und X][i] (optionally gated at the store, as pg_spmm3_gated_f32).
// A workgroup (4 waves) first stages its plan blocks in LDS (coalesced 16-B loads); each wave then owns AH of a
// block's PA a-rows (AH = PA/2: two waves per block, which halves the accumulators and raises occupancy) and runs the
// c loop over a ring of NB source-row sets (step c + NB - 1 loaded while step c is consumed; branch-free: a
// conditional load splits the round into blocks at whose joins the waitcnt pass drains every load in flight),
// reading each step's weights as LDS broadcasts (every lane the same address). A lane holds VEC = F/64 features.
// Measured at B(20,4), F=128 (tools/ngram_probe_k.py): 0.147-0.156 ms against 0.198 for the CSR window kernel;
// one wave per block 0.152-0.168; NB = 4 (a wave per SIMD fewer) 0.155; weights through the scalar cache 0.186;
// 16-B loads with a row per half-wave (half the load instructions, in-sources replicated per half) 0.215;
// 16-B loads with the half-waves on alternate steps c (every source once, partial rows summed by
// v_permlane32_swap; 196 VGPRs, 2 waves/SIMD) 0.187; the workgroup's K + PA source rows per step staged once in a
// double-buffered LDS slab (10 waves per (M, a-block), one barrier per step; 124 VGPRs + 64 KB LDS, one workgroup
// per CU) 0.280; the same slab filled by LDS-DMA (global_load_lds_dwordx4) in a ring of 3 or 4 steps ahead (90
// VGPRs, two workgroups per CU) 0.185, and 0.126 against 0.063 at F = 64, i.e. a per-step cost that does not
// shrink with the bytes; 4 x 5 plan blocks with the two blocks of a workgroup sharing their in-sources through a
// register-staged LDS slab 0.274 (this kernel on 4 x 5 blocks: 0.170). This kernel is texture-data bound (TD
// 90 % busy, ~30 cycles per 8-B wave load; PMC, profiles/r02_pmc_summary.txt).
template <int K, int VEC, int PA, int PB, int AH, int NB, bool GATED, bool BF = false>
__global__ __launch_bounds__(256) void ngram_spmm3_kernel(NgramP p) {
    static_assert(K % NB == 0, "the c loop runs in rounds of NB steps");
    using V = typename VT<VEC>::T;
    constexpr int RB = PA * PB;  // rows per plan block
    constexpr int R = AH * PB;   // rows per wave
    constexpr int WPB = PA / AH; // waves per plan block
    constexpr int BPW = 4 / WPB; // plan blocks per workgroup
    constexpr int BLK = (((2 * K + 1) * 3 * RB) + 15) / 16 * 16;
    __shared__ __attribute__((aligned(16))) float wl[BPW][BLK];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t lb = pg::xcd_logical_block(blockIdx.x, gridDim.x, p.remap != 0);
    const int64_t nblk = (p.n_rows / ((int64_t)K * K)) * (K / PA) * (K / PB);
    for (int q = threadIdx.x; q < BPW * BLK / 4; q += 256) {  // stage the workgroup's plan blocks
        const int bi = q / (BLK / 4), qq = q % (BLK / 4);
        const int64_t blk = lb * BPW + bi < nblk ? lb * BPW + bi : 0;
        reinterpret_cast<float4*>(wl[bi])[qq] = reinterpret_cast<const float4*>(p.plan + blk * BLK)[qq];
    }
    __syncthreads();
    const int64_t wb = lb * BPW + wave / WPB;
    const int half = wave % WPB;
    if (wb >= nblk) return;
    constexpr int nA = K / PA, nB = K / PB;
    const int64_t M = wb / (nA * nB);
    const int rr = (int)(wb % (nA * nB));
    const int a0 = (rr / nB) * PA + half * AH, b0 = (rr % nB) * PB;
    const float* __restrict__ W = wl[wave / WPB];
    const V* __restrict__ X = reinterpret_cast<const V*>(p.X);
    const int64_t ldxv = p.ldx / VEC;
    auto xrow = [&](int64_t row) -> V {  // this lane's VEC features of source row `row`
        if constexpr (BF) return ld_bf<VEC>(p.Xb + row * p.ldx + lane * VEC);
        else return (X + row * ldxv)[lane];
    };
    V acc[R][3];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int k = 0; k < 3; ++k) acc[r][k] = zero_v<VEC>();
    const int64_t ob = (M * K + b0) * K;         // out-source (b0 + j, c) = ob + j*K + c
    const int64_t ib = (int64_t)a0 * p.Kn2 + M;  // in-source (a0 + i, c) = c*K^(n-1) + ib + i*K^(n-2)
    auto load = [&](int c, V (&o)[PB], V (&in)[AH]) {
#pragma unroll
        for (int j = 0; j < PB; ++j) o[j] = xrow(ob + (int64_t)j * K + c);
#pragma unroll
        for (int i = 0; i < AH; ++i) in[i] = xrow((int64_t)c * p.Kn1 + ib + (int64_t)i * p.Kn2);
    };
    // the wave's rows are plan slots half*R .. half*R + R - 1 of each 3*RB-float (step, type) chunk
    auto step = [&](int c, const V (&o)[PB], const V (&in)[AH]) {
#pragma unroll
        for (int type = 0; type < 2; ++type) {
            const float4* w4 = reinterpret_cast<const float4*>(W + c * 6 * RB + type * 3 * RB + half * 3 * R);
#pragma unroll
            for (int q = 0; q < 3 * R / 4; ++q) {
                const float4 w = w4[q];
                const float wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int e = 4 * q + u, r = e / 3, k = e % 3;
                    fma_v<VEC>(acc[r][k], wv[u], type == 0 ? o[r % PB] : in[r / PB]);
                }
            }
        }
    };
    // gates (GATED): lane 5r + q loads gate q (in, out, directed, undirected, all) of the wave's row r in one
    // instruction; the epilogue reads them back with v_readlane
    float gv = 0.f;
    if constexpr (GATED) {
        static_assert(5 * R <= 64, "one gate per lane");
        if (lane < 5 * R) {
            const int r = lane / 5, q = lane - 5 * r;
            const int64_t row = (int64_t)(a0 + r / PB) * p.Kn1 + M * K + b0 + r % PB;
            const float* src = q == 0 ? p.g_in : q == 1 ? p.g_out : q == 2 ? p.g_dir : q == 3 ? p.g_und : p.g_all;
            gv = src[p.gate_scalar ? 0 : row];
        }
    }
    V bo[NB][PB], bi[NB][AH];
#pragma unroll
    for (int u = 0; u < NB - 1; ++u) load(u, bo[u], bi[u]);
#pragma unroll 1
    for (int c = 0; c < K; c += NB) {
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            const int cn = c + u + NB - 1;  // unconditional: the last round re-reads early steps (unused)
            load(cn < K ? cn : cn - K, bo[(u + NB - 1) % NB], bi[(u + NB - 1) % NB]);
            step(c + u, bo[u], bi[u]);
        }
    }
    // diagonal slots (the node itself, when it is not also one of its out-neighbours) and the stores
    const float* __restrict__ ws = W + K * 6 * RB + half * 3 * R;
#pragma unroll
    for (int i = 0; i < AH; ++i)
#pragma unroll
        for (int j = 0; j < PB; ++j) {
            const int r = i * PB + j;
            const int64_t row = (int64_t)(a0 + i) * p.Kn1 + M * K + b0 + j;
            const V xs = xrow(row);
            float s[3] = {1.f, 1.f, 1.f};
            if constexpr (GATED) {
                auto gate = [&](int q) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(gv), r * 5 + q)); };
                const float cad = gate(4) * gate(2);
                s[0] = cad * gate(0);
                s[1] = cad * gate(1);
                s[2] = gate(4) * gate(3);
            }
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                fma_v<VEC>(acc[r][k], ws[r * 3 + k], xs);
                V v = acc[r][k];
                if constexpr (GATED) v = scale_v<VEC>(v, s[k]);
                if constexpr (BF) {
                    uint16_t* dst = p.Zb + row * p.ldz + (int64_t)k * p.F + lane * VEC;
                    if (p.accumulate) v = add_v<VEC>(ld_bf<VEC>(dst), v);
                    st_bf<VEC>(dst, v);
                } else {
                    V* dst = reinterpret_cast<V*>(p.Z + row * p.ldz) + (int64_t)k * (p.zk / VEC) + lane;
                    if (p.accumulate) v = add_v<VEC>(*dst, v);
                    *dst = v;
                }
            }
        }
}

// Transposed (backward of the forward above for the symmetric n-gram matrices, A_k^T = A_k):
// dX[i] = sum_k (A_k G_k)[i], G = [G_in | G_out | G_und] ([n, 3F]). One wave per PA x PB plan block (one
// accumulator per row, so all PA*PB rows fit), the three slices of every source row gathered per step, weights
// through the scalar cache. Measured at B(20,4), F=128: 0.218 ms against 0.380 for the CSR kernel; the forward
// kernel's structure (LDS weights, two waves per block, a ring of source sets) measured 0.273 here.
template <int VEC, int PA, int PB, bool BF = false>
__global__ __launch_bounds__(256) void ngram_spmm3t_kernel(NgramP p) {
    using V = typename VT<VEC>::T;
    constexpr int R = PA * PB;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t lb = pg::xcd_logical_block(blockIdx.x, gridDim.x, p.remap != 0);
    const int pc = p.pieces > 1 ? p.pieces : 1;  // the waves of a workgroup: 4 / pc plan blocks x pc column pieces
    const int64_t wb = lb * (4 / pc) + wave / pc;
    const int64_t coff = (int64_t)(wave % pc) * 64 * VEC;
    const int nA = p.K / PA, nB = p.K / PB;
    if (wb >= (p.n_rows / ((int64_t)p.K * p.K)) * nA * nB) return;
    const int64_t M = wb / (nA * nB);
    const int rr = (int)(wb % (nA * nB));
    const int a0 = (rr / nB) * PA, b0 = (rr % nB) * PB;
    const float* __restrict__ W = p.plan + wb * p.blk;
    const V* __restrict__ G = reinterpret_cast<const V*>(p.X);
    const int64_t ldgv = p.ldx / VEC;
    const int Fv = p.F / VEC;
    auto gslice = [&](int64_t row, int k) -> V {  // this lane's VEC features of slice k of row `row`
        if constexpr (BF) return ld_bf<VEC>(p.Xb + row * p.ldx + (int64_t)k * p.F + coff + lane * VEC);
        else return G[row * ldgv + (int64_t)k * Fv + coff / VEC + lane];
    };
    V acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = zero_v<VEC>();
    const int64_t ob = (M * p.K + b0) * p.K;
    const int64_t ib = (int64_t)a0 * p.Kn2 + M;
    for (int c = 0; c < p.K; ++c) {
        V xo[PB][3], xi[PA][3];
#pragma unroll
        for (int j = 0; j < PB; ++j) {
#pragma unroll
            for (int k = 0; k < 3; ++k) xo[j][k] = gslice(ob + (int64_t)j * p.K + c, k);
        }
#pragma unroll
        for (int i = 0; i < PA; ++i) {
#pragma unroll
            for (int k = 0; k < 3; ++k) xi[i][k] = gslice((int64_t)c * p.Kn1 + ib + (int64_t)i * p.Kn2, k);
        }
        const float* __restrict__ wc = W + (int64_t)c * 6 * R;
#pragma unroll
        for (int i = 0; i < PA; ++i)
#pragma unroll
            for (int j = 0; j < PB; ++j)
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const int sl = plan_slot(i, j, PB);
                    fma_v<VEC>(acc[i * PB + j], wc[sl * 3 + k], xo[j][k]);
                    fma_v<VEC>(acc[i * PB + j], wc[3 * R + sl * 3 + k], xi[i][k]);
                }
    }
    const float* __restrict__ ws = W + (int64_t)p.K * 6 * R;
    // per a-row: its PB rows' diagonal sources and (accumulate) old dX values loaded before any of their stores, so
    // a wave waits for 4 load round trips here instead of 16 (the stores may alias the loads)
#pragma unroll
    for (int i = 0; i < PA; ++i) {
        V xs[PB][3], old[PB];
#pragma unroll
        for (int j = 0; j < PB; ++j) {
            const int64_t row = (int64_t)(a0 + i) * p.Kn1 + M * p.K + b0 + j;
#pragma unroll
            for (int k = 0; k < 3; ++k) xs[j][k] = gslice(row, k);
            old[j] = zero_v<VEC>();
            if (p.accumulate) {
                if constexpr (BF) old[j] = ld_bf<VEC>(p.Cb ? p.Cb + row * p.ldc + coff + lane * VEC
                                                           : p.Zb + row * p.ldz + coff + lane * VEC);
                else old[j] = reinterpret_cast<const V*>(p.C ? p.C + row * p.ldc + coff : p.Z + row * p.ldz + coff)[lane];
            }
        }
#pragma unroll
        for (int j = 0; j < PB; ++j) {
            const int r = i * PB + j, sl = plan_slot(i, j, PB);
            const int64_t row = (int64_t)(a0 + i) * p.Kn1 + M * p.K + b0 + j;
#pragma unroll
            for (int k = 0; k < 3; ++k) fma_v<VEC>(acc[r], ws[sl * 3 + k], xs[j][k]);
            V v = acc[r];
            if (p.accumulate) v = add_v<VEC>(old[j], v);
            if constexpr (BF) st_bf<VEC>(p.Zb + row * p.ldz + coff + lane * VEC, v);
            else reinterpret_cast<V*>(p.Z + row * p.ldz + coff)[lane] = v;
        }
    }
}

// Plan construction: one thread per CSR row scatters its entries into the row's slots (see the file comment).
__global__ __launch_bounds__(256) void ngram_plan_kernel(int K, int64_t Kn1, int64_t Kn2, int PA, int PB, int64_t n_rows,
                                                         const int64_t* rowptr, const int4* edges, float* plan,
                                                         int64_t blk, int* bad) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n_rows) return;
    const int a = (int)(i / Kn1), b = (int)(i % K);
    const int64_t M = (i % Kn1) / K;
    const int nA = K / PA, nB = K / PB;
    const int64_t wb = (M * nA + a / PA) * nB + b / PB;
    const int r = plan_slot(a % PA, b % PB, PB);
    const int R = PA * PB;
    float* W = plan + wb * blk;
    const int64_t suffix = i % Kn1, prefix = i / K;
    for (int64_t e = rowptr[i]; e < rowptr[i + 1]; ++e) {
        const int4 rec = edges[e];
        const int64_t j = rec.x;
        int64_t off;
        if (j / K == suffix) {
            off = (j % K) * 6 * R + r * 3;               // out-slot c = j mod K
        } else if (j % Kn1 == prefix) {
            off = (j / Kn1) * 6 * R + 3 * R + r * 3;     // in-slot c = j div K^(n-1)
        } else if (j == i) {
            off = (int64_t)K * 6 * R + r * 3;            // diagonal
        } else {
            atomicAdd(bad, 1);
            continue;
        }
        W[off + 0] = __int_as_float(rec.y);
        W[off + 1] = __int_as_float(rec.z);
        W[off + 2] = __int_as_float(rec.w);
    }
}

constexpr int PLAN_PA = 4, PLAN_PB = 4;

int64_t blk_floats(int K, int PA, int PB) {
    const int64_t f = ((int64_t)2 * K + 1) * 3 * PA * PB;
    return (f + 15) / 16 * 16;
}

bool pow_ok(int K, int n, int64_t n_rows, int64_t& Kn1, int64_t& Kn2) {
    if (K < 2 || n < 2 || n > 12) return false;
    int64_t v = 1;
    for (int t = 0; t < n; ++t) {
        if (v > (int64_t(1) << 40) / K) return false;
        v *= K;
        if (t == n - 3) Kn2 = v;
        if (t == n - 2) Kn1 = v;
    }
    if (n == 2) Kn2 = 1;
    return v == n_rows;
}

template <int VEC, bool T, bool BF>
int launch(const NgramP& p, hipStream_t s, bool gated) {
    const int64_t nwb = (p.n_rows / ((int64_t)p.K * p.K)) * (p.K / PLAN_PA) * (p.K / PLAN_PB);
    const unsigned nb = (unsigned)((nwb * (T && p.pieces > 1 ? p.pieces : 1) + 3) / 4);
    if constexpr (T) {
        hipLaunchKernelGGL((ngram_spmm3t_kernel<VEC, PLAN_PA, PLAN_PB, BF>), dim3(nb), dim3(256), 0, s, p);
    } else {
        if (p.K != 20) return pg::set_error(PG_ERR_UNSUPPORTED, "n-gram forward kernel built for K = 20");
        const unsigned nb2 = (unsigned)((nwb + 1) / 2);  // two waves per plan block
        if (gated) hipLaunchKernelGGL((ngram_spmm3_kernel<20, VEC, PLAN_PA, PLAN_PB, PLAN_PA / 2, 2, true, BF>), dim3(nb2), dim3(256), 0, s, p);
        else hipLaunchKernelGGL((ngram_spmm3_kernel<20, VEC, PLAN_PA, PLAN_PB, PLAN_PA / 2, 2, false, BF>), dim3(nb2), dim3(256), 0, s, p);
    }
    return PG_OK;
}

// fp32: F = 64 / 128 (forward), 64 / 128 / 256 (transposed); bf16: the transposed kernel, F = 64 / 128 / 256. (A
// bf16 forward measured slower than pg_spmm3_bf16's 16-B gathers -- 0.154 vs 0.129 ms at B(20,4), F = 128, 0.284
// vs 0.245 at F = 256: 4-B lane loads cost the texture path about what 8-B ones do -- and is not exported.)
template <bool BF>
int run(NgramP p, bool transposed, bool gated, uint32_t flags, hipStream_t s, const char* name) {
    if (BF && !transposed) return pg::set_error(PG_ERR_UNSUPPORTED, "%s: bf16 forward not built", name);
    p.remap = (flags & PG_FLAG_NO_XCD_REMAP) ? 0 : 1;
    p.zk = p.F;
    const int64_t width = transposed ? 3 * (int64_t)p.F : p.F;
    const int eb = BF ? 2 : 4;  // element bytes
    const void* xp = BF ? (const void*)p.Xb : (const void*)p.X;
    const void* zp = BF ? (const void*)p.Zb : (const void*)p.Z;
    const bool al = pg::aligned16(xp) && pg::aligned16(zp) && (p.ldx * eb) % 16 == 0 && (p.ldz * eb) % 16 == 0;
    if (!al || p.ldx < width) return pg::set_error(PG_ERR_UNSUPPORTED, "%s: needs 16-B aligned rows", name);
    int rc = PG_OK;
    if (transposed && (p.F == 64 || p.F == 128 || p.F == 256)) {
        // The 4-feature lane at F = 256 (R = 16 float4 accumulators + 24 float4 sources, 2 waves per SIMD) is latency
        // bound; at 2 features per lane the two 128-feature halves of a plan block go to two waves of one workgroup,
        // so both read a source row at about the same time (same FMAs per element, same bits:
        // profiles/r06_tsplit_probe.json). PG_FLAG_NGRAMT_WIDE / _HALVES / _NARROW pick 4 / 2 / 1 features per lane.
        int vec = (int)(p.F / 64);
        if (p.F == 256 && BF) vec = 2;
        if (flags & PG_FLAG_NGRAMT_WIDE) vec = (int)(p.F / 64);
        if ((flags & PG_FLAG_NGRAMT_HALVES) && p.F >= 128) vec = (int)(p.F / 128);
        if (flags & PG_FLAG_NGRAMT_NARROW) vec = 1;
        p.pieces = (int)(p.F / (64 * vec));
        rc = vec == 4 ? launch<4, true, BF>(p, s, false)
             : vec == 2 ? launch<2, true, BF>(p, s, false)
                        : launch<1, true, BF>(p, s, false);
        if (rc) return rc;
        return pg::check_launch(name);
    }
    switch (p.F) {
        case 64:
            if constexpr (BF) rc = launch<1, true, BF>(p, s, false);
            else rc = transposed ? launch<1, true, BF>(p, s, false) : launch<1, false, BF>(p, s, gated);
            break;
        case 128:
            if constexpr (BF) rc = launch<2, true, BF>(p, s, false);
            else rc = transposed ? launch<2, true, BF>(p, s, false) : launch<2, false, BF>(p, s, gated);
            break;
        case 256:
            if (transposed) {
                rc = launch<4, true, BF>(p, s, false);
            } else if constexpr (!BF) {
                // the F = 128 kernel on the two column halves (a 4-float-per-lane forward needs ~170 VGPRs):
                // 0.347 ms against 0.425 for the CSR kernel at B(20,4)
                NgramP q = p;
                q.F = 128;
                q.zk = 256;
                for (int h = 0; h < 2 && rc == PG_OK; ++h) {
                    q.X = p.X + 128 * h;
                    q.Z = p.Z + 128 * h;
                    rc = launch<2, false, BF>(q, s, gated);
                }
            }
            break;
        default: return pg::set_error(PG_ERR_UNSUPPORTED, "%s: F must be 64, 128 or 256", name);
    }
    if (rc) return rc;
    return pg::check_launch(name);
}

}  // namespace

extern "C" {

int64_t pg_ngram_plan_floats(int K, int n, int64_t n_rows) {
    int64_t Kn1 = 0, Kn2 = 0;
    if (!pow_ok(K, n, n_rows, Kn1, Kn2) || K % PLAN_PA || K % PLAN_PB) return -1;
    return (n_rows / ((int64_t)K * K)) * (K / PLAN_PA) * (K / PLAN_PB) * blk_floats(K, PLAN_PA, PLAN_PB);
}

int pg_ngram_plan_f32(int K, int n, int64_t n_rows, const int64_t* rowptr, const pg_edge3_t* edges, float* plan,
                      int64_t plan_floats, int* bad, void* stream) {
    int64_t Kn1 = 0, Kn2 = 0;
    PG_REQUIRE(pow_ok(K, n, n_rows, Kn1, Kn2), "n_rows %lld is not K^n (K=%d, n=%d)", (long long)n_rows, K, n);
    PG_REQUIRE(K % PLAN_PA == 0 && K % PLAN_PB == 0, "K=%d must be a multiple of %d and %d", K, PLAN_PA, PLAN_PB);
    PG_REQUIRE(plan_floats >= pg_ngram_plan_floats(K, n, n_rows), "plan buffer too small");
    PG_REQUIRE(rowptr && edges && plan && bad, "null pointer");
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(plan, 0, sizeof(float) * plan_floats, s) != hipSuccess ||
        hipMemsetAsync(bad, 0, sizeof(int), s) != hipSuccess)
        return pg::set_error(PG_ERR_HIP, "pg_ngram_plan_f32: memset failed");
    hipLaunchKernelGGL(ngram_plan_kernel, dim3((unsigned)((n_rows + 255) / 256)), dim3(256), 0, s, K, Kn1, Kn2, PLAN_PA,
                       PLAN_PB, n_rows, rowptr, reinterpret_cast<const int4*>(edges), plan,
                       blk_floats(K, PLAN_PA, PLAN_PB), bad);
    return pg::check_launch("pg_ngram_plan_f32");
}

int pg_spmm3_ngram_f32(int K, int n, int64_t n_rows, const float* plan, const float* X, int64_t ldx, int64_t F,
                       const pg_layer_args_t* gates, float* Z, int64_t ldz, uint32_t flags, void* stream) {
    int64_t Kn1 = 0, Kn2 = 0;
    PG_REQUIRE(pow_ok(K, n, n_rows, Kn1, Kn2) && K % PLAN_PA == 0 && K % PLAN_PB == 0, "bad n-gram shape");
    PG_REQUIRE(plan && X && Z, "null pointer");
    PG_REQUIRE(ldz >= 3 * F && ldx >= F, "leading dimensions too small");
    NgramP p{};
    p.K = K;
    p.n = n;
    p.Kn1 = Kn1;
    p.Kn2 = Kn2;
    p.n_rows = n_rows;
    p.plan = plan;
    p.blk = blk_floats(K, PLAN_PA, PLAN_PB);
    p.X = X;
    p.ldx = ldx;
    p.Z = Z;
    p.ldz = ldz;
    p.F = (int)F;
    if (gates) {
        PG_REQUIRE(gates->C_in && gates->C_out && gates->C_directed && gates->C_undirected && gates->C_all, "null gate");
        PG_REQUIRE(gates->gate_mode == PG_GATES_VECTOR || gates->gate_mode == PG_GATES_SCALAR, "bad gate_mode");
        PG_REQUIRE(gates->rows == nullptr, "gated propagation takes no original_indices");
        p.g_in = gates->C_in;
        p.g_out = gates->C_out;
        p.g_dir = gates->C_directed;
        p.g_und = gates->C_undirected;
        p.g_all = gates->C_all;
        p.gate_scalar = gates->gate_mode == PG_GATES_SCALAR;
    }
    return run<false>(p, false, gates != nullptr, flags, (hipStream_t)stream, "pg_spmm3_ngram_f32");
}

int pg_spmm3t_ngram_f32(int K, int n, int64_t n_rows, const float* plan, const float* G, int64_t ldg, int64_t F,
                        float* dX, int64_t lddx, int accumulate, uint32_t flags, void* stream) {
    int64_t Kn1 = 0, Kn2 = 0;
    PG_REQUIRE(pow_ok(K, n, n_rows, Kn1, Kn2) && K % PLAN_PA == 0 && K % PLAN_PB == 0, "bad n-gram shape");
    PG_REQUIRE(plan && G && dX, "null pointer");
    PG_REQUIRE(ldg >= 3 * F && lddx >= F, "leading dimensions too small");
    NgramP p{};
    p.K = K;
    p.n = n;
    p.Kn1 = Kn1;
    p.Kn2 = Kn2;
    p.n_rows = n_rows;
    p.plan = plan;
    p.blk = blk_floats(K, PLAN_PA, PLAN_PB);
    p.X = G;
    p.ldx = ldg;
    p.Z = dX;
    p.ldz = lddx;
    p.F = (int)F;
    p.accumulate = accumulate ? 1 : 0;
    return run<false>(p, true, false, flags, (hipStream_t)stream, "pg_spmm3t_ngram_f32");
}

int pg_spmm3t_ngram_bf16(int K, int n, int64_t n_rows, const float* plan, const uint16_t* G, int64_t ldg, int64_t F,
                         uint16_t* dX, int64_t lddx, int accumulate, uint32_t flags, void* stream) {
    int64_t Kn1 = 0, Kn2 = 0;
    PG_REQUIRE(pow_ok(K, n, n_rows, Kn1, Kn2) && K % PLAN_PA == 0 && K % PLAN_PB == 0, "bad n-gram shape");
    PG_REQUIRE(plan && G && dX, "null pointer");
    PG_REQUIRE(ldg >= 3 * F && lddx >= F, "leading dimensions too small");
    NgramP p{};
    p.K = K;
    p.n = n;
    p.Kn1 = Kn1;
    p.Kn2 = Kn2;
    p.n_rows = n_rows;
    p.plan = plan;
    p.blk = blk_floats(K, PLAN_PA, PLAN_PB);
    p.Xb = G;
    p.ldx = ldg;
    p.Zb = dX;
    p.ldz = lddx;
    p.F = (int)F;
    p.accumulate = accumulate ? 1 : 0;
    return run<true>(p, true, false, flags, (hipStream_t)stream, "pg_spmm3t_ngram_bf16");
}

int pg_spmm3t_ngram_add_bf16(int K, int n, int64_t n_rows, const float* plan, const uint16_t* G, int64_t ldg,
                             int64_t F, const uint16_t* C, int64_t ldc, uint16_t* dX, int64_t lddx, uint32_t flags,
                             void* stream) {
    int64_t Kn1 = 0, Kn2 = 0;
    PG_REQUIRE(pow_ok(K, n, n_rows, Kn1, Kn2) && K % PLAN_PA == 0 && K % PLAN_PB == 0, "bad n-gram shape");
    PG_REQUIRE(plan && G && C && dX, "null pointer");
    PG_REQUIRE(ldg >= 3 * F && ldc >= F && lddx >= F, "leading dimensions too small");
    PG_REQUIRE(pg::aligned16(C) && (ldc * 2) % 16 == 0, "pg_spmm3t_ngram_add_bf16: needs 16-B aligned rows");
    NgramP p{};
    p.K = K;
    p.n = n;
    p.Kn1 = Kn1;
    p.Kn2 = Kn2;
    p.n_rows = n_rows;
    p.plan = plan;
    p.blk = blk_floats(K, PLAN_PA, PLAN_PB);
    p.Xb = G;
    p.ldx = ldg;
    p.Zb = dX;
    p.ldz = lddx;
    p.Cb = C;
    p.ldc = ldc;
    p.F = (int)F;
    p.accumulate = 1;
    return run<true>(p, true, false, flags, (hipStream_t)stream, "pg_spmm3t_ngram_add_bf16");
}

}  // extern "C"
