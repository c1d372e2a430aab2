// bf16 mode of the DirectGCN hot path (BASELINE config 5: "bf16 (fp32 accumulate)").
//
// Storage is bf16 (features X, aggregates Z, layer outputs Y, and their gradients); every sum is fp32 and
// rounded once to bf16 (round-to-nearest-even, torch's float -> bfloat16 rule) when stored. Parameters
// stay fp32 (the caller's master weights); the packed contraction operand is a bf16 copy.
//
//  pg_spmm3_bf16   -- the three propagations of protgram_directgcn.py:101-112 (as pg_spmm3_f32): half the
//                     gathered bytes of fp32. Same record window and entry order, fp32 FMA accumulation
//                     (v_pk_fma_f32), so Z is within one bf16 rounding of bf16(fp32 propagate(X)).
//  pg_spmm3t_bf16  -- its transpose (backward), "gather 3, write 1".
//  pg_directgcn_dense_bf16 -- the gated contraction + epilogue of pg_directgcn_dense_f32 on
//                     v_mfma_f32_32x32x16_bf16 (16x the fp32 MFMA rate): the dense layer becomes HBM-bound.
//                     The gate scale s_q[m] is applied to Z when its tile is staged (one extra bf16
//                     rounding of s*Z); bias sums, constant, residual and leaky_relu in fp32.
// MFMA operand maps (32x32x16 bf16): lane l (r = l&31, h = l>>5) holds A[r][8h..8h+7] and B[8h..8h+7][r],
// i.e. one ds_read_b128 of a k-contiguous LDS row each; C/D: col = lane&31, row = (r&3)+8(r>>2)+4h.
#include <algorithm>

#include "pg_bf16_util.h"
#include "pg_common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
using pgbf::bf16x8;
using pgbf::f2bf;
using pgbf::pack2;
using pgbf::pack8;
using pgbf::unpack8;
__device__ __forceinline__ float bf_lo(uint32_t w) { return pgbf::lo(w); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return pgbf::hi(w); }
__device__ __forceinline__ float fb(int v) { return __int_as_float(v); }

// ------------------------------------------------------------------------------------------------
// SpMM, record-window variant (pg_spmm.hip variant C) over bf16 rows: LPR lanes x 8 features per row.
// ------------------------------------------------------------------------------------------------
struct SpmmB {
    int64_t n_rows;
    const int64_t* rowptr;
    const int32_t* row_order;
    const int4* edges;   // {col, w_in, w_out, w_und}
    const uint16_t* X;   // [.., F] bf16 (transpose: [.., 3F])
    int64_t ldx;
    uint16_t* Z;         // [n_rows, 3F] bf16 (transpose: [n_rows, F])
    int64_t ldz;
    int F;
    int remap;
};

template <int LPR, int U, bool TRANS>
__global__ __launch_bounds__(256) void spmm_bf16_kernel(SpmmB p) {
    constexpr int RPB = 256 / LPR;
    constexpr int NACC = TRANS ? 1 : 3;
    constexpr int NSL = TRANS ? 3 : 1;
    constexpr int WIN = LPR;
    __shared__ int4 win[RPB][WIN];
    const int64_t lb = pg::xcd_logical_block(blockIdx.x, gridDim.x, p.remap != 0);
    const int grp = threadIdx.x / LPR;
    const int t = threadIdx.x % LPR;
    const int64_t pos = lb * RPB + grp;
    const bool live = pos < p.n_rows;
    const int64_t row = (live && p.row_order) ? (int64_t)p.row_order[pos] : pos;
    const uint4* __restrict__ X8 = reinterpret_cast<const uint4*>(p.X);
    const int64_t ldx8 = p.ldx >> 3;
    const int F8 = p.F >> 3;
    int64_t beg = 0, end = 0;
    if (live) {
        beg = p.rowptr[row];
        end = p.rowptr[row + 1];
    }
    float acc[NACC][8];
#pragma unroll
    for (int a = 0; a < NACC; ++a)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[a][e] = 0.f;

    auto consume = [&](const int4& r, const uint4 (&xv)[NSL]) {
        float x0[8];
        unpack8(xv[0], x0);
        // fused multiply-add (v_pk_fma_f32, two features per instruction): half the VALU work of the
        // separately rounded fp32 kernels, which the VALU-bound bf16 gather needs; the single bf16
        // rounding of the result dominates the difference.
        if constexpr (!TRANS) {
            const float wi = fb(r.y), wo = fb(r.z), wu = fb(r.w);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                acc[0][e] = __builtin_fmaf(wi, x0[e], acc[0][e]);
                acc[1][e] = __builtin_fmaf(wo, x0[e], acc[1][e]);
                acc[2][e] = __builtin_fmaf(wu, x0[e], acc[2][e]);
            }
        } else {
            float x1[8], x2[8];
            unpack8(xv[1], x1);
            unpack8(xv[2], x2);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                float a = acc[0][e];
                a = __builtin_fmaf(fb(r.y), x0[e], a);
                a = __builtin_fmaf(fb(r.z), x1[e], a);
                a = __builtin_fmaf(fb(r.w), x2[e], a);
                acc[0][e] = a;
            }
        }
    };

    int4* mywin = win[grp];
    int4 nxt = (beg + t < end) ? p.edges[beg + t] : make_int4(0, 0, 0, 0);
    for (int64_t w0 = beg; w0 < end; w0 += WIN) {
        __builtin_amdgcn_wave_barrier();
        mywin[t] = nxt;
        __builtin_amdgcn_wave_barrier();
        const int64_t wn = w0 + WIN;
        if (wn + t < end) nxt = p.edges[wn + t];
        const int n = (int)((end - w0) < WIN ? (end - w0) : WIN);
        int j = 0;
        for (; j + U <= n; j += U) {
            int4 r[U];
#pragma unroll
            for (int u = 0; u < U; ++u) r[u] = mywin[j + u];
            uint4 xv[U][NSL];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint4* src = X8 + (int64_t)r[u].x * ldx8 + t;
#pragma unroll
                for (int s = 0; s < NSL; ++s) xv[u][s] = src[s * F8];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) consume(r[u], xv[u]);
        }
        for (; j < n; ++j) {
            const int4 r = mywin[j];
            const uint4* src = X8 + (int64_t)r.x * ldx8 + t;
            uint4 xv[NSL];
#pragma unroll
            for (int s = 0; s < NSL; ++s) xv[s] = src[s * F8];
            consume(r, xv);
        }
    }
    if (!live) return;
    uint4* Z8 = reinterpret_cast<uint4*>(p.Z) + row * (p.ldz >> 3) + t;
#pragma unroll
    for (int a = 0; a < NACC; ++a) Z8[a * F8] = pack8(acc[a]);
}

template <bool TRANS>
int spmm_bf16_dispatch(SpmmB p, uint32_t flags, hipStream_t s, const char* name) {
    if (p.n_rows == 0) return PG_OK;
    p.remap = (flags & PG_FLAG_NO_XCD_REMAP) ? 0 : 1;
    const bool ok = p.F % 8 == 0 && p.ldx % 8 == 0 && p.ldz % 8 == 0 && pg::aligned16(p.X) && pg::aligned16(p.Z) &&
                    pg::aligned16(p.edges);
    if (!ok) return pg::set_error(PG_ERR_UNSUPPORTED, "%s: needs F, ldx, ldz multiples of 8 and 16-B alignment", name);
    // gathers in flight per lane: 4 (default), 8 with PG_FLAG_UNROLL4. Measured at B(20,4) F=128
    // (tools/variant_probe.py): forward 0.129 / 0.133 ms (U=16: 0.201), transpose 0.208 / 0.229 ms.
    const bool deep = flags & PG_FLAG_UNROLL4;
#define PG_BF_LAUNCH(LPRv)                                                                                     \
    do {                                                                                                       \
        constexpr int RPB = 256 / (LPRv);                                                                      \
        const int64_t nb = (p.n_rows + RPB - 1) / RPB;                                                         \
        if (deep) hipLaunchKernelGGL((spmm_bf16_kernel<LPRv, 8, TRANS>), dim3((unsigned)nb), dim3(256), 0, s, p);  \
        else hipLaunchKernelGGL((spmm_bf16_kernel<LPRv, 4, TRANS>), dim3((unsigned)nb), dim3(256), 0, s, p);       \
    } while (0)
    switch (p.F) {
        case 16: PG_BF_LAUNCH(2); break;
        case 32: PG_BF_LAUNCH(4); break;
        case 64: PG_BF_LAUNCH(8); break;
        case 128: PG_BF_LAUNCH(16); break;
        case 256: PG_BF_LAUNCH(32); break;
        case 512: PG_BF_LAUNCH(64); break;
        default:
            return pg::set_error(PG_ERR_UNSUPPORTED, "%s: F=%d not in {16,32,64,128,256,512}", name, p.F);
    }
#undef PG_BF_LAUNCH
    return pg::check_launch(name);
}

// ------------------------------------------------------------------------------------------------
// Dense contraction + epilogue on bf16 MFMA
// ------------------------------------------------------------------------------------------------
constexpr int BKB = 64;   // K per tile (4 MFMA k-steps of 16)
constexpr int LDK = 72;   // LDS row in bf16 (144 B = 36 dwords: conflict-free ds_read_b128 per 16-lane group)

struct DenseB {
    int64_t M;
    int F_in, F_out, K;
    const uint16_t* Z;
    int64_t ldz;
    const uint16_t* Bp;  // [F_out, K] bf16
    const float* bsum;   // [4, F_out]
    int gate_mode;
    const float *C_in, *C_out, *C_dir, *C_und, *C_all;
    const int64_t* rows;
    const float* constant;
    int64_t ld_const;
    const uint16_t* res_x;
    int64_t ld_res;
    int proj_res;
    int act;
    float slope;
    uint16_t* Y;
    int64_t ldy;
    int remap;
    uint32_t drop_thr;  // fused layer dropout (pg_dense.hip DenseP::drop_*)
    float drop_s;
    const int64_t* drop_seed;
};

__device__ __forceinline__ float4 ld4f(const float* p) { return *reinterpret_cast<const float4*>(p); }

template <int BM, int BN, int NW>
__global__ __launch_bounds__(64 * NW) void dense_bf16_kernel(DenseB p) {
    constexpr int NT = 64 * NW;
    const uint64_t dseed = p.drop_s != 0.f ? (uint64_t)*p.drop_seed : 0ull;
    constexpr int WN = 2, WM = NW / WN;
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    static_assert(TM >= 1 && TN >= 1, "wave tile");
    constexpr int A_C = BM * BKB / 8 / NT;  // 16-B chunks per thread
    constexpr int B_C = BN * BKB / 8 / NT;
    static_assert(A_C >= 1 && B_C >= 1, "chunks");
    constexpr int TLD = BN + 4;
    constexpr int MAIN_BYTES = 2 * (BM + BN) * LDK * 2;
    constexpr int EPI_BYTES = BM * TLD * 4;
    constexpr int SMEM_BYTES = MAIN_BYTES > EPI_BYTES ? MAIN_BYTES : EPI_BYTES;
    __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM_BYTES];
    __shared__ __attribute__((aligned(16))) float Sg[BM * 4];
    __shared__ int64_t Crow[BM];
    uint16_t* As = reinterpret_cast<uint16_t*>(smem);
    uint16_t* Bs = As + 2 * BM * LDK;

    const int64_t n_mblk = (p.M + BM - 1) / BM;
    const int64_t lb = pg::xcd_logical_block(blockIdx.x, gridDim.x, p.remap != 0);
    const int64_t m0 = (lb % n_mblk) * BM;
    const int n0 = (int)(lb / n_mblk) * BN;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int wm = wave / WN, wn = wave % WN;
    const int li = lane & 31, lh = lane >> 5;

    if (tid < BM) {
        const int64_t m = m0 + tid;
        float s0 = 0.f, s1 = 0.f, s2 = 0.f;
        if (m < p.M) {
            const int64_t r = (p.gate_mode == PG_GATES_SCALAR) ? 0 : (p.rows ? p.rows[m] : m);
            const float ci = p.C_in[r], co = p.C_out[r], cd = p.C_dir[r], cu = p.C_und[r], ca = p.C_all[r];
            const float cad = ca * cd;
            s0 = cad * ci;
            s1 = cad * co;
            s2 = ca * cu;
        }
        Sg[tid * 4 + 0] = s0;
        Sg[tid * 4 + 1] = s1;
        Sg[tid * 4 + 2] = s2;
        Sg[tid * 4 + 3] = 1.f;
        Crow[tid] = m < p.M ? (p.rows ? p.rows[m] : m) : -1;
    }
    __syncthreads();

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    uint4 ra[A_C], rb[B_C];
    const int64_t mlast = p.M - 1;
    auto fetch = [&](int k0) {
#pragma unroll
        for (int q = 0; q < A_C; ++q) {
            const int idx = tid + NT * q;
            const int64_t m = min(m0 + (idx >> 3), mlast);
            const int k = k0 + 8 * (idx & 7);
            const int kc = k < p.K ? k : 0;
            const int seg = kc / p.F_in;
            const uint16_t* src = seg < 3 ? p.Z + m * p.ldz + kc : p.res_x + m * p.ld_res + (kc - 3 * p.F_in);
            ra[q] = *reinterpret_cast<const uint4*>(src);
        }
#pragma unroll
        for (int q = 0; q < B_C; ++q) {
            const int idx = tid + NT * q;
            const int n = min(n0 + (idx >> 3), p.F_out - 1);
            const int k = k0 + 8 * (idx & 7);
            rb[q] = *reinterpret_cast<const uint4*>(p.Bp + (int64_t)n * p.K + (k < p.K ? k : 0));
        }
    };
    auto stash = [&](int buf, int k0) {
        uint16_t* Ab = As + buf * BM * LDK;
        uint16_t* Bb = Bs + buf * BN * LDK;
#pragma unroll
        for (int q = 0; q < A_C; ++q) {
            const int idx = tid + NT * q;
            const int k = k0 + 8 * (idx & 7);
            uint4 v = ra[q];
            if (k >= p.K) {
                v = make_uint4(0u, 0u, 0u, 0u);
            } else {
                const int seg = k / p.F_in;
                if (seg < 3) {
                    const float sc = Sg[(idx >> 3) * 4 + seg];
                    float f[8];
                    unpack8(v, f);
#pragma unroll
                    for (int e = 0; e < 8; ++e) f[e] *= sc;
                    v = pack8(f);
                }
            }
            *reinterpret_cast<uint4*>(&Ab[(idx >> 3) * LDK + 8 * (idx & 7)]) = v;
        }
#pragma unroll
        for (int q = 0; q < B_C; ++q) {
            const int idx = tid + NT * q;
            const int k = k0 + 8 * (idx & 7);
            *reinterpret_cast<uint4*>(&Bb[(idx >> 3) * LDK + 8 * (idx & 7)]) =
                k < p.K ? rb[q] : make_uint4(0u, 0u, 0u, 0u);
        }
    };

    const int ntiles = (p.K + BKB - 1) / BKB;
    fetch(0);
    stash(0, 0);
    __syncthreads();
    for (int t = 0; t < ntiles; ++t) {
        const int cur = t & 1;
        if (t + 1 < ntiles) fetch((t + 1) * BKB);
        const uint16_t* Ab = As + cur * BM * LDK;
        const uint16_t* Bb = Bs + cur * BN * LDK;
#pragma unroll
        for (int kk = 0; kk < BKB / 16; ++kk) {
            bf16x8 a[TM], b[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
                a[i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(
                                                      &Ab[(wm * TM * 32 + i * 32 + li) * LDK + kk * 16 + 8 * lh]));
#pragma unroll
            for (int j = 0; j < TN; ++j)
                b[j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(
                                                      &Bb[(wn * TN * 32 + j * 32 + li) * LDK + kk * 16 + 8 * lh]));
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        if (t + 1 < ntiles) stash(cur ^ 1, (t + 1) * BKB);
        __syncthreads();
    }

    float* T = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int rl = wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                T[rl * TLD + wn * TN * 32 + j * 32 + li] = acc[i][j][r];
            }
    __syncthreads();

    constexpr int C4 = BN / 4;
    constexpr int ITER = BM * C4 / NT;
    const int c4 = tid % C4;
    const int nb = n0 + 4 * c4;
    const bool has_const = p.constant && p.gate_mode == PG_GATES_VECTOR;
    const bool id_res = p.res_x && !p.proj_res;
    float b0[4], b1[4], b2[4], br[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const bool ok = nb + e < p.F_out;
        b0[e] = ok ? p.bsum[nb + e] : 0.f;
        b1[e] = ok ? p.bsum[p.F_out + nb + e] : 0.f;
        b2[e] = ok ? p.bsum[2 * p.F_out + nb + e] : 0.f;
        br[e] = (ok && p.proj_res) ? p.bsum[3 * p.F_out + nb + e] : 0.f;
    }
    for (int it = 0; it < ITER; ++it) {
        const int rl = (tid + NT * it) / C4;
        const int64_t m = m0 + rl;
        if (Crow[rl] < 0 || nb >= p.F_out) continue;
        const float* sg = &Sg[rl * 4];
        const float4 v = *reinterpret_cast<const float4*>(&T[rl * TLD + 4 * c4]);
        float o[4] = {v.x, v.y, v.z, v.w};
        float cc[4] = {0.f, 0.f, 0.f, 0.f}, rr[4] = {0.f, 0.f, 0.f, 0.f};
        if (has_const) {
            const float4 c = ld4f(p.constant + Crow[rl] * p.ld_const + nb);
            cc[0] = c.x; cc[1] = c.y; cc[2] = c.z; cc[3] = c.w;
        }
        if (id_res) {
            const uint2 r2 = *reinterpret_cast<const uint2*>(p.res_x + m * p.ld_res + nb);
            rr[0] = bf_lo(r2.x); rr[1] = bf_hi(r2.x); rr[2] = bf_lo(r2.y); rr[3] = bf_hi(r2.y);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float y = o[e] + (sg[0] * b0[e] + sg[1] * b1[e] + sg[2] * b2[e]) + br[e] + cc[e] + rr[e];
            if (p.act) y = y > 0.f ? y : y * p.slope;
            if (p.drop_s != 0.f)
                y = (pg::drop_hash(dseed, (uint32_t)(m * p.F_out + nb + e)) >> 8) >= p.drop_thr ? y * p.drop_s : 0.f;
            o[e] = y;
        }
        *reinterpret_cast<uint2*>(p.Y + m * p.ldy + nb) = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
    }
}

__global__ __launch_bounds__(256) void f32_to_bf16_kernel(int64_t n, const float* in, uint16_t* out) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        out[i] = (uint16_t)f2bf(in[i]);
}

}  // namespace

extern "C" {

int pg_f32_to_bf16(int64_t n, const float* in, uint16_t* out, void* stream) {
    PG_REQUIRE(n >= 0 && (n == 0 || (in && out)), "bad arguments");
    if (n == 0) return PG_OK;
    const int nb = (int)std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, n, in, out);
    return pg::check_launch("pg_f32_to_bf16");
}

int pg_spmm3_bf16(int64_t n_rows, const int64_t* rowptr, const int32_t* row_order, const pg_edge3_t* edges,
                  const uint16_t* X, int64_t ldx, int64_t F, uint16_t* Z, int64_t ldz, uint32_t flags, void* stream) {
    PG_REQUIRE(n_rows >= 0 && F > 0 && F < (1 << 20), "bad shape");
    PG_REQUIRE(n_rows == 0 || (rowptr && edges && X && Z), "null pointer");
    PG_REQUIRE(ldx >= F && ldz >= 3 * F, "bad leading dimension");
    SpmmB p{n_rows, rowptr, row_order, reinterpret_cast<const int4*>(edges), X, ldx, Z, ldz, (int)F, 1};
    return spmm_bf16_dispatch<false>(p, flags, (hipStream_t)stream, "pg_spmm3_bf16");
}

int pg_spmm3t_bf16(int64_t n_rows, const int64_t* rowptr, const int32_t* row_order, const pg_edge3_t* edges,
                   const uint16_t* G, int64_t ldg, int64_t F, uint16_t* dX, int64_t lddx, uint32_t flags,
                   void* stream) {
    PG_REQUIRE(n_rows >= 0 && F > 0 && F < (1 << 20), "bad shape");
    PG_REQUIRE(n_rows == 0 || (rowptr && edges && G && dX), "null pointer");
    PG_REQUIRE(ldg >= 3 * F && lddx >= F, "bad leading dimension");
    SpmmB p{n_rows, rowptr, row_order, reinterpret_cast<const int4*>(edges), G, ldg, dX, lddx, (int)F, 1};
    return spmm_bf16_dispatch<true>(p, flags, (hipStream_t)stream, "pg_spmm3t_bf16");
}

int pg_directgcn_dense_bf16(const pg_layer_args_t* a, const float* packed, const uint16_t* packed_bf16,
                            uint32_t flags, void* stream) {
    PG_REQUIRE(a != nullptr && packed != nullptr && packed_bf16 != nullptr, "null args");
    PG_REQUIRE(a->M >= 0 && a->F_in > 0 && a->F_out > 0 && a->F_in < (1 << 20) && a->F_out < (1 << 20), "bad shape");
    if (a->M == 0) return PG_OK;
    PG_REQUIRE(a->Z && a->ldz >= 3 * a->F_in, "Z must be [M, >=3*F_in]");
    PG_REQUIRE(a->C_in && a->C_out && a->C_directed && a->C_undirected && a->C_all, "null gate");
    PG_REQUIRE(a->gate_mode == PG_GATES_VECTOR || a->gate_mode == PG_GATES_SCALAR, "bad gate_mode");
    PG_REQUIRE(!a->W_res || a->res_x, "W_res needs res_x");
    PG_REQUIRE(!a->res_x || a->W_res || a->F_in == a->F_out, "identity residual needs F_in == F_out");
    PG_REQUIRE(a->Y && a->ldy >= a->F_out, "bad output");
    const uint16_t* Zb = reinterpret_cast<const uint16_t*>(a->Z);
    const uint16_t* Rb = reinterpret_cast<const uint16_t*>(a->res_x);
    uint16_t* Yb = reinterpret_cast<uint16_t*>(a->Y);
    const bool ok = a->F_in % 8 == 0 && a->F_out % 4 == 0 && a->ldz % 8 == 0 && a->ldy % 4 == 0 &&
                    pg::aligned16(Zb) && pg::aligned16(packed_bf16) && (reinterpret_cast<uintptr_t>(Yb) & 7) == 0 &&
                    (!a->constant || (a->ld_const % 4 == 0 && pg::aligned16(a->constant))) &&
                    (!a->res_x || (a->ld_res % 8 == 0 && pg::aligned16(Rb)));
    if (!ok)
        return pg::set_error(PG_ERR_UNSUPPORTED, "pg_directgcn_dense_bf16: needs F_in % 8, F_out % 4, matching leading "
                                                 "dimensions and 16-B aligned buffers");
    DenseB p{};
    p.M = a->M;
    p.F_in = (int)a->F_in;
    p.F_out = (int)a->F_out;
    p.K = (int)((a->W_res ? 4 : 3) * a->F_in);
    p.Z = Zb;
    p.ldz = a->ldz;
    p.Bp = packed_bf16;
    p.bsum = packed + (int64_t)p.F_out * p.K;
    p.gate_mode = a->gate_mode;
    p.C_in = a->C_in;
    p.C_out = a->C_out;
    p.C_dir = a->C_directed;
    p.C_und = a->C_undirected;
    p.C_all = a->C_all;
    p.rows = a->rows;
    p.constant = a->constant;
    p.ld_const = a->ld_const;
    p.res_x = Rb;
    p.ld_res = a->ld_res;
    p.proj_res = a->W_res ? 1 : 0;
    p.act = a->act;
    p.slope = a->slope;
    p.Y = Yb;
    p.ldy = a->ldy;
    p.remap = (flags & PG_FLAG_NO_XCD_REMAP) ? 0 : 1;
    if (const int rc = pg::drop_params(a, p.drop_thr, p.drop_s)) return rc;
    p.drop_seed = a->drop_seed;
    PG_REQUIRE(p.drop_s == 0.f || a->M * a->F_out <= (int64_t(1) << 32), "fused dropout: M * F_out > 2^32");
    constexpr int BM = 128, BN = 128, NW = 8;
    const int64_t nb = ((p.M + BM - 1) / BM) * ((p.F_out + BN - 1) / BN);
    hipLaunchKernelGGL((dense_bf16_kernel<BM, BN, NW>), dim3((unsigned)nb), dim3(64 * NW), 0, (hipStream_t)stream, p);
    return pg::check_launch("pg_directgcn_dense_bf16");
}

}  // extern "C"
