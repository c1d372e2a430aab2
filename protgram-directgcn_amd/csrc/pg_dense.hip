// DirectGCN dense contraction + gated combine on gfx950 MFMA. Kernels (dispatch in pg_directgcn_dense_f32):
//  * dense_x3p_kernel (default, F_in = F_out = 128, no row map): split-bf16 W-stationary, software-pipelined on
//    16-row tiles (v_mfma_f32_16x16x32_bf16, exact three-way bf16 splits: fp32-level accuracy); reads the
//    unpacked weights when `packed` is NULL;
//  * dense_x3_kernel: the same on 32-row tiles without the pipeline (F_in = 64 with a projected residual);
//  * dense_kernel: the tiled fp32 GEMM described below (every other shape, row maps, projected residuals;
//    PG_FLAG_DENSE_TILED forces it).
// Tiled fp32 kernel (v_mfma_f32_32x32x2_f32):
//
// After the fused propagation Z = [A_in X | A_out X | A_und X] (pg_spmm.hip), the layer output of
// src/models/protgram_directgcn.py:100-133 is, with A(xW) = (Ax)W,
//   y[m] = sum_k s_k[m] * (Z_k[m] (W_main_k + W_shared)^T + b_main_k + b_shared_k) + constant[r(m)]
//   s_in = c_all*c_dir*c_in,  s_out = c_all*c_dir*c_out,  s_und = c_all*c_und
// i.e. ONE GEMM with K = 3*F_in (4*F_in with the model's projected residual as a 4th segment).
//
//  pg_directgcn_pack_f32  -- packs B = [W_mi+W_s | W_mo+W_s | W_u+W_s (| W_res)] ([F_out, K]) and the
//                            bias sums ([3, F_out]); packed on every call (parameters can change in place).
//  pg_directgcn_dense_f32 -- A-loader scales Z by the per-row gate (gates computed once per block into LDS,
//                            gathered through original_indices when given); epilogue adds the gated bias
//                            sums, the per-node constant, the residual and leaky_relu, then stores y once.
//
// Tiling: 512 threads = 8 waves of 32x32; block tile BM=128 x BN (128 or 64) x BK=32; operands staged
// global -> registers -> LDS (rows padded to 36 floats: conflict-free ds_read_b128) into a double
// buffer, one barrier per K tile; the next tile's global loads are in flight during the MFMAs. Each
// lane feeds its MFMAs with one ds_read_b128 per operand per 4 MFMAs by permuting K identically for A
// and B inside each group of 8 (MFMA k-step s of lane half h uses k = 4h + s): same sum, other order.
#include "pg_common.h"
#include "pg_split3.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BK = 32;
constexpr int LDSW = 36;  // padded LDS row (floats)

struct DenseP {
    int64_t M;
    int F_in, F_out, K;
    const float* Z;
    int64_t ldz;
    const float* Bp;    // packed [F_out, K]
    const float* bsum;  // packed [3, F_out]
    int gate_mode;
    const float *C_in, *C_out, *C_dir, *C_und, *C_all;
    const int64_t* rows;
    const float* constant;
    int64_t ld_const;
    const float* res_x;
    int64_t ld_res;
    int proj_res;  // residual is the 4th K segment (+ b_res in bsum row 3)
    int vec_out;   // float4 epilogue (F_out, ldy, ld_const, ld_res multiples of 4; 16-B aligned)
    int act;
    float slope;
    float* Y;
    int64_t ldy;
    int remap;
    int pregated;  // A segments 0..2 already carry their gates (pg_spmm3_gated_f32): no scaling here
    // unpacked weights (packed == NULL; the pipelined split-bf16 kernel forms W_q + W_shared and the bias sums
    // itself, with the pack kernel's fp32 adds)
    int rawW;
    const float *Wq0, *Wq1, *Wq2, *Wsh;
    const float *bm0, *bs0, *bm1, *bs1, *bm2, *bs2;
    // n-gram row map (pg_directgcn_dense_ngram_rows_f32; pipelined split-bf16 kernel only): row m of Z (middle-major
    // rows of the middles map_m0, map_m0 + 1, ...: m = 400 (M - map_m0) + 20 a + b) reads its residual row (map_res)
    // and / or writes its output row (map_y) at the global n-gram row a.M.b = a K^(n-1) + 20 M + b
    int64_t map_kn1, map_m0;
    int map_res, map_y;
    int nt_a;  // pipelined kernels: A rows and the per-node constant (read once) by non-temporal LDS-DMA
               // (PG_FLAG_DENSE_A_CACHED clears)
    int exp;  // diagnostics build only (PG_DENSE_EXP, tools/dense_exp.py): phases skipped in dense_x3p_kernel
    // fused layer dropout after the activation (drop_s = 1 / (1 - p); 0: none): pg::drop_hash of (*drop_seed, the
    // element's index m * F_out + j over the launch's rows) against drop_thr
    uint32_t drop_thr;
    float drop_s;
    const int64_t* drop_seed;
};

// the fused dropout of output element (m, j) on an activated value y (DenseP::drop_*)
__device__ __forceinline__ float drop_apply(const DenseP& p, uint64_t seed, int64_t m, int j, float y) {
    const uint32_t e = (uint32_t)(m * p.F_out + j);
    return (pg::drop_hash(seed, e) >> 8) >= p.drop_thr ? y * p.drop_s : 0.f;
}
__device__ __forceinline__ uint64_t drop_seed_of(const DenseP& p) {
    return p.drop_s != 0.f ? (uint64_t)*p.drop_seed : 0ull;
}

// Diagnostics build only: dense_x3p_kernel timing experiments, flag bits 24..28 (bit 0: no MFMAs, 1: no split,
// 2: no Y stores, 3: no A DMA, 4: no constant / residual DMA). Results are garbage in those runs.
#ifdef PG_DENSE_EXP
#define DEXP(bit) ((p.exp >> (bit)) & 1)
// per-iteration s_memtime stamps of dense_x3p_kernel (tools/dense_exp.py --stamps): blocks < DST_BLOCKS, waves 0 and
// 4 (the MFMA-first and the split-first wave of SIMD 0), iterations < DST_IT, points < DST_PT; vector stores into a
// buffer of their own (no kernel output depends on them)
constexpr int DST_BLOCKS = 64, DST_IT = 48, DST_PT = 8;
__device__ unsigned long long* g_dense_stamps = nullptr;
// the buffer pointer is read once at kernel entry (DSTAMP_INIT): re-reading the device symbol at every stamp put a
// dependent global load on the critical path
#define DSTAMP_INIT unsigned long long* const dst_base_ = g_dense_stamps
#define DSTAMP(it, pt)                                                                                             \
    do {                                                                                                           \
        if (dst_base_ && lane == 0 && (wave == 0 || wave == 4) && blockIdx.x < DST_BLOCKS && (it) < DST_IT)        \
            dst_base_[((blockIdx.x * 2 + (wave >> 2)) * DST_IT + (it)) * DST_PT + (pt)] =                          \
                __builtin_amdgcn_s_memtime();                                                                      \
    } while (0)
#else
#define DEXP(bit) 0
#define DSTAMP_INIT \
    do {            \
    } while (0)
#define DSTAMP(it, pt) \
    do {               \
    } while (0)
#endif

// global n-gram row of middle-major row m (K = 20: 400 rows per middle); see DenseP::map_*
__device__ __forceinline__ int64_t ngram_row(const DenseP& p, int64_t m) {
    const int r = (int)m;  // rows of one launch < 2^31 (checked on the host)
    const int q = r / 400, w = r - 400 * q;
    const int a = w / 20, b = w - 20 * a;
    return (int64_t)a * p.map_kn1 + (p.map_m0 + q) * 20 + b;
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float4 scale4(float4 a, float s) { return make_float4(a.x * s, a.y * s, a.z * s, a.w * s); }

__device__ __forceinline__ int seg_of(int k, int F) { return (k >= F) + (k >= 2 * F) + (k >= 3 * F); }

// one element of the logical A matrix [M, K]
__device__ __forceinline__ float a_elem(const DenseP& p, const float* sg, int64_t m, int k) {
    const int q = seg_of(k, p.F_in);
    if (q < 3) return p.pregated ? p.Z[m * p.ldz + k] : p.Z[m * p.ldz + k] * sg[q];
    return p.res_x[m * p.ld_res + (k - 3 * p.F_in)];
}

template <int BM, int BN, int NW, bool VEC>
__global__ __launch_bounds__(64 * NW) void dense_kernel(DenseP p) {
    constexpr int NT = 64 * NW;  // threads
    const uint64_t dseed = drop_seed_of(p);
    constexpr int WN = (BM == 64 && NW == 8) ? 4 : (BN == 128 || BM == 64 || NW == 8) ? 2 : 1;
    constexpr int WM = NW / WN;
    static_assert(BM / WM >= 32 && BN / WN >= 32, "wave tile too small");
    constexpr int TM = BM / WM / 32;
    constexpr int TN = BN / WN / 32;
    constexpr int A_F4 = BM * BK / 4 / NT;
    constexpr int B_F4 = BN * BK / 4 / NT;

    constexpr int TLD = BN + 4;  // epilogue tile row (floats), 16-B aligned, conflict-free float4 reads
    constexpr int MAIN_FLOATS = 2 * BM * LDSW + 2 * BN * LDSW;
    constexpr int SMEM_FLOATS = MAIN_FLOATS > BM * TLD ? MAIN_FLOATS : BM * TLD;
    __shared__ __attribute__((aligned(16))) float smem[SMEM_FLOATS];
    __shared__ __attribute__((aligned(16))) float Sg[BM * 4];
    __shared__ int64_t Crow[BM];  // constant row per tile row (original_indices), -1 past M
    static_assert(BM <= NT, "gate prologue assumes one thread per tile row");
    float (*As)[BM * LDSW] = reinterpret_cast<float (*)[BM * LDSW]>(smem);
    float (*Bs)[BN * LDSW] = reinterpret_cast<float (*)[BN * LDSW]>(smem + 2 * BM * LDSW);

    const int64_t n_mblk = (p.M + BM - 1) / BM;
    const int64_t lb = pg::xcd_logical_block(blockIdx.x, gridDim.x, p.remap != 0);
    const int64_t m0 = (lb % n_mblk) * BM;
    const int n0 = (int)(lb / n_mblk) * BN;
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int wm = wave / WN, wn = wave % WN;
    const int li = lane & 31, lh = lane >> 5;

    if (tid < BM) {  // gates, protgram_directgcn.py:116-133
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

    // Global loads are issued raw (branch-free: clamped addresses) so they stay in flight across the
    // MFMA phase; the gate scale / zero-fill is applied at stash time, just before the LDS write.
    float4 ra[A_F4], rb[B_F4];
    const int64_t mlast = p.M - 1;
    auto fetch_to = [&](int k0, float4 (&ra)[A_F4], float4 (&rb)[B_F4]) {
#pragma unroll
        for (int q = 0; q < A_F4; ++q) {
            const int idx = tid + NT * q;
            const int64_t m = min(m0 + (idx >> 3), mlast);
            const int k = k0 + 4 * (idx & 7);
            if (VEC) {
                const int kc = k < p.K ? k : 0;
                const int seg = seg_of(kc, p.F_in);
                const float* src = seg < 3 ? p.Z + m * p.ldz + kc : p.res_x + m * p.ld_res + (kc - 3 * p.F_in);
                ra[q] = ld4(src);
            } else {
                const float* sg = &Sg[(idx >> 3) * 4];
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (k + 0 < p.K) v.x = a_elem(p, sg, m, k + 0);
                if (k + 1 < p.K) v.y = a_elem(p, sg, m, k + 1);
                if (k + 2 < p.K) v.z = a_elem(p, sg, m, k + 2);
                if (k + 3 < p.K) v.w = a_elem(p, sg, m, k + 3);
                ra[q] = v;
            }
        }
#pragma unroll
        for (int q = 0; q < B_F4; ++q) {
            const int idx = tid + NT * q;
            const int n = min(n0 + (idx >> 3), p.F_out - 1);
            const int k = k0 + 4 * (idx & 7);
            const float* src = p.Bp + (int64_t)n * p.K;
            if (VEC) {
                rb[q] = ld4(src + (k < p.K ? k : 0));
            } else {
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (k + 0 < p.K) v.x = src[k + 0];
                if (k + 1 < p.K) v.y = src[k + 1];
                if (k + 2 < p.K) v.z = src[k + 2];
                if (k + 3 < p.K) v.w = src[k + 3];
                rb[q] = v;
            }
        }
    };
    auto fetch = [&](int k0) { fetch_to(k0, ra, rb); };
    auto stash_from = [&](int buf, int k0, const float4 (&ra)[A_F4], const float4 (&rb)[B_F4]) {
#pragma unroll
        for (int q = 0; q < A_F4; ++q) {
            const int idx = tid + NT * q;
            float4 v = ra[q];
            if (VEC) {
                const int k = k0 + 4 * (idx & 7);
                const int seg = seg_of(k, p.F_in);
                const float sc = k < p.K ? (p.pregated ? 1.f : Sg[(idx >> 3) * 4 + seg]) : 0.f;  // Sg[.., 3] == 1
                v = scale4(v, sc);
            }
            *reinterpret_cast<float4*>(&As[buf][(idx >> 3) * LDSW + 4 * (idx & 7)]) = v;
        }
#pragma unroll
        for (int q = 0; q < B_F4; ++q) {
            const int idx = tid + NT * q;
            float4 v = rb[q];
            if (VEC) {
                const int k = k0 + 4 * (idx & 7);
                if (k >= p.K) v = make_float4(0.f, 0.f, 0.f, 0.f);
            }
            *reinterpret_cast<float4*>(&Bs[buf][(idx >> 3) * LDSW + 4 * (idx & 7)]) = v;
        }
    };

    auto stash = [&](int buf, int k0) { stash_from(buf, k0, ra, rb); };
    auto mma = [&](int cur) {
        const float* Ab = As[cur];
        const float* Bb = Bs[cur];
#pragma unroll
        for (int g = 0; g < BK / 8; ++g) {
            float4 a[TM], b[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) a[i] = ld4(&Ab[(wm * TM * 32 + i * 32 + li) * LDSW + g * 8 + 4 * lh]);
#pragma unroll
            for (int j = 0; j < TN; ++j) b[j] = ld4(&Bb[(wn * TN * 32 + j * 32 + li) * LDSW + g * 8 + 4 * lh]);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].x, b[j].x, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].y, b[j].y, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].z, b[j].z, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].w, b[j].w, acc[i][j], 0, 0, 0);
                }
        }
    };

    const int ntiles = (p.K + BK - 1) / BK;
    fetch(0);
    stash(0, 0);
    __syncthreads();
    for (int t = 0; t < ntiles; ++t) {
        const int cur = t & 1;
        if (t + 1 < ntiles) fetch((t + 1) * BK);
        mma(cur);
        if (t + 1 < ntiles) stash(cur ^ 1, (t + 1) * BK);
        __syncthreads();
    }

    // Epilogue: park the accumulator tile in LDS (C/D map of the 32x32 MFMA: col = lane&31,
    // row = (r&3) + 8*(r>>2) + 4*(lane>>5)), then sweep it row-major with float4 per thread so the
    // constant / residual loads and the Y stores are 16-B coalesced, all loads of a batch in flight.
    float* T = smem;  // the K loop ended with a barrier: the staging buffers are free
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

    constexpr int C4 = BN / 4;            // float4 per tile row
    constexpr int ITER = BM * C4 / NT;    // float4 per thread
    constexpr int BATCH = ITER < 4 ? ITER : 4;
    const int c4 = tid % C4;              // fixed column group per thread
    const int nb = n0 + 4 * c4;
    const bool has_const = p.constant && p.gate_mode == PG_GATES_VECTOR;
    const bool id_res = p.res_x && !p.proj_res;
    const bool vec_out = p.vec_out;
    float4 b[3], br = make_float4(0.f, 0.f, 0.f, 0.f);
    {
        auto ldb = [&](const float* v) {
            float4 o;
            o.x = nb + 0 < p.F_out ? v[nb + 0] : 0.f;
            o.y = nb + 1 < p.F_out ? v[nb + 1] : 0.f;
            o.z = nb + 2 < p.F_out ? v[nb + 2] : 0.f;
            o.w = nb + 3 < p.F_out ? v[nb + 3] : 0.f;
            return o;
        };
        b[0] = ldb(p.bsum);
        b[1] = ldb(p.bsum + p.F_out);
        b[2] = ldb(p.bsum + 2 * p.F_out);
        if (p.proj_res) br = ldb(p.bsum + 3 * p.F_out);
    }
    for (int it0 = 0; it0 < ITER; it0 += BATCH) {
        float4 cv[BATCH], rv[BATCH];
        int rl[BATCH];
        int64_t mm[BATCH];
        bool ok[BATCH];
#pragma unroll
        for (int u = 0; u < BATCH; ++u) {
            rl[u] = (tid + NT * (it0 + u)) / C4;
            mm[u] = m0 + rl[u];
            ok[u] = Crow[rl[u]] >= 0 && nb < p.F_out;
            cv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            rv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (ok[u] && vec_out) {
                if (has_const) cv[u] = ld4(p.constant + Crow[rl[u]] * p.ld_const + nb);
                if (id_res) rv[u] = ld4(p.res_x + mm[u] * p.ld_res + nb);
            }
        }
#pragma unroll
        for (int u = 0; u < BATCH; ++u) {
            if (!ok[u]) continue;
            const float* sg = &Sg[rl[u] * 4];
            float4 v = ld4(&T[rl[u] * TLD + 4 * c4]);
            float o[4] = {v.x, v.y, v.z, v.w};
            const float bb0[4] = {b[0].x, b[0].y, b[0].z, b[0].w};
            const float bb1[4] = {b[1].x, b[1].y, b[1].z, b[1].w};
            const float bb2[4] = {b[2].x, b[2].y, b[2].z, b[2].w};
            const float bbr[4] = {br.x, br.y, br.z, br.w};
            float cc[4] = {cv[u].x, cv[u].y, cv[u].z, cv[u].w};
            float rr[4] = {rv[u].x, rv[u].y, rv[u].z, rv[u].w};
            if (!vec_out) {  // ragged / unaligned output: element loads with column bounds
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int n = nb + e;
                    if (n < p.F_out) {
                        if (has_const) cc[e] = p.constant[Crow[rl[u]] * p.ld_const + n];
                        if (id_res) rr[e] = p.res_x[mm[u] * p.ld_res + n];
                    }
                }
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float y = o[e] + (sg[0] * bb0[e] + sg[1] * bb1[e] + sg[2] * bb2[e]) + bbr[e] + cc[e] + rr[e];
                if (p.act) y = y > 0.f ? y : y * p.slope;
                if (p.drop_s != 0.f) y = drop_apply(p, dseed, mm[u], nb + e, y);
                o[e] = y;
            }
            if (vec_out) {
                *reinterpret_cast<float4*>(p.Y + mm[u] * p.ldy + nb) = make_float4(o[0], o[1], o[2], o[3]);
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (nb + e < p.F_out) p.Y[mm[u] * p.ldy + nb + e] = o[e];
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------------------
// Helpers of the W-stationary split-bf16 kernels below. Their tiles' A rows arrive by LDS-DMA
// (global_load_lds_dwordx4, 1 KiB per wave-instruction, lane-linear) into images whose 16-byte chunks are
// XOR-swizzled by row (chunk c of row r at c ^ (r & 15), set through the per-lane SOURCE address).
// One LDS-DMA piece: 16 B per lane from a per-lane global address to (wave-uniform base + 16 * lane).
__device__ __forceinline__ void glds16(const float* src, float* lds_base) {
    __builtin_amdgcn_global_load_lds(src, lds_base, 16, 0, 0);
}
// the same with the non-temporal cache policy (aux = 2): the A rows and the per-node constant, read once (measured:
// 0.5587 -> 0.5496 ms per bench step for the A rows, the next layer's propagation finding its input in cache, and
// 0.550 -> 0.545 ms for the constant; PG_FLAG_DENSE_A_CACHED selects the default policy for both)
__device__ __forceinline__ void glds16nt(const float* src, float* lds_base) {
    __builtin_amdgcn_global_load_lds(src, lds_base, 16, 0, 2);
}

// epilogue sum of the W-stationary kernels with every rounding step explicit (no contraction choices left to the
// compiler), so the 32-row and the pipelined 16-row split-bf16 kernels round identically:
//   acc + (s0 b0 + s1 b1 + s2 b2) + b_res + constant + residual
__device__ __forceinline__ float epi_sum(float acc, float s0, float s1, float s2, float b0, float b1, float b2,
                                         float br, float cst, float res) {
    const float gb = __fmaf_rn(s2, b2, __fmaf_rn(s1, b1, __fmul_rn(s0, b0)));
    return __fadd_rn(__fadd_rn(__fadd_rn(__fadd_rn(acc, gb), br), cst), res);
}

// ---------------------------------------------------------------------------------------------------------
// Split-bf16 W-stationary variant (PG_FLAG_DENSE_X3): fp32 accuracy on the bf16 matrix cores.
// Every fp32 operand value v is split EXACTLY into three bf16 values v = v0 + v1 + v2 (round-to-nearest-even
// at each step: v0 = bf16(v), v1 = bf16(v - v0), v2 = v - v0 - v1; both subtractions are exact in fp32 and v2
// has at most 8 significant bits, so it is a bf16). A (the aggregates) and W (the packed weights) are split,
// and the product is the sum of the six terms a_i w_j with i + j <= 2 (each an exact product, accumulated in
// fp32 by v_mfma_f32_16x16x32_bf16); the dropped terms a1 w2, a2 w1, a2 w2 are below 2^-24 |a w|, i.e. the
// size of one fp32 rounding. Six bf16 MFMAs cost 6 x 16 cycles per 16x16x32 step against 8 x 32 cycles for the
// same step on v_mfma_f32_16x16x4_f32: 2.67x fewer matrix-core cycles.
// Tile flow (32 rows, one 512-thread workgroup per CU, wave w owns output columns [16w, 16w+16) with its
// three W splits in VGPRs): fp32 rows arrive by LDS-DMA in the swizzled image described above -> every
// thread converts 3 of the tile's 1536 16-byte A units into the three bf16 images (gated here when the
// operand is not pre-gated) -> the next tile's DMA is issued -> 12 MFMA steps -> accumulators parked in LDS
// (aliasing the consumed bf16 images) -> the epilogue (epi_sum).
// bf2 / split8 / mfma_bf: pg_split3.h (shared with the split-bf16 weight gradient of pg_dense_bwd.hip)
using pgx3::bf2;
using pgx3::mfma_bf;
using pgx3::split8;

// Workgroup barrier for LDS hand-offs only: drains this wave's LDS ops, not its global loads (__syncthreads'
// release fence also waits vmcnt(0), which would drain the next tile's LDS-DMA in flight). LDS-DMA landings are
// waited for explicitly with s_waitcnt vmcnt before the barriers that publish them.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// LDS reads of LDS-DMA targets through inline asm. hipcc cannot tell which LDS-DMA (counted in vmcnt) wrote the
// bytes a ds_read touches, so before every such read it waits vmcnt(0) -- draining the DMA of the tiles in
// flight. These reads carry their own lgkmcnt wait; the DMA they depend on is retired by the explicit counted
// vmcnt waits + barriers of the tile loop.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ void lds_ld4x2(const float* p0, const float* p1, float4& a, float4& b) {
    f32x4 x, y;
    asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(x), "=&v"(y)
                 : "v"(lds_addr(p0)), "v"(lds_addr(p1))
                 : "memory");
    a = make_float4(x[0], x[1], x[2], x[3]);
    b = make_float4(y[0], y[1], y[2], y[3]);
}
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void lds_stf(float* p, float v) {
    asm volatile("ds_write_b32 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_st16(void* p, uint4 v) {
    const u32x4_t w = {v.x, v.y, v.z, v.w};
    asm volatile("ds_write_b128 %0, %1" ::"v"(lds_addr(p)), "v"(w) : "memory");
}
__device__ __forceinline__ void lds_ld4x4(const float* p0, const float* p1, const float* p2, const float* p3,
                                          float4 (&o)[4]) {
    f32x4 x0, x1, x2, x3;
    asm volatile(
        "ds_read_b128 %0, %4\n\tds_read_b128 %1, %5\n\tds_read_b128 %2, %6\n\tds_read_b128 %3, %7\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(x0), "=&v"(x1), "=&v"(x2), "=&v"(x3)
        : "v"(lds_addr(p0)), "v"(lds_addr(p1)), "v"(lds_addr(p2)), "v"(lds_addr(p3))
        : "memory");
    o[0] = make_float4(x0[0], x0[1], x0[2], x0[3]);
    o[1] = make_float4(x1[0], x1[1], x1[2], x1[3]);
    o[2] = make_float4(x2[0], x2[1], x2[2], x2[3]);
    o[3] = make_float4(x3[0], x3[1], x3[2], x3[3]);
}
// epilogue operands in one LDS round trip: three float4 (constant, residual, accumulators) and the five gate
// inputs of the row (g points at Gi[slot][0][r], rows STRIDE_BYTES apart)
template <int STRIDE_BYTES>
__device__ __forceinline__ void lds_epi(const float* p0, const float* p1, const float* p2, const float* g, float4& a,
                                        float4& b, float4& c, float (&gv)[5]) {
    f32x4 x0, x1, x2;
    asm volatile(
        "ds_read_b128 %0, %8\n\tds_read_b128 %1, %9\n\tds_read_b128 %2, %10\n\t"
        "ds_read_b32 %3, %11\n\tds_read_b32 %4, %11 offset:%c12\n\tds_read_b32 %5, %11 offset:%c13\n\t"
        "ds_read_b32 %6, %11 offset:%c14\n\tds_read_b32 %7, %11 offset:%c15\n\ts_waitcnt lgkmcnt(0)"
        : "=&v"(x0), "=&v"(x1), "=&v"(x2), "=&v"(gv[0]), "=&v"(gv[1]), "=&v"(gv[2]), "=&v"(gv[3]), "=&v"(gv[4])
        : "v"(lds_addr(p0)), "v"(lds_addr(p1)), "v"(lds_addr(p2)), "v"(lds_addr(g)), "n"(STRIDE_BYTES),
          "n"(2 * STRIDE_BYTES), "n"(3 * STRIDE_BYTES), "n"(4 * STRIDE_BYTES)
        : "memory");
    a = make_float4(x0[0], x0[1], x0[2], x0[3]);
    b = make_float4(x1[0], x1[1], x1[2], x1[3]);
    c = make_float4(x2[0], x2[1], x2[2], x2[3]);
}
// gate inputs C_in, C_out, C_dir, C_und, C_all of row r: p points at Gi[gbuf][0][r], rows BMW floats apart
template <int STRIDE_BYTES>
__device__ __forceinline__ void lds_gates5(const float* p, float (&g)[5]) {
    asm volatile(
        "ds_read_b32 %0, %5\n\tds_read_b32 %1, %5 offset:%c6\n\tds_read_b32 %2, %5 offset:%c7\n\t"
        "ds_read_b32 %3, %5 offset:%c8\n\tds_read_b32 %4, %5 offset:%c9\n\ts_waitcnt lgkmcnt(0)"
        : "=&v"(g[0]), "=&v"(g[1]), "=&v"(g[2]), "=&v"(g[3]), "=&v"(g[4])
        : "v"(lds_addr(p)), "n"(STRIDE_BYTES), "n"(2 * STRIDE_BYTES), "n"(3 * STRIDE_BYTES), "n"(4 * STRIDE_BYTES)
        : "memory");
}

// One LDS-DMA piece of 4 B per lane (lanes write consecutive dwords from wave-uniform base lds_base).
__device__ __forceinline__ void glds4(const float* src, float* lds_base) {
    __builtin_amdgcn_global_load_lds(src, lds_base, 4, 0, 0);
}

// bf16 split image layout of one 32-row tile: [k step s][row r][4 units], unit g of row r stored at slot
// g ^ ((-(r >> 2)) & 3). A wave's MFMA read of step s (lane: row lc or 16 + lc, unit kg) is then one per-lane
// address plus s * 2 KB, and every ds_read_b128 lane group (0-3,12-15,20-27 | 4-11,16-19,28-31 | ...) and every
// 8-lane ds_write_b128 group of the split pass hits 16 distinct 16-B bank slots.
__device__ __forceinline__ int a_unit(int s, int r, int g) { return 128 * s + 4 * r + (g ^ ((-(r >> 2)) & 3)); }

template <int F_IN, int KSEG, bool PRE>
__global__ __launch_bounds__(512) void dense_x3_kernel(DenseP p) {
    constexpr int K = F_IN * KSEG;
    const uint64_t dseed = drop_seed_of(p);
    constexpr int CH = K / 4;     // fp32 16-B chunks per row
    constexpr int NU = K / 8;     // bf16 16-B units per row (one MFMA operand of one lane for one k step)
    constexpr int NS = K / 32;    // MFMA k steps
    constexpr int BMW = 32;       // rows per tile (two 16x16 MFMA row blocks)
    constexpr int NI = BMW * CH / 64 / 8;  // A-row LDS-DMA instructions per wave per tile
    constexpr int NG = 3;                  // gate-input LDS-DMA instructions per tile (wave 0)
    constexpr int NCR = 4;                 // constant + residual LDS-DMA instructions per wave per tile
    (void)NCR;
    constexpr int NCV = (BMW * NU + 511) / 512;  // units converted per thread per tile
    static_assert(CH % 16 == 0 && NU % 16 == 0 && (BMW * CH) % 512 == 0 && BMW * 128 / 4 == 1024, "tile shape");
    __shared__ __attribute__((aligned(16))) float Af[BMW * K];          // fp32 rows (LDS-DMA target)
    __shared__ __attribute__((aligned(16))) uint4 As[3][BMW * NU];      // bf16 splits; Es aliases them
    __shared__ __attribute__((aligned(16))) float Cs[BMW * 128];        // constant rows (LDS-DMA)
    __shared__ __attribute__((aligned(16))) float Rs[BMW * 128];        // residual rows (LDS-DMA)
    __shared__ __attribute__((aligned(16))) float Gi[2][8][BMW];        // gate inputs C_in..C_all (LDS-DMA)
    __shared__ __attribute__((aligned(16))) float Bs[4][128];
    constexpr int ELD = 128 + 4;
    static_assert(BMW * ELD * 4 <= 3 * BMW * NU * 16, "epilogue tile must fit in the split images");
    float* Es = reinterpret_cast<float*>(&As[0][0]);

    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int lc = lane & 15, kg = lane >> 4;
    const int col = 16 * wave + lc;
    const int64_t T = (p.M + BMW - 1) / BMW;
    Bs[tid >> 7][tid & 127] = (tid >> 7) < 3 || p.proj_res ? p.bsum[(tid >> 7) * p.F_out + (tid & 127)] : 0.f;
    const int nb = gridDim.x, b = blockIdx.x;
    int64_t ntl, lo, step;
    if ((nb & 7) == 0 && nb >= 8) {  // XCD x takes a contiguous range of tiles
        const int x = b & 7, i = b >> 3, bpx = nb >> 3;
        const int64_t xlo = T * x / 8, xhi = T * (x + 1) / 8;
        ntl = (xhi - xlo - i + bpx - 1) / bpx;
        lo = xlo + i;
        step = bpx;
    } else {
        ntl = (T - b + nb - 1) / nb;
        lo = b;
        step = nb;
    }
    if (ntl < 0) ntl = 0;

    // W splits of this lane: k step s uses fp32 chunks 8s + kg and 8s + kg + 4 of column `col` (the same k
    // permutation as the A units below)
    uint4 w0[NS], w1[NS], w2[NS];
    {
        const float* src = p.Bp + (int64_t)col * K + 4 * kg;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const float4 x0 = ld4(src + 32 * s), x1 = ld4(src + 32 * s + 16);
            const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
            split8(v, w0[s], w1[s], w2[s]);
        }
    }
    const int ej = tid & 31, er = tid >> 5;  // epilogue: columns [4ej, 4ej+4) of rows er and er + 16
    const bool has_const = p.constant && p.gate_mode == PG_GATES_VECTOR;
    const bool id_res = p.res_x && !p.proj_res;

    // Every operand of a tile -- A rows, gate inputs, constant and residual rows -- arrives by LDS-DMA, so no
    // register-destination load is ever pending behind a DMA (the compiler would drain the DMA to wait for it),
    // and every wave issues the same number of pieces per tile (absent operands fetch a valid dummy row), so
    // the counted waits below are compile-time constants.
    // Per-lane offsets are recomputed at every issue from an opaque copy of the lane id (32-bit offsets from
    // per-tile uniform bases): hoisted out of the tile loop they would hold ~20 VGPRs next to the W splits.
    auto issue_A = [&](int64_t tile, float* Ad) {
        const int64_t m0 = tile * BMW;
        const int rmax = (int)min((int64_t)(BMW - 1), p.M - 1 - m0);
        const float* zb = p.Z + m0 * p.ldz;
        const float* xb = KSEG > 3 ? p.res_x + m0 * p.ld_res : zb;
        int ln = lane;
        asm volatile("" : "+v"(ln));
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int idx = (wave * NI + i) * 64 + ln;
            const int r = idx / CH, pos = idx - r * CH;
            const int k = 4 * (pos ^ (r & 15));
            const int rr = min(r, rmax);
            const float* src = (KSEG == 3 || k < 3 * F_IN) ? zb + (rr * (int)p.ldz + k)
                                                          : xb + (rr * (int)p.ld_res + (k - 3 * F_IN));
            glds16(src, Ad + (wave * NI + i) * 256);
        }
    };
    // gate inputs of the tile's rows (wave 0 only): piece i, lanes 0-31 / 32-63 fetch C_x for x = 2i / 2i + 1
    auto issue_G = [&](int64_t tile, int gbuf) {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int64_t r = p.gate_mode == PG_GATES_SCALAR ? 0 : min(tile * BMW + (ln & 31), p.M - 1);
        // per-lane choice among uniform pointers by arithmetic (an indexed choice becomes a kernarg load, whose
        // wait would drain the DMA in flight)
        const float* c0 = p.C_in;
        const float* c1 = p.C_out;
        const float* c2 = p.C_dir;
        const float* c3 = p.C_und;
        const float* c4 = p.C_all;
        asm volatile("" : "+s"(c0), "+s"(c1), "+s"(c2), "+s"(c3), "+s"(c4));
        const bool hi = ln >= 32;
        glds4((hi ? c1 : c0) + r, &Gi[gbuf][0][0]);
        glds4((hi ? c3 : c2) + r, &Gi[gbuf][2][0]);
        glds4(c4 + r, &Gi[gbuf][4][0]);
    };
    auto issue_CR = [&](int64_t tile) {
        const int64_t m0 = tile * BMW;
        const int rmax = (int)min((int64_t)(BMW - 1), p.M - 1 - m0);
        int ln = lane;
        asm volatile("" : "+v"(ln));
#pragma unroll
        for (int i = 0; i < 2; ++i) {  // wave w: rows 4w .. 4w + 3
            const int piece = 2 * wave + i;
            const int rr = min(2 * piece + (ln >> 5), rmax);
            const float* cb = has_const ? p.constant + m0 * p.ld_const + (rr * (int)p.ld_const) : p.Z + m0 * p.ldz;
            const float* rb = id_res ? p.res_x + m0 * p.ld_res + (rr * (int)p.ld_res) : p.Z + m0 * p.ldz;
            glds16(cb + 4 * (ln & 31), Cs + piece * 256);
            glds16(rb + 4 * (ln & 31), Rs + piece * 256);
        }
    };
    // s_in = c_all c_dir c_in, s_out = c_all c_dir c_out, s_und = c_all c_und (protgram_directgcn.py:116-133)
    auto gates = [&](int gbuf, int r, float& s0, float& s1, float& s2) {
        float c[5];
        lds_gates5<BMW * 4>(&Gi[gbuf][0][r], c);
        const float ci = c[0], co = c[1], cd = c[2], cu = c[3], ca = c[4];
        const float cad = ca * cd;
        s0 = cad * ci;
        s1 = cad * co;
        s2 = ca * cu;
    };
    auto tile_of = [&](int64_t kt) { return lo + min(kt, ntl - 1) * step; };  // clamped: dummy tiles past the end

    // fp32 -> three bf16 images of tile kt; thread j converts unit u of row r (rows vary fastest: conflict-free)
    auto convert = [&](const float* Af, int gb) {
#pragma unroll
        for (int i = 0; i < NCV; ++i) {
            const int j = tid + 512 * i;
            if (BMW * NU % 512 != 0 && j >= BMW * NU) break;
            const int r = j & (BMW - 1), u = j / BMW;
            const int s = u >> 2, g = u & 3;
            const int c0 = 8 * s + g;
            float4 x0, x1;
            lds_ld4x2(&Af[r * K + 4 * (c0 ^ (r & 15))], &Af[r * K + 4 * ((c0 + 4) ^ (r & 15))], x0, x1);
            float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
            if (!PRE) {
                const int q = (32 * s) / F_IN;  // K segment of this step (F_IN % 32 == 0)
                if (q < 3) {
                    float sg[3];
                    gates(gb, r, sg[0], sg[1], sg[2]);
                    const float sc = sg[q];
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] = __fmul_rn(v[e], sc);  // rounded: never contracted into the split
                }
            }
            uint4 s0, s1, s2;
            split8(v, s0, s1, s2);
            const int pos = a_unit(s, r, g);
            lds_st16(&As[0][pos], s0);
            lds_st16(&As[1][pos], s1);
            lds_st16(&As[2][pos], s2);
            __builtin_amdgcn_sched_barrier(0);  // one unit's temporaries live at a time (W holds 3 * K / 8 VGPRs)
        }
    };
    // Tile loop (four barriers per tile): wait for tile kt's A rows and gates -> convert them into the bf16
    // images -> issue CR(kt), G(kt+1), A(kt+1) (the fp32 buffer is free) -> MFMAs -> accumulators to Es (aliasing
    // the consumed images) -> wait for CR(kt) only (G / A(kt+1) stay in flight) -> epilogue. Counted waits:
    // every wave issues NCR + NI pieces per tile, wave 0 also NG.
    constexpr int WAIT_W0 = NG + NI, WAIT_WN = NI;
    if (ntl > 0) {
        if (wave == 0) issue_G(tile_of(0), 0);
        issue_A(tile_of(0), Af);
    }
    bool prev_full = false;  // the previous epilogue issued exactly 2 Y stores per thread
    for (int64_t kt = 0; kt < ntl; ++kt) {
        const int buf = (int)(kt & 1);
        const int64_t m0 = (lo + kt * step) * BMW;
        // this wave's pieces of tile kt have landed; the previous tile's two Y stores per thread (the youngest
        // vector-memory operations: vmcnt counts loads, stores and LDS-DMA in issue order) may stay in flight
        if (prev_full) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();  // every wave's pieces have landed; the previous epilogue is done with Es / Cs / Rs
        issue_CR(tile_of(kt));  // Cs / Rs are free: their DMA overlaps the split pass
        if (wave == 0) issue_G(tile_of(kt + 1), buf ^ 1);  // Gi[buf ^ 1]: tile kt-1 is done
        convert(Af, buf);
        lds_barrier();  // bf16 images ready; Af is free
        issue_A(tile_of(kt + 1), Af);
        f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
        // operands of k step s for row blocks 0 / 1 sit at one per-lane address + s * 2 KB (+ 1 KB for block 1):
        // immediate ds_read offsets, and step s + 1's six operands are read while step s's MFMAs run
        const uint4* ab0 = &As[0][a_unit(0, lc, kg)];
        const uint4* ab2 = &As[2][a_unit(0, lc, kg)];
        uint4 op[2][6];
        auto ld_ops = [&](int s, uint4 (&o)[6]) {
            o[0] = ab0[128 * s];
            o[1] = ab0[BMW * NU + 128 * s];
            o[2] = ab2[128 * s];
            o[3] = ab0[64 + 128 * s];
            o[4] = ab0[BMW * NU + 64 + 128 * s];
            o[5] = ab2[64 + 128 * s];
        };
        ld_ops(0, op[0]);
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            if (s + 1 < NS) ld_ops(s + 1, op[(s + 1) & 1]);
            const uint4 a00 = op[s & 1][0], a01 = op[s & 1][1], a02 = op[s & 1][2];
            const uint4 a10 = op[s & 1][3], a11 = op[s & 1][4], a12 = op[s & 1][5];
            acc[0] = mfma_bf(a02, w0[s], acc[0]);  // small terms first
            acc[1] = mfma_bf(a12, w0[s], acc[1]);
            acc[0] = mfma_bf(a01, w1[s], acc[0]);
            acc[1] = mfma_bf(a11, w1[s], acc[1]);
            acc[0] = mfma_bf(a00, w2[s], acc[0]);
            acc[1] = mfma_bf(a10, w2[s], acc[1]);
            acc[0] = mfma_bf(a01, w0[s], acc[0]);
            acc[1] = mfma_bf(a11, w0[s], acc[1]);
            acc[0] = mfma_bf(a00, w1[s], acc[0]);
            acc[1] = mfma_bf(a10, w1[s], acc[1]);
            acc[0] = mfma_bf(a00, w0[s], acc[0]);
            acc[1] = mfma_bf(a10, w0[s], acc[1]);
            __builtin_amdgcn_sched_barrier(0);  // keep the scheduler from hoisting later steps' reads (VGPRs)
        }
        lds_barrier();  // every wave is done reading the bf16 images: Es may overwrite them
#pragma unroll
        for (int sb = 0; sb < 2; ++sb)
#pragma unroll
            for (int i = 0; i < 4; ++i) lds_stf(&Es[(16 * sb + 4 * kg + i) * ELD + col], acc[sb][i]);
        if (wave == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WAIT_W0) : "memory");  // CR(kt)
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WAIT_WN) : "memory");
        lds_barrier();
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int rl = er + 16 * h;
            if (m0 + rl >= p.M) continue;
            float4 v, cv, rv, bb[4];
            lds_ld4x2(&Cs[rl * 128 + 4 * ej], &Rs[rl * 128 + 4 * ej], cv, rv);
            lds_ld4x4(&Es[rl * ELD + 4 * ej], &Bs[0][4 * ej], &Bs[1][4 * ej], &Bs[2][4 * ej], bb);
            v = bb[0];
            const float4 b0 = bb[1], b1 = bb[2], b2 = bb[3];
            float4 br;
            lds_ld4x2(&Bs[3][4 * ej], &Bs[3][4 * ej], br, br);
            if (!has_const) cv = make_float4(0.f, 0.f, 0.f, 0.f);
            if (!id_res) rv = make_float4(0.f, 0.f, 0.f, 0.f);
            float s0, s1, s2;
            gates(buf, rl, s0, s1, s2);
            const float o[4] = {v.x, v.y, v.z, v.w}, C4[4] = {cv.x, cv.y, cv.z, cv.w}, R4[4] = {rv.x, rv.y, rv.z, rv.w};
            const float B0[4] = {b0.x, b0.y, b0.z, b0.w}, B1[4] = {b1.x, b1.y, b1.z, b1.w},
                        B2[4] = {b2.x, b2.y, b2.z, b2.w}, BR[4] = {br.x, br.y, br.z, br.w};
            float y[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float qv = epi_sum(o[e], s0, s1, s2, B0[e], B1[e], B2[e], BR[e], C4[e], R4[e]);
                y[e] = (p.act && !(qv > 0.f)) ? qv * p.slope : qv;
                if (p.drop_s != 0.f) y[e] = drop_apply(p, dseed, m0 + rl, 4 * ej + e, y[e]);
            }
            *reinterpret_cast<float4*>(p.Y + (m0 + rl) * p.ldy + 4 * ej) = make_float4(y[0], y[1], y[2], y[3]);
        }
        prev_full = m0 + BMW <= p.M;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the dummy tile's DMA must land before the LDS is freed
}

// ---------------------------------------------------------------------------------------------------------
// Software-pipelined split-bf16 W-stationary kernel (the default for F_in = 128, F_out = 128, no row map).
// Same arithmetic as dense_x3_kernel (identical products and accumulation order per output element, hence
// bit-identical results), on 16-row tiles so that every stage has its own LDS buffer:
//   tile t:  LDS-DMA A(t) -> Af[t&1] (iteration t-2) | split(t) -> As[t&1] (iteration t-1) | MFMA(t) (iteration t)
//            | accumulators -> Es, constant/residual rows -> Cs/Rs (top of t+1) | epilogue(t) (end of t+1)
// Iteration i: [wait A(i+1)] B1 [Es <- acc(i-1); DMA CR(i-1), A(i+2), G(i+2)] then waves 0-3 run MFMA(i) and then
// split(i+1) while waves 4-7 (the other wave of each SIMD) run split(i+1) and then MFMA(i), so each SIMD's
// matrix pipe and its VALU/LDS split work overlap; [wait CR(i-1)] B2 [epilogue(i-1)]. Two barriers per tile.
// LDS: Af 2 x 24 KB, As 2 x 36 KB, Cs/Rs 16 KB, Es 8.3 KB, gate inputs 4 x 512 B, bias sums 2 KB.
__device__ __forceinline__ int a_unit16(int s, int r, int g) { return 64 * s + 4 * r + (g ^ ((-(r >> 2)) & 3)); }

// IL (the default; PG_FLAG_DENSE_NO_IL clears it): the A and gate-input LDS-DMA pieces of tile i + 2 are issued between the k-steps of
// the wave's MFMA phase instead of all at the top of the iteration (stamps: issuing the five or seven pieces at once
// took ~1,750 of an iteration's ~7,300 cycles, the memory pipeline pushing back); the constant / residual pieces stay
// first, so the counted vmcnt waits are unchanged.
// DROP: the fused layer dropout (training); the inference instantiations carry no trace of it.
template <bool PRE, bool IL, bool DROP>
__global__ __launch_bounds__(512) void dense_x3p_kernel(DenseP p) {
    constexpr int F_IN = 128, K = 384;
    constexpr int CH = K / 4;    // fp32 16-B chunks per row
    constexpr int NU = K / 8;    // bf16 16-B units per row
    constexpr int NS = K / 32;   // MFMA k steps
    constexpr int BM = 16;       // rows per tile
    constexpr int NI = BM * CH / 64 / 8;  // A-row LDS-DMA pieces per wave per tile (3)
    constexpr int NG = 2;                 // gate-input pieces per tile (wave 0)
    constexpr int NCR = 2;                // constant + residual pieces per wave per tile
    (void)NCR;
    constexpr int ELD = 128 + 4;
    static_assert(BM * CH % 512 == 0 && NI == 3, "tile shape");
    __shared__ __attribute__((aligned(16))) float Af0[BM * K];  // separate objects: the compiler tells the DMA
    __shared__ __attribute__((aligned(16))) float Af1[BM * K];  // target apart from the buffer being read
    __shared__ __attribute__((aligned(16))) uint4 As[2][3][BM * NU];
    __shared__ __attribute__((aligned(16))) float Cs[BM * 128];
    __shared__ __attribute__((aligned(16))) float Rs[BM * 128];
    __shared__ __attribute__((aligned(16))) float Es[BM * ELD];
    __shared__ __attribute__((aligned(16))) float Gi[4][8][BM];
    __shared__ __attribute__((aligned(16))) float Bs[4][128];

    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int lc = lane & 15, kg = lane >> 4;
    const int col = 16 * wave + lc;
    const bool mfma_first = wave < 4;  // waves w and w + 4 share a SIMD
    const uint64_t dseed = DROP ? drop_seed_of(p) : 0ull;
    const int64_t T = (p.M + BM - 1) / BM;
    DSTAMP_INIT;
    {
        const int q = tid >> 7, n = tid & 127;
        float bv = 0.f;
        if (p.rawW) {
            if (q < 3) bv = q == 0 ? p.bm0[n] + p.bs0[n] : q == 1 ? p.bm1[n] + p.bs1[n] : p.bm2[n] + p.bs2[n];
        } else if (q < 3 || p.proj_res) {
            bv = p.bsum[q * p.F_out + n];
        }
        Bs[q][n] = bv;
    }
    const int nb = gridDim.x, b = blockIdx.x;
    int64_t ntl, lo, step;
    if ((nb & 7) == 0 && nb >= 8) {  // XCD x takes a contiguous range of tiles
        const int x = b & 7, i = b >> 3, bpx = nb >> 3;
        const int64_t xlo = T * x / 8, xhi = T * (x + 1) / 8;
        ntl = (xhi - xlo - i + bpx - 1) / bpx;
        lo = xlo + i;
        step = bpx;
    } else {
        ntl = (T - b + nb - 1) / nb;
        lo = b;
        step = nb;
    }
    if (ntl < 0) ntl = 0;

    uint4 w0[NS], w1[NS], w2[NS];
    if (p.rawW) {  // W_q + W_shared, k step s lies in segment q = s / 4
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const float* wq = s < 4 ? p.Wq0 : s < 8 ? p.Wq1 : p.Wq2;
            const int64_t o = (int64_t)col * F_IN + (32 * s) % F_IN + 4 * kg;
            const float4 a0 = ld4(wq + o), a1 = ld4(wq + o + 16), h0 = ld4(p.Wsh + o), h1 = ld4(p.Wsh + o + 16);
            const float v[8] = {a0.x + h0.x, a0.y + h0.y, a0.z + h0.z, a0.w + h0.w,
                                a1.x + h1.x, a1.y + h1.y, a1.z + h1.z, a1.w + h1.w};
            split8(v, w0[s], w1[s], w2[s]);
        }
    } else {
        const float* src = p.Bp + (int64_t)col * K + 4 * kg;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const float4 x0 = ld4(src + 32 * s), x1 = ld4(src + 32 * s + 16);
            const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
            split8(v, w0[s], w1[s], w2[s]);
        }
    }
    const int ej = tid & 31, er = tid >> 5;  // epilogue: columns [4ej, 4ej+4) of row er
    const bool has_const = p.constant && p.gate_mode == PG_GATES_VECTOR;
    const bool id_res = p.res_x && !p.proj_res;
    auto tile_of = [&](int64_t kt) { return lo + max((int64_t)0, min(kt, ntl - 1)) * step; };

    auto issue_A_piece = [&](int64_t tile, float* Ad, int i) {
        if (DEXP(3)) return;
        const int64_t m0 = tile * BM;
        const int rmax = (int)min((int64_t)(BM - 1), p.M - 1 - m0);
        const float* zb = p.Z + m0 * p.ldz;
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int idx = (wave * NI + i) * 64 + ln;
        const int r = idx / CH, pos = idx - r * CH;
        const int k = 4 * (pos ^ r);
        const int rr = min(r, rmax);
        if (p.nt_a) glds16nt(zb + (rr * (int)p.ldz + k), Ad + (wave * NI + i) * 256);
        else glds16(zb + (rr * (int)p.ldz + k), Ad + (wave * NI + i) * 256);
    };
    auto issue_A = [&](int64_t tile, float* Ad) {
#pragma unroll
        for (int i = 0; i < NI; ++i) issue_A_piece(tile, Ad, i);
    };
    // gate inputs of a tile (wave 0): piece 0 = C_in | C_out | C_dir | C_und (16 lanes each), piece 1 = C_all
    auto issue_G = [&](int64_t tile, int slot) {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int64_t r = p.gate_mode == PG_GATES_SCALAR ? 0 : min(tile * BM + (ln & 15), p.M - 1);
        const float* c0 = p.C_in;
        const float* c1 = p.C_out;
        const float* c2 = p.C_dir;
        const float* c3 = p.C_und;
        const float* c4 = p.C_all;
        asm volatile("" : "+s"(c0), "+s"(c1), "+s"(c2), "+s"(c3), "+s"(c4));
        const int q = ln >> 4;
        const float* cq = q == 0 ? c0 : q == 1 ? c1 : q == 2 ? c2 : c3;
        glds4(cq + r, &Gi[slot][0][0]);
        glds4(c4 + r, &Gi[slot][4][0]);
    };
    auto issue_CR = [&](int64_t tile) {  // wave w: rows 2w, 2w + 1
        if (DEXP(4)) return;
        const int64_t m0 = tile * BM;
        const int rmax = (int)min((int64_t)(BM - 1), p.M - 1 - m0);
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int rr = min(2 * wave + (ln >> 5), rmax);
        const float* cb = has_const ? p.constant + m0 * p.ld_const + (rr * (int)p.ld_const) : p.Z + m0 * p.ldz;
        const float* rb = !id_res    ? p.Z + m0 * p.ldz
                          : p.map_res ? p.res_x + ngram_row(p, m0 + rr) * p.ld_res
                                      : p.res_x + m0 * p.ld_res + (rr * (int)p.ld_res);
        if (p.nt_a) glds16nt(cb + 4 * (ln & 31), Cs + wave * 256);
        else glds16(cb + 4 * (ln & 31), Cs + wave * 256);
        glds16(rb + 4 * (ln & 31), Rs + wave * 256);
    };
    auto gates = [&](int slot, int r, float& s0, float& s1, float& s2) {
        float c[5];
        lds_gates5<BM * 4>(&Gi[slot][0][r], c);
        const float cad = c[4] * c[2];
        s0 = cad * c[0];
        s1 = cad * c[1];
        s2 = c[4] * c[3];
    };
    // fp32 tile -> three bf16 images; thread j converts units j and j + 512 (row j & 15, unit j >> 4): waves 0-3
    // two units, waves 4-7 one; all of a thread's fp32 reads in one LDS round trip
    auto split_tile = [&](const float* Af, int ab, int gslot) {
        if (DEXP(1)) return;
        const int r = tid & 15;
        const bool two = tid + 512 < BM * NU;  // wave-uniform
        const int u0 = tid >> 4, u1 = u0 + 32;
        const int c00 = 8 * (u0 >> 2) + (u0 & 3), c10 = 8 * (u1 >> 2) + (u1 & 3);
        float4 x[4];
        if (two) lds_ld4x4(&Af[r * K + 4 * (c00 ^ r)], &Af[r * K + 4 * ((c00 + 4) ^ r)], &Af[r * K + 4 * (c10 ^ r)],
                           &Af[r * K + 4 * ((c10 + 4) ^ r)], x);
        else lds_ld4x2(&Af[r * K + 4 * (c00 ^ r)], &Af[r * K + 4 * ((c00 + 4) ^ r)], x[0], x[1]);
        float sg[3] = {1.f, 1.f, 1.f};
        if (!PRE) gates(gslot, r, sg[0], sg[1], sg[2]);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            if (i == 1 && !two) break;
            const int u = i ? u1 : u0;
            const int s = u >> 2, g = u & 3;
            const float4 a = x[2 * i], c = x[2 * i + 1];
            float v[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
            if (!PRE) {
                const float sc = sg[(32 * s) / F_IN];
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = __fmul_rn(v[e], sc);  // rounded: never contracted into the split
            }
            uint4 s0, s1, s2;
            split8(v, s0, s1, s2);
            const int pos = a_unit16(s, r, g);
            lds_st16(&As[ab][0][pos], s0);
            lds_st16(&As[ab][1][pos], s1);
            lds_st16(&As[ab][2][pos], s2);
        }
    };
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    // IL: the next-but-one tile's A pieces (after k-steps 2, 5, 8) and gate inputs (wave 0, after k-step 10)
    auto mfma_tile = [&](int ab, int64_t a_tile, float* a_dst, int g_slot, bool issue) {
        const uint4* a0 = &As[ab][0][a_unit16(0, lc, kg)];
        const uint4* a1 = &As[ab][1][a_unit16(0, lc, kg)];
        const uint4* a2 = &As[ab][2][a_unit16(0, lc, kg)];
        uint4 op[2][3];
        acc = f32x4{0.f, 0.f, 0.f, 0.f};
        if (DEXP(0)) {
            if (IL && issue) {
                issue_A(a_tile, a_dst);
                if (wave == 0) issue_G(a_tile, g_slot);
            }
            return;
        }
        op[0][0] = a0[0];
        op[0][1] = a1[0];
        op[0][2] = a2[0];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            if (s + 1 < NS) {
                op[(s + 1) & 1][0] = a0[64 * (s + 1)];
                op[(s + 1) & 1][1] = a1[64 * (s + 1)];
                op[(s + 1) & 1][2] = a2[64 * (s + 1)];
            }
            const uint4 x0 = op[s & 1][0], x1 = op[s & 1][1], x2 = op[s & 1][2];
            acc = mfma_bf(x2, w0[s], acc);  // small terms first (the order of dense_x3_kernel)
            acc = mfma_bf(x1, w1[s], acc);
            acc = mfma_bf(x0, w2[s], acc);
            acc = mfma_bf(x1, w0[s], acc);
            acc = mfma_bf(x0, w1[s], acc);
            acc = mfma_bf(x0, w0[s], acc);
            if constexpr (IL) {
                if (issue && (s == 2 || s == 5 || s == 8)) issue_A_piece(a_tile, a_dst, s / 3);
                if (issue && s == 10 && wave == 0) issue_G(a_tile, g_slot);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    };

    // prologue: A(0), G(0) and A(1), G(1) in flight; split(0) once A(0) has landed
    if (ntl > 0) {
        issue_A(tile_of(0), Af0);
        if (wave == 0) issue_G(tile_of(0), 0);
        issue_A(tile_of(1), Af1);
        if (wave == 0) issue_G(tile_of(1), 1);
        if (wave == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI + NG) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");
        lds_barrier();
        split_tile(Af0, 0, 0);
    }
    // bias sums of this thread's epilogue columns (Bs was published by the prologue barrier)
    float4 bq[4];
    if (ntl > 0) lds_ld4x4(&Bs[0][4 * ej], &Bs[1][4 * ej], &Bs[2][4 * ej], &Bs[3][4 * ej], bq);
    bool y_pending = false;  // the previous epilogue left exactly one Y store per thread in flight
    for (int64_t i = 0; i <= ntl && ntl > 0; ++i) {
        const int ab = (int)(i & 1);
        [[maybe_unused]] const int si = (int)i;
        DSTAMP(si, 0);
        if (y_pending) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");  // A(i+1), G(i+1) have landed
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();  // B1: A(i+1) and split(i) visible; epilogue(i-2) done with Es / Cs / Rs; As[ab ^ 1] free
        DSTAMP(si, 1);
        if (i >= 1) {
#pragma unroll
            for (int e = 0; e < 4; ++e) lds_stf(&Es[(4 * kg + e) * ELD + col], acc[e]);
        }
        issue_CR(tile_of(i - 1));
        const int64_t a_tile = tile_of(i + 2);
        float* const a_dst = ab ? Af1 : Af0;  // Af[(i + 2) & 1] = Af[ab]: split(i) is done with it
        const int g_slot = (int)((i + 2) & 3);
        const bool do_mfma = i < ntl, do_split = i + 1 < ntl;
        if (!IL || !do_mfma) {  // IL: the MFMA phase issues them (or here, past the last tile)
            issue_A(a_tile, a_dst);
            if (wave == 0) issue_G(a_tile, g_slot);
        }
        DSTAMP(si, 2);
        if (mfma_first) {
            if (do_mfma) mfma_tile(ab, a_tile, a_dst, g_slot, IL);
            DSTAMP(si, 3);
            if (do_split) split_tile(ab ? Af0 : Af1, ab ^ 1, (int)((i + 1) & 3));
        } else {
            if (do_split) split_tile(ab ? Af0 : Af1, ab ^ 1, (int)((i + 1) & 3));
            DSTAMP(si, 3);
            if (do_mfma) mfma_tile(ab, a_tile, a_dst, g_slot, IL);
        }
        DSTAMP(si, 4);
        // CR(i-1) has landed: younger are A(i+2) (+ G(i+2) on wave 0)
        if (wave == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI + NG) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");
        DSTAMP(si, 5);
        lds_barrier();  // B2: Es and Cs / Rs visible
        DSTAMP(si, 6);
        y_pending = false;
        if (i >= 1) {
            const int64_t m0 = tile_of(i - 1) * BM;
            const int gs = (int)((i - 1) & 3);
            if (m0 + er < p.M) {
                float4 cv, rv, ov;
                float c[5];
                lds_epi<BM * 4>(&Cs[er * 128 + 4 * ej], &Rs[er * 128 + 4 * ej], &Es[er * ELD + 4 * ej], &Gi[gs][0][er],
                                cv, rv, ov, c);
                if (!has_const) cv = make_float4(0.f, 0.f, 0.f, 0.f);
                if (!id_res) rv = make_float4(0.f, 0.f, 0.f, 0.f);
                const float cad = c[4] * c[2];
                const float s0 = cad * c[0], s1 = cad * c[1], s2 = c[4] * c[3];
                const float o[4] = {ov.x, ov.y, ov.z, ov.w}, C4[4] = {cv.x, cv.y, cv.z, cv.w},
                            R4[4] = {rv.x, rv.y, rv.z, rv.w};
                const float B0[4] = {bq[0].x, bq[0].y, bq[0].z, bq[0].w}, B1[4] = {bq[1].x, bq[1].y, bq[1].z, bq[1].w},
                            B2[4] = {bq[2].x, bq[2].y, bq[2].z, bq[2].w}, BR[4] = {bq[3].x, bq[3].y, bq[3].z, bq[3].w};
                float y[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float qv = epi_sum(o[e], s0, s1, s2, B0[e], B1[e], B2[e], BR[e], C4[e], R4[e]);
                    y[e] = (p.act && !(qv > 0.f)) ? qv * p.slope : qv;
                    if (DROP) y[e] = drop_apply(p, dseed, m0 + er, 4 * ej + e, y[e]);
                }
                if (!DEXP(2)) {
                    const int64_t yr = p.map_y ? ngram_row(p, m0 + er) : m0 + er;
                    *reinterpret_cast<float4*>(p.Y + yr * p.ldy + 4 * ej) = make_float4(y[0], y[1], y[2], y[3]);
                    y_pending = true;
                }
            }
        }
        DSTAMP(si, 7);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the dummy tiles' DMA must land before the LDS is freed
}

__global__ __launch_bounds__(256) void pack_kernel(int F_in, int F_out, int K, const float* W0, const float* W1,
                                                   const float* W2, const float* Ws, const float* Wr,
                                                   const float* bm0, const float* bs0, const float* bm1,
                                                   const float* bs1, const float* bm2, const float* bs2,
                                                   const float* br, float* out) {
    const int64_t total = (int64_t)F_out * K;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total + 4 * F_out; i += (int64_t)gridDim.x * 256) {
        if (i < total) {
            const int n = (int)(i / K), k = (int)(i % K);
            const int q = seg_of(k, F_in), kk = k - q * F_in;
            const int64_t w = (int64_t)n * F_in + kk;
            float v;
            if (q == 0) v = W0[w] + Ws[w];
            else if (q == 1) v = W1[w] + Ws[w];
            else if (q == 2) v = W2[w] + Ws[w];
            else v = Wr[w];
            out[i] = v;
        } else {
            const int j = (int)(i - total), q = j / F_out, n = j % F_out;
            float v;
            if (q == 0) v = bm0[n] + bs0[n];
            else if (q == 1) v = bm1[n] + bs1[n];
            else if (q == 2) v = bm2[n] + bs2[n];
            else v = br ? br[n] : 0.f;
            out[i] = v;
        }
    }
}

}  // namespace

extern "C" {

int64_t pg_directgcn_packed_floats(int64_t F_in, int64_t F_out, int has_res_proj) {
    return F_out * (has_res_proj ? 4 : 3) * F_in + 4 * F_out;
}

int pg_directgcn_pack_f32(const pg_layer_args_t* a, float* packed, void* stream) {
    PG_REQUIRE(a != nullptr && packed != nullptr, "null args");
    PG_REQUIRE(a->F_in > 0 && a->F_out > 0 && a->F_in < (1 << 20) && a->F_out < (1 << 20), "bad F_in/F_out");
    PG_REQUIRE(a->W_main_in && a->W_main_out && a->W_undirected && a->W_shared, "null weight");
    PG_REQUIRE(a->b_main_in && a->b_dir_shared_in && a->b_main_out && a->b_dir_shared_out && a->b_undirected &&
                   a->b_undirected_shared,
               "null bias");
    const int K = (int)((a->W_res ? 4 : 3) * a->F_in);
    const int64_t total = a->F_out * K + 4 * a->F_out;
    const int64_t nb = (total + 255) / 256 < 1024 ? (total + 255) / 256 : 1024;
    hipLaunchKernelGGL(pack_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, (int)a->F_in,
                       (int)a->F_out, K, a->W_main_in, a->W_main_out, a->W_undirected, a->W_shared, a->W_res,
                       a->b_main_in, a->b_dir_shared_in, a->b_main_out, a->b_dir_shared_out, a->b_undirected,
                       a->b_undirected_shared, a->b_res, packed);
    return pg::check_launch("pg_directgcn_pack_f32");
}

static int dense_launch(const pg_layer_args_t* a, const float* packed, uint32_t flags, const int64_t* ngmap,
                        void* stream) {
    PG_REQUIRE(a != nullptr, "null args");
    PG_REQUIRE(a->M >= 0 && a->F_in > 0 && a->F_out > 0 && a->F_in < (1 << 20) && a->F_out < (1 << 20),
               "bad shape M=%lld F_in=%lld F_out=%lld", (long long)a->M, (long long)a->F_in, (long long)a->F_out);
    if (a->M == 0) return PG_OK;
    PG_REQUIRE(a->Z && a->ldz >= 3 * a->F_in, "Z must be [M, >=3*F_in]");
    PG_REQUIRE(a->C_in && a->C_out && a->C_directed && a->C_undirected && a->C_all, "null gate");
    PG_REQUIRE(a->gate_mode == PG_GATES_VECTOR || a->gate_mode == PG_GATES_SCALAR, "bad gate_mode");
    PG_REQUIRE(!a->constant || a->ld_const >= a->F_out, "ld_const < F_out");
    PG_REQUIRE(!a->W_res || a->res_x, "W_res needs res_x");
    PG_REQUIRE(!a->res_x || a->W_res || a->F_in == a->F_out, "identity residual needs F_in == F_out");
    PG_REQUIRE(!a->res_x || a->ld_res >= a->F_in, "ld_res < F_in");
    PG_REQUIRE(a->Y && a->ldy >= a->F_out, "bad output");
    DenseP p{};
    p.M = a->M;
    p.F_in = (int)a->F_in;
    p.F_out = (int)a->F_out;
    p.K = (int)((a->W_res ? 4 : 3) * a->F_in);
    p.Z = a->Z;
    p.ldz = a->ldz;
    p.Bp = packed;
    p.bsum = packed ? packed + (int64_t)p.F_out * p.K : nullptr;
    if (!packed) {  // unpacked weights: only the pipelined split-bf16 kernel takes them (checked at dispatch)
        PG_REQUIRE(a->W_main_in && a->W_main_out && a->W_undirected && a->W_shared && a->b_main_in &&
                       a->b_dir_shared_in && a->b_main_out && a->b_dir_shared_out && a->b_undirected &&
                       a->b_undirected_shared,
                   "packed == NULL needs the raw weights and biases in the args");
        p.rawW = 1;
        p.Wq0 = a->W_main_in;
        p.Wq1 = a->W_main_out;
        p.Wq2 = a->W_undirected;
        p.Wsh = a->W_shared;
        p.bm0 = a->b_main_in;
        p.bs0 = a->b_dir_shared_in;
        p.bm1 = a->b_main_out;
        p.bs1 = a->b_dir_shared_out;
        p.bm2 = a->b_undirected;
        p.bs2 = a->b_undirected_shared;
    }
    p.gate_mode = a->gate_mode;
    p.C_in = a->C_in;
    p.C_out = a->C_out;
    p.C_dir = a->C_directed;
    p.C_und = a->C_undirected;
    p.C_all = a->C_all;
    p.rows = a->rows;
    p.constant = a->constant;
    p.ld_const = a->ld_const;
    p.res_x = a->res_x;
    p.ld_res = a->ld_res;
    p.proj_res = a->W_res ? 1 : 0;
    p.act = a->act;
    p.slope = a->slope;
    p.Y = a->Y;
    p.ldy = a->ldy;
    p.remap = (flags & PG_FLAG_NO_XCD_REMAP) ? 0 : 1;
    p.pregated = (flags & PG_FLAG_DENSE_PREGATED) ? 1 : 0;
    p.nt_a = (flags & PG_FLAG_DENSE_A_CACHED) ? 0 : 1;
    if (const int rc = pg::drop_params(a, p.drop_thr, p.drop_s)) return rc;
    p.drop_seed = a->drop_seed;
    PG_REQUIRE(p.drop_s == 0.f || a->M * a->F_out <= (int64_t(1) << 32), "fused dropout: M * F_out > 2^32");
#ifdef PG_DENSE_EXP
    p.exp = (int)((flags >> 24) & 31u);
#endif
    if (ngmap) {  // {Kn1, m0, map_res, map_y}
        p.map_kn1 = ngmap[0];
        p.map_m0 = ngmap[1];
        p.map_res = ngmap[2] ? 1 : 0;
        p.map_y = ngmap[3] ? 1 : 0;
    }
    p.vec_out = (a->F_out % 4 == 0) && (a->ldy % 4 == 0) && pg::aligned16(a->Y) &&
                (!a->constant || (a->ld_const % 4 == 0 && pg::aligned16(a->constant))) &&
                (!a->res_x || a->W_res || (a->ld_res % 4 == 0 && pg::aligned16(a->res_x)));
    bool vec = (a->F_in % 4 == 0) && (a->ldz % 4 == 0) && pg::aligned16(a->Z) && pg::aligned16(packed);
    if (a->res_x) vec = vec && pg::aligned16(a->res_x) && (a->ld_res % 4 == 0);
    const bool wide = a->F_out > 64;
    const int64_t BN = wide ? 128 : 64;
    const int64_t nb = ((a->M + 127) / 128) * ((a->F_out + BN - 1) / BN);
    hipStream_t s = (hipStream_t)stream;
    // split-bf16 W-stationary kernels (fp32-accurate, bf16 matrix cores): K = 384 (F_in 128: the pipelined 16-row
    // kernel) or 256 (F_in 64 with the projected residual: the 32-row kernel). The default wherever their shape
    // applies (B(20,4), F=128: 0.127-0.134 ms; the tiled fp32 kernel 0.188, an fp32 W-stationary kernel 0.162, the
    // 32-row split kernel at F_in 128 0.140 -- both removed; max |err| vs float64 1.4e-5 against 1.8e-5 for fp32
    // MFMA); PG_FLAG_DENSE_TILED selects the tiled kernel below instead.
    const bool ws_shape_ok = a->F_out == 128 && vec && p.vec_out &&
                             (!a->res_x || (a->ld_res % 4 == 0 && pg::aligned16(a->res_x)));
    if (!(flags & PG_FLAG_DENSE_TILED) && ws_shape_ok && a->ldz < (1 << 24) && a->rows == nullptr &&
        (!a->res_x || a->ld_res < (1 << 24)) &&
        ((a->F_in == 128 && !a->W_res) || (a->F_in == 64 && a->W_res))) {
        if (ngmap && a->F_in != 128)
            return pg::set_error(PG_ERR_UNSUPPORTED, "pg_directgcn_dense_ngram_rows_f32: F_in = F_out = 128 only");
        int dev = 0, ncu = 256;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
            ncu = 256;
        if (a->F_in == 128) {  // 16-row software-pipelined kernel
            if (p.rawW && !(pg::aligned16(a->W_main_in) && pg::aligned16(a->W_main_out) &&
                            pg::aligned16(a->W_undirected) && pg::aligned16(a->W_shared)))
                return pg::set_error(PG_ERR_UNSUPPORTED, "pg_directgcn_dense_f32: unpacked weights must be 16-B aligned");
            const int64_t T16 = (a->M + 15) / 16;
            const unsigned g16 = (unsigned)(T16 < ncu ? T16 : ncu);
            const bool il = (flags & PG_FLAG_DENSE_NO_IL) == 0;
            if (p.drop_s != 0.f) {
                if (p.pregated) hipLaunchKernelGGL((dense_x3p_kernel<true, true, true>), dim3(g16), dim3(512), 0, s, p);
                else hipLaunchKernelGGL((dense_x3p_kernel<false, true, true>), dim3(g16), dim3(512), 0, s, p);
            } else if (p.pregated) {
                if (il) hipLaunchKernelGGL((dense_x3p_kernel<true, true, false>), dim3(g16), dim3(512), 0, s, p);
                else hipLaunchKernelGGL((dense_x3p_kernel<true, false, false>), dim3(g16), dim3(512), 0, s, p);
            } else {
                if (il) hipLaunchKernelGGL((dense_x3p_kernel<false, true, false>), dim3(g16), dim3(512), 0, s, p);
                else hipLaunchKernelGGL((dense_x3p_kernel<false, false, false>), dim3(g16), dim3(512), 0, s, p);
            }
        } else {
            if (p.rawW)
                return pg::set_error(PG_ERR_UNSUPPORTED, "pg_directgcn_dense_f32: unpacked weights need the pipelined "
                                                         "split-bf16 kernel (F_in = F_out = 128, no row map)");
            const int64_t T = (a->M + 31) / 32;
            const unsigned g = (unsigned)(T < ncu ? T : ncu);
            if (p.pregated) hipLaunchKernelGGL((dense_x3_kernel<64, 4, true>), dim3(g), dim3(512), 0, s, p);
            else hipLaunchKernelGGL((dense_x3_kernel<64, 4, false>), dim3(g), dim3(512), 0, s, p);
        }
        return pg::check_launch("pg_directgcn_dense_f32");
    }
    if (ngmap)
        return pg::set_error(PG_ERR_UNSUPPORTED, "pg_directgcn_dense_ngram_rows_f32: needs the pipelined split-bf16 "
                                                 "kernel's shape (F_in = F_out = 128, no W_res, no row map, aligned)");
    if (p.rawW)
        return pg::set_error(PG_ERR_UNSUPPORTED, "pg_directgcn_dense_f32: unpacked weights need the pipelined "
                                                 "split-bf16 kernel (F_in = F_out = 128, no row map)");
    // tiled fp32 kernel: 128-row tiles, 8 waves of 32x32 (BM = 64 and 4-wave tilings measured slower, removed)
    if (vec) {
        if (wide) hipLaunchKernelGGL((dense_kernel<128, 128, 8, true>), dim3((unsigned)nb), dim3(512), 0, s, p);
        else hipLaunchKernelGGL((dense_kernel<128, 64, 8, true>), dim3((unsigned)nb), dim3(512), 0, s, p);
    } else {
        if (wide) hipLaunchKernelGGL((dense_kernel<128, 128, 8, false>), dim3((unsigned)nb), dim3(512), 0, s, p);
        else hipLaunchKernelGGL((dense_kernel<128, 64, 8, false>), dim3((unsigned)nb), dim3(512), 0, s, p);
    }
    return pg::check_launch("pg_directgcn_dense_f32");
}

int pg_directgcn_dense_f32(const pg_layer_args_t* a, const float* packed, uint32_t flags, void* stream) {
    return dense_launch(a, packed, flags, nullptr, stream);
}

#ifdef PG_DENSE_EXP
// diagnostics library only (tools/dense_exp.py --stamps): the stamp buffer of dense_x3p_kernel (NULL: off)
int pg_dense_set_stamps(unsigned long long* buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_dense_stamps), &buf, sizeof(buf)) == hipSuccess ? PG_OK : PG_ERR_HIP;
}
#endif

int pg_directgcn_dense_ngram_rows_f32(const pg_layer_args_t* a, const float* packed, int64_t Kn1, int64_t m0,
                                      int32_t map_res, int32_t map_y, uint32_t flags, void* stream) {
    PG_REQUIRE(a != nullptr, "null args");
    // the row map is the K = 20 grid (ngram_row): Kn1 must be K^(n-1) = 20^(n-1), not merely a multiple of 20
    int64_t pw = 20;
    while (pw < Kn1 && pw <= (int64_t(1) << 56)) pw *= 20;
    PG_REQUIRE(Kn1 >= 20 && pw == Kn1 && m0 >= 0 && m0 < Kn1,
               "bad n-gram map (Kn1 = %lld must be a power of K = 20; m0 = %lld)", (long long)Kn1, (long long)m0);
    PG_REQUIRE(a->M % 400 == 0 && a->M < (int64_t(1) << 31), "rows must be whole middles (M = %lld)", (long long)a->M);
    PG_REQUIRE(!map_res || a->res_x, "map_res needs res_x");
    PG_REQUIRE(m0 + a->M / 400 <= Kn1 / 20, "middles [%lld, %lld) past the graph's %lld", (long long)m0,
               (long long)(m0 + a->M / 400), (long long)(Kn1 / 20));
    const int64_t map[4] = {Kn1, m0, map_res, map_y};
    return dense_launch(a, packed, flags, map, stream);
}

}  // extern "C"
