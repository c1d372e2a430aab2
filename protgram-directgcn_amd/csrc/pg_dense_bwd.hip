// Backward of the fused DirectGCN dense contraction (pg_dense.hip) on gfx950 fp32 MFMA.
//
// Forward (per row m, packed B = [W_mi+W_s | W_mo+W_s | W_u+W_s (| W_res)] as [F_out, K]):
//   pre[m] = sum_q s_q[m] (Z_q[m] B_q^T + bsum_q) + bsum_3 + constant + residual,  y = leaky(pre)
// This is the autograd of src/models/protgram_directgcn.py:100-133 (the six nn.Linear calls, the bias
// adds and the c_* gate combine) plus ProtGramDirectGCN.forward :213-215 (residual, leaky_relu). Given
// dY, with dpre = dY * leaky'(y):
//   dZ_q[m]  = s_q[m] * (dpre[m] B_q)                     q = in, out, und       (dgrad_kernel)
//   dres[m]  = dpre[m] B_3                                 projected residual     (dgrad_kernel)
//   ds_q[m]  = <dpre[m] B_q, Z_q[m]> + <dpre[m], bsum_q>   -> dc_* per row        (dgrad + gate_grad_kernel)
//   dB_q     = sum_m s_q[m] dpre[m]^T Z_q[m]  (dB_3 with res_x, s_3 = 1)         (wgrad_kernel, split-K)
//   dbsum_q  = sum_m s_q[m] dpre[m]                                               (wgrad_kernel)
// dB_q is the gradient of every weight summed into segment q (W_main_q and W_shared alike), so the
// caller maps dW_main_q = dB_q, dW_shared = dB_0 + dB_1 + dB_2, dW_res = dB_3 and the bias pairs the same way.
//
// dgrad_kernel: the forward kernel's tiling (BM=128 x BN=128 x BK=32, 8 waves, double-buffered LDS,
//   K-permuted ds_read_b128 operands) with K = F_out and B = the packed weights transposed once
//   (transpose_kernel, [K, F_out]). The A loader computes dpre at stash time; the n-tile-0 blocks also
//   write dpre, the row gates (for wgrad) and the bias dots. The epilogue parks the tile in LDS, then
//   streams Z in and dZ out with float4 accesses and reduces <G_q, Z_q> per row in fixed order.
// wgrad_kernel: C[P x N] = A^T diag(s) B over row chunks of 32 (the reduction runs over rows): both
//   operands staged row-major in LDS; each MFMA k-step of lane half h reads row 4h+s with ds_read_b32
//   (32 consecutive floats per half: conflict-free). Each split writes a partial; reduce_splits_kernel
//   sums them in split order (deterministic, no atomics).
#include <algorithm>
#include <type_traits>

#include "pg_bf16_util.h"

#include "pg_common.h"
#include "pg_split3.h"

namespace {

// One row's gate partials over the C4 4-column groups of an n-tile (the per-column dots the epilogue left in T at
// stride 4), added into ds[segment] in column order -- the order of the original serial loop, so the same bits --
// with the LDS reads issued in groups of 8: C4 / 8 round trips per row instead of C4 dependent ones (the serial loop with its
// early exit and division cost the resident bf16 dgrad ~70 us of its ~300 at config 5, tools/r06_dgrad_exp.sh).
template <int C4>
__device__ __forceinline__ void row_gate_partials(const float* Trow, int n0, int N, int F_in, float (&ds)[3]) {
    constexpr int G = C4 < 8 ? C4 : 8;
#pragma unroll
    for (int c0 = 0; c0 < C4; c0 += G) {
        float tv[G];
#pragma unroll
        for (int c = 0; c < G; ++c) tv[c] = Trow[4 * (c0 + c)];
#pragma unroll
        for (int c = 0; c < G; ++c) {
            const int jj = n0 + 4 * (c0 + c);
            if (jj < N && jj < 3 * F_in) ds[(jj >= F_in) + (jj >= 2 * F_in)] += tv[c];
        }
    }
}

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BK = 32;
constexpr int LDSW = 36;

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float dot4(float4 a, float4 b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }

struct Gates {
    int gate_mode;
    const float *C_in, *C_out, *C_dir, *C_und, *C_all;
    const int64_t* rows;
};

__device__ __forceinline__ void gate_values(const Gates& g, int64_t m, float& ci, float& co, float& cd, float& cu,
                                            float& ca) {
    const int64_t r = (g.gate_mode == PG_GATES_SCALAR) ? 0 : (g.rows ? g.rows[m] : m);
    ci = g.C_in[r];
    co = g.C_out[r];
    cd = g.C_dir[r];
    cu = g.C_und[r];
    ca = g.C_all[r];
}

struct DgradP {
    int64_t M;
    int F_in, F_out, N;  // N = forward K (3 or 4 segments of F_in)
    const float* dY;
    int64_t lddy;
    const float* Y;
    int64_t ldy;
    int act;
    float slope;
    float drop_s;       // fused layer dropout's scale (pg::act_grad), 0: none
    const float* BT;    // [N, F_out]
    const float* bsum;  // [4, F_out]
    const float* Z;
    int64_t ldz;
    Gates g;
    float* dpre;
    int64_t ldp;
    float* dZ;
    int64_t lddz;
    float* dres;
    int64_t lddres;
    float* gates;  // [M, 4]
    float* dsp;    // [ntn * 3, M]
    int remap;
};

template <int BM, int BN, int NW>
__global__ __launch_bounds__(64 * NW) void dgrad_kernel(DgradP p) {
    constexpr int NT = 64 * NW;
    constexpr int WN = 2;
    constexpr int WM = NW / WN;
    constexpr int TM = BM / WM / 32;
    constexpr int TN = BN / WN / 32;
    static_assert(TM >= 1 && TN >= 1, "wave tile too small");
    constexpr int A_F4 = BM * BK / 4 / NT;
    constexpr int B_F4 = BN * BK / 4 / NT;
    constexpr int TLD = BN + 4;
    constexpr int MAIN_FLOATS = 2 * BM * LDSW + 2 * BN * LDSW;
    constexpr int SMEM_FLOATS = MAIN_FLOATS > BM * TLD ? MAIN_FLOATS : BM * TLD;
    __shared__ __attribute__((aligned(16))) float smem[SMEM_FLOATS];
    __shared__ __attribute__((aligned(16))) float Sg[BM * 4];
    __shared__ float Bd[BM * 3];
    static_assert(BM <= NT, "one thread per tile row");
    float (*As)[BM * LDSW] = reinterpret_cast<float (*)[BM * LDSW]>(smem);
    float (*Bs)[BN * LDSW] = reinterpret_cast<float (*)[BN * LDSW]>(smem + 2 * BM * LDSW);

    const int ntn = (p.N + BN - 1) / BN;
    const int64_t lb = pg::xcd_logical_block(blockIdx.x, gridDim.x, p.remap != 0);
    // n-tiles fastest: the tiles of one row block run together (same XCD under the remap) and share
    // their dY / Y rows through L2.
    const int nt = (int)(lb % ntn);
    const int64_t m0 = (lb / ntn) * BM;
    const int n0 = nt * BN;
    const bool lead = nt == 0;
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int wm = wave / WN, wn = wave % WN;
    const int li = lane & 31, lh = lane >> 5;

    if (tid < BM) {
        const int64_t m = m0 + tid;
        float4 s = make_float4(0.f, 0.f, 0.f, 1.f);
        if (m < p.M) {
            float ci, co, cd, cu, ca;
            gate_values(p.g, m, ci, co, cd, cu, ca);
            const float cad = ca * cd;
            s.x = cad * ci;
            s.y = cad * co;
            s.z = ca * cu;
            if (lead) st4(p.gates + m * 4, s);
        }
        st4(&Sg[tid * 4], s);
    }

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    float4 ra[A_F4], ry[A_F4], rb[B_F4];
    float bd[A_F4][3];
#pragma unroll
    for (int q = 0; q < A_F4; ++q) bd[q][0] = bd[q][1] = bd[q][2] = 0.f;
    const int64_t mlast = p.M - 1;
    auto fetch = [&](int k0) {
#pragma unroll
        for (int q = 0; q < A_F4; ++q) {
            const int idx = tid + NT * q;
            const int64_t m = min(m0 + (idx >> 3), mlast);
            const int k = k0 + 4 * (idx & 7);
            const int kc = k < p.F_out ? k : 0;
            ra[q] = ld4(p.dY + m * p.lddy + kc);
            if (p.act) ry[q] = ld4(p.Y + m * p.ldy + kc);
        }
#pragma unroll
        for (int q = 0; q < B_F4; ++q) {
            const int idx = tid + NT * q;
            const int n = min(n0 + (idx >> 3), p.N - 1);
            const int k = k0 + 4 * (idx & 7);
            rb[q] = ld4(p.BT + (int64_t)n * p.F_out + (k < p.F_out ? k : 0));
        }
    };
    auto stash = [&](int buf, int k0) {
#pragma unroll
        for (int q = 0; q < A_F4; ++q) {
            const int idx = tid + NT * q;
            const int k = k0 + 4 * (idx & 7);
            const int64_t m = m0 + (idx >> 3);
            float4 d = ra[q];
            if (p.act) {
                const float4 y = ry[q];
                d.x = pg::act_grad(d.x, y.x, p.slope, p.drop_s);
                d.y = pg::act_grad(d.y, y.y, p.slope, p.drop_s);
                d.z = pg::act_grad(d.z, y.z, p.slope, p.drop_s);
                d.w = pg::act_grad(d.w, y.w, p.slope, p.drop_s);
            }
            if (k >= p.F_out) d = make_float4(0.f, 0.f, 0.f, 0.f);
            if (lead && k < p.F_out && m < p.M) {
                st4(p.dpre + m * p.ldp + k, d);
#pragma unroll
                for (int s = 0; s < 3; ++s) bd[q][s] += dot4(d, ld4(p.bsum + s * p.F_out + k));
            }
            st4(&As[buf][(idx >> 3) * LDSW + 4 * (idx & 7)], d);
        }
#pragma unroll
        for (int q = 0; q < B_F4; ++q) {
            const int idx = tid + NT * q;
            const int k = k0 + 4 * (idx & 7);
            st4(&Bs[buf][(idx >> 3) * LDSW + 4 * (idx & 7)], k < p.F_out ? rb[q] : make_float4(0.f, 0.f, 0.f, 0.f));
        }
    };

    const int ntiles = (p.F_out + BK - 1) / BK;
    fetch(0);
    stash(0, 0);
    __syncthreads();
    for (int t = 0; t < ntiles; ++t) {
        const int cur = t & 1;
        if (t + 1 < ntiles) fetch((t + 1) * BK);
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
        if (t + 1 < ntiles) stash(cur ^ 1, (t + 1) * BK);
        __syncthreads();
    }

    // bias dots <dpre[m], bsum_q>: 8 consecutive lanes hold one row's K slices
    if (lead) {
#pragma unroll
        for (int q = 0; q < A_F4; ++q) {
#pragma unroll
            for (int s = 0; s < 3; ++s) {
                float v = bd[q][s];
                v += __shfl_xor(v, 1);
                v += __shfl_xor(v, 2);
                v += __shfl_xor(v, 4);
                bd[q][s] = v;
            }
            const int idx = tid + NT * q;
            if ((idx & 7) == 0) {
                Bd[(idx >> 3) * 3 + 0] = bd[q][0];
                Bd[(idx >> 3) * 3 + 1] = bd[q][1];
                Bd[(idx >> 3) * 3 + 2] = bd[q][2];
            }
        }
    }

    float* T = smem;
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
    constexpr int BATCH = ITER < 4 ? ITER : 4;
    const int c4 = tid % C4;
    const int j = n0 + 4 * c4;
    const int seg = j < p.N ? j / p.F_in : 4;  // F_in % 4 == 0: a float4 never straddles segments
    for (int it0 = 0; it0 < ITER; it0 += BATCH) {
        float4 zv[BATCH];
        int rl[BATCH];
        int64_t mm[BATCH];
#pragma unroll
        for (int u = 0; u < BATCH; ++u) {
            rl[u] = (tid + NT * (it0 + u)) / C4;
            mm[u] = m0 + rl[u];
            zv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (mm[u] < p.M && seg < 3) zv[u] = ld4(p.Z + mm[u] * p.ldz + j);
        }
#pragma unroll
        for (int u = 0; u < BATCH; ++u) {
            float part = 0.f;
            if (mm[u] < p.M && seg < 4) {
                const float4 gv = ld4(&T[rl[u] * TLD + 4 * c4]);
                if (seg < 3) {
                    const float s = Sg[rl[u] * 4 + seg];
                    if (p.dZ) st4(p.dZ + mm[u] * p.lddz + j, make_float4(s * gv.x, s * gv.y, s * gv.z, s * gv.w));
                    part = dot4(gv, zv[u]);
                } else {
                    st4(p.dres + mm[u] * p.lddres + (j - 3 * p.F_in), gv);
                }
            }
            T[rl[u] * TLD + 4 * c4] = part;  // own slot, already consumed
        }
    }
    __syncthreads();
    if (tid < BM && m0 + tid < p.M) {
        const int64_t m = m0 + tid;
        float ds[3] = {0.f, 0.f, 0.f};
        if (lead) {
            ds[0] = Bd[tid * 3 + 0];
            ds[1] = Bd[tid * 3 + 1];
            ds[2] = Bd[tid * 3 + 2];
        }
        for (int c = 0; c < C4; ++c) {
            const int jj = n0 + 4 * c;
            if (jj >= p.N) break;
            const int q = jj / p.F_in;
            if (q < 3) ds[q] += T[tid * TLD + 4 * c];
        }  // (row_gate_partials spilled 16 B per lane here)
#pragma unroll
        for (int q = 0; q < 3; ++q) p.dsp[((int64_t)nt * 3 + q) * p.M + m] = ds[q];
    }
}

// ------------------------------------------------------------------------------------------------
// dgrad_x3_kernel (round 5; the fp32 default where F_out % 32 == 0): dgrad_kernel's tiling, outputs and epilogue
// with the products on the bf16 matrix cores in the exact three-way split (pg_split3.h): every fp32 operand value
// v = v0 + v1 + v2 (bf16 each), G = sum of the six products a_i b_j with i + j <= 2 on v_mfma_f32_32x32x16_bf16,
// fp32 accumulation (the dropped terms are below 2^-24 |a b|; the forward's split-bf16 kernel makes the same
// choice). The 32x32x16 bf16 form takes 6 x 32 cycles per 16-deep k-step where v_mfma_f32_32x32x2f32 takes 8 x 64:
// 2.7x fewer matrix-core cycles, which at B(20,4) F = 128 turns dgrad_kernel's 0.23 ms of fp32 MFMA time into a
// memory-bound kernel. A = dpre (split once per k-tile while staging, as bf16 images), B = the packed weights
// transposed and split once per backward (transpose_split3_kernel: BT3 [3][N][F_out] bf16). LDS per buffer: three
// A and three B images of BM / BN rows x 32 k (rows padded to 40 bf16 = 80 B: conflict-free ds_read_b128).
// Built without SLP vectorisation (see dgrad_bf16_kernel).
constexpr int XBK = 32;
constexpr int XLDK = 40;

__device__ __forceinline__ f32x16 mfma32_bf(uint4 a, uint4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(pgx3::bf16x8_t, a),
                                                   __builtin_bit_cast(pgx3::bf16x8_t, b), c, 0, 0, 0);
}

// exact three-way split of 4 fp32 values into three bf16x4 (8-B) pieces
__device__ __forceinline__ void split4(float4 v, uint2& s0, uint2& s1, uint2& s2) {
    float a = v.x, b = v.y, c = v.z, d = v.w, fa, fb, fc, fd;
    uint32_t w0 = pgx3::bf2(a, b, fa, fb), w1 = pgx3::bf2(c, d, fc, fd);
    s0 = make_uint2(w0, w1);
    a -= fa; b -= fb; c -= fc; d -= fd;
    w0 = pgx3::bf2(a, b, fa, fb);
    w1 = pgx3::bf2(c, d, fc, fd);
    s1 = make_uint2(w0, w1);
    a -= fa; b -= fb; c -= fc; d -= fd;
    w0 = pgx3::bf2(a, b, fa, fb);
    w1 = pgx3::bf2(c, d, fc, fd);
    s2 = make_uint2(w0, w1);
}

template <int BM, int BN, int NW>
__global__ __launch_bounds__(64 * NW, 3) void dgrad_x3_kernel(DgradP p, const uint16_t* BT3) {
    constexpr int NT = 64 * NW;
    constexpr int WN = 2;
    constexpr int WM = NW / WN;
    constexpr int TM = BM / WM / 32;
    constexpr int TN = BN / WN / 32;
    static_assert(TM >= 1 && TN >= 1, "wave tile too small");
    constexpr int A_F4 = BM * XBK / 4 / NT;  // fp32 float4 pieces of dY (and Y) per thread per k-tile
    constexpr int B_C = BN * XBK / 8 / NT;   // bf16x8 pieces of each B split per thread per k-tile
    static_assert(A_F4 >= 1 && B_C >= 1, "tile shape");
    constexpr int TLD = BN + 4;
    constexpr int IMG = XLDK;                              // u16 per image row
    constexpr int MAIN_U16 = 3 * (BM + BN) * IMG;          // one buffer of three A and three B images
    constexpr int SMEM_BYTES = MAIN_U16 * 2 > BM * TLD * 4 ? MAIN_U16 * 2 : BM * TLD * 4;
    __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM_BYTES];
    __shared__ __attribute__((aligned(16))) float Sg[BM * 4];
    __shared__ float Bd[BM * 3];
    uint16_t* const img = reinterpret_cast<uint16_t*>(smem);
    auto Aimg = [&](int buf, int sp) { return img + (buf * 3 + sp) * BM * IMG; };  // buf = 0: one LDS buffer
    auto Bimg = [&](int buf, int sp) { return img + 3 * BM * IMG + (buf * 3 + sp) * BN * IMG; };

    const int ntn = (p.N + BN - 1) / BN;
    const int64_t lb = pg::xcd_logical_block(blockIdx.x, gridDim.x, p.remap != 0);
    const int nt = (int)(lb % ntn);
    const int64_t m0 = (lb / ntn) * BM;
    const int n0 = nt * BN;
    const bool lead = nt == 0;
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int wm = wave / WN, wn = wave % WN;
    const int li = lane & 31, lh = lane >> 5;

    if (tid < BM) {
        const int64_t m = m0 + tid;
        float4 sv = make_float4(0.f, 0.f, 0.f, 1.f);
        if (m < p.M) {
            float ci, co, cd, cu, ca;
            gate_values(p.g, m, ci, co, cd, cu, ca);
            const float cad = ca * cd;
            sv.x = cad * ci;
            sv.y = cad * co;
            sv.z = ca * cu;
            if (lead) st4(p.gates + m * 4, sv);
        }
        st4(&Sg[tid * 4], sv);
    }

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    float4 ra[A_F4], ry[A_F4];
    uint4 rb[B_C][3];
    float bd[A_F4][3];
#pragma unroll
    for (int q = 0; q < A_F4; ++q) bd[q][0] = bd[q][1] = bd[q][2] = 0.f;
    const int64_t mlast = p.M - 1;
    const int64_t bsplit = (int64_t)p.N * p.F_out;  // elements per BT3 split
    auto fetch = [&](int k0) {
#pragma unroll
        for (int q = 0; q < A_F4; ++q) {
            const int idx = tid + NT * q;
            const int64_t m = min(m0 + (idx >> 3), mlast);
            const int k = k0 + 4 * (idx & 7);
            const int kc = k < p.F_out ? k : 0;
            ra[q] = ld4(p.dY + m * p.lddy + kc);
            if (p.act) ry[q] = ld4(p.Y + m * p.ldy + kc);
        }
#pragma unroll
        for (int q = 0; q < B_C; ++q) {
            const int idx = tid + NT * q;
            const int n = min(n0 + (idx >> 2), p.N - 1);
            const int k = k0 + 8 * (idx & 3);
            const int64_t o = (int64_t)n * p.F_out + (k < p.F_out ? k : 0);
#pragma unroll
            for (int sp = 0; sp < 3; ++sp) rb[q][sp] = *reinterpret_cast<const uint4*>(BT3 + sp * bsplit + o);
        }
    };
    auto stash = [&](int buf, int k0) {
#pragma unroll
        for (int q = 0; q < A_F4; ++q) {
            const int idx = tid + NT * q;
            const int k = k0 + 4 * (idx & 7);
            const int64_t m = m0 + (idx >> 3);
            float4 d = ra[q];
            if (p.act) {
                const float4 y = ry[q];
                d.x = pg::act_grad(d.x, y.x, p.slope, p.drop_s);
                d.y = pg::act_grad(d.y, y.y, p.slope, p.drop_s);
                d.z = pg::act_grad(d.z, y.z, p.slope, p.drop_s);
                d.w = pg::act_grad(d.w, y.w, p.slope, p.drop_s);
            }
            if (k >= p.F_out) d = make_float4(0.f, 0.f, 0.f, 0.f);
            if (lead && k < p.F_out && m < p.M) {
                st4(p.dpre + m * p.ldp + k, d);
#pragma unroll
                for (int sg = 0; sg < 3; ++sg) bd[q][sg] += dot4(d, ld4(p.bsum + sg * p.F_out + k));
            }
            uint2 s0, s1, s2;
            split4(d, s0, s1, s2);
            const int o = (idx >> 3) * IMG + 4 * (idx & 7);
            *reinterpret_cast<uint2*>(Aimg(buf, 0) + o) = s0;
            *reinterpret_cast<uint2*>(Aimg(buf, 1) + o) = s1;
            *reinterpret_cast<uint2*>(Aimg(buf, 2) + o) = s2;
        }
#pragma unroll
        for (int q = 0; q < B_C; ++q) {
            const int idx = tid + NT * q;
            const int k = k0 + 8 * (idx & 3);
            const int o = (idx >> 2) * IMG + 8 * (idx & 3);
#pragma unroll
            for (int sp = 0; sp < 3; ++sp)
                *reinterpret_cast<uint4*>(Bimg(buf, sp) + o) = k < p.F_out ? rb[q][sp] : make_uint4(0u, 0u, 0u, 0u);
        }
    };

    // one LDS buffer (so that three workgroups fit a CU and one's epilogue overlaps another's k-loop): the next
    // k-tile's operands wait in registers during this tile's MFMAs, then are split into the buffer between two
    // barriers
    const int ntiles = (p.F_out + XBK - 1) / XBK;
    fetch(0);
    stash(0, 0);
    __syncthreads();
    for (int t = 0; t < ntiles; ++t) {
        const int cur = 0;
        if (t + 1 < ntiles) fetch((t + 1) * XBK);
#pragma unroll
        for (int kk = 0; kk < XBK / 16; ++kk) {
            uint4 a[TM][3], b[TN][3];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int sp = 0; sp < 3; ++sp)
                    a[i][sp] = *reinterpret_cast<const uint4*>(Aimg(cur, sp) + (wm * TM * 32 + i * 32 + li) * IMG +
                                                               kk * 16 + 8 * lh);
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int sp = 0; sp < 3; ++sp)
                    b[j][sp] = *reinterpret_cast<const uint4*>(Bimg(cur, sp) + (wn * TN * 32 + j * 32 + li) * IMG +
                                                               kk * 16 + 8 * lh);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {  // small terms first (the order of every split-bf16 kernel here)
                    acc[i][j] = mfma32_bf(a[i][2], b[j][0], acc[i][j]);
                    acc[i][j] = mfma32_bf(a[i][1], b[j][1], acc[i][j]);
                    acc[i][j] = mfma32_bf(a[i][0], b[j][2], acc[i][j]);
                    acc[i][j] = mfma32_bf(a[i][1], b[j][0], acc[i][j]);
                    acc[i][j] = mfma32_bf(a[i][0], b[j][1], acc[i][j]);
                    acc[i][j] = mfma32_bf(a[i][0], b[j][0], acc[i][j]);
                }
        }
        if (t + 1 < ntiles) {
            __syncthreads();
            stash(0, (t + 1) * XBK);
        }
        __syncthreads();
    }

    // bias dots <dpre[m], bsum_q>: 8 consecutive lanes hold one row's K slices
    if (lead) {
#pragma unroll
        for (int q = 0; q < A_F4; ++q) {
#pragma unroll
            for (int sg = 0; sg < 3; ++sg) {
                float v = bd[q][sg];
                v += __shfl_xor(v, 1);
                v += __shfl_xor(v, 2);
                v += __shfl_xor(v, 4);
                bd[q][sg] = v;
            }
            const int idx = tid + NT * q;
            if ((idx & 7) == 0) {
                Bd[(idx >> 3) * 3 + 0] = bd[q][0];
                Bd[(idx >> 3) * 3 + 1] = bd[q][1];
                Bd[(idx >> 3) * 3 + 2] = bd[q][2];
            }
        }
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
    constexpr int BATCH = ITER < 4 ? ITER : 4;
    const int c4 = tid % C4;
    const int j = n0 + 4 * c4;
    const int seg = j < p.N ? j / p.F_in : 4;  // F_in % 4 == 0: a float4 never straddles segments
    for (int it0 = 0; it0 < ITER; it0 += BATCH) {
        float4 zv[BATCH];
        int rl[BATCH];
        int64_t mm[BATCH];
#pragma unroll
        for (int u = 0; u < BATCH; ++u) {
            rl[u] = (tid + NT * (it0 + u)) / C4;
            mm[u] = m0 + rl[u];
            zv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (mm[u] < p.M && seg < 3) zv[u] = ld4(p.Z + mm[u] * p.ldz + j);
        }
#pragma unroll
        for (int u = 0; u < BATCH; ++u) {
            float part = 0.f;
            if (mm[u] < p.M && seg < 4) {
                const float4 gv = ld4(&T[rl[u] * TLD + 4 * c4]);
                if (seg < 3) {
                    const float sc = Sg[rl[u] * 4 + seg];
                    if (p.dZ) st4(p.dZ + mm[u] * p.lddz + j, make_float4(sc * gv.x, sc * gv.y, sc * gv.z, sc * gv.w));
                    part = dot4(gv, zv[u]);
                } else {
                    st4(p.dres + mm[u] * p.lddres + (j - 3 * p.F_in), gv);
                }
            }
            T[rl[u] * TLD + 4 * c4] = part;  // own slot, already consumed
        }
    }
    __syncthreads();
    if (tid < BM && m0 + tid < p.M) {
        const int64_t m = m0 + tid;
        float ds[3] = {0.f, 0.f, 0.f};
        if (lead) {
            ds[0] = Bd[tid * 3 + 0];
            ds[1] = Bd[tid * 3 + 1];
            ds[2] = Bd[tid * 3 + 2];
        }
        row_gate_partials<C4>(&T[tid * TLD], n0, p.N, p.F_in, ds);
#pragma unroll
        for (int q = 0; q < 3; ++q) p.dsp[((int64_t)nt * 3 + q) * p.M + m] = ds[q];
    }
}

// ------------------------------------------------------------------------------------------------
// dgrad_span_kernel (round 5): dgrad_x3_kernel's arithmetic with each workgroup's n-tile spanning ALL THREE segments
// of a 64-feature block (columns (q, f) for q = in, out, und and f in [64 nt, 64 nt + 64)), so a lane holds
// G_in, G_out, G_und of the same (row, feature) in its accumulators (TN = 3, one per segment). That makes the
// transposed propagation's diagonal term free ("Transposed middle-tile kernel"):
//   E[m, f] = sum_q Wdiag_q[m] dZ_q[m, f]  (+ dpre[m, f] for the model's identity residual)
// is written next to dZ, and the off-diagonal transposed kernel (pg_spmm3t_ngram_mid_offdiag_f32) accumulates into E,
// which then is the layer input's whole gradient. The epilogue runs from the accumulators (no tile in LDS): dZ / E
// stores and Z loads are 128-B row pieces of 32 lanes; the gate partials <G_q, Z_q> go through LDS, summed per row in
// feature order. Two workgroups of four waves per CU; wave (wm, wn): rows 32 wm.., features 64 nt + 32 wn + lane%32.
struct SpanP {
    const float* wdiag;  // [M or rows, 3]: Wdiag_in, _out, _und per row (NgramPlan.diag3())
    float* E;
    int64_t lde;
    int e_res;           // add dpre (identity residual)
};

template <int BM, int NW>
__global__ __launch_bounds__(64 * NW, 2) void dgrad_span_kernel(DgradP p, const uint16_t* BT3, SpanP sp) {
    constexpr int NT = 64 * NW;
    constexpr int WN = 2, WM = NW / WN;
    static_assert(BM == 32 * WM, "one 32-row MFMA tile per wave");
    constexpr int FB = 64;                 // features per workgroup
    constexpr int BNC = 3 * FB;            // B columns per workgroup (three segments)
    constexpr int A_F4 = BM * XBK / 4 / NT;
    constexpr int B_C = BNC * XBK / 8 / NT;
    static_assert(A_F4 >= 1 && B_C >= 1 && BNC * XBK % (8 * NT) == 0, "tile shape");
    constexpr int IMG = XLDK;
    constexpr int MAIN_U16 = 3 * (BM + BNC) * IMG;
    constexpr int PBYTES = BM * (3 * FB + 4) * 4;  // the epilogue's G tile, then <G_q, Z_q> products per (row, q, feature)
    constexpr int SMEM_BYTES = MAIN_U16 * 2 > PBYTES ? MAIN_U16 * 2 : PBYTES;
    __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM_BYTES];
    __shared__ __attribute__((aligned(16))) float Sg[BM * 4];
    __shared__ float Wd[BM * 3];
    __shared__ float Bd[BM * 3];
    uint16_t* const img = reinterpret_cast<uint16_t*>(smem);
    auto Aimg = [&](int spl) { return img + spl * BM * IMG; };
    auto Bimg = [&](int spl) { return img + 3 * BM * IMG + spl * BNC * IMG; };

    const int ntn = p.F_in / FB;
    const int64_t lb = pg::xcd_logical_block(blockIdx.x, gridDim.x, p.remap != 0);
    const int nt = (int)(lb % ntn);
    const int64_t m0 = (lb / ntn) * BM;
    const bool lead = nt == 0;
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int wm = wave / WN, wn = wave % WN;
    const int li = lane & 31, lh = lane >> 5;
    const int f = nt * FB + wn * 32 + li;  // this lane's feature (epilogue)

    if (tid < BM) {
        const int64_t m = m0 + tid;
        float4 sv = make_float4(0.f, 0.f, 0.f, 1.f);
        float w0 = 0.f, w1 = 0.f, w2 = 0.f;
        if (m < p.M) {
            float ci, co, cd, cu, ca;
            gate_values(p.g, m, ci, co, cd, cu, ca);
            const float cad = ca * cd;
            sv.x = cad * ci;
            sv.y = cad * co;
            sv.z = ca * cu;
            if (lead) st4(p.gates + m * 4, sv);
            w0 = sp.wdiag[m * 3 + 0];
            w1 = sp.wdiag[m * 3 + 1];
            w2 = sp.wdiag[m * 3 + 2];
        }
        st4(&Sg[tid * 4], sv);
        Wd[tid * 3 + 0] = w0;
        Wd[tid * 3 + 1] = w1;
        Wd[tid * 3 + 2] = w2;
    }

    f32x16 acc[3];
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

    float4 ra[A_F4], ry[A_F4];
    float bd[A_F4][3];
#pragma unroll
    for (int q = 0; q < A_F4; ++q) bd[q][0] = bd[q][1] = bd[q][2] = 0.f;
    const int64_t mlast = p.M - 1;
    const int64_t bsplit = (int64_t)p.N * p.F_out;
    // B a k-tile ahead in named registers (an array here stays in scratch memory)
    static_assert(B_C == 3, "three B pieces per thread");
    uint4 rb00, rb01, rb02, rb10, rb11, rb12, rb20, rb21, rb22;
    auto fetch = [&](int k0) {
#pragma unroll
        for (int q = 0; q < A_F4; ++q) {
            const int idx = tid + NT * q;
            const int64_t m = min(m0 + (idx >> 3), mlast);
            const int k = k0 + 4 * (idx & 7);
            ra[q] = ld4(p.dY + m * p.lddy + k);
            if (p.act) ry[q] = ld4(p.Y + m * p.ldy + k);
        }
        // B (the split packed weights, 295 KB at F = 128: L2-resident), a k-tile ahead like A
        auto bsrc = [&](int q) {
            const int idx = tid + NT * q;
            const int c = idx >> 2;  // workgroup column: (wn_c, segment, lane)
            const int n = (c % 96) / 32 * p.F_in + nt * FB + (c / 96) * 32 + (c % 32);
            return BT3 + (int64_t)n * p.F_out + k0 + 8 * (idx & 3);
        };
        const uint16_t* b0 = bsrc(0);
        const uint16_t* b1 = bsrc(1);
        const uint16_t* b2 = bsrc(2);
        rb00 = *reinterpret_cast<const uint4*>(b0);
        rb01 = *reinterpret_cast<const uint4*>(b0 + bsplit);
        rb02 = *reinterpret_cast<const uint4*>(b0 + 2 * bsplit);
        rb10 = *reinterpret_cast<const uint4*>(b1);
        rb11 = *reinterpret_cast<const uint4*>(b1 + bsplit);
        rb12 = *reinterpret_cast<const uint4*>(b1 + 2 * bsplit);
        rb20 = *reinterpret_cast<const uint4*>(b2);
        rb21 = *reinterpret_cast<const uint4*>(b2 + bsplit);
        rb22 = *reinterpret_cast<const uint4*>(b2 + 2 * bsplit);
    };
    auto stash = [&](int k0) {
#pragma unroll
        for (int q = 0; q < A_F4; ++q) {
            const int idx = tid + NT * q;
            const int k = k0 + 4 * (idx & 7);
            const int64_t m = m0 + (idx >> 3);
            float4 d = ra[q];
            if (p.act) {
                const float4 y = ry[q];
                d.x = pg::act_grad(d.x, y.x, p.slope, p.drop_s);
                d.y = pg::act_grad(d.y, y.y, p.slope, p.drop_s);
                d.z = pg::act_grad(d.z, y.z, p.slope, p.drop_s);
                d.w = pg::act_grad(d.w, y.w, p.slope, p.drop_s);
            }
            if (lead && m < p.M) {
                st4(p.dpre + m * p.ldp + k, d);
#pragma unroll
                for (int sg = 0; sg < 3; ++sg) bd[q][sg] += dot4(d, ld4(p.bsum + sg * p.F_out + k));
            }
            uint2 s0, s1, s2;
            split4(d, s0, s1, s2);
            const int o = (idx >> 3) * IMG + 4 * (idx & 7);
            *reinterpret_cast<uint2*>(Aimg(0) + o) = s0;
            *reinterpret_cast<uint2*>(Aimg(1) + o) = s1;
            *reinterpret_cast<uint2*>(Aimg(2) + o) = s2;
        }
        auto bdst = [&](int q) {
            const int idx = tid + NT * q;
            return (idx >> 2) * IMG + 8 * (idx & 3);
        };
        const int o0 = bdst(0), o1 = bdst(1), o2 = bdst(2);
        *reinterpret_cast<uint4*>(Bimg(0) + o0) = rb00;
        *reinterpret_cast<uint4*>(Bimg(1) + o0) = rb01;
        *reinterpret_cast<uint4*>(Bimg(2) + o0) = rb02;
        *reinterpret_cast<uint4*>(Bimg(0) + o1) = rb10;
        *reinterpret_cast<uint4*>(Bimg(1) + o1) = rb11;
        *reinterpret_cast<uint4*>(Bimg(2) + o1) = rb12;
        *reinterpret_cast<uint4*>(Bimg(0) + o2) = rb20;
        *reinterpret_cast<uint4*>(Bimg(1) + o2) = rb21;
        *reinterpret_cast<uint4*>(Bimg(2) + o2) = rb22;
        (void)k0;
    };

    const int ntiles = p.F_out / XBK;
    fetch(0);
    stash(0);
    __syncthreads();
    for (int t = 0; t < ntiles; ++t) {
        if (t + 1 < ntiles) fetch((t + 1) * XBK);
#pragma unroll
        for (int kk = 0; kk < XBK / 16; ++kk) {
            uint4 a[3], b[3][3];
#pragma unroll
            for (int spl = 0; spl < 3; ++spl)
                a[spl] = *reinterpret_cast<const uint4*>(Aimg(spl) + (wm * 32 + li) * IMG + kk * 16 + 8 * lh);
#pragma unroll
            for (int j = 0; j < 3; ++j)
#pragma unroll
                for (int spl = 0; spl < 3; ++spl)
                    b[j][spl] = *reinterpret_cast<const uint4*>(Bimg(spl) + (wn * 96 + j * 32 + li) * IMG + kk * 16 +
                                                                8 * lh);
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                acc[j] = mfma32_bf(a[2], b[j][0], acc[j]);
                acc[j] = mfma32_bf(a[1], b[j][1], acc[j]);
                acc[j] = mfma32_bf(a[0], b[j][2], acc[j]);
                acc[j] = mfma32_bf(a[1], b[j][0], acc[j]);
                acc[j] = mfma32_bf(a[0], b[j][1], acc[j]);
                acc[j] = mfma32_bf(a[0], b[j][0], acc[j]);
            }
        }
        if (t + 1 < ntiles) {
            __syncthreads();
            stash((t + 1) * XBK);
        }
        __syncthreads();
    }

    if (lead) {
#pragma unroll
        for (int q = 0; q < A_F4; ++q) {
#pragma unroll
            for (int sg = 0; sg < 3; ++sg) {
                float v = bd[q][sg];
                v += __shfl_xor(v, 1);
                v += __shfl_xor(v, 2);
                v += __shfl_xor(v, 4);
                bd[q][sg] = v;
            }
            const int idx = tid + NT * q;
            if ((idx & 7) == 0) {
                Bd[(idx >> 3) * 3 + 0] = bd[q][0];
                Bd[(idx >> 3) * 3 + 1] = bd[q][1];
                Bd[(idx >> 3) * 3 + 2] = bd[q][2];
            }
        }
    }

    // epilogue through LDS: the accumulators are parked as T [BM][3 x 64] (the k-loop ended with a barrier); thread
    // item (row rl, features 4c..4c+3 of the block) reads G_q for q = in, out, und, writes dZ_q = s_q G_q and
    // E = sum_q Wdiag_q dZ_q (+ dpre, recomputed from dY and Y: the value the k-loop split exactly) as float4 row pieces,
    // and leaves its products G_q Z_q in its own T slots for the per-row gate partials (summed in feature order)
    constexpr int TLD = BNC + 4;
    constexpr int C4 = FB / 4;
    constexpr int ITEMS = BM * C4 / NT;
    static_assert(BM * TLD * 4 <= SMEM_BYTES && BM * C4 % NT == 0, "epilogue tile");
    (void)f;
    float* T = reinterpret_cast<float*>(smem);
    const int c4 = tid % C4;
    const int fo = nt * FB + 4 * c4;  // this thread's first feature
    float4 zv[ITEMS][3], dy[ITEMS], yy[ITEMS];
#pragma unroll
    for (int u = 0; u < ITEMS; ++u) {  // loads first: their latency overlaps the parking of the accumulators
        const int rl = (tid + NT * u) / C4;
        const int64_t m = min(m0 + rl, mlast);
#pragma unroll
        for (int q = 0; q < 3; ++q) zv[u][q] = ld4(p.Z + m * p.ldz + q * p.F_in + fo);
        if (sp.e_res) {
            dy[u] = ld4(p.dY + m * p.lddy + fo);
            yy[u] = p.act ? ld4(p.Y + m * p.ldy + fo) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int rl = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
            T[rl * TLD + j * FB + wn * 32 + li] = acc[j][r];
        }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < ITEMS; ++u) {
        const int rl = (tid + NT * u) / C4;
        const int64_t m = m0 + rl;
        float4 g[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) g[q] = ld4(&T[rl * TLD + q * FB + 4 * c4]);
        float4 e = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const float sq = Sg[rl * 4 + q], wq = Wd[rl * 3 + q];
            const float4 dz = make_float4(sq * g[q].x, sq * g[q].y, sq * g[q].z, sq * g[q].w);
            if (m < p.M && p.dZ) st4(p.dZ + m * p.lddz + q * p.F_in + fo, dz);
            e = make_float4(__fmaf_rn(wq, dz.x, e.x), __fmaf_rn(wq, dz.y, e.y), __fmaf_rn(wq, dz.z, e.z),
                            __fmaf_rn(wq, dz.w, e.w));
            st4(&T[rl * TLD + q * FB + 4 * c4], make_float4(g[q].x * zv[u][q].x, g[q].y * zv[u][q].y,
                                                            g[q].z * zv[u][q].z, g[q].w * zv[u][q].w));
        }
        if (sp.e_res) {
            float4 d = dy[u];
            if (p.act) {
                d.x = pg::act_grad(d.x, yy[u].x, p.slope, p.drop_s);
                d.y = pg::act_grad(d.y, yy[u].y, p.slope, p.drop_s);
                d.z = pg::act_grad(d.z, yy[u].z, p.slope, p.drop_s);
                d.w = pg::act_grad(d.w, yy[u].w, p.slope, p.drop_s);
            }
            e = make_float4(e.x + d.x, e.y + d.y, e.z + d.z, e.w + d.w);
        }
        if (m < p.M) st4(sp.E + m * sp.lde + fo, e);
    }
    __syncthreads();
    // gate partials: thread (row tid / 4, q = tid % 4 < 3) sums its row's 64 products of segment q in feature order
    if (tid < 4 * BM) {
        const int rl = tid >> 2, q = tid & 3;
        const int64_t m = m0 + rl;
        if (q < 3 && m < p.M) {
            float ds = lead ? Bd[rl * 3 + q] : 0.f;
            const float* row = T + rl * TLD + q * FB;
            for (int c = 0; c < FB; ++c) ds += row[c];
            p.dsp[((int64_t)nt * 3 + q) * p.M + m] = ds;
        }
    }
}

// ds_q[m] = sum over n-tiles (fixed order) -> dL/dc_* per row (chain rule of s_q(c), :116-133)
__global__ __launch_bounds__(256) void gate_grad_kernel(int64_t M, int ntn, const float* dsp, Gates g, float* dgate) {
    for (int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x; m < M; m += (int64_t)gridDim.x * 256) {
        float d0 = 0.f, d1 = 0.f, d2 = 0.f;
        for (int t = 0; t < ntn; ++t) {
            d0 += dsp[((int64_t)t * 3 + 0) * M + m];
            d1 += dsp[((int64_t)t * 3 + 1) * M + m];
            d2 += dsp[((int64_t)t * 3 + 2) * M + m];
        }
        float ci, co, cd, cu, ca;
        gate_values(g, m, ci, co, cd, cu, ca);
        const float cad = ca * cd;
        dgate[0 * M + m] = d0 * cad;                       // c_in
        dgate[1 * M + m] = d1 * cad;                       // c_out
        dgate[2 * M + m] = ca * (d0 * ci + d1 * co);        // c_directed
        dgate[3 * M + m] = d2 * ca;                        // c_undirected
        dgate[4 * M + m] = cd * (d0 * ci + d1 * co) + d2 * cu;  // c_all
    }
}

// BT3[sp][c][r] = split sp of in[r][c] (the exact three-way bf16 split of pg_split3.h); R x C, once per backward
__global__ __launch_bounds__(256) void transpose_split3_kernel(int R, int C, const float* in, uint16_t* out) {
    const int64_t total = (int64_t)R * C;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int c = (int)(i / R), r = (int)(i % R);
        float v = in[(int64_t)r * C + c], fa, fb;
        const uint32_t w0 = pgx3::bf2(v, 0.f, fa, fb);
        v -= fa;
        const uint32_t w1 = pgx3::bf2(v, 0.f, fa, fb);
        v -= fa;
        const uint32_t w2 = pgx3::bf2(v, 0.f, fa, fb);
        out[i] = (uint16_t)(w0 & 0xffffu);
        out[total + i] = (uint16_t)(w1 & 0xffffu);
        out[2 * total + i] = (uint16_t)(w2 & 0xffffu);
    }
}

__global__ __launch_bounds__(256) void transpose_kernel(int R, int C, const float* in, float* out) {
    // out[c][r] = in[r][c]; tiny (the packed weights), run once per backward
    const int64_t total = (int64_t)R * C;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int c = (int)(i / R), r = (int)(i % R);
        out[i] = in[(int64_t)r * C + c];
    }
}

struct WgradP {
    int64_t M;
    int P, N, F_in;
    const float* A;  // [M, P]
    int64_t lda;
    const float* Z;  // segments 0..2
    int64_t ldz;
    const float* R;  // segment 3 (projected residual input) or null
    int64_t ldr;
    const float* gates;  // [M, 4] or null (all scales 1)
    int64_t rows_per_split;
    int64_t part_stride;
    float* part;  // [splits, P*N + 4*P]
};

constexpr int WROWS = 32;  // rows per K step
constexpr int WLD = 132;   // LDS row (floats)

template <int NW>
__global__ __launch_bounds__(64 * NW) void wgrad_kernel(WgradP p) {
    constexpr int NT = 64 * NW;
    constexpr int BI = 128, BJ = 128;
    constexpr int WJ = 2, WI = NW / WJ;
    constexpr int TI = BI / WI / 32, TJ = BJ / WJ / 32;
    constexpr int F4 = WROWS * 32 / NT;  // float4 per thread per operand (rows of 128 floats = 32 float4)
    static_assert(TI >= 1 && TJ >= 1 && F4 >= 1, "tile");
    __shared__ __attribute__((aligned(16))) float smem[4 * WROWS * WLD];
    float (*As)[WROWS * WLD] = reinterpret_cast<float (*)[WROWS * WLD]>(smem);
    float (*Bs)[WROWS * WLD] = reinterpret_cast<float (*)[WROWS * WLD]>(smem + 2 * WROWS * WLD);

    const int j0 = blockIdx.x * BJ, i0 = blockIdx.y * BI;
    const int64_t r0 = (int64_t)blockIdx.z * p.rows_per_split;
    const int64_t rend = min(r0 + p.rows_per_split, p.M);
    const bool do_db = blockIdx.x == 0;
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int wi = wave / WJ, wj = wave % WJ;
    const int li = lane & 31, lh = lane >> 5;
    const int c4 = tid & 31;
    const int ia = i0 + 4 * c4, jb = j0 + 4 * c4;
    const bool ia_ok = ia < p.P, jb_ok = jb < p.N;
    const int seg = jb_ok ? jb / p.F_in : 0;
    const float* bsrc = seg < 3 ? p.Z + jb : p.R + (jb - 3 * p.F_in);
    const int64_t ldb = seg < 3 ? p.ldz : p.ldr;

    f32x16 acc[TI][TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    float db[4][4];
#pragma unroll
    for (int q = 0; q < 4; ++q) db[q][0] = db[q][1] = db[q][2] = db[q][3] = 0.f;

    float4 ra[F4], rb[F4], rs[F4];
    const int64_t mlast = p.M - 1;
    auto fetch = [&](int64_t base) {
#pragma unroll
        for (int q = 0; q < F4; ++q) {
            const int row = (tid + NT * q) >> 5;
            const int64_t m = min(base + row, mlast);
            ra[q] = ld4(p.A + m * p.lda + (ia_ok ? ia : 0));
            rb[q] = ld4((jb_ok ? bsrc : p.Z) + m * ldb);
            rs[q] = p.gates ? ld4(p.gates + m * 4) : make_float4(1.f, 1.f, 1.f, 1.f);
        }
    };
    auto stash = [&](int buf, int64_t base) {
#pragma unroll
        for (int q = 0; q < F4; ++q) {
            const int row = (tid + NT * q) >> 5;
            const bool ok = base + row < rend;
            const float4 s = rs[q];
            const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);
            const float4 a = (ok && ia_ok) ? ra[q] : zero;
            const float sc = seg == 0 ? s.x : seg == 1 ? s.y : seg == 2 ? s.z : 1.f;
            const float4 b = (ok && jb_ok) ? make_float4(rb[q].x * sc, rb[q].y * sc, rb[q].z * sc, rb[q].w * sc) : zero;
            if (do_db) {
                const float sv[4] = {s.x, s.y, s.z, 1.f};
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    db[t][0] += sv[t] * a.x;
                    db[t][1] += sv[t] * a.y;
                    db[t][2] += sv[t] * a.z;
                    db[t][3] += sv[t] * a.w;
                }
            }
            st4(&As[buf][row * WLD + 4 * c4], a);
            st4(&Bs[buf][row * WLD + 4 * c4], b);
        }
    };

    const int64_t nsteps = (rend - r0 + WROWS - 1) / WROWS;
    if (nsteps > 0) {
        fetch(r0);
        stash(0, r0);
    }
    __syncthreads();
    for (int64_t t = 0; t < nsteps; ++t) {
        const int cur = (int)(t & 1);
        const int64_t nb = r0 + (t + 1) * WROWS;
        if (t + 1 < nsteps) fetch(nb);
        const float* Ab = As[cur];
        const float* Bb = Bs[cur];
#pragma unroll
        for (int g = 0; g < WROWS / 8; ++g) {
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int row = g * 8 + 4 * lh + s;
                float a[TI], b[TJ];
#pragma unroll
                for (int i = 0; i < TI; ++i) a[i] = Ab[row * WLD + wi * TI * 32 + i * 32 + li];
#pragma unroll
                for (int j = 0; j < TJ; ++j) b[j] = Bb[row * WLD + wj * TJ * 32 + j * 32 + li];
#pragma unroll
                for (int i = 0; i < TI; ++i)
#pragma unroll
                    for (int j = 0; j < TJ; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
            }
        }
        if (t + 1 < nsteps) stash(cur ^ 1, nb);
        __syncthreads();
    }

    float* out = p.part + (int64_t)blockIdx.z * p.part_stride;
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int oi = i0 + wi * TI * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                const int oj = j0 + wj * TJ * 32 + j * 32 + li;
                if (oi < p.P && oj < p.N) out[(int64_t)oi * p.N + oj] = acc[i][j][r];
            }

    if (do_db) {  // 16 row groups x 32 column groups x 16 sums -> fixed-order reduction over row groups
        constexpr int RG = NT / 32;
        float* D = smem;  // the K loop ended with a barrier
        const int rg = tid >> 5;
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int e = 0; e < 4; ++e) D[(rg * 32 + c4) * 16 + q * 4 + e] = db[q][e];
        __syncthreads();
        for (int w = tid; w < 32 * 16; w += NT) {
            const int cc = w & 31, qe = w >> 5;
            float v = 0.f;
            for (int g2 = 0; g2 < RG; ++g2) v += D[(g2 * 32 + cc) * 16 + qe];
            const int i = i0 + 4 * cc + (qe & 3);
            if (i < p.P) out[(int64_t)p.P * p.N + (qe >> 2) * p.P + i] = v;
        }
    }
}

// Split-bf16 weight gradient (round 5; the fp32 default where F_out % 128 == 0 and F_in % 128 == 0, no projected
// residual): the partial C[P x N] = A^T diag(s) B of one row split on v_mfma_f32_32x32x16_bf16 with exact three-way
// bf16 splits of both operands (pg_split3.h: six products, fp32-level accuracy). wgrad_kernel's v_mfma_f32_32x32x2f32
// takes 64 cycles per 2-deep k-step, the six bf16 products 6 x 32 per 16-deep one: 2.7x fewer matrix-core cycles,
// which moves the B(20,4) F = 128 weight gradient (15.7 GFLOP, 0.33 GB of operands) from the fp32 matrix cores'
// bound (~0.10 ms at peak, 0.175 ms measured) to about the HBM one.
// One 512-thread workgroup per (row split, 128 x 384 output tile), one per CU (LDS 100 KB; the tiles of a split on
// one XCD at neighbouring times, wgrad_tile_of, so they share the split's rows through its L2): each 16-row step is
// staged ONCE for the whole tile -- A = dpre (128 columns) and B = s_q Z_q (384 columns), 8 rows x 2 columns per
// thread, loaded two steps ahead through buffer descriptors -- split into three bf16 images and stored transposed, image [split][k-group][column]
// of 16-B units (the 8 rows of a k-group of one column: one MFMA operand of one lane), double-buffered (one barrier
// per step). Reads are conflict-free (16 lanes of a ds_read_b128 group read 16 consecutive columns, 256 B); the
// writes of a thread's two columns are 2-way conflicted (16 LDS-array cycles for a 13-cycle store). Wave w owns
// output rows 64 (w & 1).. (two 32-row tiles) and columns 96 (w >> 1).. (three 32-column tiles): 6 A and 3 x 3 B
// operand reads for 36 MFMAs per step. The A threads also sum the bias gradients (s_q dpre per column, in row order);
// the n-tile-0 workgroups reduce them over their two k-groups.
constexpr int WX_BP = 128, WX_BN = 384, WX_COLS = WX_BP + WX_BN, WX_K = 16;

// blockIdx.x -> (split, tile) with the `tiles` workgroups of a split on one XCD (hardware dispatch: block b on XCD
// b % 8), dispatched together: b = xcd + 8 (tiles j + tile) for split 8 j + xcd. Splits past `splits` get tile -1.
__device__ __forceinline__ void wgrad_tile_of(int b, int tiles, int splits, int& split, int& tile) {
    const int xcd = b & 7, q = b >> 3;
    split = 8 * (q / tiles) + xcd;
    tile = q % tiles;
    if (split >= splits) tile = -1;
}

__global__ __launch_bounds__(512, 1) void wgrad_x3_kernel(WgradP p, int splits) {
    __shared__ __attribute__((aligned(16))) uint4 U[2][3][2][WX_COLS];
    __shared__ float Db[2][4][WX_BP];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, li = lane & 31, kh = lane >> 5;
    const int n_tiles = min(p.N, 3 * p.F_in) / WX_BN;  // the gated segments (a projected residual's: wgrad_bf16_kernel)
    int split, tile;
    wgrad_tile_of((int)blockIdx.x, (p.P / WX_BP) * n_tiles, splits, split, tile);
    if (tile < 0) return;  // whole workgroup: no barrier reached
    const int pt = tile / n_tiles, nt = tile % n_tiles;
    const int64_t r0 = (int64_t)split * p.rows_per_split;
    const int64_t rend = min(r0 + p.rows_per_split, p.M);
    // staging role, from the wave index in a scalar register (so the buffer descriptors below are wave-uniform):
    // waves 0-1 stage A (k-group = wave), waves 2-4 / 5-7 B (k-group 0 / 1), 64 column pairs per wave
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const bool isA = wv < 2;
    const int kg = isA ? wv : (wv - 2) / 3;
    const int pair = (isA ? 0 : 64 * ((wv - 2) % 3)) + lane;
    const int col0 = (isA ? 0 : WX_BP) + 2 * pair;              // staged column (image index)
    const int gcol = isA ? WX_BP * pt + 2 * pair : WX_BN * nt + 2 * pair;
    const int seg = isA ? 3 : gcol / p.F_in;  // 3: unscaled (A)
    const float* src = isA ? p.A + WX_BP * pt : p.Z + WX_BN * nt;  // wave-uniform; the lane's columns: + 2 pair
    const int64_t ld = isA ? p.lda : p.ldz;
    // Two register slots of one step's rows each (x: the operand values, gq: the row's scale of this thread's segment),
    // loaded two steps ahead through buffer descriptors over the split's rows: rows past the split read as 0 (the
    // hardware's range check), so the loads and splits carry no clamps or selects. The bias sums need the three
    // gates of every row in the A threads: the B thread at the first column of a segment writes its scales to Gs with
    // the images, and the A threads add the step's sums after the barrier, from the split-time values they keep (va,
    // vb). A segment's bias belongs to the n-tile holding its first column, the unscaled one (q = 3) to n-tile 0.
    __shared__ float Gs[2][3][WX_K];
    const int gsel = seg < 3 ? seg : 0;
    const bool gwriter = !isA && gcol % p.F_in == 0;
    const int64_t nr64 = rend - r0;
    const int nrows = __builtin_amdgcn_readfirstlane(nr64 > 0 ? (int)nr64 : 0);  // scalar (descriptor word 2)
    const auto rs_x = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src + r0 * ld), 0, nrows * (int)ld * 4,
                                                        0x00020000);
    const auto rs_g = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.gates + r0 * 4), 0, nrows * 16, 0x00020000);
    const int ld4b = (int)ld * 4;
    const int xoff = 8 * kg * ld4b + 8 * pair, goff = (8 * kg * 4 + gsel) * 4;
    auto load = [&](float2 (&x)[8], float (&gq)[8], int step) {  // step < 2^31 / (16 ld) (host-checked)
        const int sx = step * WX_K * ld4b, sg = step * WX_K * 16;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
            const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs_x, xoff + sx + e * ld4b, 0, 0);
            x[e] = make_float2(__uint_as_float(v.x), __uint_as_float(v.y));
            gq[e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_g, goff + sg + e * 16, 0, 0));
        }
    };
    float db[4][2];
#pragma unroll
    for (int t = 0; t < 4; ++t) db[t][0] = db[t][1] = 0.f;
    float va[8], vb[8];
    auto split_store = [&](const float2 (&x)[8], const float (&gq)[8], int buf) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float sc = isA ? 1.f : gq[e];
            va[e] = __fmul_rn(x[e].x, sc);
            vb[e] = __fmul_rn(x[e].y, sc);
        }
        uint4 a0, a1, a2, b0, b1, b2;
        pgx3::split8(va, a0, a1, a2);
        pgx3::split8(vb, b0, b1, b2);
        U[buf][0][kg][col0] = a0;
        U[buf][1][kg][col0] = a1;
        U[buf][2][kg][col0] = a2;
        U[buf][0][kg][col0 + 1] = b0;
        U[buf][1][kg][col0 + 1] = b1;
        U[buf][2][kg][col0 + 1] = b2;
        if (gwriter) {
#pragma unroll
            for (int e = 0; e < 8; ++e) Gs[buf][seg][8 * kg + e] = gq[e];
        }
    };
    auto bias_step = [&](int cur) {  // A threads, after the barrier: the step's rows' bias sums, in row order
        if (!isA) return;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int row = 8 * kg + e;
            const float sv[4] = {Gs[cur][0][row], Gs[cur][1][row], Gs[cur][2][row], 1.f};
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                db[t][0] += sv[t] * va[e];
                db[t][1] += sv[t] * vb[e];
            }
        }
    };
    if (tid < 2 * 3 * WX_K) (&Gs[0][0][0])[tid] = 0.f;  // segments that start in another n-tile stay 0
    f32x16 acc[2][3];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int ih = wave & 1, jq = wave >> 1;
    auto mfma_step = [&](int cur) {
        uint4 a[2][3];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int sp = 0; sp < 3; ++sp) a[i][sp] = U[cur][sp][kh][64 * ih + 32 * i + li];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            uint4 b[3];
#pragma unroll
            for (int sp = 0; sp < 3; ++sp) b[sp] = U[cur][sp][kh][WX_BP + 96 * jq + 32 * j + li];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                acc[i][j] = mfma32_bf(a[i][2], b[0], acc[i][j]);
                acc[i][j] = mfma32_bf(a[i][1], b[1], acc[i][j]);
                acc[i][j] = mfma32_bf(a[i][0], b[2], acc[i][j]);
                acc[i][j] = mfma32_bf(a[i][1], b[0], acc[i][j]);
                acc[i][j] = mfma32_bf(a[i][0], b[1], acc[i][j]);
                acc[i][j] = mfma32_bf(a[i][0], b[0], acc[i][j]);
            }
        }
    };
    // step t: slot t & 1 takes step t + 2's rows, the MFMAs read image t & 1, slot (t + 1) & 1 (step t + 1's rows,
    // loaded a step ago) is split into image (t + 1) & 1; one barrier
    float2 x0[8], x1[8];
    float g0[8], g1[8];
    const int64_t nsteps = (rend - r0 + WX_K - 1) / WX_K;
    __syncthreads();  // Gs zeroed
    // Loads and splits are unconditional (past the last step: clamped rows, zero images, zero bias terms): VMEM
    // loads under a branch would make the compiler's wait counts assume the worst at the join -- waiting for the
    // newest step's loads before splitting the older one -- and undo the two-step prefetch
    load(x0, g0, 0);
    load(x1, g1, 1);
    split_store(x0, g0, 0);
    __syncthreads();
    for (int t = 0; t < (int)nsteps; t += 2) {
        bias_step(0);
        load(x0, g0, t + 2);
        mfma_step(0);
        split_store(x1, g1, 1);
        __syncthreads();
        bias_step(1);
        load(x1, g1, t + 3);
        if (t + 1 < nsteps) mfma_step(1);
        split_store(x0, g0, 0);
        __syncthreads();
    }
    float* out = p.part + (int64_t)split * p.part_stride;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int oi = WX_BP * pt + 64 * ih + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * kh;
                const int oj = WX_BN * nt + 96 * jq + 32 * j + li;
                out[(int64_t)oi * p.N + oj] = acc[i][j][r];
            }
    if (isA) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            Db[kg][t][2 * pair] = db[t][0];
            Db[kg][t][2 * pair + 1] = db[t][1];
        }
    }
    __syncthreads();
    {
        const int t = tid >> 7, c = tid & 127;  // 4 x 128 sums, k-groups in fixed order
        const int first = t * p.F_in;            // the segment's first column (q = 3: n-tile 0)
        const bool mine = t == 3 ? nt == 0 : (first >= WX_BN * nt && first < WX_BN * (nt + 1));
        if (mine) out[(int64_t)p.P * p.N + t * p.P + WX_BP * pt + c] = Db[0][t][c] + Db[1][t][c];
    }
}

// out[c] = sum_s part[s][c]. A block owns 32 consecutive float4 columns (512 contiguous bytes per split);
// its 8 thread groups take every 8th split and are combined in group order: deterministic, and enough
// loads in flight to stream the partials at HBM rate.
constexpr int RS_COLS = 32, RS_GROUPS = 8;
__global__ __launch_bounds__(256) void reduce_splits_kernel(int64_t n4, int splits, int64_t stride, const float* part,
                                                            float* out) {
    __shared__ float4 acc_s[RS_GROUPS][RS_COLS];
    const int c = threadIdx.x % RS_COLS, grp = threadIdx.x / RS_COLS;
    const int64_t i = (int64_t)blockIdx.x * RS_COLS + c;
    float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
    if (i < n4) {
        int k = grp;
        for (; k + RS_GROUPS < splits; k += 2 * RS_GROUPS) {  // two independent chains
            const float4 u = ld4(part + (int64_t)k * stride + 4 * i);
            const float4 v = ld4(part + (int64_t)(k + RS_GROUPS) * stride + 4 * i);
            s0.x += u.x; s0.y += u.y; s0.z += u.z; s0.w += u.w;
            s1.x += v.x; s1.y += v.y; s1.z += v.z; s1.w += v.w;
        }
        if (k < splits) {
            const float4 u = ld4(part + (int64_t)k * stride + 4 * i);
            s0.x += u.x; s0.y += u.y; s0.z += u.z; s0.w += u.w;
        }
    }
    acc_s[grp][c] = make_float4(s0.x + s1.x, s0.y + s1.y, s0.z + s1.z, s0.w + s1.w);
    __syncthreads();
    if (grp == 0 && i < n4) {
        float4 t = acc_s[0][c];
        for (int g = 1; g < RS_GROUPS; ++g) {
            const float4 v = acc_s[g][c];
            t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
        }
        st4(out + 4 * i, t);
    }
}

void launch_reduce(int64_t n4, int splits, int64_t stride, const float* part, float* out, hipStream_t s) {
    const int64_t nb = (n4 + RS_COLS - 1) / RS_COLS;
    hipLaunchKernelGGL(reduce_splits_kernel, dim3((unsigned)nb), dim3(RS_COLS * RS_GROUPS), 0, s, n4, splits, stride,
                       part, out);
}

// ------------------------------------------------------------------------------------------------
// bf16 mode: the same two products on v_mfma_f32_32x32x16_bf16 (bf16 operands, fp32 sums)
// ------------------------------------------------------------------------------------------------
constexpr int BKB = 64;  // K per dgrad tile (4 MFMA k-steps)
constexpr int LDKB = 72; // dgrad LDS row in bf16 (144 B: conflict-free ds_read_b128)

struct DgradB {
    int64_t M;
    int F_in, F_out, N;
    const uint16_t* dY;
    int64_t lddy;
    const uint16_t* Y;
    int64_t ldy;
    int act;
    float slope;
    float drop_s;        // fused layer dropout's scale (pg::act_grad), 0: none
    const uint16_t* BT;  // [N, F_out] bf16
    const float* bsum;   // [4, F_out]
    const uint16_t* Z;
    int64_t ldz;
    Gates g;
    uint16_t* dpre;
    int64_t ldp;
    uint16_t* dZ;
    int64_t lddz;
    uint16_t* dres;
    int64_t lddres;
    float* gates;
    float* dsp;
    int remap;
    float* dpre32;  // optional fp32 copy of dpre (the rounded values), or null
    int64_t ldp32;
};

// Reproducibility (round 5). With packed-FP32 VALU math (v_pk_fma_f32 / v_pk_mul_f32, formed by the SLP vectoriser
// from the lead tile's bias dots) this kernel's segment-0 gate partials came out wrong for 4-row groups (lanes 48-63
// of a wave; up to 0.8 % of one partial) in about half of the runs with cold caches, while its accumulators, its A
// images and its epilogue products were bit-identical (stage dumps of a diagnostics build, tools/r05_dgrad_dbg.py);
// padding after the wave's own MFMAs did not help, the same source built without SLP vectorisation is reproducible.
// pg_dense_bwd.hip is therefore compiled with -fno-slp-vectorize (Makefile). The occupancy bound is 2 waves per SIMD
// (154 VGPRs): at 4 (128 VGPRs) the compiler spilled 76 B per lane to scratch and the kernel ran 5 % slower.
template <int BM, int BN, int NW>
__global__ __launch_bounds__(64 * NW, 2) void dgrad_bf16_kernel(DgradB p) {
    using namespace pgbf;
    constexpr int NT = 64 * NW;
    constexpr int WN = 2, WM = NW / WN;
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    static_assert(TM >= 1 && TN >= 1, "wave tile");
    constexpr int A_C = BM * BKB / 8 / NT;
    constexpr int B_C = BN * BKB / 8 / NT;
    static_assert(A_C >= 1 && B_C >= 1, "chunks");
    constexpr int TLD = BN + 4;
    constexpr int MAIN_BYTES = 2 * (BM + BN) * LDKB * 2;
    constexpr int EPI_BYTES = BM * TLD * 4;
    constexpr int SMEM_BYTES = MAIN_BYTES > EPI_BYTES ? MAIN_BYTES : EPI_BYTES;
    __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM_BYTES];
    __shared__ __attribute__((aligned(16))) float Sg[BM * 4];
    __shared__ float Bd[BM * 3];
    uint16_t* As = reinterpret_cast<uint16_t*>(smem);
    uint16_t* Bs = As + 2 * BM * LDKB;

    const int ntn = (p.N + BN - 1) / BN;
    const int64_t lb = pg::xcd_logical_block(blockIdx.x, gridDim.x, p.remap != 0);
    const int nt = (int)(lb % ntn);
    const int64_t m0 = (lb / ntn) * BM;
    const int n0 = nt * BN;
    const bool lead = nt == 0;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int wm = wave / WN, wn = wave % WN;
    const int li = lane & 31, lh = lane >> 5;

    if (tid < BM) {
        const int64_t m = m0 + tid;
        float4 sv = make_float4(0.f, 0.f, 0.f, 1.f);
        if (m < p.M) {
            float ci, co, cd, cu, ca;
            gate_values(p.g, m, ci, co, cd, cu, ca);
            const float cad = ca * cd;
            sv.x = cad * ci;
            sv.y = cad * co;
            sv.z = ca * cu;
            if (lead) st4(p.gates + m * 4, sv);
        }
        st4(&Sg[tid * 4], sv);
    }

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    uint4 ra[A_C], ry[A_C], rb[B_C];
    float bd[A_C][3];
#pragma unroll
    for (int q = 0; q < A_C; ++q) bd[q][0] = bd[q][1] = bd[q][2] = 0.f;
    const int64_t mlast = p.M - 1;
    auto fetch = [&](int k0) {
#pragma unroll
        for (int q = 0; q < A_C; ++q) {
            const int idx = tid + NT * q;
            const int64_t m = min(m0 + (idx >> 3), mlast);
            const int k = k0 + 8 * (idx & 7);
            const int kc = k < p.F_out ? k : 0;
            ra[q] = *reinterpret_cast<const uint4*>(p.dY + m * p.lddy + kc);
            if (p.act) ry[q] = *reinterpret_cast<const uint4*>(p.Y + m * p.ldy + kc);
        }
#pragma unroll
        for (int q = 0; q < B_C; ++q) {
            const int idx = tid + NT * q;
            const int n = min(n0 + (idx >> 3), p.N - 1);
            const int k = k0 + 8 * (idx & 7);
            rb[q] = *reinterpret_cast<const uint4*>(p.BT + (int64_t)n * p.F_out + (k < p.F_out ? k : 0));
        }
    };
    auto stash = [&](int buf, int k0) {
        uint16_t* Ab = As + buf * BM * LDKB;
        uint16_t* Bb = Bs + buf * BN * LDKB;
#pragma unroll
        for (int q = 0; q < A_C; ++q) {
            const int idx = tid + NT * q;
            const int k = k0 + 8 * (idx & 7);
            const int64_t m = m0 + (idx >> 3);
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (k < p.F_out) {
                float d[8];
                unpack8(ra[q], d);
                if (p.act) {
                    float y[8];
                    unpack8(ry[q], y);
#pragma unroll
                    for (int e = 0; e < 8; ++e) d[e] = pg::act_grad(d[e], y[e], p.slope, p.drop_s);
                }
                v = pack8(d);
                if (lead && m < p.M) {
                    *reinterpret_cast<uint4*>(p.dpre + m * p.ldp + k) = v;
                    float dr[8];
                    unpack8(v, dr);  // the rounded gradient, as the products below see it
                    if (p.dpre32) {
                        st4(p.dpre32 + m * p.ldp32 + k, make_float4(dr[0], dr[1], dr[2], dr[3]));
                        st4(p.dpre32 + m * p.ldp32 + k + 4, make_float4(dr[4], dr[5], dr[6], dr[7]));
                    }
#pragma unroll
                    for (int sg = 0; sg < 3; ++sg) {
                        const float4 b0 = ld4(p.bsum + sg * p.F_out + k), b1 = ld4(p.bsum + sg * p.F_out + k + 4);
                        bd[q][sg] += dr[0] * b0.x + dr[1] * b0.y + dr[2] * b0.z + dr[3] * b0.w + dr[4] * b1.x +
                                     dr[5] * b1.y + dr[6] * b1.z + dr[7] * b1.w;
                    }
                }
            }
            *reinterpret_cast<uint4*>(&Ab[(idx >> 3) * LDKB + 8 * (idx & 7)]) = v;
        }
#pragma unroll
        for (int q = 0; q < B_C; ++q) {
            const int idx = tid + NT * q;
            const int k = k0 + 8 * (idx & 7);
            *reinterpret_cast<uint4*>(&Bb[(idx >> 3) * LDKB + 8 * (idx & 7)]) =
                k < p.F_out ? rb[q] : make_uint4(0u, 0u, 0u, 0u);
        }
    };

    const int ntiles = (p.F_out + BKB - 1) / BKB;
    fetch(0);
    stash(0, 0);
    __syncthreads();
    for (int t = 0; t < ntiles; ++t) {
        const int cur = t & 1;
        if (t + 1 < ntiles) fetch((t + 1) * BKB);
        const uint16_t* Ab = As + cur * BM * LDKB;
        const uint16_t* Bb = Bs + cur * BN * LDKB;
#pragma unroll
        for (int kk = 0; kk < BKB / 16; ++kk) {
            bf16x8 a[TM], b[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
                a[i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(
                                                      &Ab[(wm * TM * 32 + i * 32 + li) * LDKB + kk * 16 + 8 * lh]));
#pragma unroll
            for (int j = 0; j < TN; ++j)
                b[j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(
                                                      &Bb[(wn * TN * 32 + j * 32 + li) * LDKB + kk * 16 + 8 * lh]));
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        if (t + 1 < ntiles) stash(cur ^ 1, (t + 1) * BKB);
        __syncthreads();
    }

    if (lead) {
#pragma unroll
        for (int q = 0; q < A_C; ++q) {
#pragma unroll
            for (int sg = 0; sg < 3; ++sg) {
                float v = bd[q][sg];
                v += __shfl_xor(v, 1);
                v += __shfl_xor(v, 2);
                v += __shfl_xor(v, 4);
                bd[q][sg] = v;
            }
            const int idx = tid + NT * q;
            if ((idx & 7) == 0) {
                Bd[(idx >> 3) * 3 + 0] = bd[q][0];
                Bd[(idx >> 3) * 3 + 1] = bd[q][1];
                Bd[(idx >> 3) * 3 + 2] = bd[q][2];
            }
        }
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
    constexpr int BATCH = ITER < 4 ? ITER : 4;
    const int c4 = tid % C4;
    const int j = n0 + 4 * c4;
    const int seg = j < p.N ? j / p.F_in : 4;
    for (int it0 = 0; it0 < ITER; it0 += BATCH) {
        uint2 zv[BATCH];
        int rl[BATCH];
        int64_t mm[BATCH];
#pragma unroll
        for (int u = 0; u < BATCH; ++u) {
            rl[u] = (tid + NT * (it0 + u)) / C4;
            mm[u] = m0 + rl[u];
            zv[u] = make_uint2(0u, 0u);
            if (mm[u] < p.M && seg < 3) zv[u] = *reinterpret_cast<const uint2*>(p.Z + mm[u] * p.ldz + j);
        }
        float part[BATCH];  // the gate dots before the batch's stores: one wait for its Z loads, not one per item
#pragma unroll
        for (int u = 0; u < BATCH; ++u)
            part[u] = mm[u] < p.M && seg < 3 ? dot4(ld4(&T[rl[u] * TLD + 4 * c4]), unpack4(zv[u])) : 0.f;
#pragma unroll
        for (int u = 0; u < BATCH; ++u) {
            if (mm[u] < p.M && seg < 4) {
                const float4 gv = ld4(&T[rl[u] * TLD + 4 * c4]);
                if (seg < 3) {
                    const float sc = Sg[rl[u] * 4 + seg];
                    if (p.dZ)
                        *reinterpret_cast<uint2*>(p.dZ + mm[u] * p.lddz + j) =
                            pack4(make_float4(sc * gv.x, sc * gv.y, sc * gv.z, sc * gv.w));
                } else {
                    *reinterpret_cast<uint2*>(p.dres + mm[u] * p.lddres + (j - 3 * p.F_in)) = pack4(gv);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < BATCH; ++u) T[rl[u] * TLD + 4 * c4] = part[u];  // own slots
    }
    __syncthreads();
    if (tid < BM && m0 + tid < p.M) {
        const int64_t m = m0 + tid;
        float ds[3] = {0.f, 0.f, 0.f};
        if (lead) {
            ds[0] = Bd[tid * 3 + 0];
            ds[1] = Bd[tid * 3 + 1];
            ds[2] = Bd[tid * 3 + 2];
        }
        for (int c = 0; c < C4; ++c) {
            const int jj = n0 + 4 * c;
            if (jj >= p.N) break;
            const int q = jj / p.F_in;
            if (q < 3) ds[q] += T[tid * TLD + 4 * c];
        }  // (row_gate_partials spilled 16 B per lane here)
#pragma unroll
        for (int q = 0; q < 3; ++q) p.dsp[((int64_t)nt * 3 + q) * p.M + m] = ds[q];
    }
}

// Resident-A form of dgrad_bf16_kernel (round 5, the default where F_out <= 256 and F_out % 64 == 0): one 256-thread
// workgroup owns 64 rows for ALL n-tiles. dpre of its rows (the A operand, 64 x F_out bf16) is computed once into LDS
// (dgrad_bf16_kernel recomputes it from dY and Y for each of the N / 128 n-tiles), then the workgroup walks the
// n-tiles with the B k-tiles double-buffered a tile ahead (crossing n-tile boundaries) and the Z rows of each n-tile's
// epilogue loaded during its last k-tile. Same products in the same order, same per-thread bias-dot order, same
// epilogue: every output is bit-identical to dgrad_bf16_kernel's (PG_FLAG_DGRAD_BF16_TILED keeps that kernel).
// diagnostics build only (-DPG_DGRAD_EXP=mask, tools/r06_dgrad_exp.sh): phases of dgrad_bf16r_kernel skipped
#ifndef PG_DGRAD_EXP
#define PG_DGRAD_EXP 0
#endif
#define GXP(bit) ((PG_DGRAD_EXP >> (bit)) & 1)
// non-temporal forms of the resident dgrad's once-touched streams (PG_DGRAD_NT bits: 0 the dY / Y loads, 1 the
// epilogue's Z loads, 2 its dZ stores); A/B builds via tools/r06_ab_lib2.sh
#ifndef PG_DGRAD_NT
#define PG_DGRAD_NT 7  // all three: config 5 3.904 -> 3.875 ms (mean of 3 interleaved runs, profiles/r06_ab_train_dgrad_nt.txt)
#endif
typedef unsigned int pg_u4v __attribute__((ext_vector_type(4)));
typedef unsigned int pg_u2v __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ uint4 ld16u(const uint16_t* q) {
    if constexpr (NT) {
        const pg_u4v x = __builtin_nontemporal_load(reinterpret_cast<const pg_u4v*>(q));
        return make_uint4(x.x, x.y, x.z, x.w);
    }
    return *reinterpret_cast<const uint4*>(q);
}
template <bool NT>
__device__ __forceinline__ uint2 ld8u(const uint16_t* q) {
    if constexpr (NT) {
        const pg_u2v x = __builtin_nontemporal_load(reinterpret_cast<const pg_u2v*>(q));
        return make_uint2(x.x, x.y);
    }
    return *reinterpret_cast<const uint2*>(q);
}
template <bool NT>
__device__ __forceinline__ void st8u(uint16_t* q, uint2 v) {
    if constexpr (NT) {
        const pg_u2v x = {v.x, v.y};
        __builtin_nontemporal_store(x, reinterpret_cast<pg_u2v*>(q));
    } else {
        *reinterpret_cast<uint2*>(q) = v;
    }
}
constexpr int RB_BM = 64, RB_NW = 4, RB_FMAX = 256;
__global__ __launch_bounds__(64 * RB_NW, 2) void dgrad_bf16r_kernel(DgradB p) {
    using namespace pgbf;
    constexpr int BM = RB_BM, BN = 128, NW = RB_NW, NT = 64 * NW;
    constexpr int WN = 2, WM = NW / WN;
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    static_assert(TM == 1 && TN == 2, "wave tile");
    constexpr int LDA = RB_FMAX + 8;                 // resident A row (bf16): 528 B, conflict-free ds_read_b128
    constexpr int A_C = BM * BKB / 8 / NT;           // 16-B pieces of one A k-tile per thread (2)
    constexpr int B_C = BN * BKB / 8 / NT;           // of one B k-tile (4)
    constexpr int KT_MAX = RB_FMAX / BKB;
    constexpr int TLD = BN + 4;
    constexpr int B_BYTES = 2 * BN * LDKB * 2;
    static_assert(BM * TLD * 4 <= B_BYTES, "the epilogue tile aliases the B buffers");
    constexpr int C4 = BN / 4;
    constexpr int ITER = BM * C4 / NT;               // epilogue items per thread (8)
    __shared__ __attribute__((aligned(16))) uint16_t As[BM * LDA];
    __shared__ __attribute__((aligned(16))) unsigned char bsm[B_BYTES];
    __shared__ __attribute__((aligned(16))) float Sg[BM * 4];
    __shared__ float Bd[BM * 3];
    uint16_t* const Bs = reinterpret_cast<uint16_t*>(bsm);
    float* const T = reinterpret_cast<float*>(bsm);

    const int ntn = (p.N + BN - 1) / BN;
    const int KT = p.F_out / BKB;
    const int64_t m0 = pg::xcd_logical_block(blockIdx.x, gridDim.x, p.remap != 0) * BM;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int wm = wave / WN, wn = wave % WN;
    const int li = lane & 31, lh = lane >> 5;
    const int64_t mlast = p.M - 1;

    if (tid < BM) {
        const int64_t m = m0 + tid;
        float4 sv = make_float4(0.f, 0.f, 0.f, 1.f);
        if (m < p.M) {
            float ci, co, cd, cu, ca;
            gate_values(p.g, m, ci, co, cd, cu, ca);
            const float cad = ca * cd;
            sv.x = cad * ci;
            sv.y = cad * co;
            sv.z = ca * cu;
            st4(p.gates + m * 4, sv);
        }
        st4(&Sg[tid * 4], sv);
    }

    // B k-tile g = nt * KT + kt -> registers, two tiles ahead in two named sets (an array of registers here stays in
    // scratch memory): tile g + 1 waits in one set while tile g + 2 loads into the other
    static_assert(B_C == 4, "four B pieces per thread");
    struct B4 {
        uint4 a, b, c, d;
    };
    B4 S0, S1;
    auto loadB = [&](int g) __attribute__((always_inline)) {
        const int nt = g / KT, k0 = (g - nt * KT) * BKB;
        auto src = [&](int q) {
            const int idx = tid + NT * q;
            const int n = min(nt * BN + (idx >> 3), p.N - 1);
            return reinterpret_cast<const uint4*>(p.BT + (int64_t)n * p.F_out + k0 + 8 * (idx & 7));
        };
        B4 r;
        if (GXP(1)) {
            r.a = r.b = r.c = r.d = make_uint4(g, tid, 0u, 0u);
            return r;
        }
        r.a = *src(0);
        r.b = *src(1);
        r.c = *src(2);
        r.d = *src(3);
        return r;
    };
    auto stashB = [&](B4 r, int buf) __attribute__((always_inline)) {
        uint16_t* Bb = Bs + buf * BN * LDKB;
        auto dst = [&](int q) {
            const int idx = tid + NT * q;
            return reinterpret_cast<uint4*>(&Bb[(idx >> 3) * LDKB + 8 * (idx & 7)]);
        };
        *dst(0) = r.a;
        *dst(1) = r.b;
        *dst(2) = r.c;
        *dst(3) = r.d;
    };

    // A = dpre of the 64 rows, all k-tiles' loads in flight at once; the bias dots <dpre, bsum_q> accumulate per
    // thread over the k-tiles in order, as in dgrad_bf16_kernel (thread (row, 8-column piece) = (idx >> 3, idx & 7))
    {
        uint4 ra[KT_MAX][A_C], ry[KT_MAX][A_C];
#pragma unroll
        for (int t = 0; t < KT_MAX; ++t)
#pragma unroll
            for (int q = 0; q < A_C; ++q) {
                const int idx = tid + NT * q;
                const int64_t m = min(m0 + (idx >> 3), mlast);
                const int k = (t < KT ? t : 0) * BKB + 8 * (idx & 7);
                if (GXP(5)) {
                    ra[t][q] = make_uint4(m, k, 0u, 0u);
                    ry[t][q] = ra[t][q];
                    continue;
                }
                ra[t][q] = ld16u<(PG_DGRAD_NT & 1) != 0>(p.dY + m * p.lddy + k);
                if (p.act) ry[t][q] = ld16u<(PG_DGRAD_NT & 1) != 0>(p.Y + m * p.ldy + k);
            }
        S0 = loadB(0);
        float bd[A_C][3];
#pragma unroll
        for (int q = 0; q < A_C; ++q) bd[q][0] = bd[q][1] = bd[q][2] = 0.f;
#pragma unroll
        for (int t = 0; t < KT_MAX; ++t) {
            if (t >= KT) break;
#pragma unroll
            for (int q = 0; q < A_C; ++q) {
                const int idx = tid + NT * q;
                const int k = t * BKB + 8 * (idx & 7);
                const int64_t m = m0 + (idx >> 3);
                float d[8];
                unpack8(ra[t][q], d);
                if (p.act) {
                    float y[8];
                    unpack8(ry[t][q], y);
#pragma unroll
                    for (int e = 0; e < 8; ++e) d[e] = pg::act_grad(d[e], y[e], p.slope, p.drop_s);
                }
                const uint4 v = pack8(d);
                if (m < p.M) {
                    if (!GXP(2)) *reinterpret_cast<uint4*>(p.dpre + m * p.ldp + k) = v;
                    float dr[8];
                    unpack8(v, dr);
                    if (p.dpre32 && !GXP(2)) {
                        st4(p.dpre32 + m * p.ldp32 + k, make_float4(dr[0], dr[1], dr[2], dr[3]));
                        st4(p.dpre32 + m * p.ldp32 + k + 4, make_float4(dr[4], dr[5], dr[6], dr[7]));
                    }
#pragma unroll
                    for (int sg = 0; sg < 3; ++sg) {
                        const float4 b0 = ld4(p.bsum + sg * p.F_out + k), b1 = ld4(p.bsum + sg * p.F_out + k + 4);
                        bd[q][sg] += dr[0] * b0.x + dr[1] * b0.y + dr[2] * b0.z + dr[3] * b0.w + dr[4] * b1.x +
                                     dr[5] * b1.y + dr[6] * b1.z + dr[7] * b1.w;
                    }
                }
                *reinterpret_cast<uint4*>(&As[(idx >> 3) * LDA + k]) = v;
            }
        }
#pragma unroll
        for (int q = 0; q < A_C; ++q) {
#pragma unroll
            for (int sg = 0; sg < 3; ++sg) {
                float v = bd[q][sg];
                v += __shfl_xor(v, 1);
                v += __shfl_xor(v, 2);
                v += __shfl_xor(v, 4);
                bd[q][sg] = v;
            }
            const int idx = tid + NT * q;
            if ((idx & 7) == 0) {
                Bd[(idx >> 3) * 3 + 0] = bd[q][0];
                Bd[(idx >> 3) * 3 + 1] = bd[q][1];
                Bd[(idx >> 3) * 3 + 2] = bd[q][2];
            }
        }
    }
    const int G = ntn * KT;
    if (G > 1) S1 = loadB(1);
    stashB(S0, 0);
    __syncthreads();

    const int c4 = tid % C4;
    f32x16 acc[TN];
    uint2 zv[ITER];
    auto epilogue = [&](int nt) __attribute__((always_inline)) {  // the B buffers are free: T aliases them
        const int n0 = nt * BN;
        const int j = n0 + 4 * c4;
        const int seg = j < p.N ? j / p.F_in : 4;
#pragma unroll
        for (int jj = 0; jj < TN; ++jj)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int rl = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                T[rl * TLD + wn * TN * 32 + jj * 32 + li] = acc[jj][r];
            }
        __syncthreads();
        // the gate dots first: every use of the Z rows precedes this epilogue's stores, so the compiler waits for
        // the Z loads once; with a dot after each dZ store it drained the whole memory queue (vmcnt(0): the stores
        // and the next B k-tile) at every one of the 8 items. Same products and order: the same bits.
        float part[ITER];
#pragma unroll
        for (int u = 0; u < ITER; ++u) {
            const int rl = (tid + NT * u) / C4;
            const float4 gv = ld4(&T[rl * TLD + 4 * c4]);
            part[u] = m0 + rl < p.M && seg < 3 ? dot4(gv, unpack4(zv[u])) : 0.f;
        }
#pragma unroll
        for (int u = 0; u < ITER; ++u) {
            const int rl = (tid + NT * u) / C4;
            const int64_t mm = m0 + rl;
            if (mm < p.M && seg < 4) {
                const float4 gv = ld4(&T[rl * TLD + 4 * c4]);
                if (seg < 3) {
                    const float sc = Sg[rl * 4 + seg];
                    if (p.dZ && !GXP(0))
                        st8u<(PG_DGRAD_NT & 4) != 0>(p.dZ + mm * p.lddz + j,
                                                     pack4(make_float4(sc * gv.x, sc * gv.y, sc * gv.z, sc * gv.w)));
                } else if (!GXP(0)) {
                    *reinterpret_cast<uint2*>(p.dres + mm * p.lddres + (j - 3 * p.F_in)) = pack4(gv);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < ITER; ++u) T[((tid + NT * u) / C4) * TLD + 4 * c4] = part[u];  // own slots
        __syncthreads();
        if (tid < BM && m0 + tid < p.M && !GXP(7)) {
            const int64_t m = m0 + tid;
            float ds[3] = {0.f, 0.f, 0.f};
            if (nt == 0) {
                ds[0] = Bd[tid * 3 + 0];
                ds[1] = Bd[tid * 3 + 1];
                ds[2] = Bd[tid * 3 + 2];
            }
            row_gate_partials<C4>(&T[tid * TLD], n0, p.N, p.F_in, ds);
#pragma unroll
            for (int q = 0; q < 3; ++q) p.dsp[((int64_t)nt * 3 + q) * p.M + m] = ds[q];
        }
        __syncthreads();  // T is read before the next n-tile's first B k-tile overwrites it
    };
    auto acc_sink = [&](int nt) __attribute__((always_inline)) {  // diagnostics: keep the products live
        float t = 0.f;
#pragma unroll
        for (int jj = 0; jj < TN; ++jj)
#pragma unroll
            for (int r = 0; r < 16; ++r) t += acc[jj][r];
        if (t == 12345.f) p.dsp[nt] = t;
    };
    // tile g: MFMAs on buffer g & 1 (tile g, stashed); tile g + 2 loads into one register set while tile g + 1 goes
    // from the other to the other buffer -- after the epilogue when g ends an n-tile (even g: load S0, stash S1)
    auto step = [&](int g, auto odd) __attribute__((always_inline)) {  // odd: tile g + 2 loads into S1, g + 1 is in S0
        const int nt = g / KT, kt = g - nt * KT;
        if (kt == 0) {
#pragma unroll
            for (int jj = 0; jj < TN; ++jj)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[jj][r] = 0.f;
        }
        {  // unconditional (the last steps re-read tile G - 1, unused): with a load on every path the compiler's
           // wait before the stash below counts the 4 younger loads (vmcnt(4)) instead of draining everything,
           // epilogue stores included (vmcnt(0)), at every k-tile
            const int gl = g + 2 < G ? g + 2 : G - 1;
            if constexpr (decltype(odd)::value) S1 = loadB(gl);
            else S0 = loadB(gl);
        }
        if (kt == KT - 1) {  // this n-tile's Z rows for the epilogue
            const int j = nt * BN + 4 * c4;
            const bool zseg = j < p.N && j / p.F_in < 3;
#pragma unroll
            for (int u = 0; u < ITER; ++u) {
                const int64_t m = min(m0 + (tid + NT * u) / C4, mlast);
                zv[u] = zseg && !GXP(6) ? ld8u<(PG_DGRAD_NT & 2) != 0>(p.Z + m * p.ldz + j) : make_uint2(m, j);
            }
        }
        const uint16_t* Bb = Bs + (g & 1) * BN * LDKB;
#pragma unroll
        for (int kk = 0; kk < BKB / 16; ++kk) {
            const bf16x8 a = __builtin_bit_cast(
                bf16x8, *reinterpret_cast<const uint4*>(&As[(wm * 32 + li) * LDA + kt * BKB + kk * 16 + 8 * lh]));
            bf16x8 b[TN];
#pragma unroll
            for (int jj = 0; jj < TN; ++jj)
                b[jj] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(
                                                      &Bb[(wn * TN * 32 + jj * 32 + li) * LDKB + kk * 16 + 8 * lh]));
#pragma unroll
            for (int jj = 0; jj < TN; ++jj) {
                if (GXP(3)) acc[jj][kk] += (float)a[jj] * (float)b[jj][kk];
                else acc[jj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b[jj], acc[jj], 0, 0, 0);
            }
        }
        auto stash_next = [&]() __attribute__((always_inline)) {
            if constexpr (decltype(odd)::value) stashB(S0, (g + 1) & 1);
            else stashB(S1, (g + 1) & 1);
        };
        if (kt + 1 < KT) {
            stash_next();
            __syncthreads();
        } else {
            __syncthreads();
            if (!GXP(4)) epilogue(nt);
            else acc_sink(nt);
            if (g + 1 < G) {
                stash_next();
                __syncthreads();
            }
        }
    };
    for (int g = 0; g < G; g += 2) {
        step(g, std::false_type{});
        if (g + 1 < G) step(g + 1, std::true_type{});
    }
}

// pg_dense_grads_layout_f32: thread i < F_out F_in / 4 moves one float4 of every segment and writes W_shared's sum;
// the next 6 F_out threads the bias pairs
__global__ __launch_bounds__(256) void grads_layout_kernel(int F_out, int F_in, int S, const float* dB,
                                                           const float* dbsum, float* out) {
    const int64_t nw4 = (int64_t)F_out * F_in / 4, plane = (int64_t)F_out * F_in;
    const int64_t total = nw4 + 6 * (int64_t)F_out;
    const int K = S * F_in;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        if (i < nw4) {
            const int n = (int)(i / (F_in / 4)), k = 4 * (int)(i % (F_in / 4));
            const float* row = dB + (int64_t)n * K + k;
            const float4 a = ld4(row), b = ld4(row + F_in), c = ld4(row + 2 * F_in);
            const int64_t o = (int64_t)n * F_in + k;
            st4(out + o, a);
            st4(out + plane + o, b);
            st4(out + 2 * plane + o, c);
            if (S == 4) st4(out + 3 * plane + o, ld4(row + 3 * F_in));
            float4 w;
            w.x = __fadd_rn(__fadd_rn(a.x, b.x), c.x);
            w.y = __fadd_rn(__fadd_rn(a.y, b.y), c.y);
            w.z = __fadd_rn(__fadd_rn(a.z, b.z), c.z);
            w.w = __fadd_rn(__fadd_rn(a.w, b.w), c.w);
            st4(out + S * plane + o, w);
        } else {
            const int j = (int)(i - nw4);  // [2][3][F_out]
            const int q = (j / F_out) % 3, n = j % F_out;
            out[(S + 1) * plane + j] = dbsum[(int64_t)q * F_out + n];
        }
    }
}

struct WgradB {
    int64_t M;
    int P, N, F_in;
    const uint16_t* A;  // dpre [M, P] bf16
    int64_t lda;
    const uint16_t* Z;  // [M, >= 3 F_in] bf16
    int64_t ldz;
    const uint16_t* R;  // segment 3 (projected residual input) bf16, or null
    int64_t ldr;
    const float* gates; // [M, 4]
    int64_t rows_per_split;
    int64_t part_stride;
    float* part;
    int col0;           // wgrad_bf16_kernel: first output column (the projected residual's columns after the staged
                        // kernel's 3 F_in; then no bias sums here)
};

constexpr int WRB = 32;  // rows per K step (2 MFMA k-steps)
constexpr int LDM = 40;  // transposed LDS row in bf16: 32 rows + 8 pad (80 B: conflict-free ds_read_b128)

// C[P x N] = A^T diag(s) B with both operands staged TRANSPOSED in LDS (rows of the K step along the LDS
// row), so each MFMA operand (8 consecutive K = rows) is one ds_read_b128. Waves 0-3 stage A (and sum
// the bias gradients), waves 4-7 stage s*B; a thread owns a row pair x 8 columns and writes each column's
// two rows as one 32-bit LDS word.
__global__ __launch_bounds__(512, 4) void wgrad_bf16_kernel(WgradB p) {
    using namespace pgbf;
    constexpr int BI = 128, BJ = 128;
    __shared__ __attribute__((aligned(16))) uint16_t At[2][BI * LDM];
    __shared__ __attribute__((aligned(16))) uint16_t Bt[2][BJ * LDM];
    const int j0 = p.col0 + blockIdx.x * BJ, i0 = blockIdx.y * BI;
    const int64_t r0 = (int64_t)blockIdx.z * p.rows_per_split;
    const int64_t rend = min(r0 + p.rows_per_split, p.M);
    const bool do_db = blockIdx.x == 0 && p.col0 == 0;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int wi = wave >> 1, wj = wave & 1;  // wave tile 32 (i) x 64 (j)
    const int li = lane & 31, lh = lane >> 5;
    const int half = tid >> 8, lt = tid & 255;
    const int rp = lt & 15, cg = lt >> 4;
    const int col = (half ? j0 : i0) + 8 * cg;
    const bool col_ok = col < (half ? p.N : p.P);
    const int seg = (half && col_ok) ? col / p.F_in : 0;
    const uint16_t* src = half ? (seg < 3 ? p.Z + col : p.R + (col - 3 * p.F_in)) : p.A + col;
    const int64_t ld = half ? (seg < 3 ? p.ldz : p.ldr) : p.lda;
    const bool need_s = half || do_db;

    f32x16 acc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    float db[4][8];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 8; ++e) db[q][e] = 0.f;

    uint4 v0, v1;
    float4 s0 = make_float4(1.f, 1.f, 1.f, 1.f), s1 = s0;
    const int64_t mlast = p.M - 1;
    auto fetch = [&](int64_t base) {
        const int64_t ma = min(base + 2 * rp, mlast), mb = min(base + 2 * rp + 1, mlast);
        v0 = col_ok ? *reinterpret_cast<const uint4*>(src + ma * ld) : make_uint4(0u, 0u, 0u, 0u);
        v1 = col_ok ? *reinterpret_cast<const uint4*>(src + mb * ld) : make_uint4(0u, 0u, 0u, 0u);
        if (need_s && p.gates) {
            s0 = ld4(p.gates + ma * 4);
            s1 = ld4(p.gates + mb * 4);
        }
    };
    auto stash = [&](int buf, int64_t base) {
        const bool oka = col_ok && base + 2 * rp < rend, okb = col_ok && base + 2 * rp + 1 < rend;
        float fa[8], fb2[8];
        unpack8(v0, fa);
        unpack8(v1, fb2);
        uint32_t ba[8], bb[8];
        if (half) {
            const float sa = seg == 0 ? s0.x : seg == 1 ? s0.y : seg == 2 ? s0.z : 1.f;
            const float sb = seg == 0 ? s1.x : seg == 1 ? s1.y : seg == 2 ? s1.z : 1.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                ba[e] = oka ? f2bf(fa[e] * sa) : 0u;
                bb[e] = okb ? f2bf(fb2[e] * sb) : 0u;
            }
        } else {
            const uint32_t wa[4] = {v0.x, v0.y, v0.z, v0.w}, wb[4] = {v1.x, v1.y, v1.z, v1.w};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                ba[e] = oka ? ((e & 1) ? wa[e >> 1] >> 16 : wa[e >> 1] & 0xffffu) : 0u;
                bb[e] = okb ? ((e & 1) ? wb[e >> 1] >> 16 : wb[e >> 1] & 0xffffu) : 0u;
            }
            if (do_db) {
                const float sa[4] = {s0.x, s0.y, s0.z, 1.f}, sb[4] = {s1.x, s1.y, s1.z, 1.f};
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int e = 0; e < 8; ++e)
                        db[q][e] += (oka ? sa[q] * fa[e] : 0.f) + (okb ? sb[q] * fb2[e] : 0.f);
            }
        }
        uint16_t* T = half ? Bt[buf] : At[buf];
#pragma unroll
        for (int e = 0; e < 8; ++e)
            *reinterpret_cast<uint32_t*>(&T[(8 * cg + e) * LDM + 2 * rp]) = ba[e] | (bb[e] << 16);
    };

    const int64_t nsteps = (rend - r0 + WRB - 1) / WRB;
    if (nsteps > 0) {
        fetch(r0);
        stash(0, r0);
    }
    __syncthreads();
    for (int64_t t = 0; t < nsteps; ++t) {
        const int cur = (int)(t & 1);
        const int64_t nb = r0 + (t + 1) * WRB;
        if (t + 1 < nsteps) fetch(nb);
#pragma unroll
        for (int ks = 0; ks < WRB / 16; ++ks) {
            const bf16x8 a = __builtin_bit_cast(
                bf16x8, *reinterpret_cast<const uint4*>(&At[cur][(wi * 32 + li) * LDM + ks * 16 + 8 * lh]));
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const bf16x8 b = __builtin_bit_cast(
                    bf16x8, *reinterpret_cast<const uint4*>(&Bt[cur][(wj * 64 + j * 32 + li) * LDM + ks * 16 + 8 * lh]));
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[j], 0, 0, 0);
            }
        }
        if (t + 1 < nsteps) stash(cur ^ 1, nb);
        __syncthreads();
    }

    float* out = p.part + (int64_t)blockIdx.z * p.part_stride;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int oi = i0 + wi * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
            const int oj = j0 + wj * 64 + j * 32 + li;
            if (oi < p.P && oj < p.N) out[(int64_t)oi * p.N + oj] = acc[j][r];
        }
    if (do_db && !half) {  // sum the 16 row pairs of each column group (16 consecutive lanes)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                float v = db[q][e];
                v += __shfl_xor(v, 1, 16);
                v += __shfl_xor(v, 2, 16);
                v += __shfl_xor(v, 4, 16);
                v += __shfl_xor(v, 8, 16);
                db[q][e] = v;
            }
        if (rp == 0 && col_ok) {
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int e = 0; e < 8; ++e)
                    if (col + e < p.P) out[(int64_t)p.P * p.N + q * p.P + col + e] = db[q][e];
        }
    }
}

__global__ __launch_bounds__(256) void transpose_u16_kernel(int R, int C, const uint16_t* in, uint16_t* out) {
    const int64_t total = (int64_t)R * C;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int c = (int)(i / R), r = (int)(i % R);
        out[i] = in[(int64_t)r * C + c];
    }
}

constexpr int DG_BM = 128, DG_BN = 128, DG_NW = 8, WG_NW = 8;
constexpr int X3_BM = 64, X3_NW = 4;  // dgrad_x3_kernel: 64-row blocks of 4 waves, three workgroups per CU

struct BwdPlan {
    int K, ntn, splits;
    int64_t rows_per_split, part_stride;
    int64_t off_bt, off_dsp, off_part, total;
};

struct SplitPlan {
    int splits;
    int64_t rows_per_split;
};

// Row splits for wgrad_kernel: about 512 blocks (2 per CU), whole 32-row chunks per split.
SplitPlan split_rows(int64_t M, int64_t tiles) {
    SplitPlan sp{};
    int64_t splits = (512 + tiles - 1) / tiles;
    const int64_t chunks = (M + WROWS - 1) / WROWS;
    if (splits > chunks) splits = chunks;
    if (splits < 1) splits = 1;
    sp.rows_per_split = ((chunks + splits - 1) / splits) * WROWS;
    if (sp.rows_per_split < WROWS) sp.rows_per_split = WROWS;
    sp.splits = (int)((M + sp.rows_per_split - 1) / sp.rows_per_split);
    if (sp.splits < 1) sp.splits = 1;
    return sp;
}

// Staged bf16 weight gradient (round 5; the bf16 mode's default where F_in, F_out % 128 == 0, no projected residual):
// wgrad_x3_kernel's structure on bf16 operands, one product per pair instead of six. One 512-thread workgroup per
// (row split, 128 x 384 output tile), one per CU; every 32-row step is staged once for the whole tile (A = dpre,
// B = bf16(s_q Z_q) rounded as wgrad_bf16_kernel rounds it, 8 rows x 4 columns per thread) through buffer descriptors
// two steps ahead, repacked into [k-group][column] units of 8 rows, double-buffered; wave w owns output rows
// 64 (w & 1).. and columns 96 (w >> 1)... The workgroups of one row split (its 128 x 384 tiles) are numbered onto
// one XCD at neighbouring times (blockIdx -> (split, tile), see wgrad_tile_of), so the tiles that read the same rows
// share them through that XCD's L2. wgrad_bf16_kernel (128 x 128 tiles, one step of prefetch) re-read dpre once per
// 128-column tile: 984 MB at F = 256 against the 656 MB here.
constexpr int WB_K = 32;  // rows per step (4 k-groups of 8)

__global__ __launch_bounds__(512, 1) void wgrad_bfs_kernel(WgradB p, int splits) {
    __shared__ __attribute__((aligned(16))) uint4 U[2][4][WX_COLS];
    __shared__ float Db[4][4][WX_BP];
    __shared__ float Gs[2][3][WB_K];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, li = lane & 31, kh = lane >> 5;
    const int n_tiles = p.N / WX_BN;
    int split, tile;
    wgrad_tile_of((int)blockIdx.x, (p.P / WX_BP) * n_tiles, splits, split, tile);
    if (tile < 0) return;  // whole workgroup: no barrier reached
    const int pt = tile / n_tiles, nt = tile % n_tiles;
    const int64_t r0 = (int64_t)split * p.rows_per_split;
    const int64_t rend = min(r0 + p.rows_per_split, p.M);
    // staging role: waves 0-1 stage A (128 columns: 32 quads x 4 k-groups), waves 2-7 B (384 columns: 96 x 4); the
    // wave index in a scalar register keeps the buffer descriptors wave-uniform
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const bool isA = wv < 2;
    const int u = isA ? tid : tid - 128;
    const int kg = isA ? (u >> 5) : (u / 96);
    const int quad = isA ? (u & 31) : (u % 96);
    const int col0 = (isA ? 0 : WX_BP) + 4 * quad;
    const int gcol = isA ? WX_BP * pt + 4 * quad : WX_BN * nt + 4 * quad;
    const int seg = isA ? 3 : gcol / p.F_in;
    const uint16_t* src = isA ? p.A + WX_BP * pt : p.Z + WX_BN * nt;
    const int64_t ld = isA ? p.lda : p.ldz;
    const int gsel = seg < 3 ? seg : 0;
    const bool gwriter = !isA && gcol % p.F_in == 0;
    const int64_t nr64 = rend - r0;
    const int nrows = __builtin_amdgcn_readfirstlane(nr64 > 0 ? (int)nr64 : 0);
    const auto rs_x = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(src + r0 * ld), 0, nrows * (int)ld * 2,
                                                        0x00020000);
    const auto rs_g = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.gates + r0 * 4), 0, nrows * 16, 0x00020000);
    const int ld2b = (int)ld * 2;
    const int xoff = 8 * kg * ld2b + 8 * quad, goff = (8 * kg * 4 + gsel) * 4;
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    auto load = [&](uint2 (&x)[8], float (&gq)[8], int step) {  // step < 2^31 / (32 ld) (host-checked)
        const int sx = step * WB_K * ld2b, sg = step * WB_K * 16;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs_x, xoff + sx + e * ld2b, 0, 0);
            x[e] = make_uint2(v.x, v.y);
            gq[e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_g, goff + sg + e * 16, 0, 0));
        }
    };
    float db[4][4];
#pragma unroll
    for (int t = 0; t < 4; ++t) db[t][0] = db[t][1] = db[t][2] = db[t][3] = 0.f;
    uint2 xa[8];  // A threads: the staged rows, kept for the bias sums after the barrier
    auto pack_store = [&](const uint2 (&x)[8], const float (&gq)[8], int buf) {
        uint32_t w[4][4];  // [column][row pair]
        if (isA) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint2 r0v = x[2 * i], r1v = x[2 * i + 1];
                w[0][i] = (r0v.x & 0xffffu) | (r1v.x << 16);
                w[1][i] = (r0v.x >> 16) | (r1v.x & 0xffff0000u);
                w[2][i] = (r0v.y & 0xffffu) | (r1v.y << 16);
                w[3][i] = (r0v.y >> 16) | (r1v.y & 0xffff0000u);
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) xa[e] = x[e];
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float f[2][4];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const uint2 v = x[2 * i + h];
                    const float s = gq[2 * i + h];
                    f[h][0] = __fmul_rn(pgbf::lo(v.x), s);
                    f[h][1] = __fmul_rn(pgbf::hi(v.x), s);
                    f[h][2] = __fmul_rn(pgbf::lo(v.y), s);
                    f[h][3] = __fmul_rn(pgbf::hi(v.y), s);
                }
                float d0, d1;
#pragma unroll
                for (int c = 0; c < 4; ++c) w[c][i] = pgx3::bf2(f[0][c], f[1][c], d0, d1);  // RNE, as f2bf
            }
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) U[buf][kg][col0 + c] = make_uint4(w[c][0], w[c][1], w[c][2], w[c][3]);
        if (gwriter) {
#pragma unroll
            for (int e = 0; e < 8; ++e) Gs[buf][seg][8 * kg + e] = gq[e];
        }
    };
    auto bias_step = [&](int cur) {  // A threads, after the barrier: the step's rows in order
        if (!isA) return;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int row = 8 * kg + e;
            const float sv[4] = {Gs[cur][0][row], Gs[cur][1][row], Gs[cur][2][row], 1.f};
            const float f[4] = {pgbf::lo(xa[e].x), pgbf::hi(xa[e].x), pgbf::lo(xa[e].y), pgbf::hi(xa[e].y)};
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int c = 0; c < 4; ++c) db[t][c] += sv[t] * f[c];
        }
    };
    if (tid < 2 * 3 * WB_K) (&Gs[0][0][0])[tid] = 0.f;
    f32x16 acc[2][3];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int ih = wave & 1, jq = wave >> 1;
    auto mfma_step = [&](int cur) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {  // k-groups 2 ks + kh
            const int g = 2 * ks + kh;
            uint4 a[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) a[i] = U[cur][g][64 * ih + 32 * i + li];
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const uint4 b = U[cur][g][WX_BP + 96 * jq + 32 * j + li];
#pragma unroll
                for (int i = 0; i < 2; ++i) acc[i][j] = mfma32_bf(a[i], b, acc[i][j]);
            }
        }
    };
    uint2 x0[8], x1[8];
    float g0[8], g1[8];
    const int64_t nsteps = (rend - r0 + WB_K - 1) / WB_K;
    __syncthreads();  // Gs zeroed
    // loads and packs unconditional (past the last step: zero rows), as in wgrad_x3_kernel
    load(x0, g0, 0);
    load(x1, g1, 1);
    pack_store(x0, g0, 0);
    __syncthreads();
    for (int t = 0; t < (int)nsteps; t += 2) {
        bias_step(0);
        load(x0, g0, t + 2);
        mfma_step(0);
        pack_store(x1, g1, 1);
        __syncthreads();
        bias_step(1);
        load(x1, g1, t + 3);
        if (t + 1 < nsteps) mfma_step(1);
        pack_store(x0, g0, 0);
        __syncthreads();
    }
    float* out = p.part + (int64_t)split * p.part_stride;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int oi = WX_BP * pt + 64 * ih + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * kh;
                const int oj = WX_BN * nt + 96 * jq + 32 * j + li;
                out[(int64_t)oi * p.N + oj] = acc[i][j][r];
            }
    if (isA) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int c = 0; c < 4; ++c) Db[kg][t][4 * quad + c] = db[t][c];
    }
    __syncthreads();
    {
        const int t = tid >> 7, c = tid & 127;  // 4 x 128 sums, k-groups in fixed order
        const int first = t * p.F_in;
        const bool mine = t == 3 ? nt == 0 : (first >= WX_BN * nt && first < WX_BN * (nt + 1));
        if (mine) out[(int64_t)p.P * p.N + t * p.P + WX_BP * pt + c] = ((Db[0][t][c] + Db[1][t][c]) + Db[2][t][c]) + Db[3][t][c];
    }
}

// ------------------------------------------------------------------------------------------------
// Any-shape path (F_in / F_out not multiples of 4, unaligned or odd leading dimensions): the same outputs as
// dgrad_kernel + wgrad_kernel from plain per-element loops. Sums run in another order (within fp32 rounding of
// the vector path); these shapes are off the model's hot path.
// ------------------------------------------------------------------------------------------------
constexpr int GEN_MAX_FOUT = 8192;  // dpre row staged in LDS

// one 256-thread block per row (grid-stride): dpre, gates, dZ / dres, and ds_q into dsp tile 0
__global__ __launch_bounds__(256) void dgrad_generic_kernel(DgradP p) {
    __shared__ float dp[GEN_MAX_FOUT];
    __shared__ float red[3][256];
    const int tid = threadIdx.x;
    for (int64_t m = blockIdx.x; m < p.M; m += gridDim.x) {
        float ci, co, cd, cu, ca;
        gate_values(p.g, m, ci, co, cd, cu, ca);
        const float cad = ca * cd;
        const float s[3] = {cad * ci, cad * co, ca * cu};
        if (tid == 0) {
            p.gates[m * 4 + 0] = s[0];
            p.gates[m * 4 + 1] = s[1];
            p.gates[m * 4 + 2] = s[2];
            p.gates[m * 4 + 3] = 1.f;
        }
        float ds[3] = {0.f, 0.f, 0.f};
        for (int o = tid; o < p.F_out; o += 256) {
            float d = p.dY[m * p.lddy + o];
            if (p.act) d = pg::act_grad(d, p.Y[m * p.ldy + o], p.slope, p.drop_s);
            dp[o] = d;
            p.dpre[m * p.ldp + o] = d;
#pragma unroll
            for (int q = 0; q < 3; ++q) ds[q] += d * p.bsum[q * p.F_out + o];
        }
        __syncthreads();
        for (int j = tid; j < p.N; j += 256) {
            const float* bt = p.BT + (int64_t)j * p.F_out;
            float G = 0.f;
            for (int o = 0; o < p.F_out; ++o) G += dp[o] * bt[o];
            const int seg = j / p.F_in;
            if (seg < 3) {
                ds[seg] += G * p.Z[m * p.ldz + j];
                if (p.dZ) p.dZ[m * p.lddz + j] = s[seg] * G;
            } else {
                p.dres[m * p.lddres + (j - 3 * p.F_in)] = G;
            }
        }
#pragma unroll
        for (int q = 0; q < 3; ++q) red[q][tid] = ds[q];
        __syncthreads();
        for (int w = 128; w > 0; w >>= 1) {
            if (tid < w)
#pragma unroll
                for (int q = 0; q < 3; ++q) red[q][tid] += red[q][tid + w];
            __syncthreads();
        }
        if (tid < 3) p.dsp[(int64_t)tid * p.M + m] = red[tid][0];
        __syncthreads();  // dp / red are reused by the next row
    }
}

// partial [split][F_out * K + 4 F_out]: dB[o][j] = sum_m s_seg(j)[m] dpre[m][o] A[m][j] (A = Z, or res_x in
// segment 3 with s = 1), dbsum[q][o] = sum_m s_q[m] dpre[m][o] (q = 3: the projected residual's bias, else 0)
struct WgradGenP {
    int64_t M;
    int F_in, F_out, K, proj;
    const float *dpre, *Z, *R, *gates;
    int64_t ldp, ldz, ldr;
    int64_t rows_per_split, part_stride;
    float* part;
};

__global__ __launch_bounds__(256) void wgrad_generic_kernel(WgradGenP w) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t n = (int64_t)w.F_out * (w.K + 4);
    if (idx >= n) return;
    const int64_t m0 = (int64_t)blockIdx.y * w.rows_per_split;
    const int64_t m1 = m0 + w.rows_per_split < w.M ? m0 + w.rows_per_split : w.M;
    float acc = 0.f;
    int64_t out;
    if (idx < (int64_t)w.F_out * w.K) {  // dB[o][j], j fastest
        const int o = (int)(idx / w.K), j = (int)(idx % w.K);
        const int seg = j / w.F_in;
        for (int64_t m = m0; m < m1; ++m) {
            const float a = seg < 3 ? w.Z[m * w.ldz + j] : w.R[m * w.ldr + (j - 3 * w.F_in)];
            const float sv = seg < 3 ? w.gates[m * 4 + seg] : 1.f;
            acc += sv * w.dpre[m * w.ldp + o] * a;
        }
        out = idx;
    } else {
        const int64_t t = idx - (int64_t)w.F_out * w.K;
        const int q = (int)(t / w.F_out), o = (int)(t % w.F_out);
        if (q < 3 || w.proj)
            for (int64_t m = m0; m < m1; ++m) acc += (q < 3 ? w.gates[m * 4 + q] : 1.f) * w.dpre[m * w.ldp + o];
        out = (int64_t)w.F_out * w.K + (int64_t)q * w.F_out + o;
    }
    w.part[(int64_t)blockIdx.y * w.part_stride + out] = acc;
}

__global__ __launch_bounds__(256) void reduce_generic_kernel(int64_t n, int splits, int64_t stride, const float* part,
                                                             float* out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float acc = 0.f;
    for (int k = 0; k < splits; ++k) acc += part[(int64_t)k * stride + i];
    out[i] = acc;
}

int64_t up4(int64_t v) { return (v + 3) / 4 * 4; }

// the split-bf16 weight gradient (wgrad_x3_kernel: 128 x 384 output tiles) takes these shapes
bool wgrad_x3_shape(int64_t F_in, int64_t F_out, bool proj) {
    return F_in % (WX_BN / 3) == 0 && F_out % WX_BP == 0 && !proj;
}

// x3w: the row splits of wgrad_x3_kernel (one 512-thread workgroup per CU over all output tiles, 16-row steps)
// instead of wgrad_kernel's (512 workgroups of 128 x 128 tiles, 32-row steps); the workspace covers both
BwdPlan plan_of(int64_t M, int64_t F_in, int64_t F_out, bool proj, bool x3w = false) {
    BwdPlan b{};
    b.K = (int)((proj ? 4 : 3) * F_in);
    b.ntn = (b.K + DG_BN - 1) / DG_BN;
    if (x3w) {
        const int64_t tiles = (F_out / WX_BP) * (std::min<int64_t>(b.K, 3 * F_in) / WX_BN);
        const int64_t steps = std::max<int64_t>((M + WX_K - 1) / WX_K, 1);
        const int64_t splits = std::min<int64_t>(std::max<int64_t>((256 + tiles - 1) / tiles, 1), steps);
        b.rows_per_split = ((steps + splits - 1) / splits) * WX_K;
        b.splits = (int)std::max<int64_t>((M + b.rows_per_split - 1) / b.rows_per_split, 1);
    } else {
        const SplitPlan sp = split_rows(M, ((F_out + 127) / 128) * ((b.K + 127) / 128));
        b.splits = sp.splits;
        b.rows_per_split = sp.rows_per_split;
    }
    b.part_stride = up4(F_out * b.K + 4 * F_out);
    b.off_bt = 0;  // BT (fp32), or BT3 (three bf16 splits, dgrad_x3_kernel), or the bf16 BT
    b.off_dsp = up4(2 * (int64_t)b.K * F_out);
    b.off_part = b.off_dsp + up4((int64_t)b.ntn * 3 * M);
    b.total = b.off_part + (int64_t)b.splits * b.part_stride;
    // (the bf16 backward stages the gated segments even with a projected residual)
    if (!x3w && wgrad_x3_shape(F_in, F_out, false)) b.total = std::max(b.total, plan_of(M, F_in, F_out, proj, true).total);
    return b;
}

}  // namespace

extern "C" {

int64_t pg_directgcn_dense_bwd_workspace(const pg_layer_args_t* a) {
    if (!a || a->M < 0 || a->F_in <= 0 || a->F_out <= 0) return -1;
    return plan_of(a->M, a->F_in, a->F_out, a->W_res != nullptr).total;
}

}  // extern "C"

namespace {
// the fp32 backward; span != nullptr: pg_directgcn_dense_bwd_span_f32 (dgrad_span_kernel, E = diagonal term of the
// transposed propagation (+ residual), PG_ERR_UNSUPPORTED unless its shape conditions hold)
int dense_bwd_f32_impl(const pg_layer_args_t* a, const float* packed, const pg_layer_grad_args_t* g, uint32_t flags,
                       void* stream, const SpanP* span) {
    PG_REQUIRE(a != nullptr && packed != nullptr && g != nullptr, "null args");
    PG_REQUIRE(a->M >= 0 && a->F_in > 0 && a->F_out > 0 && a->F_in < (1 << 20) && a->F_out < (1 << 20),
               "bad shape M=%lld F_in=%lld F_out=%lld", (long long)a->M, (long long)a->F_in, (long long)a->F_out);
    PG_REQUIRE(a->C_in && a->C_out && a->C_directed && a->C_undirected && a->C_all, "null gate");
    PG_REQUIRE(a->gate_mode == PG_GATES_VECTOR || a->gate_mode == PG_GATES_SCALAR, "bad gate_mode");
    PG_REQUIRE(!a->W_res || a->res_x, "W_res needs res_x");
    PG_REQUIRE(g->dY && g->dpre && g->dgate && g->gates && g->dW && g->work, "null gradient buffer");
    PG_REQUIRE(!a->act || a->Y, "act needs the forward output Y");
    PG_REQUIRE(!a->W_res || g->dres, "W_res needs dres");
    uint32_t drop_thr = 0;
    float drop_s = 0.f;
    if (const int rc = pg::drop_params(a, drop_thr, drop_s, false)) return rc;
    const bool proj = a->W_res != nullptr;
    const bool x3w = wgrad_x3_shape(a->F_in, a->F_out, proj) && !(flags & PG_FLAG_WGRAD_F32MFMA);
    const BwdPlan pl = plan_of(a->M, a->F_in, a->F_out, proj, x3w);
    PG_REQUIRE(g->work_floats >= pl.total, "workspace too small: %lld < %lld floats", (long long)g->work_floats,
               (long long)pl.total);
    // vector paths only: every row / column block is float4
    const bool vec = a->F_in % 4 == 0 && a->F_out % 4 == 0 && a->ldz % 4 == 0 && g->lddy % 4 == 0 &&
                     g->ldp % 4 == 0 && (!a->act || a->ldy % 4 == 0) &&
                     (!proj || (a->ld_res % 4 == 0 && g->lddres % 4 == 0 && pg::aligned16(a->res_x) &&
                                pg::aligned16(g->dres))) &&
                     pg::aligned16(a->Z) && pg::aligned16(g->dY) && pg::aligned16(g->dpre) && (!g->dZ || (pg::aligned16(g->dZ) && g->lddz % 4 == 0)) &&
                     pg::aligned16(g->gates) && pg::aligned16(g->dW) && pg::aligned16(g->work) &&
                     pg::aligned16(packed) && (!a->act || pg::aligned16(a->Y));
    PG_REQUIRE(a->ldz >= 3 * a->F_in && (!g->dZ || g->lddz >= 3 * a->F_in) && g->lddy >= a->F_out && g->ldp >= a->F_out,
               "leading dimensions too small");
    PG_REQUIRE(vec || a->F_out <= GEN_MAX_FOUT, "F_out %lld > %d on the any-shape path", (long long)a->F_out,
               GEN_MAX_FOUT);
    hipStream_t s = (hipStream_t)stream;
    const int K = pl.K;
    const int F_in = (int)a->F_in, F_out = (int)a->F_out;
    float* work = g->work;
    float* BT = work + pl.off_bt;
    float* dsp = work + pl.off_dsp;
    float* part = work + pl.off_part;
    if (a->M == 0) {  // no rows: all parameter gradients are zero
        if (hipMemsetAsync(g->dW, 0, sizeof(float) * ((int64_t)F_out * K + 4 * F_out), s) != hipSuccess)
            return pg::set_error(PG_ERR_HIP, "pg_directgcn_dense_bwd_f32: memset failed");
        return PG_OK;
    }
    // the split-bf16 dgrad where the k-tiles are whole (F_out % 32 == 0); PG_FLAG_DGRAD_F32MFMA keeps the fp32 MFMAs
    const bool x3 = vec && a->F_out % XBK == 0 && (span || !(flags & PG_FLAG_DGRAD_F32MFMA));
    if (span) {
        const bool ok = x3 && !proj && a->F_in % 64 == 0 && a->rows == nullptr && g->dZ != nullptr &&
                        (!span->e_res || a->F_in == a->F_out) && pg::aligned16(span->E) && span->lde % 4 == 0;
        if (!ok)
            return pg::set_error(PG_ERR_UNSUPPORTED, "pg_directgcn_dense_bwd_span_f32: needs F_in %% 64 == 0, "
                                 "F_out %% 32 == 0, no projected residual, no row map, dZ, aligned buffers and "
                                 "F_in == F_out with e_res");
    }
    uint16_t* BT3 = reinterpret_cast<uint16_t*>(BT);
    {
        const int64_t total = (int64_t)K * F_out;
        const int nb = (int)std::min<int64_t>((total + 255) / 256, 1024);
        if (x3) hipLaunchKernelGGL(transpose_split3_kernel, dim3(nb), dim3(256), 0, s, F_out, K, packed, BT3);
        else hipLaunchKernelGGL(transpose_kernel, dim3(nb), dim3(256), 0, s, F_out, K, packed, BT);
    }
    Gates gt{a->gate_mode, a->C_in, a->C_out, a->C_directed, a->C_undirected, a->C_all, a->rows};
    if (!vec) {  // any shape: per-element kernels (same outputs, sums in another order)
        DgradP p{};
        p.M = a->M;
        p.F_in = F_in;
        p.F_out = F_out;
        p.N = K;
        p.dY = g->dY;
        p.lddy = g->lddy;
        p.Y = a->Y;
        p.ldy = a->ldy;
        p.act = a->act;
        p.slope = a->slope;
        p.drop_s = drop_s;
        p.BT = BT;
        p.bsum = packed + (int64_t)F_out * K;
        p.Z = a->Z;
        p.ldz = a->ldz;
        p.g = gt;
        p.dpre = g->dpre;
        p.ldp = g->ldp;
        p.dZ = g->dZ;
        p.lddz = g->lddz;
        p.dres = g->dres;
        p.lddres = g->lddres;
        p.gates = g->gates;
        p.dsp = dsp;
        const unsigned nb = (unsigned)std::min<int64_t>(a->M, 8192);
        hipLaunchKernelGGL(dgrad_generic_kernel, dim3(nb), dim3(256), 0, s, p);
        const int gb = (int)std::min<int64_t>((a->M + 255) / 256, 2048);
        hipLaunchKernelGGL(gate_grad_kernel, dim3(gb), dim3(256), 0, s, a->M, 1, (const float*)dsp, gt, g->dgate);
        WgradGenP w{};
        w.M = a->M;
        w.F_in = F_in;
        w.F_out = F_out;
        w.K = K;
        w.proj = proj ? 1 : 0;
        w.dpre = g->dpre;
        w.ldp = g->ldp;
        w.Z = a->Z;
        w.ldz = a->ldz;
        w.R = a->res_x;
        w.ldr = a->ld_res;
        w.gates = g->gates;
        w.rows_per_split = pl.rows_per_split;
        w.part_stride = pl.part_stride;
        w.part = part;
        const int64_t n = (int64_t)F_out * (K + 4);
        hipLaunchKernelGGL(wgrad_generic_kernel, dim3((unsigned)((n + 255) / 256), (unsigned)pl.splits), dim3(256), 0, s,
                           w);
        hipLaunchKernelGGL(reduce_generic_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, pl.splits,
                           pl.part_stride, (const float*)part, g->dW);
        return pg::check_launch("pg_directgcn_dense_bwd_f32");
    }
    {
        DgradP p{};
        p.M = a->M;
        p.F_in = F_in;
        p.F_out = F_out;
        p.N = K;
        p.dY = g->dY;
        p.lddy = g->lddy;
        p.Y = a->Y;
        p.ldy = a->ldy;
        p.act = a->act;
        p.slope = a->slope;
        p.drop_s = drop_s;
        p.BT = BT;
        p.bsum = packed + (int64_t)F_out * K;
        p.Z = a->Z;
        p.ldz = a->ldz;
        p.g = gt;
        p.dpre = g->dpre;
        p.ldp = g->ldp;
        p.dZ = g->dZ;
        p.lddz = g->lddz;
        p.dres = g->dres;
        p.lddres = g->lddres;
        p.gates = g->gates;
        p.dsp = dsp;
        p.remap = (flags & PG_FLAG_NO_XCD_REMAP) ? 0 : 1;
        const int64_t nb = ((a->M + DG_BM - 1) / DG_BM) * pl.ntn;
        if (span)
            hipLaunchKernelGGL((dgrad_span_kernel<X3_BM, X3_NW>),
                               dim3((unsigned)(((a->M + X3_BM - 1) / X3_BM) * (a->F_in / 64))), dim3(64 * X3_NW), 0, s,
                               p, (const uint16_t*)BT3, *span);
        else if (x3)
            hipLaunchKernelGGL((dgrad_x3_kernel<X3_BM, DG_BN, X3_NW>), dim3((unsigned)(((a->M + X3_BM - 1) / X3_BM) * pl.ntn)),
                               dim3(64 * X3_NW), 0, s, p, (const uint16_t*)BT3);
        else hipLaunchKernelGGL((dgrad_kernel<DG_BM, DG_BN, DG_NW>), dim3((unsigned)nb), dim3(64 * DG_NW), 0, s, p);
    }
    {
        const int nb = (int)std::min<int64_t>((a->M + 255) / 256, 2048);
        hipLaunchKernelGGL(gate_grad_kernel, dim3(nb), dim3(256), 0, s, a->M, span ? (int)(a->F_in / 64) : pl.ntn,
                           (const float*)dsp, gt, g->dgate);
    }
    {
        WgradP w{};
        w.M = a->M;
        w.P = F_out;
        w.N = K;
        w.F_in = F_in;
        w.A = g->dpre;
        w.lda = g->ldp;
        w.Z = a->Z;
        w.ldz = a->ldz;
        w.R = a->res_x;
        w.ldr = a->ld_res;
        w.gates = g->gates;
        w.rows_per_split = pl.rows_per_split;
        w.part_stride = pl.part_stride;
        w.part = part;
        if (x3w) {
            const int tiles = (F_out / WX_BP) * (K / WX_BN);
            hipLaunchKernelGGL(wgrad_x3_kernel, dim3((unsigned)(8 * ((pl.splits + 7) / 8) * tiles)), dim3(512), 0, s, w,
                               (int)pl.splits);
        } else {
            dim3 grid((unsigned)((K + 127) / 128), (unsigned)((F_out + 127) / 128), (unsigned)pl.splits);
            hipLaunchKernelGGL((wgrad_kernel<WG_NW>), grid, dim3(64 * WG_NW), 0, s, w);
        }
    }
    // F_out % 4 == 0, so part_stride == F_out*K + 4*F_out == the dW buffer
    launch_reduce(pl.part_stride / 4, pl.splits, pl.part_stride, part, g->dW, s);
    return pg::check_launch(span ? "pg_directgcn_dense_bwd_span_f32" : "pg_directgcn_dense_bwd_f32");
}
}  // namespace

extern "C" {

int pg_directgcn_dense_bwd_f32(const pg_layer_args_t* a, const float* packed, const pg_layer_grad_args_t* g,
                               uint32_t flags, void* stream) {
    return dense_bwd_f32_impl(a, packed, g, flags, stream, nullptr);
}

int pg_directgcn_dense_bwd_span_f32(const pg_layer_args_t* a, const float* packed, const pg_layer_grad_args_t* g,
                                    const float* wdiag, float* E, int64_t lde, int e_res, uint32_t flags,
                                    void* stream) {
    PG_REQUIRE(wdiag != nullptr && E != nullptr && a != nullptr && g != nullptr, "null args");
    PG_REQUIRE(lde >= a->F_in, "lde too small");
    const SpanP sp{wdiag, E, lde, e_res ? 1 : 0};
    return dense_bwd_f32_impl(a, packed, g, flags, stream, &sp);
}

int64_t pg_gemm_at_b_workspace(int64_t M, int64_t P, int64_t N) {
    if (M < 0 || P <= 0 || N <= 0) return -1;
    const SplitPlan sp = split_rows(M, ((P + 127) / 128) * ((N + 127) / 128));
    return (int64_t)sp.splits * up4(P * N + 4 * P);
}

int pg_dense_grads_layout_f32(int64_t F_out, int64_t F_in, int32_t S, const float* dB, const float* dbsum, float* out,
                              void* stream) {
    PG_REQUIRE(F_out > 0 && F_in > 0 && F_out < (1 << 20) && F_in < (1 << 20) && (S == 3 || S == 4), "bad shape");
    PG_REQUIRE(dB && dbsum && out, "null pointer");
    if (F_in % 4 || !pg::aligned16(dB) || !pg::aligned16(out))
        return pg::set_error(PG_ERR_UNSUPPORTED, "pg_dense_grads_layout_f32: needs F_in %% 4 == 0 and aligned buffers");
    const int64_t n4 = F_out * F_in / 4 + 6 * F_out;
    const int nb = (int)std::min<int64_t>((n4 + 255) / 256, 2048);
    hipLaunchKernelGGL(grads_layout_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, (int)F_out, (int)F_in, (int)S,
                       dB, dbsum, out);
    return pg::check_launch("pg_dense_grads_layout_f32");
}

int pg_gemm_at_b_f32(int64_t M, int64_t P, int64_t N, const float* A, int64_t lda, const float* B, int64_t ldb,
                     float* out, float* work, int64_t work_floats, void* stream) {
    PG_REQUIRE(M >= 0 && P > 0 && N > 0 && P < (1 << 20) && N < (1 << 20), "bad shape M=%lld P=%lld N=%lld",
               (long long)M, (long long)P, (long long)N);
    PG_REQUIRE(out != nullptr && (M == 0 || (A && B && work)), "null buffer");
    PG_REQUIRE(lda >= P && ldb >= N, "leading dimensions too small");
    hipStream_t s = (hipStream_t)stream;
    if (M == 0) {
        if (hipMemsetAsync(out, 0, sizeof(float) * (P * N + P), s) != hipSuccess)
            return pg::set_error(PG_ERR_HIP, "pg_gemm_at_b_f32: memset failed");
        return PG_OK;
    }
    if (P % 4 || N % 4 || lda % 4 || ldb % 4 || !pg::aligned16(A) || !pg::aligned16(B) || !pg::aligned16(out) ||
        !pg::aligned16(work))
        return pg::set_error(PG_ERR_UNSUPPORTED,
                             "pg_gemm_at_b_f32: needs P, N, lda, ldb multiples of 4 and 16-B aligned buffers");
    const SplitPlan sp = split_rows(M, ((P + 127) / 128) * ((N + 127) / 128));
    const int64_t stride = up4(P * N + 4 * P);
    PG_REQUIRE(work_floats >= (int64_t)sp.splits * stride, "workspace too small: %lld < %lld floats",
               (long long)work_floats, (long long)sp.splits * stride);
    WgradP w{};
    w.M = M;
    w.P = (int)P;
    w.N = (int)N;
    w.F_in = (int)N;  // one segment, unit scales
    w.A = A;
    w.lda = lda;
    w.Z = B;
    w.ldz = ldb;
    w.R = nullptr;
    w.ldr = 0;
    w.gates = nullptr;
    w.rows_per_split = sp.rows_per_split;
    w.part_stride = stride;
    w.part = work;
    dim3 grid((unsigned)((N + 127) / 128), (unsigned)((P + 127) / 128), (unsigned)sp.splits);
    hipLaunchKernelGGL((wgrad_kernel<WG_NW>), grid, dim3(64 * WG_NW), 0, s, w);
    launch_reduce((P * N + P) / 4, sp.splits, stride, work, out, s);  // C, then colsum(A) (db row 0)
    return pg::check_launch("pg_gemm_at_b_f32");
}

int pg_directgcn_dense_bwd_bf16(const pg_layer_args_t* a, const float* packed, const uint16_t* packed_bf16,
                                const pg_layer_grad_args_t* g, uint32_t flags, void* stream) {
    PG_REQUIRE(a != nullptr && packed != nullptr && packed_bf16 != nullptr && g != nullptr, "null args");
    PG_REQUIRE(a->M >= 0 && a->F_in > 0 && a->F_out > 0 && a->F_in < (1 << 20) && a->F_out < (1 << 20), "bad shape");
    PG_REQUIRE(a->C_in && a->C_out && a->C_directed && a->C_undirected && a->C_all, "null gate");
    PG_REQUIRE(a->gate_mode == PG_GATES_VECTOR || a->gate_mode == PG_GATES_SCALAR, "bad gate_mode");
    PG_REQUIRE(!a->W_res || a->res_x, "W_res needs res_x");
    PG_REQUIRE(g->dY && g->dpre && g->dgate && g->gates && g->dW && g->work, "null gradient buffer");
    PG_REQUIRE(!a->act || a->Y, "act needs the forward output Y");
    PG_REQUIRE(!a->W_res || g->dres, "W_res needs dres");
    uint32_t drop_thr = 0;
    float drop_s = 0.f;
    if (const int rc = pg::drop_params(a, drop_thr, drop_s, false)) return rc;
    const bool proj = a->W_res != nullptr;
    // the staged weight gradient (wgrad_bfs_kernel) where its tiles fit; PG_FLAG_WGRAD_BF16_TILED keeps the 128 x 128
    // tiles of wgrad_bf16_kernel
    // (with a projected residual, its F_in columns then run on wgrad_bf16_kernel beside it)
    const bool bfs = wgrad_x3_shape(a->F_in, a->F_out, false) && !(flags & PG_FLAG_WGRAD_BF16_TILED) &&
                     a->ldz % 4 == 0 && g->ldp % 4 == 0 && (reinterpret_cast<uintptr_t>(a->Z) & 7) == 0 &&
                     (reinterpret_cast<uintptr_t>(g->dpre) & 7) == 0;
    const BwdPlan pl = plan_of(a->M, a->F_in, a->F_out, proj, bfs);
    PG_REQUIRE(g->work_floats >= pl.total, "workspace too small");
    const uint16_t* Zb = reinterpret_cast<const uint16_t*>(a->Z);
    const uint16_t* Yb = reinterpret_cast<const uint16_t*>(a->Y);
    const uint16_t* Rb = reinterpret_cast<const uint16_t*>(a->res_x);
    const uint16_t* dYb = reinterpret_cast<const uint16_t*>(g->dY);
    uint16_t* dpb = reinterpret_cast<uint16_t*>(g->dpre);
    uint16_t* dZb = reinterpret_cast<uint16_t*>(g->dZ);
    uint16_t* drb = reinterpret_cast<uint16_t*>(g->dres);
    const bool ok = a->F_in % 8 == 0 && a->F_out % 8 == 0 && a->ldz % 8 == 0 && g->lddy % 8 == 0 && g->ldp % 8 == 0 &&
                    (!a->act || a->ldy % 8 == 0) && (!dZb || (g->lddz % 4 == 0 && (reinterpret_cast<uintptr_t>(dZb) & 7) == 0)) &&
                    (!proj || (a->ld_res % 8 == 0 && g->lddres % 4 == 0 && pg::aligned16(Rb) &&
                               (reinterpret_cast<uintptr_t>(drb) & 7) == 0)) &&
                    pg::aligned16(Zb) && pg::aligned16(dYb) && pg::aligned16(dpb) && pg::aligned16(g->gates) &&
                    pg::aligned16(g->dW) && pg::aligned16(g->work) && pg::aligned16(packed) &&
                    pg::aligned16(packed_bf16) && (!a->act || pg::aligned16(Yb));
    if (!ok)
        return pg::set_error(PG_ERR_UNSUPPORTED, "pg_directgcn_dense_bwd_bf16: needs F_in, F_out and leading dims "
                                                 "multiples of 8 and aligned buffers");
    PG_REQUIRE(a->ldz >= 3 * a->F_in && (!dZb || g->lddz >= 3 * a->F_in) && g->lddy >= a->F_out &&
                   g->ldp >= a->F_out,
               "leading dimensions too small");
    hipStream_t s = (hipStream_t)stream;
    const int K = pl.K;
    const int F_in = (int)a->F_in, F_out = (int)a->F_out;
    if (a->M == 0) {
        if (hipMemsetAsync(g->dW, 0, sizeof(float) * ((int64_t)F_out * K + 4 * F_out), s) != hipSuccess)
            return pg::set_error(PG_ERR_HIP, "pg_directgcn_dense_bwd_bf16: memset failed");
        return PG_OK;
    }
    uint16_t* BT = reinterpret_cast<uint16_t*>(g->work + pl.off_bt);
    float* dsp = g->work + pl.off_dsp;
    float* part = g->work + pl.off_part;
    {
        const int64_t total = (int64_t)K * F_out;
        const int nb = (int)std::min<int64_t>((total + 255) / 256, 1024);
        hipLaunchKernelGGL(transpose_u16_kernel, dim3(nb), dim3(256), 0, s, F_out, K, packed_bf16, BT);
    }
    Gates gt{a->gate_mode, a->C_in, a->C_out, a->C_directed, a->C_undirected, a->C_all, a->rows};
    {
        DgradB p{};
        p.M = a->M;
        p.F_in = F_in;
        p.F_out = F_out;
        p.N = K;
        p.dY = dYb;
        p.lddy = g->lddy;
        p.Y = Yb;
        p.ldy = a->ldy;
        p.act = a->act;
        p.slope = a->slope;
        p.drop_s = drop_s;
        p.BT = BT;
        p.bsum = packed + (int64_t)F_out * K;
        p.Z = Zb;
        p.ldz = a->ldz;
        p.g = gt;
        p.dpre = dpb;
        p.ldp = g->ldp;
        p.dZ = dZb;
        p.lddz = g->lddz;
        p.dres = drb;
        p.lddres = g->lddres;
        p.gates = g->gates;
        p.dsp = dsp;
        p.remap = (flags & PG_FLAG_NO_XCD_REMAP) ? 0 : 1;
        PG_REQUIRE(!g->dpre_f32 || (g->ldp_f32 >= F_out && g->ldp_f32 % 4 == 0 && pg::aligned16(g->dpre_f32)),
                   "dpre_f32 needs ldp_f32 >= F_out, a multiple of 4, and a 16-B aligned buffer");
        p.dpre32 = g->dpre_f32;
        p.ldp32 = g->ldp_f32;
        // resident-A kernel: 64-row workgroups, two per CU; below 256 rows per CU (a P = 8 rank's 20,000 rows: 313
        // workgroups) they underfill the GPU and the per-n-tile kernel's N / 128 times as many workgroups run faster
        int dev = 0, ncu = 256;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
            ncu = 256;
        const bool big = a->M >= (int64_t)256 * ncu;
        if (F_out <= RB_FMAX && F_out % BKB == 0 && !(flags & PG_FLAG_DGRAD_BF16_TILED) &&
            (big || (flags & PG_FLAG_DGRAD_BF16_RESIDENT))) {
            const int64_t nb = (a->M + RB_BM - 1) / RB_BM;
            hipLaunchKernelGGL(dgrad_bf16r_kernel, dim3((unsigned)nb), dim3(64 * RB_NW), 0, s, p);
        } else {
            const int64_t nb = ((a->M + DG_BM - 1) / DG_BM) * pl.ntn;
            hipLaunchKernelGGL((dgrad_bf16_kernel<DG_BM, DG_BN, DG_NW>), dim3((unsigned)nb), dim3(64 * DG_NW), 0, s, p);
        }
    }
    {
        const int nb = (int)std::min<int64_t>((a->M + 255) / 256, 2048);
        hipLaunchKernelGGL(gate_grad_kernel, dim3(nb), dim3(256), 0, s, a->M, pl.ntn, (const float*)dsp, gt, g->dgate);
    }
    {
        WgradB w{};
        w.M = a->M;
        w.P = F_out;
        w.N = K;
        w.F_in = F_in;
        w.A = dpb;
        w.lda = g->ldp;
        w.Z = Zb;
        w.ldz = a->ldz;
        w.R = Rb;
        w.ldr = a->ld_res;
        w.gates = g->gates;
        w.rows_per_split = pl.rows_per_split;
        w.part_stride = pl.part_stride;
        w.part = part;
        if (bfs) {
            const int tiles = (F_out / WX_BP) * (3 * F_in / WX_BN);
            const unsigned nb = (unsigned)(8 * ((pl.splits + 7) / 8) * tiles);
            hipLaunchKernelGGL(wgrad_bfs_kernel, dim3(nb), dim3(512), 0, s, w, (int)pl.splits);
            if (proj) {  // the residual's columns [3 F_in, 4 F_in): the same partial buffers, no bias sums
                WgradB wr = w;
                wr.col0 = 3 * F_in;
                dim3 grid((unsigned)((F_in + 127) / 128), (unsigned)((F_out + 127) / 128), (unsigned)pl.splits);
                hipLaunchKernelGGL(wgrad_bf16_kernel, grid, dim3(512), 0, s, wr);
            }
        } else {
            dim3 grid((unsigned)((K + 127) / 128), (unsigned)((F_out + 127) / 128), (unsigned)pl.splits);
            hipLaunchKernelGGL(wgrad_bf16_kernel, grid, dim3(512), 0, s, w);
        }
    }
    launch_reduce(pl.part_stride / 4, pl.splits, pl.part_stride, part, g->dW, s);
    return pg::check_launch("pg_directgcn_dense_bwd_bf16");
}

}  // extern "C"
