// DirectGCN dense contraction + gated combine on gfx950 fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// After the fused propagation Z = [A_in X | A_out X | A_und X] (pg_spmm.hip), the layer output of
// src/models/protgram_directgcn.py:100-133 is, with A(xW) = (Ax)W,
//   y[m] = sum_k s_k[m] * (Z_k[m] (W_main_k + W_shared)^T + b_main_k + b_shared_k) + constant[r(m)]
//   s_in = c_all*c_dir*c_in,  s_out = c_all*c_dir*c_out,  s_und = c_all*c_und
// i.e. ONE GEMM with K = 3*F_in. This kernel reads the reference's parameters as they are:
//   * B tile: (W_main_k + W_shared) summed while staging (W is a few hundred KB, L2-resident);
//   * A tile: Z scaled by the per-row gate s_k while staging (gates computed once per block into LDS,
//     gathered through original_indices when given);
//   * epilogue: gated bias sums, per-node constant, the model's residual (identity, or a projected
//     residual as a 4th K segment against W_res) and leaky_relu -- then the single store of y.
// So a DirectGCN layer forward is exactly two launches (spmm3 + this), with no framework glue.
//
// Tiling: 256 threads = 4 waves; block tile BM=128 x BN (128 or 64) x BK=32; fp32 operands staged
// global -> registers -> LDS (rows padded to 36 floats: conflict-free ds_read_b128); the next K tile
// is prefetched into registers during the MFMA phase. Each lane feeds its MFMAs with one
// ds_read_b128 per operand per 4 MFMAs by permuting K identically for A and B inside each group of
// 8 (MFMA k-step s of lane half h uses k = 4h + s): same sum, different order.
#include "pg_common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 128;
constexpr int BK = 32;
constexpr int LDSW = 36;  // padded LDS row (floats)

struct LayerP {
    int64_t M, F_in, F_out, K;
    const float* Z;
    int64_t ldz;
    const float* W[3];
    const float* Ws;
    const float* bm[3];
    const float* bs[3];
    int gate_mode;
    const float *C_in, *C_out, *C_dir, *C_und, *C_all;
    const int64_t* rows;
    const float* constant;
    int64_t ld_const;
    const float* res_x;
    int64_t ld_res;
    const float* W_res;
    const float* b_res;
    int act;
    float slope;
    float* Y;
    int64_t ldy;
    int remap;
};

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float4 add4(float4 a, float4 b) {
    return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float4 scale4(float4 a, float s) { return make_float4(a.x * s, a.y * s, a.z * s, a.w * s); }

// One element of the logical A matrix [M, K]: gated aggregates, then the residual input segment.
__device__ __forceinline__ float a_elem(const LayerP& p, const float* sg, int64_t m, int64_t k) {
    const int64_t q = k / p.F_in;
    if (q < 3) return p.Z[m * p.ldz + k] * sg[q];
    return p.res_x[m * p.ld_res + (k - 3 * p.F_in)];
}

// One element of the logical B^T matrix [N, K].
__device__ __forceinline__ float w_elem(const LayerP& p, int64_t n, int64_t k) {
    const int64_t q = k / p.F_in, kk = k - q * p.F_in;
    if (q < 3) return p.W[q][n * p.F_in + kk] + p.Ws[n * p.F_in + kk];
    return p.W_res[n * p.F_in + kk];
}

template <int BN, bool VEC>
__global__ __launch_bounds__(256) void layer_dense_kernel(LayerP p) {
    constexpr int WN = (BN == 128) ? 2 : 1;
    constexpr int WM = 4 / WN;
    constexpr int TM = BM / WM / 32;
    constexpr int TN = BN / WN / 32;
    constexpr int A_F4 = BM * BK / 4 / 256;
    constexpr int W_F4 = BN * BK / 4 / 256;

    __shared__ __attribute__((aligned(16))) float As[BM * LDSW];
    __shared__ __attribute__((aligned(16))) float Bs[BN * LDSW];
    __shared__ float Sg[BM * 4];  // per-row gates s_in, s_out, s_und

    const int64_t n_mblk = (p.M + BM - 1) / BM;
    const int64_t lb = pg::xcd_logical_block(blockIdx.x, gridDim.x, p.remap != 0);
    const int64_t m0 = (lb % n_mblk) * BM;
    const int64_t n0 = (lb / n_mblk) * BN;
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int wm = wave / WN, wn = wave % WN;
    const int li = lane & 31, lh = lane >> 5;

    // Gates (protgram_directgcn.py:116-133): c_x = C_x_vec[r(m)] or the scalar C_x.
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
    }
    __syncthreads();

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    float4 ra[A_F4], rb[W_F4];
    auto fetch = [&](int64_t k0) {
#pragma unroll
        for (int q = 0; q < A_F4; ++q) {
            const int idx = tid + 256 * q;
            const int r = idx >> 3;
            const int64_t m = m0 + r, k = k0 + 4 * (idx & 7);
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (m < p.M) {
                const float* sg = &Sg[r * 4];
                if (VEC && k + 3 < p.K) {  // F_in % 4 == 0: the 4 elements share one segment
                    const int64_t seg = k / p.F_in;
                    v = seg < 3 ? scale4(ld4(p.Z + m * p.ldz + k), sg[seg])
                                : ld4(p.res_x + m * p.ld_res + (k - 3 * p.F_in));
                } else {
                    if (k + 0 < p.K) v.x = a_elem(p, sg, m, k + 0);
                    if (k + 1 < p.K) v.y = a_elem(p, sg, m, k + 1);
                    if (k + 2 < p.K) v.z = a_elem(p, sg, m, k + 2);
                    if (k + 3 < p.K) v.w = a_elem(p, sg, m, k + 3);
                }
            }
            ra[q] = v;
        }
#pragma unroll
        for (int q = 0; q < W_F4; ++q) {
            const int idx = tid + 256 * q;
            const int64_t n = n0 + (idx >> 3), k = k0 + 4 * (idx & 7);
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (n < p.F_out) {
                if (VEC && k + 3 < p.K) {
                    const int64_t seg = k / p.F_in, kk = k - seg * p.F_in;
                    v = seg < 3 ? add4(ld4(p.W[seg] + n * p.F_in + kk), ld4(p.Ws + n * p.F_in + kk))
                                : ld4(p.W_res + n * p.F_in + kk);
                } else {
                    if (k + 0 < p.K) v.x = w_elem(p, n, k + 0);
                    if (k + 1 < p.K) v.y = w_elem(p, n, k + 1);
                    if (k + 2 < p.K) v.z = w_elem(p, n, k + 2);
                    if (k + 3 < p.K) v.w = w_elem(p, n, k + 3);
                }
            }
            rb[q] = v;
        }
    };

    fetch(0);
    for (int64_t k0 = 0; k0 < p.K; k0 += BK) {
        __syncthreads();
#pragma unroll
        for (int q = 0; q < A_F4; ++q) {
            const int idx = tid + 256 * q;
            *reinterpret_cast<float4*>(&As[(idx >> 3) * LDSW + 4 * (idx & 7)]) = ra[q];
        }
#pragma unroll
        for (int q = 0; q < W_F4; ++q) {
            const int idx = tid + 256 * q;
            *reinterpret_cast<float4*>(&Bs[(idx >> 3) * LDSW + 4 * (idx & 7)]) = rb[q];
        }
        __syncthreads();
        if (k0 + BK < p.K) fetch(k0 + BK);
#pragma unroll
        for (int g = 0; g < BK / 8; ++g) {
            float4 a[TM], b[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) a[i] = ld4(&As[(wm * TM * 32 + i * 32 + li) * LDSW + g * 8 + 4 * lh]);
#pragma unroll
            for (int j = 0; j < TN; ++j) b[j] = ld4(&Bs[(wn * TN * 32 + j * 32 + li) * LDSW + g * 8 + 4 * lh]);
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
    }

    // Epilogue. C/D map of the 32x32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
    const bool vec_gates = p.gate_mode == PG_GATES_VECTOR;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int64_t n = n0 + wn * TN * 32 + j * 32 + li;
        if (n >= p.F_out) continue;
        float bsum[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) bsum[q] = p.bm[q][n] + p.bs[q][n];
        const float rbias = (p.W_res && p.b_res) ? p.b_res[n] : 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int rl = wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                const int64_t m = m0 + rl;
                if (m >= p.M) continue;
                const float* sg = &Sg[rl * 4];
                float v = acc[i][j][r] + (sg[0] * bsum[0] + sg[1] * bsum[1] + sg[2] * bsum[2]);
                if (vec_gates && p.constant) {
                    const int64_t cr = p.rows ? p.rows[m] : m;
                    v += p.constant[cr * p.ld_const + n];
                }
                if (p.res_x) v += p.W_res ? rbias : p.res_x[m * p.ld_res + n];
                if (p.act) v = v > 0.f ? v : v * p.slope;
                p.Y[m * p.ldy + n] = v;
            }
    }
}

}  // namespace

extern "C" int pg_directgcn_dense_f32(const pg_layer_args_t* a, uint32_t flags, void* stream) {
    PG_REQUIRE(a != nullptr, "null args");
    PG_REQUIRE(a->M >= 0 && a->F_in > 0 && a->F_out > 0, "bad shape M=%lld F_in=%lld F_out=%lld", (long long)a->M,
               (long long)a->F_in, (long long)a->F_out);
    if (a->M == 0) return PG_OK;
    PG_REQUIRE(a->Z && a->ldz >= 3 * a->F_in, "Z must be [M, >=3*F_in]");
    PG_REQUIRE(a->W_main_in && a->W_main_out && a->W_undirected && a->W_shared, "null weight");
    PG_REQUIRE(a->b_main_in && a->b_dir_shared_in && a->b_main_out && a->b_dir_shared_out && a->b_undirected &&
                   a->b_undirected_shared,
               "null bias");
    PG_REQUIRE(a->C_in && a->C_out && a->C_directed && a->C_undirected && a->C_all, "null gate");
    PG_REQUIRE(a->gate_mode == PG_GATES_VECTOR || a->gate_mode == PG_GATES_SCALAR, "bad gate_mode");
    PG_REQUIRE(!a->constant || a->ld_const >= a->F_out, "ld_const < F_out");
    PG_REQUIRE(!a->W_res || a->res_x, "W_res needs res_x");
    PG_REQUIRE(!a->res_x || a->W_res || a->F_in == a->F_out, "identity residual needs F_in == F_out");
    PG_REQUIRE(!a->res_x || a->ld_res >= a->F_in, "ld_res < F_in");
    PG_REQUIRE(a->Y && a->ldy >= a->F_out, "bad output");
    LayerP p{};
    p.M = a->M;
    p.F_in = a->F_in;
    p.F_out = a->F_out;
    p.K = (a->W_res ? 4 : 3) * a->F_in;
    p.Z = a->Z;
    p.ldz = a->ldz;
    p.W[0] = a->W_main_in;
    p.W[1] = a->W_main_out;
    p.W[2] = a->W_undirected;
    p.Ws = a->W_shared;
    p.bm[0] = a->b_main_in;
    p.bm[1] = a->b_main_out;
    p.bm[2] = a->b_undirected;
    p.bs[0] = a->b_dir_shared_in;
    p.bs[1] = a->b_dir_shared_out;
    p.bs[2] = a->b_undirected_shared;
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
    p.W_res = a->W_res;
    p.b_res = a->b_res;
    p.act = a->act;
    p.slope = a->slope;
    p.Y = a->Y;
    p.ldy = a->ldy;
    p.remap = (flags & PG_FLAG_NO_XCD_REMAP) ? 0 : 1;
    bool vec = (a->F_in % 4 == 0) && (a->ldz % 4 == 0) && pg::aligned16(a->Z) && pg::aligned16(a->W_main_in) &&
               pg::aligned16(a->W_main_out) && pg::aligned16(a->W_undirected) && pg::aligned16(a->W_shared);
    if (a->W_res) vec = vec && pg::aligned16(a->W_res);
    if (a->res_x) vec = vec && pg::aligned16(a->res_x) && (a->ld_res % 4 == 0);
    const bool wide = a->F_out > 64;
    const int64_t BN = wide ? 128 : 64;
    const int64_t nb = ((a->M + BM - 1) / BM) * ((a->F_out + BN - 1) / BN);
    hipStream_t s = (hipStream_t)stream;
    if (wide) {
        if (vec) hipLaunchKernelGGL((layer_dense_kernel<128, true>), dim3((unsigned)nb), dim3(256), 0, s, p);
        else hipLaunchKernelGGL((layer_dense_kernel<128, false>), dim3((unsigned)nb), dim3(256), 0, s, p);
    } else {
        if (vec) hipLaunchKernelGGL((layer_dense_kernel<64, true>), dim3((unsigned)nb), dim3(256), 0, s, p);
        else hipLaunchKernelGGL((layer_dense_kernel<64, false>), dim3((unsigned)nb), dim3(256), 0, s, p);
    }
    return pg::check_launch("pg_directgcn_dense_f32");
}
