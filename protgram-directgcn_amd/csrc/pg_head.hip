// Fused prediction head of ProtGramDirectGCN (src/models/protgram_directgcn.py:218-222):
//   logits = W2 relu(W1 h + b1) + b2            (decoder_fc: Linear -> ReLU -> Dropout(eval) -> Linear)
//   logp   = log_softmax(logits)                (F.log_softmax(.., dim=-1))
//   emb    = h / (||h||_2 + eps)                (EmbeddingProcessor.l2_normalize_torch, models_utils.py:139-147)
// One pass over h: a persistent block walks 64-row tiles, staging each in LDS (the next tile's rows are
// already in flight into registers), writes their embeddings, runs both decoder products on fp32 MFMA
// (v_mfma_f32_32x32x2_f32, B operands straight from the L1/L2-resident weights), and finishes the row
// softmax in LDS. Replaces 6+ framework launches and two re-reads of h.
// Fast path: F <= 256, H <= 128, C <= 64 (F, H multiples of 4); other shapes use a one-wave-per-row
// fallback kernel. The model's own shape (F = 128 -> 64 -> C <= 32) runs head_x3_kernel (split-bf16 decoder 1;
// head_f128_kernel, its fp32-MFMA predecessor, with -DPG_HEAD_FP32). A persistent form of head_x3_kernel (W1 splits
// and W2 kept in registers across a block's 32-row tiles, next tile's rows loaded behind the math; 128 VGPRs, four
// blocks per CU) measured 0.062 ms against 0.050 for one tile per block; two 32-row tiles per block (W1 splits loaded
// once per block; 128 VGPRs, occupancy 4) made the bench step 0.547 -> 0.580 ms (round 3). Round 4: unconditional W2
// loads (no per-lane branch join, whose vmcnt(0) waited on the h rows an HBM round trip early) 47.6 -> 45.8 us per
// launch (bench HIP events, two runs); W1 loaded first with its split pinned ahead of the h rows' arrival measured
// 47.5 us (112 VGPRs, occupancy 4; forcing 5 spills), so the split stays where the compiler puts it.
#include "pg_common.h"
#include "pg_split3.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int HB = 64;  // rows per block

struct HeadP {
    int64_t M;
    int F, H, C;
    const float* h;
    const uint16_t* hb;  // bf16 input instead of h (bf16 mode), or null
    int64_t ldh;
    const float *W1, *b1, *W2, *b2;
    float eps;
    float* logp;
    int64_t ldp;
    float* emb;
    int64_t lde;
};

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

template <int FMAX, int HMAX, int CMAX>
__global__ __launch_bounds__(256) void head_kernel(HeadP p) {
    constexpr int HLD = FMAX + 4, ZLD = HMAX + 4, LLD = CMAX + 1;
    static_assert(HB * LLD <= HB * HLD, "logits alias the h tile");
    constexpr int PF = HB * FMAX / 4 / 256;  // float4 of the h tile per thread
    __shared__ __attribute__((aligned(16))) float Hs[HB * HLD];
    __shared__ __attribute__((aligned(16))) float Zs[HB * ZLD];
    float* Ls = Hs;  // logits reuse the h tile once both decoder products are done
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int li = lane & 31, lh = lane >> 5;
    const int F4 = p.F >> 2;
    const int64_t ntiles = (p.M + HB - 1) / HB;

    // Persistent: the block walks tiles blockIdx.x, +gridDim.x, ...; the next tile's h rows are loaded
    // into registers while the current tile is computed (HBM latency hidden behind the MFMA / softmax).
    float4 hv[PF];
    auto load = [&](int64_t t) {
#pragma unroll
        for (int q = 0; q < PF; ++q) {
            const int idx = tid + 256 * q;
            const int r = idx / (FMAX / 4), c4 = idx % (FMAX / 4);
            const int64_t m = t * HB + r;
            if (m < p.M && c4 < F4) {
                if (p.hb) {
                    const uint2 w = *reinterpret_cast<const uint2*>(p.hb + m * p.ldh + 4 * c4);
                    hv[q] = make_float4(__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
                                        __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u));
                } else {
                    hv[q] = ld4(p.h + m * p.ldh + 4 * c4);
                }
            } else {
                hv[q] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
    };
    int64_t t = blockIdx.x;
    if (t < ntiles) load(t);
    for (; t < ntiles; t += gridDim.x) {
        const int64_t m0 = t * HB;
        // 1. stage h rows (rows past M and columns past F are zero)
#pragma unroll
        for (int q = 0; q < PF; ++q) {
            const int idx = tid + 256 * q;
            const int r = idx / (FMAX / 4), c4 = idx % (FMAX / 4);
            *reinterpret_cast<float4*>(&Hs[r * HLD + 4 * c4]) = hv[q];
        }
        __syncthreads();
        if (t + gridDim.x < ntiles) load(t + gridDim.x);

        // 2. embeddings: one 16-lane group per row, 16 rows per wave pass
        {
            const int g = lane >> 4, tt = lane & 15;
            for (int r = wave * 4 + g; r < HB; r += 16) {
                float ss = 0.f;
                for (int c4 = tt; c4 < F4; c4 += 16) {
                    const float4 v = ld4(&Hs[r * HLD + 4 * c4]);
                    ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
                }
#pragma unroll
                for (int o = 8; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 16);
                const int64_t m = m0 + r;
                if (m < p.M) {
                    const float inv = 1.0f / (sqrtf(ss) + p.eps);
                    for (int c4 = tt; c4 < F4; c4 += 16) {
                        float4 v = ld4(&Hs[r * HLD + 4 * c4]);
                        v = make_float4(v.x * inv, v.y * inv, v.z * inv, v.w * inv);
                        *reinterpret_cast<float4*>(p.emb + m * p.lde + 4 * c4) = v;
                    }
                }
            }
        }

        // 3. z = relu(h W1^T + b1): (HB/32) x (H/32) tiles of 32x32, K = F. A from LDS, B (= W1 rows)
        //    from the L2-resident weights, 4 k at a time with the K permutation of pg_dense.hip.
        {
            const int ntile_n = (p.H + 31) / 32;
            for (int tile = wave; tile < 2 * ntile_n; tile += 4) {
                const int tm = tile / ntile_n, tn = tile % ntile_n;
                const int j = tn * 32 + li;
                const bool jok = j < p.H;
                const float* w1row = p.W1 + (int64_t)(jok ? j : 0) * p.F;
                constexpr int KG = FMAX / 8;
                float4 bf[KG];
#pragma unroll
                for (int g = 0; g < KG; ++g) {
                    const int k = g * 8 + 4 * lh;
                    bf[g] = (jok && k < p.F) ? ld4(w1row + k) : make_float4(0.f, 0.f, 0.f, 0.f);
                }
                f32x16 acc;
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
                for (int g = 0; g < KG; ++g) {
                    const int k = g * 8 + 4 * lh;
                    const float4 a = k < p.F ? ld4(&Hs[(tm * 32 + li) * HLD + k]) : make_float4(0.f, 0.f, 0.f, 0.f);
                    const float4 b = bf[g];
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b.x, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b.y, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b.z, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b.w, acc, 0, 0, 0);
                }
                const float bj = jok ? p.b1[j] : 0.f;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                    const float z = acc[r] + bj;
                    if (j < ZLD - 4) Zs[row * ZLD + j] = jok ? (z > 0.f ? z : 0.f) : 0.f;
                }
            }
        }
        __syncthreads();  // Zs complete; Hs free (-> Ls)

        // 4. logits = z W2^T + b2: (HB/32) x (C/32) tiles, K = H
        {
            const int ntile_n = (p.C + 31) / 32;
            for (int tile = wave; tile < 2 * ntile_n; tile += 4) {
                const int tm = tile / ntile_n, tn = tile % ntile_n;
                const int c = tn * 32 + li;
                const bool cok = c < p.C;
                const float* w2row = p.W2 + (int64_t)(cok ? c : 0) * p.H;
                constexpr int KG = HMAX / 8;
                float4 bf[KG];
#pragma unroll
                for (int g = 0; g < KG; ++g) {
                    const int k = g * 8 + 4 * lh;
                    bf[g] = (cok && k < p.H) ? ld4(w2row + k) : make_float4(0.f, 0.f, 0.f, 0.f);
                }
                f32x16 acc;
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
                for (int g = 0; g < KG; ++g) {
                    const int k = g * 8 + 4 * lh;
                    const float4 a = k < p.H ? ld4(&Zs[(tm * 32 + li) * ZLD + k]) : make_float4(0.f, 0.f, 0.f, 0.f);
                    const float4 b = bf[g];
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b.x, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b.y, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b.z, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b.w, acc, 0, 0, 0);
                }
                const float bc = cok ? p.b2[c] : 0.f;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                    if (cok) Ls[row * LLD + c] = acc[r] + bc;
                }
            }
        }
        __syncthreads();

        // 5. log_softmax per row (max-shifted, as torch): 4 lanes per row
        {
            const int r = tid >> 2, tt = tid & 3;
            const int64_t m = m0 + r;
            float mx = -INFINITY;
            for (int c = tt; c < p.C; c += 4) mx = fmaxf(mx, Ls[r * LLD + c]);
            mx = fmaxf(mx, __shfl_xor(mx, 1, 4));
            mx = fmaxf(mx, __shfl_xor(mx, 2, 4));
            float se = 0.f;
            for (int c = tt; c < p.C; c += 4) se += expf(Ls[r * LLD + c] - mx);
            se += __shfl_xor(se, 1, 4);
            se += __shfl_xor(se, 2, 4);
            const float lse = mx + logf(se);
            if (m < p.M)
                for (int c = tt; c < p.C; c += 4) p.logp[m * p.ldp + c] = Ls[r * LLD + c] - lse;
        }
        __syncthreads();  // Ls (= Hs) is read before the next tile is staged
    }
}

// The model's own head shape (F = 128 -> H = 64 -> C <= 32; ProtGramDirectGCN's decoder is F -> F/2 -> C):
// one 32-row tile per 256-thread block, no persistent loop, small enough (LDS 30 KB, <= 128 VGPRs) for four
// blocks per CU, so one block's loads, MFMAs and softmax overlap the others'. Decoder products on
// v_mfma_f32_16x16x4f32 with a K permutation (lane (i, q) supplies k = 4q + 16m + t for t = 0..3 as four
// consecutive MFMAs, the weights in the same order); both weight fragments stay in registers for the block.
// Rows of the LDS tiles are padded by 8 floats: the (row, 4q) float4 reads of one ds_read_b128 lane group hit 16
// distinct 16-B bank slots.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) void head_f128_kernel(HeadP p) {
    constexpr int BM = 32, F = 128, H = 64, CP = 32;
    constexpr int HLD = F + 8, ZLD = H + 8, LLD = CP + 1;
    __shared__ __attribute__((aligned(16))) float Hs[BM * HLD];
    __shared__ __attribute__((aligned(16))) float Zs[BM * ZLD];
    __shared__ __attribute__((aligned(16))) float Ls[BM * LLD];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int li = lane & 15, q = lane >> 4;
    const int64_t m0 = (int64_t)blockIdx.x * BM;
    // 1. h tile (4 float4 per thread, 512-B rows), then the weight fragments while the loads are in flight
    float4 hv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int r = (tid >> 5) + 8 * k;
        const int64_t m = m0 + r;
        if (m >= p.M) {
            hv[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        } else if (p.hb) {  // bf16 mode: widened exactly
            const uint2 w = *reinterpret_cast<const uint2*>(p.hb + m * p.ldh + 4 * (tid & 31));
            hv[k] = make_float4(__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
                                __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u));
        } else {
            hv[k] = ld4(p.h + m * p.ldh + 4 * (tid & 31));
        }
    }
    float4 w1f[8], w2f[4];
    {
        const float* w1row = p.W1 + (int64_t)(16 * wave + li) * F + 4 * q;  // decoder 1: wave w owns hidden 16w..16w+15
#pragma unroll
        for (int m = 0; m < 8; ++m) w1f[m] = ld4(w1row + 16 * m);
        const int c = 16 * (wave >> 1) + li;  // decoder 2: row block wave & 1, classes 16 (wave >> 1) + li
        const bool cok = c < p.C;
        const float* w2row = p.W2 + (int64_t)(cok ? c : 0) * H + 4 * q;
#pragma unroll
        for (int m = 0; m < 4; ++m) w2f[m] = cok ? ld4(w2row + 16 * m) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const float b1v = p.b1[16 * wave + li];
    const int c2 = 16 * (wave >> 1) + li;
    const float b2v = c2 < p.C ? p.b2[c2] : 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) *reinterpret_cast<float4*>(&Hs[((tid >> 5) + 8 * k) * HLD + 4 * (tid & 31)]) = hv[k];
    __syncthreads();
    // 2. embeddings: 8 threads per row, 16 columns each
    {
        const int r = tid >> 3, part = tid & 7;
        float4 v[4];
        float ss = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v[k] = ld4(&Hs[r * HLD + 16 * part + 4 * k]);
            ss += v[k].x * v[k].x + v[k].y * v[k].y + v[k].z * v[k].z + v[k].w * v[k].w;
        }
        ss += __shfl_xor(ss, 1, 8);
        ss += __shfl_xor(ss, 2, 8);
        ss += __shfl_xor(ss, 4, 8);
        const int64_t m = m0 + r;
        if (m < p.M) {
            const float inv = 1.0f / (sqrtf(ss) + p.eps);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                *reinterpret_cast<float4*>(p.emb + m * p.lde + 16 * part + 4 * k) =
                    make_float4(v[k].x * inv, v[k].y * inv, v[k].z * inv, v[k].w * inv);
        }
    }
    // 3. z = relu(h W1^T + b1): wave w computes hidden columns 16w..16w+15 for both 16-row blocks
    {
        f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int m = 0; m < 8; ++m) {
#pragma unroll
            for (int rb = 0; rb < 2; ++rb) {
                const float4 a = ld4(&Hs[(16 * rb + li) * HLD + 4 * q + 16 * m]);
                acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, w1f[m].x, acc[rb], 0, 0, 0);
                acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, w1f[m].y, acc[rb], 0, 0, 0);
                acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, w1f[m].z, acc[rb], 0, 0, 0);
                acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, w1f[m].w, acc[rb], 0, 0, 0);
            }
        }
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float z = acc[rb][i] + b1v;
                Zs[(16 * rb + 4 * q + i) * ZLD + 16 * wave + li] = z > 0.f ? z : 0.f;
            }
    }
    __syncthreads();
    // 4. logits = z W2^T + b2: wave w -> rows 16 (w & 1).., classes 16 (w >> 1)..
    {
        const int rb = wave & 1;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const float4 a = ld4(&Zs[(16 * rb + li) * ZLD + 4 * q + 16 * m]);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, w2f[m].x, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, w2f[m].y, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, w2f[m].z, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, w2f[m].w, acc, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) Ls[(16 * rb + 4 * q + i) * LLD + c2] = acc[i] + b2v;
    }
    __syncthreads();
    // 5. log_softmax (max-shifted, as torch): 8 threads per row
    {
        const int r = tid >> 3, part = tid & 7;
        const int64_t m = m0 + r;
        float mx = -INFINITY;
        for (int c = part; c < p.C; c += 8) mx = fmaxf(mx, Ls[r * LLD + c]);
        mx = fmaxf(mx, __shfl_xor(mx, 1, 8));
        mx = fmaxf(mx, __shfl_xor(mx, 2, 8));
        mx = fmaxf(mx, __shfl_xor(mx, 4, 8));
        float se = 0.f;
        for (int c = part; c < p.C; c += 8) se += expf(Ls[r * LLD + c] - mx);
        se += __shfl_xor(se, 1, 8);
        se += __shfl_xor(se, 2, 8);
        se += __shfl_xor(se, 4, 8);
        const float lse = mx + logf(se);
        if (m < p.M)
            for (int c = part; c < p.C; c += 8) p.logp[m * p.ldp + c] = Ls[r * LLD + c] - lse;
    }
}

// Split-bf16 variant of head_f128_kernel (the default for its shape): decoder 1 (K = 128, 75 % of the head's
// matrix work) on v_mfma_f32_16x16x32_bf16 with exact three-way bf16 splits of h and W1 (pg_split3.h: six
// products per k step, fp32-level accuracy) -- 48 bf16 MFMAs per wave instead of 64 fp32 16x16x4 ones at twice
// the cycles each. The h tile never goes through LDS as fp32: each thread keeps its 4 rows x 4 columns in
// registers, reduces the row norms across the row's 32 lanes, writes the embeddings, and stores its three bf16
// splits (half a 16-B operand unit per row) into row-swizzled images. Decoder 2 and the softmax as head_f128.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) void head_x3_kernel(HeadP p) {
    constexpr int BM = 32, F = 128, H = 64, CP = 32;
    constexpr int ZLD = H + 8, LLD = CP + 1;
    constexpr int NU = F / 8;  // bf16 operand units per row
    __shared__ __attribute__((aligned(16))) uint4 As[3][BM * NU];  // 24 KB; Zs aliases it after decoder 1
    __shared__ __attribute__((aligned(16))) float Ls[BM * LLD];
    float* Zs = reinterpret_cast<float*>(&As[0][0]);
    static_assert(BM * ZLD * 4 <= 3 * BM * NU * 16, "Zs fits the split images");
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int li = lane & 15, q = lane >> 4;
    const int64_t m0 = (int64_t)blockIdx.x * BM;
    const int c4 = tid & 31;  // this thread's float4 column of every row it holds
    // 1. h rows (tid >> 5) + 8k, columns 4 c4 .. 4 c4 + 3
    float4 hv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t m = m0 + (tid >> 5) + 8 * k;
        if (m >= p.M) {
            hv[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        } else if (p.hb) {  // bf16 mode: widened exactly
            const uint2 w = *reinterpret_cast<const uint2*>(p.hb + m * p.ldh + 4 * c4);
            hv[k] = make_float4(__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
                                __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u));
        } else {
            hv[k] = ld4(p.h + m * p.ldh + 4 * c4);
        }
    }
    // W1 splits: wave w owns hidden columns 16w + li; k step s takes k = 32 s + 8 q .. + 7
    uint4 w0[4], w1[4], w2[4];
    {
        const float* w1row = p.W1 + (int64_t)(16 * wave + li) * F + 8 * q;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const float4 x0 = ld4(w1row + 32 * s), x1 = ld4(w1row + 32 * s + 4);
            const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
            pgx3::split8(v, w0[s], w1[s], w2[s]);
        }
    }
    float4 w2f[4];
    {
        // classes c >= C load row 0 instead of zeros: their logit columns (Ls[.., c]) are never read by the softmax,
        // and unconditional loads keep the compiler from waiting on every load in flight (h included) at a
        // per-lane branch join (a vmcnt(0) one HBM round trip early)
        const int c = 16 * (wave >> 1) + li;
        const float* w2row = p.W2 + (int64_t)(c < p.C ? c : 0) * H + 4 * q;
#pragma unroll
        for (int m = 0; m < 4; ++m) w2f[m] = ld4(w2row + 16 * m);
    }
    const float b1v = p.b1[16 * wave + li];
    const int c2 = 16 * (wave >> 1) + li;
    const float b2v = c2 < p.C ? p.b2[c2] : 0.f;
    // 2. embeddings from registers (row norm: 4-column partials, butterfly over the row's 32 lanes) and the
    //    split images
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int r = (tid >> 5) + 8 * k;
        const float4 v = hv[k];
        float ss = v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) ss += __shfl_xor(ss, o, 32);
        const int64_t m = m0 + r;
        if (m < p.M) {
            const float inv = 1.0f / (sqrtf(ss) + p.eps);
            *reinterpret_cast<float4*>(p.emb + m * p.lde + 4 * c4) = make_float4(v.x * inv, v.y * inv, v.z * inv, v.w * inv);
        }
        uint32_t s0[2], s1[2], s2[2];
        {
            float fa, fb;
            float a = v.x, b = v.y;
            s0[0] = pgx3::bf2(a, b, fa, fb); a -= fa; b -= fb;
            s1[0] = pgx3::bf2(a, b, fa, fb); a -= fa; b -= fb;
            s2[0] = pgx3::bf2(a, b, fa, fb);
            a = v.z; b = v.w;
            s0[1] = pgx3::bf2(a, b, fa, fb); a -= fa; b -= fb;
            s1[1] = pgx3::bf2(a, b, fa, fb); a -= fa; b -= fb;
            s2[1] = pgx3::bf2(a, b, fa, fb);
        }
        const int u = c4 >> 1;
        uint2* d0 = reinterpret_cast<uint2*>(&As[0][r * NU + (u ^ (r & 15))]) + (c4 & 1);
        uint2* d1 = reinterpret_cast<uint2*>(&As[1][r * NU + (u ^ (r & 15))]) + (c4 & 1);
        uint2* d2 = reinterpret_cast<uint2*>(&As[2][r * NU + (u ^ (r & 15))]) + (c4 & 1);
        *d0 = make_uint2(s0[0], s0[1]);
        *d1 = make_uint2(s1[0], s1[1]);
        *d2 = make_uint2(s2[0], s2[1]);
    }
    __syncthreads();
    // 3. z = relu(h W1^T + b1): wave w -> hidden columns 16w.., both 16-row blocks
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
            const int r = 16 * rb + li, u = 4 * s + q;
            const int pos = r * NU + (u ^ (r & 15));
            acc[rb] = pgx3::mfma_x3(As[0][pos], As[1][pos], As[2][pos], w0[s], w1[s], w2[s], acc[rb]);
        }
    }
    __syncthreads();  // every wave is done with the split images before Zs overwrites them
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float z = acc[rb][i] + b1v;
            Zs[(16 * rb + 4 * q + i) * ZLD + 16 * wave + li] = z > 0.f ? z : 0.f;
        }
    __syncthreads();
    // 4. logits = z W2^T + b2: wave w -> rows 16 (w & 1).., classes 16 (w >> 1)..
    {
        const int rb = wave & 1;
        f32x4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const float4 x = ld4(&Zs[(16 * rb + li) * ZLD + 4 * q + 16 * m]);
            a = __builtin_amdgcn_mfma_f32_16x16x4f32(x.x, w2f[m].x, a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x4f32(x.y, w2f[m].y, a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x4f32(x.z, w2f[m].z, a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x4f32(x.w, w2f[m].w, a, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) Ls[(16 * rb + 4 * q + i) * LLD + c2] = a[i] + b2v;
    }
    __syncthreads();
    // 5. log_softmax (max-shifted, as torch): 8 threads per row
    {
        const int r = tid >> 3, part = tid & 7;
        const int64_t m = m0 + r;
        float mx = -INFINITY;
        for (int c = part; c < p.C; c += 8) mx = fmaxf(mx, Ls[r * LLD + c]);
        mx = fmaxf(mx, __shfl_xor(mx, 1, 8));
        mx = fmaxf(mx, __shfl_xor(mx, 2, 8));
        mx = fmaxf(mx, __shfl_xor(mx, 4, 8));
        float se = 0.f;
        for (int c = part; c < p.C; c += 8) se += expf(Ls[r * LLD + c] - mx);
        se += __shfl_xor(se, 1, 8);
        se += __shfl_xor(se, 2, 8);
        se += __shfl_xor(se, 4, 8);
        const float lse = mx + logf(se);
        if (m < p.M)
            for (int c = part; c < p.C; c += 8) p.logp[m * p.ldp + c] = Ls[r * LLD + c] - lse;
    }
}

// General shapes: one wave per row, VALU.
__global__ __launch_bounds__(256) void head_generic_kernel(HeadP p) {
    extern __shared__ float sm[];  // per wave: F + H + C floats
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t m = (int64_t)blockIdx.x * 4 + wave;
    float* hs = sm + wave * (p.F + p.H + p.C);
    float* zs = hs + p.F;
    float* ls = zs + p.H;
    if (m >= p.M) return;
    float ss = 0.f;
    for (int f = lane; f < p.F; f += 64) {
        const float v = p.h[m * p.ldh + f];
        hs[f] = v;
        ss += v * v;
    }
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
    const float inv = 1.0f / (sqrtf(ss) + p.eps);
    for (int f = lane; f < p.F; f += 64) p.emb[m * p.lde + f] = hs[f] * inv;
    __builtin_amdgcn_wave_barrier();
    for (int j = lane; j < p.H; j += 64) {
        float z = p.b1[j];
        for (int f = 0; f < p.F; ++f) z += p.W1[(int64_t)j * p.F + f] * hs[f];
        zs[j] = z > 0.f ? z : 0.f;
    }
    __builtin_amdgcn_wave_barrier();
    float mx = -INFINITY;
    for (int c = lane; c < p.C; c += 64) {
        float l = p.b2[c];
        for (int k = 0; k < p.H; ++k) l += p.W2[(int64_t)c * p.H + k] * zs[k];
        ls[c] = l;
        mx = fmaxf(mx, l);
    }
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    __builtin_amdgcn_wave_barrier();
    float se = 0.f;
    for (int c = lane; c < p.C; c += 64) se += expf(ls[c] - mx);
    for (int o = 32; o > 0; o >>= 1) se += __shfl_xor(se, o);
    const float lse = mx + logf(se);
    for (int c = lane; c < p.C; c += 64) p.logp[m * p.ldp + c] = ls[c] - lse;
}

}  // namespace

namespace {
int head_launch(int64_t M, int64_t F, int64_t H, int64_t C, const float* h, const uint16_t* hb, int64_t ldh,
                const float* W1, const float* b1, const float* W2, const float* b2, float eps, float* logp, int64_t ldp,
                float* emb, int64_t lde, void* stream) {
    PG_REQUIRE(M >= 0 && F > 0 && H > 0 && C > 0 && F < (1 << 16) && H < (1 << 16) && C < (1 << 16), "bad shape");
    if (M == 0) return PG_OK;
    PG_REQUIRE((h || hb) && W1 && b1 && W2 && b2 && logp && emb, "null pointer");
    PG_REQUIRE(ldh >= F && lde >= F && ldp >= C, "bad leading dimension");
    HeadP p{M, (int)F, (int)H, (int)C, h, hb, ldh, W1, b1, W2, b2, eps, logp, ldp, emb, lde};
    hipStream_t s = (hipStream_t)stream;
    const bool in_ok = hb ? ((reinterpret_cast<uintptr_t>(hb) & 7) == 0) : pg::aligned16(h);
    const bool vec = F % 4 == 0 && H % 4 == 0 && ldh % 4 == 0 && lde % 4 == 0 && in_ok &&
                     pg::aligned16(emb) && pg::aligned16(W1) && pg::aligned16(W2);
    if (hb && !(vec && F <= 256 && H <= 128 && C <= 64))
        return pg::set_error(PG_ERR_UNSUPPORTED, "pg_directgcn_head_bf16: needs F <= 256, H <= 128, C <= 64, "
                                                 "F, H, ldh multiples of 4");
    const int64_t ntiles = (M + HB - 1) / HB;
    // persistent grid: blocks per CU as VGPRs allow (179 / 256 VGPRs), tiles split evenly over one wave
    auto grid_of = [&](int64_t per_cu) {
        const int64_t slots = 256 * per_cu;
        const int64_t per_block = (ntiles + slots - 1) / slots;
        return (unsigned)((ntiles + per_block - 1) / per_block);
    };
    if (vec && F == 128 && H == 64 && C <= 32 && ldh % 4 == 0 && lde % 4 == 0) {
#ifdef PG_HEAD_FP32
        hipLaunchKernelGGL(head_f128_kernel, dim3((unsigned)((M + 31) / 32)), dim3(256), 0, s, p);
#else
        hipLaunchKernelGGL(head_x3_kernel, dim3((unsigned)((M + 31) / 32)), dim3(256), 0, s, p);
#endif
    } else if (vec && F <= 128 && H <= 64 && C <= 32) {
        hipLaunchKernelGGL((head_kernel<128, 64, 32>), dim3(grid_of(2)), dim3(256), 0, s, p);
    } else if (vec && F <= 256 && H <= 128 && C <= 64) {
        hipLaunchKernelGGL((head_kernel<256, 128, 64>), dim3(grid_of(1)), dim3(256), 0, s, p);
    } else {
        const size_t shm = 4 * (size_t)(F + H + C) * sizeof(float);
        PG_REQUIRE(shm <= 160 * 1024, "head too wide for the generic kernel");
        hipLaunchKernelGGL(head_generic_kernel, dim3((unsigned)((M + 3) / 4)), dim3(256), shm, s, p);
    }
    return pg::check_launch("pg_directgcn_head_f32");
}
}  // namespace

extern "C" int pg_directgcn_head_f32(int64_t M, int64_t F, int64_t H, int64_t C, const float* h, int64_t ldh,
                                     const float* W1, const float* b1, const float* W2, const float* b2, float eps,
                                     float* logp, int64_t ldp, float* emb, int64_t lde, void* stream) {
    return head_launch(M, F, H, C, h, nullptr, ldh, W1, b1, W2, b2, eps, logp, ldp, emb, lde, stream);
}

extern "C" int pg_directgcn_head_bf16(int64_t M, int64_t F, int64_t H, int64_t C, const uint16_t* h, int64_t ldh,
                                      const float* W1, const float* b1, const float* W2, const float* b2, float eps,
                                      float* logp, int64_t ldp, float* emb, int64_t lde, void* stream) {
    return head_launch(M, F, H, C, nullptr, h, ldh, W1, b1, W2, b2, eps, logp, ldp, emb, lde, stream);
}
