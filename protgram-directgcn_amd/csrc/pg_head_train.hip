// Training step of ProtGramDirectGCN's prediction head, forward and backward in one pass over the rows
// (src/models/protgram_directgcn.py:218-222 in train mode, and the autograd of the trainer's loss on it,
// protgram_directgcn_trainer.py:91-100):
//   a      = dropout(relu(h W1^T + b1))                      decoder_fc[0..2] (Linear, ReLU, Dropout(p))
//   logits = a W2^T + b2                                      decoder_fc[3]
//   loss   = lw * sum_m -log_softmax(logits[m])[y[m]]          F.nll_loss(.., reduction mean): lw = weight / M
// and, for a loss gradient s (the GradScaler scale, or 1), with dl = s * lw * (softmax(logits) - onehot(y)):
//   dW2 = dl^T a,  db2 = sum dl,  da = (dl W2) * (a > 0) / (1 - p),  dW1 = da^T h,  db1 = sum da,  dh = da W1.
// The framework path runs ~20 launches for this (two library GEMMs forward, two backward, two weight-gradient
// reductions over all M rows, the softmax, the gather and a dozen elementwise passes) and moves h, the hidden
// activations and the logits through HBM several times; here each row block reads h once and writes dh once.
//
// One 512-thread workgroup per CU walks 64-row tiles (persistent, the next tile's h rows loaded into registers behind
// the current tile's math). Every product is a set of 16x16 tiles on fp32 MFMA (v_mfma_f32_16x16x4_f32, fp32
// operands and sums, as the library GEMMs it replaces), operands from LDS: the weights (W1 [H][F], W2 [C][H], staged
// once per workgroup), the h tile, a (the dropout output), dl and da. Phases per tile (barriers between them):
//   A  a = h W1^T: 16 tiles of 16x16, two per wave
//   B  logits = a W2^T: 8 tiles, one per wave
//   C  log-softmax, loss, dl: eight lanes per row
//   D  dW2 += dl^T a (one tile per wave, accumulated in registers over the workgroup's tiles); da = dl W2 (two tiles
//      per wave); db2 column sums
//   E  dh = da W1 (four tiles per wave, stored); dW1 += da^T h (four tiles per wave, accumulated); db1 column sums
// Each accumulated weight-gradient tile belongs to one wave, so a workgroup writes one partial per tile; a second
// kernel adds the partials of all workgroups in workgroup order (deterministic, no atomics).
// Dropout keeps element (m, j) when hash(seed, m, j) >= p * 2^24 (a counter-based draw: the same mask in the forward
// and backward phases, nothing stored); seed is a device int64 the caller draws from torch's generator per step.
// Shapes: F = 128, H = 64, C <= 32 (the model's F = 128 head: hidden = final_dim / 2, protgram_directgcn.py:173-177);
// others: PG_ERR_UNSUPPORTED, the caller runs the framework path.
#include <algorithm>
#include <cmath>

#include "pg_common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int TC = 32;  // classes, padded
constexpr int NT = 512;
// The tiling is written for F = 128 (H = 64, 64-row tiles, W1 staged in LDS) and F = 256 (H = 128, 32-row tiles, W1
// read from the L2-resident weights); only F = 128 is launched (shape_ok). Row strides are 18 mod 32 floats: the
// 16x16x4 operand reads (16 rows x 2 k per 32-lane half) fall on distinct banks.
template <int F> struct HT {
    static constexpr int H = F / 2, TR = F == 128 ? 64 : 32;
    static constexpr bool W1L = F == 128;  // W1 in LDS
    static constexpr int LDH = F + 18, LDW1 = F + 18, LDA = H + 18, LDW2 = H + 18, LDL = TC + 18;
    static constexpr int HT4 = TR * F / 4 / NT;  // float4 of the h tile per thread
    // per-workgroup partial: dW1 [H][F], db1 [H], dW2 [C][H], db2 [C], loss
    static constexpr int P_DW1 = 0, P_DB1 = H * F, P_DW2 = P_DB1 + H, P_DB2 = P_DW2 + TC * H, P_LOSS = P_DB2 + TC;
    static constexpr int P_STRIDE = (P_LOSS + 1 + 3) / 4 * 4;
    static constexpr int LDS_FLOATS = (W1L ? H * LDW1 : 0) + TC * LDW2 + TR * LDH + 2 * TR * LDA + TR * LDL;
    // tiles of 16x16 per wave: A = TR x H, dW2 = 32 x H, da = TR x H, dh = TR x F, dW1 = H x F
    static constexpr int QA = (TR / 16) * (H / 16) / 8, QW2 = 2 * (H / 16) / 8, QD = (TR / 16) * (H / 16) / 8;
    static constexpr int QE = (TR / 16) * (F / 16) / 8, QW1 = (H / 16) * (F / 16) / 8;
    static_assert(HT4 * NT * 4 == TR * F && QA >= 1 && QW2 >= 1 && QD >= 1 && QE >= 1 && QW1 >= 1, "tiling");
};

struct HeadTrainP {
    int64_t M;
    int C;
    const float* h;
    int64_t ldh;
    const float *W1, *b1, *W2, *b2;
    const int64_t* y;
    float lw;           // loss weight per row (weight / M)
    uint32_t drop_thr;  // keep when (hash >> 8) >= drop_thr (p * 2^24); 0: no dropout
    float inv_keep;     // 1 / (1 - p)
    const int64_t* seed;
    const float* scale;  // the loss gradient (GradScaler's scale) or null (1)
    float* dh;
    int64_t lddh;
    float* part;  // [gridDim.x][P_STRIDE]
};

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// counter-based dropout draw (a murmur3-style finalizer of the element's index mixed with the seed)
__device__ __forceinline__ uint32_t drop_hash(uint64_t seed, int64_t m, int j, int H) {
    uint64_t x = seed ^ (0x9E3779B97F4A7C15ull * (uint64_t)(m * H + j + 1));
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return (uint32_t)x;
}

template <int F>
__global__ __launch_bounds__(NT) void head_train_kernel(HeadTrainP p) {
    using T = HT<F>;
    constexpr int H = T::H, TR = T::TR, LDH = T::LDH, LDW1 = T::LDW1, LDA = T::LDA, LDW2 = T::LDW2, LDL = T::LDL;
    __shared__ float lds[T::LDS_FLOATS];
    float* W1s = lds;                                   // W1 [H][F] (F = 128 only)
    float* W2s = W1s + (T::W1L ? H * LDW1 : 0);         // W2 [C][H], rows >= C zero
    float* Hs = W2s + TC * LDW2;                        // the h tile
    float* As = Hs + TR * LDH;                          // a (after relu and dropout)
    float* Ds = As + TR * LDA;                          // da
    float* Ls = Ds + TR * LDA;                          // logits, then dl
    __shared__ float red[NT / 64];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int l16 = lane & 15, kq = lane >> 4;
    const int64_t ntiles = (p.M + TR - 1) / TR;
    const uint64_t seed = p.drop_thr ? (uint64_t)p.seed[0] : 0;
    const float gscale = p.scale ? p.scale[0] : 1.f;
    // W1[j][k] for a 16x16x4 operand: LDS image or the global (L2-resident) weights
    auto w1 = [&](int j, int k) -> float { return T::W1L ? W1s[j * LDW1 + k] : p.W1[j * F + k]; };

    if (T::W1L)
        for (int i = tid; i < H * F; i += NT) W1s[(i / F) * LDW1 + i % F] = p.W1[i];
    for (int i = tid; i < TC * H; i += NT) W2s[(i / H) * LDW2 + i % H] = i / H < p.C ? p.W2[i] : 0.f;

    float4 hv[T::HT4];
    auto load = [&](int64_t t) {
#pragma unroll
        for (int q = 0; q < T::HT4; ++q) {
            const int idx = tid + NT * q, r = idx / (F / 4), c4 = idx % (F / 4);
            const int64_t m = t * TR + r;
            hv[q] = m < p.M ? *reinterpret_cast<const float4*>(p.h + m * p.ldh + 4 * c4) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto stash = [&]() {
#pragma unroll
        for (int q = 0; q < T::HT4; ++q) {
            const int idx = tid + NT * q, r = idx / (F / 4), c4 = idx % (F / 4);
            float* d = &Hs[r * LDH + 4 * c4];
            d[0] = hv[q].x;
            d[1] = hv[q].y;
            d[2] = hv[q].z;
            d[3] = hv[q].w;
        }
    };

    // persistent accumulators: dW1 tiles wave + 8 q (q < QW1, of the (H/16) x (F/16) grid), dW2 tiles (q < QW2, of
    // 2 x (H/16)), the bias column sums (db1: threads 0..H-1, db2: threads 256..256+C-1) and the loss
    f32x4 accW1[T::QW1], accW2[T::QW2];
#pragma unroll
    for (int q = 0; q < T::QW1; ++q) accW1[q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < T::QW2; ++q) accW2[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    float dbias = 0.f, lossp = 0.f;

    int64_t t = blockIdx.x;
    if (t < ntiles) load(t);
    for (; t < ntiles; t += gridDim.x) {
        const int64_t m0 = t * TR;
        stash();
        __syncthreads();  // h tile (and, the first time, the weights) staged
        if (t + gridDim.x < ntiles) load(t + gridDim.x);

        // A: a = dropout(relu(h W1^T + b1)); the wave's tiles share their column tile, chains interleaved
        {
            constexpr int CT = H / 16;
            f32x4 acc[T::QA];
#pragma unroll
            for (int q = 0; q < T::QA; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
            const int ct = wave % CT;
#pragma unroll 4
            for (int k = 0; k < F; k += 4) {
                const float b = w1(16 * ct + l16, k + kq);
#pragma unroll
                for (int q = 0; q < T::QA; ++q)
                    acc[q] = mfma16(Hs[(16 * ((wave + 8 * q) / CT) + l16) * LDH + k + kq], b, acc[q]);
            }
            const int j = 16 * ct + l16;
            const float bj = p.b1[j];
#pragma unroll
            for (int q = 0; q < T::QA; ++q)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = 16 * ((wave + 8 * q) / CT) + 4 * kq + r;
                    float v = fmaxf(acc[q][r] + bj, 0.f);
                    if (p.drop_thr) v = (drop_hash(seed, m0 + row, j, H) >> 8) >= p.drop_thr ? v * p.inv_keep : 0.f;
                    As[row * LDA + j] = v;
                }
        }
        __syncthreads();

        // B: logits = a W2^T + b2: (TR / 16) x 2 tiles
        if (wave < (TR / 16) * 2) {
            const int rt = wave >> 1, ct = wave & 1;
            f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
            const float* ap = &As[(16 * rt + l16) * LDA + kq];
            const float* bp = &W2s[(16 * ct + l16) * LDW2 + kq];
#pragma unroll 8
            for (int k = 0; k < H; k += 4) acc = mfma16(ap[k], bp[k], acc);
            const int c = 16 * ct + l16;
            const float bc = c < p.C ? p.b2[c] : 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) Ls[(16 * rt + 4 * kq + r) * LDL + c] = acc[r] + bc;
        }
        __syncthreads();

        // C: log-softmax, loss and dl = s lw (softmax - onehot(y)); eight lanes per row, classes part, part + 8, ..
        if (wave < TR / 8) {
            const int row = 8 * wave + (lane >> 3), part = lane & 7;
            const int64_t m = m0 + row;
            const bool ok = m < p.M;
            const int64_t yl = ok ? p.y[m] : -1;
            const int yv = (int)yl;
            // a label outside [0, C) makes the loss NaN (F.nll_loss raises on it; ops.head_train checks the labels
            // on the host once per label tensor, this covers what that check cannot see, e.g. a captured step)
            if (ok && part == 0 && (yl < 0 || yl >= p.C)) lossp += __builtin_nanf("");
            float x[TC / 8];
            float mx = -INFINITY;
#pragma unroll
            for (int u = 0; u < TC / 8; ++u) {
                const int c = part + 8 * u;
                x[u] = c < p.C ? Ls[row * LDL + c] : -INFINITY;
                mx = fmaxf(mx, x[u]);
            }
#pragma unroll
            for (int o = 1; o < 8; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 8));
            float se = 0.f;
#pragma unroll
            for (int u = 0; u < TC / 8; ++u) se += part + 8 * u < p.C ? expf(x[u] - mx) : 0.f;
#pragma unroll
            for (int o = 1; o < 8; o <<= 1) se += __shfl_xor(se, o, 8);
            const float lse = logf(se);
            const float g = gscale * p.lw;
#pragma unroll
            for (int u = 0; u < TC / 8; ++u) {
                const int c = part + 8 * u;
                float dl = 0.f;
                if (ok && c < p.C) {
                    const float lp = (x[u] - mx) - lse;  // log_softmax as torch computes it
                    if (c == yv) lossp -= lp;
                    dl = (expf(lp) - (c == yv ? 1.f : 0.f)) * g;
                }
                Ls[row * LDL + c] = dl;
            }
        }
        __syncthreads();

        // D: dW2 += dl^T a (tiles wave + 8 q of 2 x (H/16)); da = (dl W2) * (a > 0) / (1 - p); db2 column sums
#pragma unroll
        for (int q = 0; q < T::QW2; ++q) {
            const int tt = wave + 8 * q, ct = tt / (H / 16), ht = tt % (H / 16);
#pragma unroll 4
            for (int k = 0; k < TR; k += 4)
                accW2[q] = mfma16(Ls[(k + kq) * LDL + 16 * ct + l16], As[(k + kq) * LDA + 16 * ht + l16], accW2[q]);
        }
        {
            constexpr int CT = H / 16;
            f32x4 acc[T::QD];
#pragma unroll
            for (int q = 0; q < T::QD; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
            const int ht = wave % CT;
#pragma unroll
            for (int k = 0; k < TC; k += 4) {
                const float b = W2s[(k + kq) * LDW2 + 16 * ht + l16];
#pragma unroll
                for (int q = 0; q < T::QD; ++q)
                    acc[q] = mfma16(Ls[(16 * ((wave + 8 * q) / CT) + l16) * LDL + k + kq], b, acc[q]);
            }
            const int j = 16 * ht + l16;
            const float ik = p.drop_thr ? p.inv_keep : 1.f;
#pragma unroll
            for (int q = 0; q < T::QD; ++q)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = 16 * ((wave + 8 * q) / CT) + 4 * kq + r;
                    Ds[row * LDA + j] = As[row * LDA + j] > 0.f ? acc[q][r] * ik : 0.f;
                }
        }
        if (tid >= 256 && tid < 256 + TC) {  // db2: rows in order
            float s = 0.f;
            for (int r = 0; r < TR; ++r) s += Ls[r * LDL + (tid - 256)];
            dbias += s;
        }
        __syncthreads();

        // E: dh = da W1 (tiles wave + 8 q of (TR/16) x (F/16), stored); dW1 += da^T h (tiles wave + 8 q of
        // (H/16) x (F/16)); db1 column sums
        {
            constexpr int FT = F / 16;
            f32x4 acc[T::QE];
#pragma unroll
            for (int q = 0; q < T::QE; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
            for (int k = 0; k < H; k += 4) {
#pragma unroll
                for (int q = 0; q < T::QE; ++q) {
                    const int tt = wave + 8 * q;
                    acc[q] = mfma16(Ds[(16 * (tt / FT) + l16) * LDA + k + kq], w1(k + kq, 16 * (tt % FT) + l16), acc[q]);
                }
            }
#pragma unroll
            for (int q = 0; q < T::QE; ++q) {
                const int tt = wave + 8 * q, f = 16 * (tt % FT) + l16;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int64_t m = m0 + 16 * (tt / FT) + 4 * kq + r;
                    if (m < p.M) p.dh[m * p.lddh + f] = acc[q][r];
                }
            }
#pragma unroll 1
            for (int k = 0; k < TR; k += 4) {
#pragma unroll
                for (int q = 0; q < T::QW1; ++q) {
                    const int tt = wave + 8 * q;
                    accW1[q] = mfma16(Ds[(k + kq) * LDA + 16 * (tt / FT) + l16], Hs[(k + kq) * LDH + 16 * (tt % FT) + l16],
                                      accW1[q]);
                }
            }
        }
        if (tid < H) {  // db1: rows in order
            float s = 0.f;
            for (int r = 0; r < TR; ++r) s += Ds[r * LDA + tid];
            dbias += s;
        }
        __syncthreads();  // the tile's LDS is read out before the next tile is staged
    }

    // this workgroup's partial
    float* out = p.part + (int64_t)blockIdx.x * T::P_STRIDE;
#pragma unroll
    for (int q = 0; q < T::QW1; ++q) {
        const int tt = wave + 8 * q, ht = tt / (F / 16), ft = tt % (F / 16);
#pragma unroll
        for (int r = 0; r < 4; ++r) out[T::P_DW1 + (16 * ht + 4 * kq + r) * F + 16 * ft + l16] = accW1[q][r];
    }
#pragma unroll
    for (int q = 0; q < T::QW2; ++q) {
        const int tt = wave + 8 * q, ct = tt / (H / 16), ht = tt % (H / 16);
#pragma unroll
        for (int r = 0; r < 4; ++r) out[T::P_DW2 + (16 * ct + 4 * kq + r) * H + 16 * ht + l16] = accW2[q][r];
    }
    if (tid < H) out[T::P_DB1 + tid] = dbias;
    if (tid >= 256 && tid < 256 + TC) out[T::P_DB2 + tid - 256] = dbias;
    // loss: lanes in order within the wave, then waves in order
    float v = lossp;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    if (lane == 0) red[wave] = v;
    __syncthreads();
    if (tid == 0) {
        float s = 0.f;
        for (int w = 0; w < NT / 64; ++w) s += red[w];
        out[T::P_LOSS] = s * p.lw;
    }
}

// grads[i] = sum over workgroups of part[b][i], i <= P_LOSS: dW1, db1, dW2 (C rows), db2, loss. A block owns 32
// consecutive entries; its 8 thread groups take every 8th partial and are combined in group order (deterministic).
template <int F>
__global__ __launch_bounds__(256) void head_train_reduce_kernel(int nparts, int C, const float* part, float* grads,
                                                                float* loss) {
    using T = HT<F>;
    constexpr int H = T::H;
    __shared__ float acc_s[8][32];
    const int c = threadIdx.x & 31, grp = threadIdx.x >> 5;
    const int i = blockIdx.x * 32 + c;
    float s = 0.f;
    if (i <= T::P_LOSS)
        for (int b = grp; b < nparts; b += 8) s += part[(int64_t)b * T::P_STRIDE + i];
    acc_s[grp][c] = s;
    __syncthreads();
    if (grp != 0 || i > T::P_LOSS) return;
    s = acc_s[0][c];
    for (int g = 1; g < 8; ++g) s += acc_s[g][c];
    if (i < T::P_DW2) grads[i] = s;                                                       // dW1, db1
    else if (i < T::P_DB2) { if ((i - T::P_DW2) / H < C) grads[i] = s; }                  // dW2 rows < C
    else if (i < T::P_LOSS) { if (i - T::P_DB2 < C) grads[T::P_DW2 + C * H + (i - T::P_DB2)] = s; }  // db2
    else loss[0] = s;
}

template <int F>
int grid_of(int64_t M) {
    const int64_t ntiles = (M + HT<F>::TR - 1) / HT<F>::TR;
    return (int)std::max<int64_t>(1, std::min<int64_t>(ntiles, 256));
}

template <int F>
int launch(const HeadTrainP& p, int64_t C, float* grads, float* loss, hipStream_t s) {
    const int grid = grid_of<F>(p.M);
    hipLaunchKernelGGL(head_train_kernel<F>, dim3((unsigned)grid), dim3(NT), 0, s, p);
    hipLaunchKernelGGL(head_train_reduce_kernel<F>, dim3((HT<F>::P_LOSS + 1 + 31) / 32), dim3(256), 0, s, grid, (int)C,
                       (const float*)p.part, grads, loss);
    return pg::check_launch("pg_head_train_f32");
}

// F = 256 (config 5) is not taken: its 128 KB W1 does not fit the LDS beside the tiles, and read from L2 per MFMA
// operand the kernel measured 760 us against ~0.66 ms for the framework ops it would replace (round 5)
bool shape_ok(int64_t F, int64_t H, int64_t C) { return F == 128 && H == F / 2 && C >= 1 && C <= TC; }

// ---------------------------------------------------------------------------------------------------------------
// bf16 mode, F = 256, H = 128 (config 5: dims [.., 256], hidden = 128, protgram_directgcn.py:173-177): the same step on
// the bf16 h the layers produce, dh returned in bf16 (the gradient of the bf16 h; rounded once). The model's fp32
// decoder on a 256-wide h does 3 x 10.5 GFLOP of products per step; on the fp32 matrix cores that alone is 0.2 ms, so
// the products run on v_mfma_f32_16x16x32_bf16 / _16x16x16_bf16 with two-term bf16 splits of the fp32 operands
// (v = hi + lo, hi = bf16(v), lo = bf16(v - hi): |v - hi - lo| <= 2^-16 |v|) and fp32 accumulation: h is exact in bf16,
// so z = h W1^T takes two products (W1 hi, lo), dW1 = da^T h two (da hi, lo), the others three (hi hi, hi lo, lo hi;
// the dropped lo lo term is below 2^-16 of the product). Every product is thus within ~2^-15 relative of the fp32
// one -- far below the 2^-8 rounding of the bf16 h and dh around it.
// One 512-thread workgroup per CU, persistent over 16-row tiles. LDS: W1 split into two bf16 planes [128][256] (staged
// once per workgroup, rows padded to 528 B), the h tile, a (split), da (split), the logits / dl rows (133 KB + 30 KB).
// W2 (C <= 32 rows) lives in registers in the two operand layouts it is read in. Per tile (six barriers):
//   A  z = h W1^T + b1 (wave w: hidden columns 16w..16w+15), a = dropout(relu(z)) -> the a image (hi, lo)
//   B  logits = a W2^T + b2 (waves 0, 1: classes 0..15, 16..31)
//   C  log-softmax, loss, dl = s lw (softmax - onehot(y)) -> dl (hi, lo) in place of its row's logits
//   D  dW2 += dl^T a (K = the 16 rows: 16x16x16, operands by ds_read_b64_tr_b16); D2 da = (dl W2) * mask -> da image
//   E  dh = da W1 (wave w: features 32w..32w+31; W1's k = j rows by transposed reads) -> bf16 staging -> HBM
//   F  dW1 += da^T h (wave w: hidden rows 16w.., all 256 features; 16x16x16 on transposed reads)
// Partials per workgroup, summed in workgroup order by a second kernel (deterministic), as head_train_kernel.
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

namespace h5 {
constexpr int F = 256, H = 128, TR = 16;
constexpr int RW1 = F + 8;     // W1 plane row (elements): 528 B, 16-B aligned rows for ds_read_b128
constexpr int RH = F + 8;      // h tile row
constexpr int RA = H + 8;      // a / da image row: 272 B
constexpr int RL = 36;         // logits row (floats): 144 B; dl (bf16) hi at bytes 0..63, lo at 64..127 of the row
constexpr int W1B = 2 * H * RW1 * 2, HB = TR * RH * 2, AB = 2 * TR * RA * 2, LB = TR * RL * 4;
constexpr int LDS_BYTES = W1B + HB + 2 * AB + LB;
static_assert(LDS_BYTES <= 163840, "LDS");
static_assert(TR * F * 2 <= AB, "dh staging fits the a image");
constexpr int P_DW1 = 0, P_DB1 = H * F, P_DW2 = P_DB1 + H, P_DB2 = P_DW2 + TC * H, P_LOSS = P_DB2 + TC;
constexpr int P_STRIDE = (P_LOSS + 1 + 3) / 4 * 4;
}  // namespace h5

__device__ __forceinline__ void split2(float v, uint16_t& hi, uint16_t& lo) {
    const __bf16 h = (__bf16)v;
    hi = __builtin_bit_cast(uint16_t, h);
    lo = __builtin_bit_cast(uint16_t, (__bf16)(v - (float)h));
}
__device__ __forceinline__ f32x4 mfma32(uint4 a, uint4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                   0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16k(s16x4 a, s16x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}
// ds_read_b64_tr_b16: per 16-lane group, 4 rows x 16 columns delivered column-major (lane i: column i, element q = row
// q); lane 4q + p supplies the address of row q, columns 4p .. 4p + 3
__device__ __forceinline__ s16x4 tr16(const void* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}
__device__ __forceinline__ uint4 cat8(s16x4 a, s16x4 b) {
    const uint2 x = __builtin_bit_cast(uint2, a), y = __builtin_bit_cast(uint2, b);
    return make_uint4(x.x, x.y, y.x, y.y);
}

__global__ __launch_bounds__(NT) void head_train5_kernel(HeadTrainP p, const uint16_t* hb, uint16_t* dhb) {
    using namespace h5;
    extern __shared__ __attribute__((aligned(16))) char L5[];
    uint16_t* W1P = reinterpret_cast<uint16_t*>(L5);                  // [2][H][RW1]
    uint16_t* HI = reinterpret_cast<uint16_t*>(L5 + W1B);             // [TR][RH]
    uint16_t* AI = reinterpret_cast<uint16_t*>(L5 + W1B + HB);        // [2][TR][RA]; the dh staging [TR][F] after D
    uint16_t* DI = reinterpret_cast<uint16_t*>(L5 + W1B + HB + AB);   // [2][TR][RA]
    char* LF = L5 + W1B + HB + 2 * AB;                                 // [TR][RL] floats; dl bf16 in place
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int l16 = lane & 15, g = lane >> 4, tq = l16 >> 2, tp = lane & 3;  // tr16 address roles: row tq, cols 4 tp
    const int64_t ntiles = (p.M + TR - 1) / TR;
    const uint64_t seed = p.drop_thr ? (uint64_t)p.seed[0] : 0;
    const float gscale = p.scale ? p.scale[0] : 1.f;
    const float ik = p.drop_thr ? p.inv_keep : 1.f;

    // W1 -> two bf16 planes (once per workgroup)
    for (int i = tid; i < H * F / 4; i += NT) {
        const int j = (4 * i) / F, f = (4 * i) % F;
        const float4 v = *reinterpret_cast<const float4*>(p.W1 + (int64_t)j * F + f);
        const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            uint16_t hi, lo;
            split2(e[u], hi, lo);
            W1P[j * RW1 + f + u] = hi;
            W1P[H * RW1 + j * RW1 + f + u] = lo;
        }
    }
    // W2 in registers: B of the logits (waves 0, 1; class c = 16 w + l16, hidden 32 s + 8 g ..) and B of da (hidden
    // j = 16 w + l16, classes 8 g ..), each split in two
    uint4 w2t[2][H / 32], w2b[2];
    {
        const int c = 16 * (wave & 1) + l16;
#pragma unroll
        for (int s = 0; s < H / 32; ++s) {
            uint16_t hi[8], lo[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) split2(c < p.C ? p.W2[c * H + 32 * s + 8 * g + e] : 0.f, hi[e], lo[e]);
            w2t[0][s] = make_uint4(hi[0] | (uint32_t)hi[1] << 16, hi[2] | (uint32_t)hi[3] << 16, hi[4] | (uint32_t)hi[5] << 16,
                                   hi[6] | (uint32_t)hi[7] << 16);
            w2t[1][s] = make_uint4(lo[0] | (uint32_t)lo[1] << 16, lo[2] | (uint32_t)lo[3] << 16, lo[4] | (uint32_t)lo[5] << 16,
                                   lo[6] | (uint32_t)lo[7] << 16);
        }
        const int j = 16 * wave + l16;
        uint16_t hi[8], lo[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) split2(8 * g + e < p.C ? p.W2[(8 * g + e) * H + j] : 0.f, hi[e], lo[e]);
        w2b[0] = make_uint4(hi[0] | (uint32_t)hi[1] << 16, hi[2] | (uint32_t)hi[3] << 16, hi[4] | (uint32_t)hi[5] << 16,
                            hi[6] | (uint32_t)hi[7] << 16);
        w2b[1] = make_uint4(lo[0] | (uint32_t)lo[1] << 16, lo[2] | (uint32_t)lo[3] << 16, lo[4] | (uint32_t)lo[5] << 16,
                            lo[6] | (uint32_t)lo[7] << 16);
    }
    const float b1j = p.b1[16 * wave + l16];
    const float b2c = (wave < 2 && 16 * wave + l16 < p.C) ? p.b2[16 * wave + l16] : 0.f;

    f32x4 accW1[F / 16], accW2[2];
#pragma unroll
    for (int q = 0; q < F / 16; ++q) accW1[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    accW2[0] = accW2[1] = f32x4{0.f, 0.f, 0.f, 0.f};
    float db1p = 0.f, db2p = 0.f, lossp = 0.f;

    // h tile: thread t carries row t >> 5, features 8 (t & 31) .. + 7 (one 16-B piece)
    const int hr = tid >> 5, hc = 8 * (tid & 31);
    auto load_h = [&](int64_t t) -> uint4 {
        const int64_t m = t * TR + hr;
        return m < p.M ? *reinterpret_cast<const uint4*>(hb + m * p.ldh + hc) : make_uint4(0u, 0u, 0u, 0u);
    };
    int64_t t = blockIdx.x;
    uint4 hv = t < ntiles ? load_h(t) : make_uint4(0u, 0u, 0u, 0u);
    for (; t < ntiles; t += gridDim.x) {
        const int64_t m0 = t * TR;
        *reinterpret_cast<uint4*>(&HI[hr * RH + hc]) = hv;
        __syncthreads();  // B0: h tile (and, the first time, W1) staged; the previous tile's staging is stored
        if (t + gridDim.x < ntiles) hv = load_h(t + gridDim.x);

        // A: z = h W1^T + b1, wave w: hidden columns 16 w + l16; rows 4 g + r
        float dsc[4];
        {
            f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
            const uint16_t* ha = &HI[l16 * RH + 8 * g];
            const uint16_t* wh = &W1P[(16 * wave + l16) * RW1 + 8 * g];
#pragma unroll
            for (int s = 0; s < F / 32; ++s) {
                const uint4 a = *reinterpret_cast<const uint4*>(ha + 32 * s);
                const uint4 bh = *reinterpret_cast<const uint4*>(wh + 32 * s);
                const uint4 bl = *reinterpret_cast<const uint4*>(wh + H * RW1 + 32 * s);
                acc = mfma32(a, bl, acc);
                acc = mfma32(a, bh, acc);
            }
            const int j = 16 * wave + l16;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 4 * g + r;
                const float z = acc[r] + b1j;
                bool keep = z > 0.f;
                if (p.drop_thr) keep = keep && (drop_hash(seed, m0 + row, j, H) >> 8) >= p.drop_thr;
                dsc[r] = keep ? ik : 0.f;
                const float a = keep ? (p.drop_thr ? z * p.inv_keep : z) : 0.f;
                uint16_t hi, lo;
                split2(a, hi, lo);
                AI[row * RA + j] = hi;
                AI[TR * RA + row * RA + j] = lo;
            }
        }
        __syncthreads();  // B1

        // B: logits = a W2^T + b2 (waves 0, 1)
        if (wave < 2) {
            f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
            const uint16_t* aa = &AI[l16 * RA + 8 * g];
#pragma unroll
            for (int s = 0; s < H / 32; ++s) {
                const uint4 ah = *reinterpret_cast<const uint4*>(aa + 32 * s);
                const uint4 al = *reinterpret_cast<const uint4*>(aa + TR * RA + 32 * s);
                acc = mfma32(al, w2t[0][s], acc);
                acc = mfma32(ah, w2t[1][s], acc);
                acc = mfma32(ah, w2t[0][s], acc);
            }
            const int c = 16 * wave + l16;
            float* lf = reinterpret_cast<float*>(LF);
#pragma unroll
            for (int r = 0; r < 4; ++r) lf[(4 * g + r) * RL + c] = acc[r] + b2c;
        }
        __syncthreads();  // B2

        // C: log-softmax, loss, dl (thread: row tid >> 5, class tid & 31); dl (hi, lo) replaces the row's logits
        {
            const int row = tid >> 5, c = tid & 31;
            const int64_t m = m0 + row;
            const bool ok = m < p.M;
            const int64_t yl = ok ? p.y[m] : -1;
            if (ok && c == 0 && (yl < 0 || yl >= p.C)) lossp += __builtin_nanf("");  // as head_train_kernel
            float* lrow = reinterpret_cast<float*>(LF + row * RL * 4);
            const float x = c < p.C ? lrow[c] : -INFINITY;
            float mx = x;
#pragma unroll
            for (int o = 16; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 32));
            float se = c < p.C ? expf(x - mx) : 0.f;
#pragma unroll
            for (int o = 16; o > 0; o >>= 1) se += __shfl_xor(se, o, 32);
            const float lse = logf(se);
            float dl = 0.f;
            if (ok && c < p.C) {
                const float lp = (x - mx) - lse;
                if (c == (int)yl) lossp -= lp;
                dl = (expf(lp) - (c == (int)yl ? 1.f : 0.f)) * (gscale * p.lw);
            }
            db2p += dl;
            uint16_t hi, lo;
            split2(dl, hi, lo);
            uint16_t* drow = reinterpret_cast<uint16_t*>(lrow);
            drow[c] = hi;
            drow[32 + c] = lo;
        }
        __syncthreads();  // B3

        // D: dW2 += dl^T a: rows c (class tiles 0, 1), K = the tile's 16 rows, columns j = 16 w ..
        {
            const uint16_t* dlt = reinterpret_cast<const uint16_t*>(LF + (4 * g + tq) * RL * 4) + 4 * tp;
            const uint16_t* at = &AI[(4 * g + tq) * RA + 16 * wave + 4 * tp];
            const s16x4 ah = tr16(at), al = tr16(at + TR * RA);
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                const s16x4 dh_ = tr16(dlt + 16 * ct), dlo = tr16(dlt + 32 + 16 * ct);
                accW2[ct] = mfma16k(dlo, ah, accW2[ct]);
                accW2[ct] = mfma16k(dh_, al, accW2[ct]);
                accW2[ct] = mfma16k(dh_, ah, accW2[ct]);
            }
        }
        // D2: da = (dl W2) * dropout / relu mask: rows 4 g + r, column j = 16 w + l16, K = the 32 classes
        {
            const uint16_t* drow = reinterpret_cast<const uint16_t*>(LF + l16 * RL * 4) + 8 * g;
            const uint4 dh_ = *reinterpret_cast<const uint4*>(drow), dlo = *reinterpret_cast<const uint4*>(drow + 32);
            f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
            acc = mfma32(dlo, w2b[0], acc);
            acc = mfma32(dh_, w2b[1], acc);
            acc = mfma32(dh_, w2b[0], acc);
            const int j = 16 * wave + l16;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float da = acc[r] * dsc[r];
                db1p += da;
                uint16_t hi, lo;
                split2(da, hi, lo);
                DI[(4 * g + r) * RA + j] = hi;
                DI[TR * RA + (4 * g + r) * RA + j] = lo;
            }
        }
        __syncthreads();  // B4: da staged; a is dead (its image becomes the dh staging)

        // E: dh = da W1, wave w: features 16 (2 w + u) + l16, rows 4 g + r; K = hidden j (W1 rows, transposed reads)
        {
            f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
            const uint16_t* da = &DI[l16 * RA + 8 * g];
#pragma unroll
            for (int s = 0; s < H / 32; ++s) {
                const uint4 ah = *reinterpret_cast<const uint4*>(da + 32 * s);
                const uint4 al = *reinterpret_cast<const uint4*>(da + TR * RA + 32 * s);
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const uint16_t* wb = &W1P[(32 * s + 8 * g + tq) * RW1 + 16 * (2 * wave + u) + 4 * tp];
                    const uint4 bh = cat8(tr16(wb), tr16(wb + 4 * RW1));
                    const uint4 bl = cat8(tr16(wb + H * RW1), tr16(wb + H * RW1 + 4 * RW1));
                    acc[u] = mfma32(al, bh, acc[u]);
                    acc[u] = mfma32(ah, bl, acc[u]);
                    acc[u] = mfma32(ah, bh, acc[u]);
                }
            }
            uint16_t* st = AI;  // [TR][F] bf16
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    st[(4 * g + r) * F + 16 * (2 * wave + u) + l16] = __builtin_bit_cast(uint16_t, (__bf16)acc[u][r]);
        }
        // F: dW1 += da^T h: rows j = 16 w + .., columns f, K = the tile's 16 rows
        {
            const uint16_t* dt = &DI[(4 * g + tq) * RA + 16 * wave + 4 * tp];
            const s16x4 dh_ = tr16(dt), dlo = tr16(dt + TR * RA);
            const uint16_t* ht = &HI[(4 * g + tq) * RH + 4 * tp];
#pragma unroll
            for (int ft = 0; ft < F / 16; ++ft) {
                const s16x4 hx = tr16(ht + 16 * ft);
                accW1[ft] = mfma16k(dlo, hx, accW1[ft]);
                accW1[ft] = mfma16k(dh_, hx, accW1[ft]);
            }
        }
        __syncthreads();  // B5: dh staged; h and da read
        {
            const int64_t m = m0 + hr;
            if (m < p.M)
                *reinterpret_cast<uint4*>(dhb + m * p.lddh + hc) = *reinterpret_cast<const uint4*>(&AI[hr * F + hc]);
        }
    }

    // this workgroup's partial: dW1 rows 16 w + 4 g + r, columns 16 ft + l16; dW2 rows 16 ct + 4 g + r, columns
    // 16 w + l16; db1 (column j = 16 w + l16: the four row groups g in order); db2 (classes: the 16 rows in order)
    float* out = p.part + (int64_t)blockIdx.x * P_STRIDE;
#pragma unroll
    for (int ft = 0; ft < F / 16; ++ft)
#pragma unroll
        for (int r = 0; r < 4; ++r) out[P_DW1 + (16 * wave + 4 * g + r) * F + 16 * ft + l16] = accW1[ft][r];
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int r = 0; r < 4; ++r) out[P_DW2 + (16 * ct + 4 * g + r) * H + 16 * wave + l16] = accW2[ct][r];
    __syncthreads();
    float* red = reinterpret_cast<float*>(LF);  // [16][32] scratch (the tile loop is done with it)
    __shared__ float redw[NT / 64];
    if (tid < 256) red[tid] = 0.f;
    __syncthreads();
    {  // db1: g = 0..3 in order
        for (int gg = 0; gg < 4; ++gg) {
            if (g == gg) red[16 * wave + l16] += db1p;
            __syncthreads();
        }
        if (tid < H) out[P_DB1 + tid] = red[tid];
        __syncthreads();
        red[tid] = db2p;  // db2: thread (row tid >> 5, class tid & 31)
        __syncthreads();
        if (tid < TC) {
            float s_ = 0.f;
            for (int r = 0; r < TR; ++r) s_ += red[r * 32 + tid];
            out[P_DB2 + tid] = s_;
        }
    }
    float v = lossp;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    if (lane == 0) redw[wave] = v;
    __syncthreads();
    if (tid == 0) {
        float s_ = 0.f;
        for (int w = 0; w < NT / 64; ++w) s_ += redw[w];
        out[P_LOSS] = s_ * p.lw;
    }
}

// the F = 256 partials summed as head_train_reduce_kernel does for F = 128
__global__ __launch_bounds__(256) void head_train5_reduce_kernel(int nparts, int C, const float* part, float* grads,
                                                                 float* loss) {
    using namespace h5;
    __shared__ float acc_s[8][32];
    const int c = threadIdx.x & 31, grp = threadIdx.x >> 5;
    const int i = blockIdx.x * 32 + c;
    float s = 0.f;
    if (i <= P_LOSS)
        for (int b = grp; b < nparts; b += 8) s += part[(int64_t)b * P_STRIDE + i];
    acc_s[grp][c] = s;
    __syncthreads();
    if (grp != 0 || i > P_LOSS) return;
    s = acc_s[0][c];
    for (int g = 1; g < 8; ++g) s += acc_s[g][c];
    if (i < P_DW2) grads[i] = s;
    else if (i < P_DB2) { if ((i - P_DW2) / H < C) grads[i] = s; }
    else if (i < P_LOSS) { if (i - P_DB2 < C) grads[P_DW2 + C * H + (i - P_DB2)] = s; }
    else loss[0] = s;
}

int grid5(int64_t M) {
    const int64_t ntiles = (M + h5::TR - 1) / h5::TR;
    return (int)std::max<int64_t>(1, std::min<int64_t>(ntiles, 256));
}

}  // namespace

extern "C" {

int64_t pg_head_train_bf16_workspace(int64_t M, int64_t F, int64_t H, int64_t C) {
    if (M < 0 || F != h5::F || H != h5::H || C < 1 || C > TC) return -1;
    return (int64_t)grid5(M) * h5::P_STRIDE;
}

int pg_head_train_bf16(int64_t M, int64_t F, int64_t H, int64_t C, const uint16_t* h, int64_t ldh, const float* W1,
                       const float* b1, const float* W2, const float* b2, const int64_t* y, float loss_weight,
                       float drop_p, const int64_t* seed, const float* grad_scale, uint16_t* dh, int64_t lddh,
                       float* grads, float* loss, float* work, int64_t work_floats, void* stream) {
    if (F != h5::F || H != h5::H || C < 1 || C > TC)
        return pg::set_error(PG_ERR_UNSUPPORTED, "pg_head_train_bf16: F = 256, H = 128, C <= 32 only");
    PG_REQUIRE(M >= 0 && h && W1 && b1 && W2 && b2 && y && dh && grads && loss && work, "null argument");
    PG_REQUIRE(ldh >= F && lddh >= F && ldh % 8 == 0 && lddh % 8 == 0 && pg::aligned16(h) && pg::aligned16(dh),
               "h, dh: 16-B aligned bf16 rows of F elements");
    PG_REQUIRE(pg::aligned16(W1), "W1: 16-B aligned");
    PG_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "drop_p in [0, 1)");
    PG_REQUIRE(drop_p == 0.f || seed, "dropout needs a seed");
    PG_REQUIRE(work_floats >= pg_head_train_bf16_workspace(M, F, H, C), "workspace too small");
    HeadTrainP p{};
    p.M = M;
    p.C = (int)C;
    p.ldh = ldh;
    p.W1 = W1;
    p.b1 = b1;
    p.W2 = W2;
    p.b2 = b2;
    p.y = y;
    p.lw = loss_weight;
    p.drop_thr = drop_p > 0.f ? (uint32_t)std::min(16777215.0, std::ceil((double)drop_p * 16777216.0)) : 0u;
    p.inv_keep = drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.f;
    p.seed = seed;
    p.scale = grad_scale;
    p.lddh = lddh;
    p.part = work;
    hipStream_t s = (hipStream_t)stream;
    static bool attr_set = false;  // dynamic LDS above the 64 KiB default (set once; idempotent)
    if (!attr_set) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(head_train5_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, h5::LDS_BYTES) != hipSuccess)
            return pg::set_error(PG_ERR_HIP, "pg_head_train_bf16: cannot raise the LDS limit");
        attr_set = true;
    }
    const int grid = grid5(M);
    hipLaunchKernelGGL(head_train5_kernel, dim3((unsigned)grid), dim3(NT), h5::LDS_BYTES, s, p, h, dh);
    hipLaunchKernelGGL(head_train5_reduce_kernel, dim3((h5::P_LOSS + 1 + 31) / 32), dim3(256), 0, s, grid, (int)C,
                       (const float*)p.part, grads, loss);
    return pg::check_launch("pg_head_train_bf16");
}

int64_t pg_head_train_workspace(int64_t M, int64_t F, int64_t H, int64_t C) {
    if (M < 0 || !shape_ok(F, H, C)) return -1;
    return (int64_t)grid_of<128>(M) * HT<128>::P_STRIDE;
}

int pg_head_train_f32(int64_t M, int64_t F, int64_t H, int64_t C, const float* h, int64_t ldh, const float* W1,
                      const float* b1, const float* W2, const float* b2, const int64_t* y, float loss_weight,
                      float drop_p, const int64_t* seed, const float* grad_scale, float* dh, int64_t lddh,
                      float* grads, float* loss, float* work, int64_t work_floats, void* stream) {
    if (!shape_ok(F, H, C))
        return pg::set_error(PG_ERR_UNSUPPORTED, "pg_head_train_f32: F = 128, H = 64, C <= 32 only");
    PG_REQUIRE(M >= 0 && h && W1 && b1 && W2 && b2 && y && dh && grads && loss && work, "null argument");
    PG_REQUIRE(ldh >= F && lddh >= F && ldh % 4 == 0 && pg::aligned16(h), "h: aligned rows of F floats");
    PG_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "drop_p in [0, 1)");
    PG_REQUIRE(drop_p == 0.f || seed, "dropout needs a seed");
    PG_REQUIRE(work_floats >= pg_head_train_workspace(M, F, H, C), "workspace too small");
    HeadTrainP p{};
    p.M = M;
    p.C = (int)C;
    p.h = h;
    p.ldh = ldh;
    p.W1 = W1;
    p.b1 = b1;
    p.W2 = W2;
    p.b2 = b2;
    p.y = y;
    p.lw = loss_weight;
    p.drop_thr = drop_p > 0.f ? (uint32_t)std::min(16777215.0, std::ceil((double)drop_p * 16777216.0)) : 0u;
    p.inv_keep = drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.f;
    p.seed = seed;
    p.scale = grad_scale;
    p.dh = dh;
    p.lddh = lddh;
    p.part = work;
    hipStream_t s = (hipStream_t)stream;
    return launch<128>(p, C, grads, loss, s);
}

}  // extern "C"
