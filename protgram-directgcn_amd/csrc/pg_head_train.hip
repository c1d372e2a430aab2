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

}  // namespace

extern "C" {

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
