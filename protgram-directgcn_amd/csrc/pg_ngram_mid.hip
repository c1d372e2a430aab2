// N-gram MIDDLE-tile propagation on the fp32 matrix cores (gfx950 v_mfma_f32_16x16x4_f32): the three DirectGCN
// aggregates of a graph over all K^n n-grams, one middle (n-2)-gram at a time.
//
// Structure (pg_ngram_spmm.hip has the derivation): row i = a.M.b (a = first letter, M = the middle
// n-2 letters, b = last letter). Its out-sources are M.b.c, its in-sources c.a.M (c = 0..K-1). For one middle M and
// one 16-feature column chunk f:
//   out-phase, per b:  P[(k, a), f] = sum_c Wout_k[a, b, c] X[M.b.c, f]      a GEMM (3K rows (k,a)) x (K) x (16)
//   in-phase,  per a:  Z[(k, b), f] = P[(k, a) of b] + sum_c Win_k[a, b, c] X[c.a.M, f] + Wdiag_k[a, b] X[a.M.b, f]
// Each phase is 20 dense 60 x 20 x 16 products (rows padded to 64): 80 MFMA tiles of 16 x 16 (K = 20 = 5 steps of
// 4), shared by 8 compute waves (10 tiles each). The out-phase results are handed to the in-phase through an LDS
// partial buffer laid out in the in-phase's accumulator order (the two phases group the rows differently: by b, then
// by a), read back as the in-phase MFMAs' initial accumulators.
//
// Operands: the weights are the MFMA A fragments, loaded ONCE per work item into registers (the plan is stored in
// fragment order, 256 B per fragment: one coalesced dword per lane) and reused for every column chunk of the item;
// the source rows are the B fragments, read from LDS, where two loader waves bring each chunk's 800 source rows and
// 400 self rows by LDS-DMA (64 B per row chunk), one phase ahead of their use. A work item is (M, group of NCG
// consecutive 16-feature chunks); the kernel is persistent (one workgroup of 8 compute + 2 loader waves per CU).
//
// Plan layout (pg_ngram_mplan_f32, built from the CSR; slot rules as pg_ngram_plan_f32: an entry goes to its
// out-slot, else its in-slot, else the diagonal; a missing transition leaves 0; an entry that fits no slot marks the
// plan invalid), per middle, XMB floats:
//   out  [b][m][s][lane]  lane l holds A[i = 16 m + (l & 15)][c = 4 s + (l >> 4)] = Wout_k[a, b, c], (k, a) = divmod(i, K)
//   in   [a][m][s][lane]  the same with (k, b) = divmod(i, K) and Win
//   diag [a][b][k]
// Rows i >= 3K are zero padding.
//
// Numerics: each aggregate is the same sum of w*x terms as the reference's propagate(), accumulated in fp32 by the
// MFMA (exact fp32 FMA chain, k-ordered: out-slots, in-slots, then the diagonal by a VALU FMA): within fp32 rounding
// of the reference (|d| <= 1e-5 + 1e-5|ref|), like pg_spmm3_ngram_f32. Zero weights add 0 * x: X must be finite.
#include "pg_common.h"

namespace {

typedef float f4_t __attribute__((ext_vector_type(4)));

constexpr int XK = 20;               // alphabet (the LDS image, the tile map and the plan are sized for K = 20)
constexpr int XR = XK * XK;          // rows per middle
constexpr int XCW = 8;               // compute waves
constexpr int XLW = 4;               // loader waves
constexpr int XTHREADS = 64 * (XCW + XLW);
constexpr int XTILES = 80;           // per phase: K (b or a) x 4 row tiles of 16 (3K = 60 rows, padded to 64)
constexpr int XTPW = XTILES / XCW;   // tiles per compute wave
constexpr int XS = XK / 4;           // K-steps of 4 per tile
constexpr int XFC = 16;              // features per column chunk
// plan
constexpr int XPO = 0;                              // out fragments
constexpr int XPI = XK * 4 * XS * 64;               // in fragments (25,600 floats after the out ones)
constexpr int XPD = 2 * XPI;                        // diagonal weights [a][b][k]
constexpr int XMB = XPD + XR * 3;                   // floats per middle: 52,400
// LDS image (bytes)
constexpr int LOUT = 0;                             // out-sources [b][c][16 f]   400 rows x 64 B
constexpr int LIN = LOUT + XR * 64;                 // in-sources  [a][c][16 f]
constexpr int LSELF = LIN + XR * 64;                // self rows   [a][b][16 f]
constexpr int LPART = LSELF + XR * 64;              // partial     [a][row k K + b (3K)][16 f] fp32
constexpr int LDIAG = LPART + XK * 3 * XK * 64;     // diagonal weights [a][b][k]
constexpr int LBYTES = LDIAG + XR * 3 * 4;          // 158,400 B
static_assert(LBYTES <= 163840, "LDS image exceeds 160 KiB");
static_assert(XTILES % XCW == 0 && XTPW % 2 == 0, "tiles per wave");

struct XP {
    int64_t Kn1, Kn2;      // K^(n-1), K^(n-2) (= number of middles)
    const float* plan;
    const float* X;
    int64_t ldx;
    float* Z;
    int64_t ldz;
    int F;
    int nch;               // F / 16
    int ncg;               // chunks per work item
    int ngrp;              // work items per middle = ceil(nch / ncg)
    int items;             // K^(n-2) * ngrp
    int remap;
    unsigned long long* stamps;  // diagnostics build only (PG_MID_STAMPS): s_memtime per block, chunk and point
};

#ifdef PG_MID_STAMPS
constexpr int XSTAMP_CH = 32, XSTAMP_PT = 8;
#define XSTAMP(ci, pt)                                                                                              \
    do {                                                                                                            \
        if (p.stamps && lane == 0 && (ci) < XSTAMP_CH)                                                              \
            p.stamps[((int64_t)blockIdx.x * 2 + (wave >= XCW)) * XSTAMP_CH * XSTAMP_PT + (ci) * XSTAMP_PT + (pt)] = \
                __builtin_amdgcn_s_memtime();                                                                       \
    } while (0)
#else
#define XSTAMP(ci, pt) \
    do {               \
    } while (0)
#endif

__device__ __forceinline__ void glds16(const float* src, const void* lds_base) {
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

struct Chunk {
    int M, ch, first;  // middle, chunk index, first chunk of its work item
};

__global__ __launch_bounds__(XTHREADS) void ngram_x_kernel(XP p) {
    extern __shared__ __attribute__((aligned(16))) char L[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int first = (int)pg::xcd_logical_block(blockIdx.x, gridDim.x, p.remap != 0);
    const int stride = gridDim.x;

    // the chunk stream of this workgroup: items first, first + stride, ..., each NCG chunks (fewer in a last group)
    auto chunk_at = [&](int item, int cc) -> Chunk {
        const int M = item / p.ngrp;
        const int g = item - M * p.ngrp;
        return Chunk{M, g * p.ncg + cc, cc == 0};
    };
    auto chunks_of = [&](int item) {
        const int g = item % p.ngrp;
        const int n = p.nch - g * p.ncg;
        return n < p.ncg ? n : p.ncg;
    };

    if (wave >= XCW) {  // ---------------- loader waves: LDS-DMA only (same barrier sequence as the compute waves)
        const int lw = wave - XCW;
        // one region of 400 rows x 64 B = 25 wave-instructions, split over the loader waves
        auto dma_rows = [&](int region, int kind, int M, int ch) {
            const float* xc = p.X + ch * XFC;
#pragma unroll 1
            for (int it = lw; it < XR * 4 / 64; it += XLW) {
                const int P = it * 64 + lane;
                const int rl = P >> 2, q = P & 3;
                const int u = rl / XK, v = rl - u * XK;
                int64_t row;
                if (kind == 0) row = (int64_t)M * XR + u * XK + v;                   // out: (b = u, c = v) -> M.b.c
                else if (kind == 1) row = v * p.Kn1 + u * p.Kn2 + M;                 // in:  (a = u, c = v) -> c.a.M
                else row = u * p.Kn1 + (int64_t)M * XK + v;                          // self: (a = u, b = v) -> a.M.b
                glds16(xc + row * p.ldx + q * 4, L + region + it * 1024);
            }
        };
        auto dma_diag = [&](int M) {  // 4,800 B = 300 pieces: wave-instructions 0..4 (the last one partial)
            const float* d = p.plan + (int64_t)M * XMB + XPD;
#pragma unroll 1
            for (int it = lw; it < 5; it += XLW) {
                const int P = it * 64 + lane;
                if (P < XR * 3 / 4) glds16(d + P * 4, L + LDIAG + it * 1024);
            }
        };
        int item = first, cc = 0;
        if (item < p.items) {
            const Chunk c0 = chunk_at(item, 0);
            dma_rows(LOUT, 0, c0.M, c0.ch);
            dma_rows(LIN, 1, c0.M, c0.ch);
            dma_rows(LSELF, 2, c0.M, c0.ch);
            dma_diag(c0.M);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_barrier" ::: "memory");  // S(-1)
        int ci = 0;
#pragma unroll 1
        while (item < p.items) {
            int nitem = item, ncc = cc + 1;  // next chunk of the stream
            if (ncc >= chunks_of(item)) {
                nitem = item + stride;
                ncc = 0;
            }
            const bool more = nitem < p.items;
            const Chunk nx = more ? chunk_at(nitem, ncc) : Chunk{0, 0, 0};
            XSTAMP(ci, 0);
            asm volatile("s_barrier" ::: "memory");  // M(t): out-phase done, partial written, out-region free
            XSTAMP(ci, 1);
            if (more) dma_rows(LOUT, 0, nx.M, nx.ch);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            XSTAMP(ci, 2);
            asm volatile("s_barrier" ::: "memory");  // S(t): in-phase done; in / self / diag / partial free
            XSTAMP(ci, 3);
            if (more) {
                dma_rows(LIN, 1, nx.M, nx.ch);
                dma_rows(LSELF, 2, nx.M, nx.ch);
                if (nx.first) dma_diag(nx.M);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            XSTAMP(ci, 4);
            item = nitem;
            cc = ncc;
            ++ci;
        }
        return;
    }

    // ---------------- compute waves
    // Tile assignment: wave w owns, in both phases, the row tile m = w & 3 of the columns b (out) / a (in) =
    // 2 j + (w >> 2), j = 0..9, so every LDS address below is a per-lane base plus a compile-time offset in j and s.
    const int q4 = lane >> 4, fl = lane & 15;
    const int mw = wave & 3, wb = wave >> 2;
    float Ao[XTPW][XS], Ai[XTPW][XS];  // A fragments of this wave's out / in tiles (item-resident)
    auto load_A = [&](int M) {
        const float* pm = p.plan + (int64_t)M * XMB + lane;
#pragma unroll
        for (int j = 0; j < XTPW; ++j) {
            const int t = (2 * j + wb) * 4 + mw;  // tile t = (b or a) * 4 + m
#pragma unroll
            for (int s = 0; s < XS; ++s) {
                Ao[j][s] = pm[XPO + (t * XS + s) * 64];
                Ai[j][s] = pm[XPI + (t * XS + s) * 64];
            }
        }
    };
    // this lane's four accumulator rows i = 16 mw + 4 q4 + r: (k, a) in the out-phase, (k, b) in the in-phase
    int rk[4], rv[4];
    bool rok[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = 16 * mw + 4 * q4 + r;
        rok[r] = i < 3 * XK;
        rk[r] = rok[r] ? i / XK : 0;
        rv[r] = rok[r] ? i - rk[r] * XK : 0;
    }
    // LDS byte offsets: sources [row][16 f] (64 B rows); partial [a][row k K + b][16 f]
    const int src_lane = (q4 * 16 + fl) * 4;                 // + (col * K + 4 s) * 64
    int part_w[4], part_r[4], self_r[4], diag_r[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        part_w[r] = LPART + ((rv[r] * 3 * XK + rk[r] * XK + wb) * 16 + fl) * 4;  // out: a = rv, row k K + b; + 2 j * 64
        part_r[r] = LPART + ((wb * 3 * XK + 16 * mw + 4 * q4 + r) * 16 + fl) * 4;  // in: + 2 j * 60 * 64
        self_r[r] = LSELF + ((wb * XK + rv[r]) * 16 + fl) * 4;                     // in: (a, b = rv); + 2 j * K * 64
        diag_r[r] = LDIAG + ((wb * XK + rv[r]) * 3 + rk[r]) * 4;                   // + 2 j * K * 12
    }
    asm volatile("s_barrier" ::: "memory");  // S(-1)
    int item = first, cc = 0, ci = 0;
#pragma unroll 1
    while (item < p.items) {
        const Chunk cu = chunk_at(item, cc);
        XSTAMP(ci, 0);
        if (cu.first) load_A(cu.M);
        // ---- out-phase: tiles (b = 2 j + wb, m = mw); hand-over of row (k, a) to the in-phase row k K + b of a
#pragma unroll
        for (int j = 0; j < XTPW; j += 2) {
            f4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < XS; ++s) {
                const float x0 = *reinterpret_cast<const float*>(L + LOUT + src_lane + ((2 * j + wb) * XK + 4 * s) * 64);
                const float x1 =
                    *reinterpret_cast<const float*>(L + LOUT + src_lane + ((2 * j + 2 + wb) * XK + 4 * s) * 64);
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(Ao[j][s], x0, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(Ao[j + 1][s], x1, acc1, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (rok[r]) {
                    *reinterpret_cast<float*>(L + part_w[r] + 2 * j * 64) = acc0[r];
                    *reinterpret_cast<float*>(L + part_w[r] + (2 * j + 2) * 64) = acc1[r];
                }
            asm volatile("" ::: "memory");
        }
        XSTAMP(ci, 1);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // M(t)
        XSTAMP(ci, 2);
        // ---- in-phase: tiles (a = 2 j + wb, m = mw): rows (k, b); initial accumulators from the partial buffer
        const int M = cu.M;
        float* zb[4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
            zb[r] = p.Z + ((int64_t)wb * p.Kn1 + (int64_t)M * XK + rv[r]) * p.ldz + (int64_t)rk[r] * p.F + cu.ch * XFC + fl;
        const int64_t zstep = 2 * p.Kn1 * p.ldz;  // a -> a + 2
#pragma unroll
        for (int j = 0; j < XTPW; j += 2) {
            f4_t acc0, acc1;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                acc0[r] = *reinterpret_cast<const float*>(L + part_r[r] + 2 * j * 3 * XK * 64);
                acc1[r] = *reinterpret_cast<const float*>(L + part_r[r] + (2 * j + 2) * 3 * XK * 64);
            }
#pragma unroll
            for (int s = 0; s < XS; ++s) {
                const float x0 = *reinterpret_cast<const float*>(L + LIN + src_lane + ((2 * j + wb) * XK + 4 * s) * 64);
                const float x1 =
                    *reinterpret_cast<const float*>(L + LIN + src_lane + ((2 * j + 2 + wb) * XK + 4 * s) * 64);
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(Ai[j][s], x0, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(Ai[j + 1][s], x1, acc1, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (rok[r]) {
                    const float w0 = *reinterpret_cast<const float*>(L + diag_r[r] + 2 * j * XK * 12);
                    const float w1 = *reinterpret_cast<const float*>(L + diag_r[r] + (2 * j + 2) * XK * 12);
                    const float s0 = *reinterpret_cast<const float*>(L + self_r[r] + 2 * j * XK * 64);
                    const float s1 = *reinterpret_cast<const float*>(L + self_r[r] + (2 * j + 2) * XK * 64);
                    zb[r][(int64_t)j * zstep] = __builtin_fmaf(w0, s0, acc0[r]);
                    zb[r][(int64_t)(j + 1) * zstep] = __builtin_fmaf(w1, s1, acc1[r]);
                }
            asm volatile("" ::: "memory");
        }
        XSTAMP(ci, 3);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // S(t)
        XSTAMP(ci, 4);
        ++ci;
        if (++cc >= chunks_of(item)) {
            item += stride;
            cc = 0;
        }
    }
}

// Plan construction: one thread per CSR row scatters its entries into the fragment-ordered slots.
__global__ __launch_bounds__(256) void ngram_mplan_kernel(int64_t Kn1, int64_t n_rows, const int64_t* rowptr,
                                                          const int4* edges, float* plan, int* bad) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n_rows) return;
    const int K = XK;
    const int a = (int)(i / Kn1), b = (int)(i % K);
    const int64_t M = (i % Kn1) / K;
    float* W = plan + M * XMB;
    const int64_t suffix = i % Kn1, prefix = i / K;
    for (int64_t e = rowptr[i]; e < rowptr[i + 1]; ++e) {
        const int4 rec = edges[e];
        const int64_t j = rec.x;
        const float w3[3] = {__int_as_float(rec.y), __int_as_float(rec.z), __int_as_float(rec.w)};
        int type, c;
        if (j / K == suffix) {
            type = 0;  // out-slot c = j mod K
            c = (int)(j % K);
        } else if (j % Kn1 == prefix) {
            type = 1;  // in-slot c = j div K^(n-1)
            c = (int)(j / Kn1);
        } else if (j == i) {
            type = 2;  // diagonal
            c = 0;
        } else {
            atomicAdd(bad, 1);
            continue;
        }
        for (int k = 0; k < 3; ++k) {
            int64_t off;
            if (type == 2) {
                off = XPD + ((int64_t)(a * K + b) * 3 + k);
            } else {
                const int grp = type == 0 ? b : a;           // out fragments per b, in fragments per a
                const int rr = k * K + (type == 0 ? a : b);  // tile row (k, a) / (k, b)
                const int m = rr >> 4, li = rr & 15;
                const int s = c >> 2, lk = c & 3;
                off = (type == 0 ? XPO : XPI) + ((int64_t)((grp * 4 + m) * XS + s) * 64 + lk * 16 + li);
            }
            W[off] = w3[k];
        }
    }
}

bool mid_shape(int K, int n, int64_t n_rows, int64_t& Kn1, int64_t& Kn2) {
    if (K != XK || n < 2 || n > 12) return false;
    int64_t v = 1;
    for (int t = 0; t < n; ++t) {
        if (v > (int64_t(1) << 40) / K) return false;
        v *= K;
    }
    if (v != n_rows) return false;
    Kn1 = n_rows / K;
    Kn2 = Kn1 / K;
    return true;
}

int grid_cap() {  // one persistent workgroup per CU (device-properties cache: immutable once read)
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (cus[dev] == 0) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
        cus[dev] = v;
    }
    return cus[dev];
}

}  // namespace

extern "C" {

int64_t pg_ngram_mplan_floats(int K, int n, int64_t n_rows) {
    int64_t Kn1 = 0, Kn2 = 0;
    if (!mid_shape(K, n, n_rows, Kn1, Kn2)) return -1;
    return Kn2 * XMB;
}

int pg_ngram_mplan_f32(int K, int n, int64_t n_rows, const int64_t* rowptr, const pg_edge3_t* edges, float* plan,
                       int64_t plan_floats, int* bad, void* stream) {
    int64_t Kn1 = 0, Kn2 = 0;
    PG_REQUIRE(mid_shape(K, n, n_rows, Kn1, Kn2), "n_rows %lld is not K^n with K = %d (K=%d, n=%d)", (long long)n_rows,
               XK, K, n);
    PG_REQUIRE(plan_floats >= pg_ngram_mplan_floats(K, n, n_rows), "plan buffer too small");
    PG_REQUIRE(rowptr && edges && plan && bad, "null pointer");
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(plan, 0, sizeof(float) * plan_floats, s) != hipSuccess ||
        hipMemsetAsync(bad, 0, sizeof(int), s) != hipSuccess)
        return pg::set_error(PG_ERR_HIP, "pg_ngram_mplan_f32: memset failed");
    hipLaunchKernelGGL(ngram_mplan_kernel, dim3((unsigned)((n_rows + 255) / 256)), dim3(256), 0, s, Kn1, n_rows, rowptr,
                       reinterpret_cast<const int4*>(edges), plan, bad);
    return pg::check_launch("pg_ngram_mplan_f32");
}

static int mid_launch(int K, int n, int64_t n_rows, const float* plan, const float* X, int64_t ldx, int64_t F,
                      const pg_layer_args_t* gates, float* Z, int64_t ldz, uint32_t flags, unsigned long long* stamps,
                      void* stream) {
    int64_t Kn1 = 0, Kn2 = 0;
    PG_REQUIRE(mid_shape(K, n, n_rows, Kn1, Kn2), "bad n-gram shape (K must be %d, n_rows = K^n)", XK);
    PG_REQUIRE(plan && X && Z, "null pointer");
    PG_REQUIRE(ldz >= 3 * F && ldx >= F, "leading dimensions too small");
    if (gates)
        return pg::set_error(PG_ERR_UNSUPPORTED, "pg_spmm3_ngram_mid_f32: no gated store (the dense kernel gates)");
    if (F <= 0 || F % XFC)
        return pg::set_error(PG_ERR_UNSUPPORTED, "pg_spmm3_ngram_mid_f32: F must be a multiple of %d", XFC);
    if (!pg::aligned16(X) || !pg::aligned16(plan) || (ldx * 4) % 16)
        return pg::set_error(PG_ERR_UNSUPPORTED, "pg_spmm3_ngram_mid_f32: needs 16-B aligned X rows");
    PG_REQUIRE(Kn2 * (F / XFC) < (int64_t(1) << 30), "too many work items");
    XP p{};
    p.Kn1 = Kn1;
    p.Kn2 = Kn2;
    p.plan = plan;
    p.X = X;
    p.ldx = ldx;
    p.Z = Z;
    p.ldz = ldz;
    p.F = (int)F;
    p.nch = (int)(F / XFC);
    // chunks per work item: the weights (A fragments) load once per item; smaller items balance the persistent grid
    const int req = (int)((flags >> 24) & 15u);
    p.ncg = req ? req : 4;
    if (p.ncg > p.nch) p.ncg = p.nch;
    p.ngrp = (p.nch + p.ncg - 1) / p.ncg;
    p.items = (int)(Kn2 * p.ngrp);
    p.remap = (flags & PG_FLAG_NO_XCD_REMAP) ? 0 : 1;
    p.stamps = stamps;
    const int64_t cap = grid_cap();
    const unsigned grid = (unsigned)(p.items < cap ? p.items : cap);
    hipStream_t s = (hipStream_t)stream;
    static bool attr_set = false;  // the kernel's dynamic LDS exceeds the 64 KiB default (set once; idempotent)
    if (!attr_set) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(ngram_x_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                                LBYTES) != hipSuccess)
            return pg::set_error(PG_ERR_HIP, "pg_spmm3_ngram_mid_f32: cannot raise the LDS limit");
        attr_set = true;
    }
    hipLaunchKernelGGL(ngram_x_kernel, dim3(grid), dim3(XTHREADS), LBYTES, s, p);
    return pg::check_launch("pg_spmm3_ngram_mid_f32");
}

int pg_spmm3_ngram_mid_f32(int K, int n, int64_t n_rows, const float* plan, const float* X, int64_t ldx, int64_t F,
                           const pg_layer_args_t* gates, float* Z, int64_t ldz, uint32_t flags, void* stream) {
    return mid_launch(K, n, n_rows, plan, X, ldx, F, gates, Z, ldz, flags, nullptr, stream);
}

#ifdef PG_MID_STAMPS
// diagnostics library only (tools/mid_stamps.py): the same launch with per-block time stamps
int pg_mid_stamped(int K, int n, int64_t n_rows, const float* plan, const float* X, int64_t ldx, int64_t F, float* Z,
                   int64_t ldz, uint32_t flags, unsigned long long* stamps, void* stream) {
    return mid_launch(K, n, n_rows, plan, X, ldx, F, nullptr, Z, ldz, flags, stamps, stream);
}
#endif
}  // extern "C"
