// Transposed middle-tile propagation of one middle-partition rank (shard.MiddleTrainer's backward; the autograd of
// protgram_directgcn.py:101-112 restricted to the rank's owned rows): dX = sum_k A_k^T G_k with G = dZ of the OWNED
// rows only. A rank holds the rows a.M.b of its middles M; A_k[a.M.b, .] reads the out-sources M.b.c (prefix M),
// the in-sources c.a.M (suffix M) and the row itself (pg_ngram_mid.hip, forward). So the transpose sends each owned
// middle's gradient to exactly three row sets, every row of which is reached from ONE middle of the rank:
//   P[M.b.c, f] = sum_{k,a} Wout_k[a,b,c] G_k[a.M.b, f]     (per b: a 20 x 60 x 16 product, rows c, K = (k, a))
//   S[c.a.M, f] = sum_{k,b} Win_k[a,b,c]  G_k[a.M.b, f]     (per a: the same with K = (k, b))
//   D[a.M.b, f] = sum_k Wdiag_k[a,b] G_k[a.M.b, f]
// The kernel writes the three parts as separate fp32 row blocks of T [3 * n_own, ldt] (no atomics, one writer per
// row: deterministic), each middle-major in its own order:
//   D: row        l*400 + a*20 + b  (= the owned-row order of G)
//   P: n_own   +  l*400 + b*20 + c
//   S: 2 n_own +  l*400 + c*20 + a
// (l = the middle's position in the rank's range). A global row may be reached by two or three parts (a ghost row
// by P and S of different middles; an owned row by D and, when its prefix / suffix middle is owned too, P / S):
// the caller sums them per row with pg_rows_gather_sum, which also folds in the rows received from the other ranks.
//
// Work unit: (middle, direction, group of cpw 16-feature chunks), one workgroup of 8 waves. The direction's 40
// output tiles of 16 rows c (two per b or a: c = 0..15, 16..31 with 20..31 zero weights) x 16 features are dealt 5
// per wave; their MFMA A fragments (the weights, W^T[c][K]) stay in registers for all chunks of the group, loaded
// once from the scatter plan (pg_ngram_scatter_plan: the forward plan re-laid in that fragment order, lane-
// contiguous 256-B fragments). The B fragments (G rows, K = 60 rows (k, a) or (k, b)) come from an LDS image of the
// middle's 400 x 3 row chunks, written in the direction's order [row K][column b or a][16 f] (row-group stride
// padded so that the four K-rows of one MFMA step hit disjoint banks), and refilled per chunk from registers that
// were loaded one chunk ahead. The out-direction workgroups also write D.
#include "pg_bf16_util.h"
#include "pg_common.h"

namespace {

typedef float f4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u4_t __attribute__((ext_vector_type(4)));

constexpr int SK = 20;                        // alphabet (the plan is sized for K = 20)
constexpr int SR = SK * SK;                   // rows per middle
constexpr int SSTEP = 3 * SK / 4;             // K-steps of 4 over the 60 rows (k, x)
constexpr int SDIR = SK * 2 * SSTEP * 64;     // fragments per direction: [col][ct][s][lane] = 38,400 floats
constexpr int SDG = 2 * SDIR;                 // diagonal weights [a][b][k]
constexpr int SMB = SDG + SR * 3;             // floats per middle: 78,000
constexpr int SWAVES = 8;
constexpr int STHREADS = 64 * SWAVES;
constexpr int STPW = SK * 2 / SWAVES;         // tiles per wave: 5
constexpr int SOOB = 1 << 30;                 // a buffer-store offset past every descriptor's range: dropped
// forward plan (pg_ngram_mid.hip): out [b][m][s][lane], in [a][m][s][lane], diag [a][b][k]; 52,400 floats
constexpr int FPI = SK * 4 * 5 * 64, FPD = 2 * FPI, FMB = FPD + SR * 3;

struct SP {
    const float* splan;
    const void* G;
    int64_t ldg;      // elements
    float* T;
    int64_t ldt;      // elements
    int64_t n_own;    // n_mid * 400
    int F, nch, cpw, ngrp, remap;
    int exp;          // diagnostics build only (PG_SCATTER_EXP): bits skip phases (0 MFMA + B reads, 1 stores, 2 D, 3 DMA)
};
#ifdef PG_SCATTER_EXP
#define SEXP(bit) ((p.exp >> (bit)) & 1)
#else
#define SEXP(bit) 0
#endif

// LDS-DMA of one 16-B piece per lane (global_load_lds_dwordx4: lane i's 16 B land at M0 + 16 i), as inline asm so
// that the compiler's wait insertion does not see it (the builtin form makes it wait for every outstanding
// vector-memory operation at control-flow joins); the kernel counts these operations itself. M0 saved and restored.
__device__ __forceinline__ void dma16(const void* src, uint32_t lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds)
                 : "memory");
}

// s_waitcnt vmcnt(n) for a wave-uniform n in 0..24
__device__ __forceinline__ void vm_wait(int n) {
    switch (n) {
#define PG_VMW(k)                                                  \
    case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); \
        break;
        PG_VMW(0) PG_VMW(20)
#undef PG_VMW
        default: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    }
}

template <bool BF>
struct SL {
    static constexpr int ES = BF ? 2 : 4;
    static constexpr int RB = 16 * ES;                  // bytes per 16-feature row chunk
    static constexpr int PPS = RB / 16;                 // 16-B pieces per row chunk
    static constexpr int ROWB = (SK + 1) * RB;          // bytes per K-row: 20 columns + 1 pad column (bank offset)
    static constexpr int PPR = ROWB / 16;               // pieces per K-row (the pad column's pieces fetch a dummy)
    static constexpr int NPC = 3 * SK * PPR;            // pieces per chunk image
    static constexpr int NI = (NPC + 63) / 64;          // wave-instructions per image (the last may be partial)
    static constexpr int IMG = NI * 1024;               // bytes per image buffer (the partial tail lands in padding)
    static constexpr int NW = (NI + SWAVES - 1) / SWAVES;  // instructions per wave (max)
};
static_assert(2 * SL<false>::IMG <= 163840 && 2 * SL<true>::IMG <= 163840, "two chunk images exceed 160 KiB");

template <bool BF>
__global__ __launch_bounds__(STHREADS) void ngram_scatter_kernel(SP p) {
    using C = SL<BF>;
    using ET = std::conditional_t<BF, uint16_t, float>;
    constexpr int ES = C::ES, RB = C::RB, PPS = C::PPS, PPR = C::PPR, NI = C::NI, NW = C::NW;
    // two chunk images [K-row i = (k, x)][column (b or a), pad][16 f], double-buffered by chunk parity
    __shared__ __attribute__((aligned(1024))) char Gs[2 * C::IMG];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t lb = pg::xcd_logical_block(blockIdx.x, gridDim.x, p.remap != 0);
    const int per_mid = 2 * p.ngrp;                // neighbouring logical blocks share the middle (one XCD's L2)
    const int l = (int)(lb / per_mid);
    const int rem = (int)(lb - (int64_t)l * per_mid);
    const int d = rem & 1, grp = rem >> 1;         // direction 0: out (P, + D), 1: in (S)
    const int ch0 = grp * p.cpw, ch1 = min(p.nch, ch0 + p.cpw);
    if (ch0 >= ch1) return;                        // whole workgroup (uniform): no barrier pending

    // this wave's tiles t = wave + 8 j: column x = t >> 1 = (wave >> 1) + 4 j (b for out, a for in), ct = wave & 1
    const int q4 = lane >> 4, fl = lane & 15;
    const int ct = wave & 1, x0 = wave >> 1;
    float A[STPW][SSTEP];
    {
        const float* pw = p.splan + (int64_t)l * SMB + d * SDIR + lane;
#pragma unroll
        for (int j = 0; j < STPW; ++j)
#pragma unroll
            for (int s = 0; s < SSTEP; ++s) A[j][s] = pw[((wave + 8 * j) * SSTEP + s) * 64];
    }
    // this wave's DMA pieces: instruction n = wave + 8 u, piece P = 64 n + lane in LDS order -> K-row i, column x,
    // 16-B part h; out: i = (k, a), x = b; in: i = (k, b), x = a; G row a*20 + b, slice k. Pad-column pieces and the
    // last instruction's spare lanes fetch the middle's first piece (a valid address) into padding.
    const int nw = (NI - wave + SWAVES - 1) / SWAVES;  // wave-uniform: instructions of this wave
    int goff[NW];
#pragma unroll
    for (int u = 0; u < NW; ++u) {
        const int P = (wave + SWAVES * u) * 64 + lane;
        const int i = P / PPR, q = P - i * PPR;
        const int x = q / PPS, h = q - x * PPS;
        const int k = i / SK, y = i - k * SK;
        const int a = d == 0 ? y : x, b = d == 0 ? x : y;
        goff[u] = (P < C::NPC && x < SK) ? (int)((a * SK + b) * p.ldg + k * p.F + h * (16 / ES)) : 0;
    }
    const ET* gbase = reinterpret_cast<const ET*>(p.G) + (int64_t)l * SR * p.ldg;
    const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)Gs;
    auto dma = [&](int ch) {
        const ET* g = gbase + ch * 16;
        const uint32_t dst = lds0 + (uint32_t)((ch - ch0) & 1) * C::IMG + (uint32_t)wave * 1024;
#pragma unroll
        for (int u = 0; u < NW; ++u)
            if (u < nw) dma16(g + goff[u], dst + (uint32_t)(SWAVES * u) * 1024);
    };
    // out-direction D: items (row r, 4 features), weights of the item rows in registers
    constexpr int ND = (SR * 4 + STHREADS - 1) / STHREADS;
    float wd[ND][3];
    if (d == 0) {
#pragma unroll
        for (int u = 0; u < ND; ++u) {
            const int it = tid + u * STHREADS, r = min(it >> 2, SR - 1);
#pragma unroll
            for (int k = 0; k < 3; ++k) wd[u][k] = p.splan[(int64_t)l * SMB + SDG + r * 3 + k];
        }
    }
    // output rows of this lane's accumulator rows c = 16 ct + 4 q4 + r (valid: c < 20): descriptors over the
    // middle's 400 rows of its part (P for out, S for in) and of D, from block-uniform values
    const int ldt = (int)p.ldt;
    const int64_t tbase = (d == 0 ? p.n_own : 2 * p.n_own) + (int64_t)l * SR;
    const int nbytes = SR * ldt * 4;  // < 2^30 (host-checked)
    const auto rs_part = __builtin_amdgcn_make_buffer_rsrc(p.T + tbase * p.ldt, 0, nbytes, 0x00020000);
    const auto rs_diag = __builtin_amdgcn_make_buffer_rsrc(p.T + (int64_t)l * SR * p.ldt, 0, nbytes, 0x00020000);
    const int n_st = d == 0 ? STPW * 4 + ND : STPW * 4;  // vector-memory operations a wave issues per chunk after its DMA
    const int lane_lds = (q4 * C::ROWB + x0 * RB + fl * ES);  // + 4 s ROWB + 4 j RB

    if (!SEXP(3)) dma(ch0);
#pragma unroll 1
    for (int ch = ch0; ch < ch1; ++ch) {
        // chunk ch's DMA was issued before the previous chunk's stores: wait for it, not for them
        vm_wait(ch == ch0 ? 0 : n_st);
        __syncthreads();  // every wave's pieces of chunk ch landed; the other image is no longer read
        if (ch + 1 < ch1 && !SEXP(3)) dma(ch + 1);
        const char* img = Gs + ((ch - ch0) & 1) * C::IMG;
        f4_t acc[STPW];
#pragma unroll
        for (int j = 0; j < STPW; ++j) acc[j] = f4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < SSTEP; ++s) {
            if (SEXP(0)) break;
            float bv[STPW];
#pragma unroll
            for (int j = 0; j < STPW; ++j) {
                const char* q = img + lane_lds + 4 * s * C::ROWB + 4 * j * RB;
                if constexpr (BF) bv[j] = __uint_as_float((uint32_t)(*reinterpret_cast<const uint16_t*>(q)) << 16);
                else bv[j] = *reinterpret_cast<const float*>(q);
            }
#pragma unroll
            for (int j = 0; j < STPW; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(A[j][s], bv[j], acc[j], 0, 0, 0);
        }
        // stores through buffer descriptors over this middle's 400 rows of its part (and of D): the lanes of the
        // padding rows c >= 20 (and the D loop's spare items) get an offset past the range, which the hardware drops
        // -- every wave issues the same count of stores per chunk (n_st), which the wait above relies on
#pragma unroll
        for (int j = 0; j < STPW; ++j) {
            const int x = x0 + 4 * j;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int c = 16 * ct + 4 * q4 + r;
                const int row = d == 0 ? x * SK + c : c * SK + x;
                const int off = c < SK ? (row * ldt + ch * 16 + fl) * 4 : SOOB;
                if (!SEXP(1)) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[j][r]), rs_part, off, 0, 0);
            }
        }
        if (d == 0 && !SEXP(2)) {  // D rows: sum_k Wdiag_k[a, b] G_k[a.M.b, f] (out image: K-row (k, a), column b)
#pragma unroll
            for (int u = 0; u < ND; ++u) {
                const int it = tid + u * STHREADS;
                const int r = min(it >> 2, SR - 1), f4 = (it & 3) * 4;
                const int a = r / SK, b = r - a * SK;
                u4_t o;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float v = 0.f;
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        const char* q = img + (k * SK + a) * C::ROWB + b * RB + (f4 + e) * ES;
                        float gv;
                        if constexpr (BF) gv = __uint_as_float((uint32_t)(*reinterpret_cast<const uint16_t*>(q)) << 16);
                        else gv = *reinterpret_cast<const float*>(q);
                        v = __builtin_fmaf(wd[u][k], gv, v);
                    }
                    o[e] = __float_as_uint(v);
                }
                const int off = it < SR * 4 ? (r * ldt + ch * 16 + f4) * 4 : SOOB;
                if (!SEXP(1)) __builtin_amdgcn_raw_buffer_store_b128(o, rs_diag, off, 0, 0);
            }
        }
    }
}

// scatter plan of middles [m0, m0 + n_mid) from the forward middle plan: per middle [dir][x][ct][s][lane] fragments
// W^T[c = 16 ct + (lane & 15)][K = 4 s + (lane >> 4)] (0 for c >= 20), then the diagonal [a][b][k] copied
__global__ __launch_bounds__(256) void scatter_plan_kernel(const float* mplan, int64_t m0, int64_t n_mid, float* sp) {
    const int64_t total = n_mid * SMB;
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
        const int64_t l = t / SMB;
        const int e = (int)(t - l * SMB);
        const float* fm = mplan + (m0 + l) * FMB;
        float v = 0.f;
        if (e >= SDG) {
            v = fm[FPD + (e - SDG)];
        } else {
            const int dir = e / SDIR, q = e - dir * SDIR;
            const int lane = q & 63, s = (q >> 6) % SSTEP, xc = (q >> 6) / SSTEP;
            const int x = xc >> 1, ctl = xc & 1;
            const int c = 16 * ctl + (lane & 15), i = 4 * s + (lane >> 4);  // i = (k, a) out / (k, b) in: the forward row
            if (c < SK) {
                const int m = i >> 4, il = i & 15;
                v = fm[dir * FPI + ((x * 4 + m) * 5 + (c >> 2)) * 64 + il + 16 * (c & 3)];
            }
        }
        sp[t] = v;
    }
}

}  // namespace

extern "C" {

int pg_ngram_scatter_plan(int K, int n, const float* mplan, int64_t m0, int64_t n_mid, float* splan, void* stream) {
    PG_REQUIRE(K == SK, "pg_ngram_scatter_plan: the middle-tile kernels take K = 20 (got %d)", K);
    PG_REQUIRE(n >= 3 && n <= 7, "pg_ngram_scatter_plan: n-gram length %d outside 3..7", n);
    int64_t Kn2 = 1;
    for (int i = 0; i < n - 2; ++i) Kn2 *= K;
    PG_REQUIRE(m0 >= 0 && n_mid >= 0 && m0 + n_mid <= Kn2, "pg_ngram_scatter_plan: middles [%lld, %lld) outside [0, %lld)",
               (long long)m0, (long long)(m0 + n_mid), (long long)Kn2);
    if (n_mid == 0) return PG_OK;
    PG_REQUIRE(mplan && splan, "pg_ngram_scatter_plan: null pointer");
    const int64_t blocks = (n_mid * SMB + 255) / 256;
    hipLaunchKernelGGL(scatter_plan_kernel, dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(256), 0,
                       (hipStream_t)stream, mplan, m0, n_mid, splan);
    return pg::check_launch("pg_ngram_scatter_plan");
}

}  // extern "C"

namespace {

int grid_cap() {  // CUs of the current device (cached; immutable once read)
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

template <bool BF>
int scatter_launch(const float* splan, int64_t n_mid, const void* G, int64_t ldg, int64_t F, float* T, int64_t ldt,
                   uint32_t flags, void* stream, const char* name) {
    PG_REQUIRE(n_mid >= 0 && F >= 0, "%s: negative size", name);
    if (n_mid == 0 || F == 0) return PG_OK;
    PG_REQUIRE(splan && G && T, "%s: null pointer", name);
    PG_REQUIRE(F % 16 == 0, "%s: F = %lld must be a multiple of 16", name, (long long)F);
    PG_REQUIRE(ldg >= 3 * F && ldt >= F, "%s: row strides smaller than the rows", name);
    PG_REQUIRE(ldg % (BF ? 8 : 4) == 0 && pg::aligned16(G) && pg::aligned16(T) && ldt % 4 == 0,
               "%s: G rows must be 16-B aligned pieces (ldg %% %d == 0, 16-B base) and T 16-B aligned", name, BF ? 8 : 4);
    PG_REQUIRE((int64_t)SR * ldg < (int64_t)1 << 31, "%s: a middle's G rows exceed 2^31 elements", name);
    PG_REQUIRE((int64_t)SR * ldt * 4 < (int64_t)1 << 30, "%s: a middle's T rows exceed 2^30 bytes", name);
    SP p;
    p.splan = splan;
    p.G = G;
    p.ldg = ldg;
    p.T = T;
    p.ldt = ldt;
    p.n_own = n_mid * SR;
    p.F = (int)F;
    p.nch = (int)(F / 16);
    // chunks per workgroup: the (middle, direction) pairs' chunks split into as many equal groups as one round of
    // workgroups (one per CU: the kernel's registers allow one) holds, at least one group per pair (more pairs than
    // CUs: whole pairs, several rounds). A workgroup loads its pair's weights once, so fewer, longer groups amortise
    // them; measured at config 5's rank shapes (50 middles, F = 256): 8 chunks (200 workgroups) 49.6 us, 4 chunks
    // 54.3, 2 chunks 60.2, 16 chunks (100 workgroups) 76.2, a persistent walker over the item stream with weight
    // reloads at pair changes (256 workgroups) 59.0
    const int64_t pairs = n_mid * 2;
    int64_t groups = grid_cap() / pairs;
    groups = groups < 1 ? 1 : (groups > p.nch ? p.nch : groups);
    int64_t cpw = (p.nch + groups - 1) / groups;
    int64_t forced = (flags >> PG_FLAG_SCATTER_CPW_SHIFT) & 31;
#ifdef PG_SCATTER_EXP
    p.exp = (int)forced;  // the diagnostics build reads bits 24..28 as phase skips, at 8 chunks per workgroup
    forced = 8;
#else
    p.exp = 0;
#endif
    if (forced) cpw = forced;
    cpw = cpw < 1 ? 1 : (cpw > p.nch ? p.nch : cpw);
    p.cpw = (int)cpw;
    p.ngrp = (int)((p.nch + cpw - 1) / cpw);
    p.remap = (flags & PG_FLAG_NO_XCD_REMAP) ? 0 : 1;
    const int64_t blocks = n_mid * 2 * p.ngrp;
    PG_REQUIRE(blocks < ((int64_t)1 << 31), "%s: grid too large", name);
    hipLaunchKernelGGL(ngram_scatter_kernel<BF>, dim3((unsigned)blocks), dim3(STHREADS), 0, (hipStream_t)stream, p);
    return pg::check_launch(name);
}

}  // namespace

extern "C" {

int pg_spmm3t_ngram_scatter_f32(const float* splan, int64_t n_mid, const float* G, int64_t ldg, int64_t F, float* T,
                                int64_t ldt, uint32_t flags, void* stream) {
    return scatter_launch<false>(splan, n_mid, G, ldg, F, T, ldt, flags, stream, "pg_spmm3t_ngram_scatter_f32");
}

int pg_spmm3t_ngram_scatter_bf16(const float* splan, int64_t n_mid, const uint16_t* G, int64_t ldg, int64_t F,
                                 float* T, int64_t ldt, uint32_t flags, void* stream) {
    return scatter_launch<true>(splan, n_mid, G, ldg, F, T, ldt, flags, stream, "pg_spmm3t_ngram_scatter_bf16");
}

}  // extern "C"
