// N-gram MIDDLE-tile propagation on the fp32 matrix cores (gfx950 v_mfma_f32_16x16x4_f32): the three DirectGCN
// aggregates of a graph over all K^n n-grams, one middle (n-2)-gram at a time.
//
// Structure (pg_ngram_spmm.hip has the derivation): row i = a.M.b (a = first letter, M = the middle
// n-2 letters, b = last letter). Its out-sources are M.b.c, its in-sources c.a.M (c = 0..K-1). For one middle M and
// one 16-feature column chunk f:
//   out-phase, per b:  P[(k, a), f] = sum_c Wout_k[a, b, c] X[M.b.c, f] + Wdiag_k[a, b] X[a.M.b, f]
//                      (a GEMM (3K rows (k,a)) x (K) x (16), plus the diagonal by a VALU FMA)
//   in-phase,  per a:  Z[(k, b), f] = P[(k, a) of b] + sum_c Win_k[a, b, c] X[c.a.M, f]
// Each phase is 20 dense 60 x 20 x 16 products (rows padded to 64): 80 MFMA tiles of 16 x 16 (K = 20 = 5 steps of
// 4), shared by 8 compute waves (10 tiles each). The out-phase results are handed to the in-phase through an LDS
// partial buffer laid out in the in-phase's accumulator order (the two phases group the rows differently: by b, then
// by a), read back as the in-phase MFMAs' initial accumulators.
//
// Operands: the weights are the MFMA A fragments, loaded into registers once per middle a workgroup visits (the plan is stored in
// fragment order, 256 B per fragment: one coalesced dword per lane) and reused for every column chunk of it;
// the source rows are the B fragments, read from LDS, where four loader waves bring each chunk's 800 source rows and
// 400 self rows by LDS-DMA (64 B per row chunk), one phase ahead of their use. The kernel is persistent (one workgroup
// of 8 compute + 4 loader waves per CU), each workgroup walking a contiguous range of the (middle, 16-feature chunk)
// stream.
//
// Plan layout (pg_ngram_mplan_f32, built from the CSR; slot rules as pg_ngram_plan_f32: an entry goes to its
// out-slot, else its in-slot, else the diagonal; a missing transition leaves 0; an entry that fits no slot marks the
// plan invalid), per middle, XMB floats:
//   out  [b][m][s][lane]  lane l holds A[i = 16 m + (l & 15)][c = 4 s + (l >> 4)] = Wout_k[a, b, c], (k, a) = divmod(i, K)
//   in   [a][m][s][lane]  the same with (k, b) = divmod(i, K) and Win
//   diag [a][b][k]
// The padding rows i = 3K..3K+3 (60..63) repeat rows 56..59 (the compute waves' lanes of those rows then need no
// branch: they write what the lanes of rows 56..59 write).
//
// Numerics: each aggregate is the same sum of w*x terms as the reference's propagate(), accumulated in fp32 (the
// MFMA sums in groups of 4 c: out-slots, then the diagonal by a VALU FMA, then in-slots) in another order than the
// reference's scatter_add: within fp32 rounding of it (|d| <= 1e-5 + 1e-5|ref|), like pg_spmm3_ngram_f32. Zero
// weights add 0 * x: X must be finite.
#include <type_traits>

#include "pg_bf16_util.h"
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
constexpr int XCB = XK + 1;                         // in-source c-block rows (one pad row: bank offset 16)
// LDS image (bytes) of the fp32 kernel (BF = false: X and Z fp32) and of the bf16 one (BF = true: X and Z bf16 rows,
// the same fp32 weights, partial buffer and sums; Z rounded once at the store). Source regions hold one 16-feature
// row chunk per row (64 B fp32, 32 B bf16), rounded up to whole LDS-DMA wave-instructions (1 KiB).
template <bool BF>
struct ML {
    static constexpr int ES = BF ? 2 : 4;                           // bytes per source element
    static constexpr int RB = XFC * ES;                             // bytes per source row chunk
    static constexpr int PPR = RB / 16;                             // 16-B LDS-DMA pieces per row chunk
    static constexpr int EPP = 16 / ES;                             // elements per piece
    static constexpr int OUTB = (XR * RB + 1023) / 1024 * 1024;      // out / self region bytes
    static constexpr int LOUT = 0;                                  // out-sources [b][c][16 f]
    static constexpr int LIN = LOUT + OUTB;                         // in-sources  [c][a (+pad)][16 f]
    static constexpr int LINB = (XK * XCB * RB + 1023) / 1024 * 1024;
    static constexpr int LSELF = LIN + LINB;                        // self rows   [a][b][16 f]
    static constexpr int LPART = LSELF + OUTB;                      // partial     [a][row k K + b (3K)][16 f] fp32
    static constexpr int LDIAG = LPART + XK * 3 * XK * 64;          // diagonal weights [a][b][k]
    static constexpr int LBYTES = LDIAG + XR * 3 * 4;               // 160,448 B fp32; 122,560 B bf16
    static constexpr int LMAP = LBYTES;                             // mapped kernel: node rows of a middle's 400
    static constexpr int LBYTES_MAP = LMAP + 2 * XR * 4;            //   self rows, double-buffered by middle parity
    static constexpr int NOI = OUTB / 1024, NII = LINB / 1024;      // wave-instructions per region
};
static_assert(ML<false>::LBYTES == 160448 && ML<false>::OUTB == XR * 64, "fp32 LDS image");
static_assert(ML<true>::LBYTES_MAP <= 163840 && ML<false>::LBYTES_MAP <= 163840, "LDS image exceeds 160 KiB");
static_assert(XTILES % XCW == 0 && XTPW % 2 == 0, "tiles per wave");

struct XP {
    int64_t Kn1, Kn2;      // K^(n-1), K^(n-2) (= number of middles)
    int64_t m0;            // first middle of the launch (the chunk stream covers middles m0 .. m0 + chunks / nch - 1)
    int64_t zsa, zsm;      // Z row of a.M.b = a zsa + (M - m0) zsm + b: (K^(n-1), K) global, (K, K^2) middle-major
    const float* plan;
    const void* X;         // fp32 or (bf16 kernel) bf16 rows
    int64_t ldx;           // elements
    void* Z;               // fp32 or (bf16 kernel) bf16 rows
    int64_t ldz;           // elements
    int F;
    int nch;               // F / 16
    int chunks;            // length of the (middle, chunk) stream a workgroup pair / workgroup walks, middle-major
    int cstride;           // 2: workgroup pairs split each middle's chunks odd / even (see the kernel); 1: no pairs
    int remap;
    int early_in;          // loader: out / self DMA of chunk t + 1 waited for at W(t), not S(t) (PG_FLAG_MID_LOADER_SYNC clears)
    int exp;               // diagnostics build only: timing experiments (bit 0: no Z stores, 1: no out/self DMA, 2: no in DMA)
    const int* gmap;       // mapped kernel: grid row (base-K n-gram) -> node row of X / Z, -1 = n-gram not in the graph
    unsigned long long* stamps;  // diagnostics build only (PG_MID_STAMPS): s_memtime per block, chunk and point
};

#ifdef PG_MID_STAMPS
constexpr int XSTAMP_CH = 32, XSTAMP_PT = 8, XSTAMP_LAST = XSTAMP_CH - 1;  // chunk slots; the last: entry/exit
#define XSTAMP(ci, pt)                                                                                              \
    do {                                                                                                            \
        if (p.stamps && lane == 0 && ((ci) < XSTAMP_LAST || (pt) >= 5))                                                              \
            p.stamps[((int64_t)blockIdx.x * 2 + (wave >= XCW)) * XSTAMP_CH * XSTAMP_PT + (ci) * XSTAMP_PT + (pt)] = \
                __builtin_amdgcn_s_memtime();                                                                       \
    } while (0)
#define XEXP(bit) ((p.exp >> (bit)) & 1)
#else
#define XEXP(bit) 0
#define XSTAMP(ci, pt) \
    do {               \
    } while (0)
#endif

// Hide a per-lane LDS offset from the optimiser: the per-tile compile-time parts then stay ds_read/ds_write
// immediate offsets (< 64 KiB) instead of being folded with the region base into one constant per tile, each
// needing its own register.
__device__ __forceinline__ int opaque(int v) {
    asm volatile("" : "+v"(v));
    return v;
}

__device__ __forceinline__ void glds16(const void* src, const void* lds_base) {
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// Loader wave lw after issuing the next chunk's in-source pieces: wait until everything it issued before them (the
// out / self / diagonal pieces) has landed, leaving its own in-source pieces (the youngest vector-memory operations;
// vmcnt counts in issue order) in flight. NII = in-source wave-instructions per region, dealt round-robin.
template <int NII>
__device__ __forceinline__ void wait_all_but_in(int lw) {
    const int nin = (NII - lw + XLW - 1) / XLW;  // wave-uniform
    static_assert((NII + XLW - 1) / XLW <= 8, "in pieces per loader wave");
    switch (nin) {
        case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}

// one source element from the LDS image as fp32 (bf16: exact widening)
template <bool BF>
__device__ __forceinline__ float lds_src(const char* q) {
    if constexpr (BF) return __uint_as_float((uint32_t)(*reinterpret_cast<const uint16_t*>(q)) << 16);
    else return *reinterpret_cast<const float*>(q);
}

struct Chunk {
    int M, ch, first;  // middle, chunk index, first chunk of this middle in the workgroup's range
};

// MAP (pg_spmm3_ngram_mid_map_f32: a graph whose nodes are a subset of the K^n grid plus others, e.g. the builder's
// padded sequences): X rows are read and Z rows written at node rows gmap[grid row] instead of at the grid rows. The
// loader waves fetch the node rows of a middle's 1,200 source rows one middle ahead (registers); the 400 self-row
// entries also go to an LDS row map (double-buffered by middle parity) that the store-out reads, and rows whose
// n-gram is absent (-1) are not stored (their DMA reads row 0: its weights are 0). Z rows of nodes off the grid are
// left to the caller (the residual CSR pass).
template <bool BF, bool MAP>
__global__ __launch_bounds__(XTHREADS) void ngram_mid_kernel(XP p) {
    using C = ML<BF>;
    using ET = std::conditional_t<BF, uint16_t, float>;
    constexpr int LOUT = C::LOUT, LIN = C::LIN, LSELF = C::LSELF, LPART = C::LPART, LDIAG = C::LDIAG;
    constexpr int RB = C::RB, ES = C::ES;
    extern __shared__ __attribute__((aligned(16))) char L[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    XSTAMP(XSTAMP_LAST, 5);  // kernel entry
    // This workgroup's share of the chunk stream: a contiguous range [g0, g1) of it in middle-major order (ranges
    // differ by at most one step: no tail of whole middles; the weights reload only where the middle changes;
    // neighbouring ranges, which share a middle, sit on the same XCD). With cstride 2, the two workgroups of a pair
    // (logical blocks 2i, 2i + 1: same XCD) walk the same range, one the even and one the odd 16-feature chunks of
    // each middle, in step: a 64-B row piece is half of a 128-B line, and the partner's read of the other half,
    // issued at about the same time, hits in L2 (alone, each half-line read fetched the whole line from HBM: 2x the
    // X bytes), and the partners' 64-B stores of one line merge in L2 before it is written back.
    const int64_t lb = pg::xcd_logical_block(blockIdx.x, gridDim.x, p.remap != 0);
    const int half = p.cstride == 2 ? (int)(lb & 1) : 0;
    const int64_t lu = p.cstride == 2 ? lb >> 1 : lb, nu = p.cstride == 2 ? gridDim.x >> 1 : gridDim.x;
    const int g0 = (int)(lu * p.chunks / nu), g1 = (int)((lu + 1) * p.chunks / nu);
    const int nchu = p.nch / p.cstride;  // chunks of one middle in a workgroup's stream
    auto chunk_at = [&](int g) -> Chunk {
        const int Mr = g / nchu;
        const int j = g - Mr * nchu;
        return Chunk{(int)p.m0 + Mr, j * p.cstride + half, g == g0 || j == 0};
    };

    if (wave >= XCW) {  // ---------------- loader waves: LDS-DMA only (same barrier sequence as the compute waves)
        const int lw = wave - XCW;
        // One region = 400 rows x 64 B = 25 wave-instructions fp32, 400 x 32 B = 12.5 -> 13 bf16 (in-sources: 420 rows
        // with the pad rows, 27 / 14), split over the loader waves; piece order = LDS order; the in-sources are fetched
        // c-major (one wave-instruction: rows c.a.M of one c, within 4 MB). The per-lane part of every piece's element
        // offset does not depend on the middle or the chunk: computed once here (64-bit, in registers), so a DMA costs
        // one add per instruction. Pieces past the last row of a region (bf16: rows 400..415) fetch row 0 of the
        // middle (a valid address) into the region's padding.
        constexpr int NO = (C::NOI + XLW - 1) / XLW, NI = (C::NII + XLW - 1) / XLW;
        constexpr int PPR = C::PPR, EPP = C::EPP;
        int64_t off_o[NO], off_i[NI], off_s[NO];
        const int64_t ldx = p.ldx;
#pragma unroll
        for (int t = 0; t < NO; ++t) {
            const int it = lw + t * XLW;
            int rl = (int)((unsigned)(it * 64 + lane) / PPR);
            const int q = lane & (PPR - 1);  // 64 % PPR == 0
            if constexpr (C::OUTB != XR * C::RB) {  // bf16: the region's padding rows
                if (rl >= XR) rl = 0;
            }
            off_o[t] = (int64_t)rl * ldx + q * EPP;                                  // out: row M.b.c = 400 M + rl
            const int a = rl / XK, b = rl - a * XK;
            off_s[t] = (a * p.Kn1 + b) * ldx + q * EPP;                               // self: a.M.b = a K^(n-1) + 20 M + b
        }
#pragma unroll
        for (int t = 0; t < NI; ++t) {
            const int it = lw + t * XLW;
            const int rl = (int)((unsigned)(it * 64 + lane) / PPR), q = lane & (PPR - 1);
            const int c = rl / XCB, a = rl - c * XCB;
            off_i[t] = (a >= XK || c >= XK) ? q * EPP : (c * p.Kn1 + a * p.Kn2) * ldx + q * EPP;  // in: c.a.M; pad: row M
        }
        // MAP: per-lane grid offsets of the pieces' rows (out: M K^2 + go_o, self: 20 M + go_s, in: M + go_i; -1 =
        // an in-source pad piece) and the node rows of the current middle (cr_*) and of the next one (nr_*)
        [[maybe_unused]] int go_o[NO], go_s[NO], go_i[NI], cr_o[NO], cr_s[NO], cr_i[NI], nr_o[NO], nr_s[NO], nr_i[NI];
        [[maybe_unused]] const int qe = (lane & (PPR - 1)) * EPP;
        if constexpr (MAP) {
#pragma unroll
            for (int t = 0; t < NO; ++t) {
                const int it = lw + t * XLW;
                int rl = (int)((unsigned)(it * 64 + lane) / PPR);
                if (rl >= XR) rl = 0;
                go_o[t] = rl;
                const int a = rl / XK, b = rl - a * XK;
                go_s[t] = a * (int)p.Kn1 + b;
            }
#pragma unroll
            for (int t = 0; t < NI; ++t) {
                const int it = lw + t * XLW;
                const int rl = (int)((unsigned)(it * 64 + lane) / PPR);
                const int c = rl / XCB, a = rl - c * XCB;
                go_i[t] = (a >= XK || c >= XK) ? -1 : c * (int)p.Kn1 + a * (int)p.Kn2;
            }
        }
        auto fetch_map = [&](int M, int (&o)[NO], int (&s_)[NO], int (&i_)[NI]) {
            const int* gm = p.gmap;
#pragma unroll
            for (int t = 0; t < NO; ++t) {
                o[t] = gm[M * XR + go_o[t]];
                s_[t] = gm[M * XK + go_s[t]];
            }
#pragma unroll
            for (int t = 0; t < NI; ++t) i_[t] = go_i[t] < 0 ? 0 : gm[M + go_i[t]];
        };
        auto put_map = [&](int M) {  // the self pieces' node rows -> the LDS row map of middle M's parity
            int* mb = reinterpret_cast<int*>(L + C::LMAP + (M & 1) * XR * 4);
#pragma unroll
            for (int t = 0; t < NO; ++t) {
                const int it = lw + t * XLW;
                const int rl = (int)((unsigned)(it * 64 + lane) / PPR);
                if (it < C::NOI && rl < XR && (lane & (PPR - 1)) == 0) mb[rl] = cr_s[t];
            }
        };
        auto dma_rows = [&](int region, int kind, int M, int ch) {
            const ET* xc = reinterpret_cast<const ET*>(p.X) + ch * XFC;
            if constexpr (MAP) {
                (void)M;
                if (kind == 0) {
#pragma unroll
                    for (int t = 0; t < NO; ++t)
                        if (lw + t * XLW < C::NOI)
                            glds16(xc + (int64_t)max(cr_o[t], 0) * ldx + qe, L + region + (lw + t * XLW) * 1024);
                } else if (kind == 1) {
#pragma unroll
                    for (int t = 0; t < NI; ++t)
                        if (lw + t * XLW < C::NII)
                            glds16(xc + (int64_t)max(cr_i[t], 0) * ldx + qe, L + region + (lw + t * XLW) * 1024);
                } else {
#pragma unroll
                    for (int t = 0; t < NO; ++t)
                        if (lw + t * XLW < C::NOI)
                            glds16(xc + (int64_t)max(cr_s[t], 0) * ldx + qe, L + region + (lw + t * XLW) * 1024);
                }
                return;
            }
            if (kind == 0) {
                const ET* base = xc + (int64_t)M * XR * ldx;
#pragma unroll
                for (int t = 0; t < NO; ++t)
                    if (lw + t * XLW < C::NOI) glds16(base + off_o[t], L + region + (lw + t * XLW) * 1024);
            } else if (kind == 1) {
                const ET* base = xc + (int64_t)M * ldx;
#pragma unroll
                for (int t = 0; t < NI; ++t)
                    if (lw + t * XLW < C::NII) glds16(base + off_i[t], L + region + (lw + t * XLW) * 1024);
            } else {
                const ET* base = xc + (int64_t)M * XK * ldx;
#pragma unroll
                for (int t = 0; t < NO; ++t)
                    if (lw + t * XLW < C::NOI) glds16(base + off_s[t], L + region + (lw + t * XLW) * 1024);
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
        const int mlast = (int)p.Kn2 - 1;
        if (g0 < g1) {
            const Chunk c0 = chunk_at(g0);
            if constexpr (MAP) {
                fetch_map(c0.M, cr_o, cr_s, cr_i);
                fetch_map(min(c0.M + 1, mlast), nr_o, nr_s, nr_i);  // one middle ahead
                put_map(c0.M);
            }
            dma_rows(LOUT, 0, c0.M, c0.ch);
            dma_rows(LIN, 1, c0.M, c0.ch);
            dma_rows(LSELF, 2, c0.M, c0.ch);
            dma_diag(c0.M);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if constexpr (MAP) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        XSTAMP(XSTAMP_LAST, 6);
        asm volatile("s_barrier" ::: "memory");  // S(-1)
        [[maybe_unused]] int ci = 0;  // chunk slot of the diagnostics build's time stamps
#pragma unroll 1
        for (int g = g0; g < g1; ++g) {
            const bool more = g + 1 < g1;
            const Chunk nx = more ? chunk_at(g + 1) : Chunk{0, 0, 0};
            XSTAMP(ci, 0);
            asm volatile("s_barrier" ::: "memory");  // M(t): out-phase done, partial written; out / self / diag free
            XSTAMP(ci, 1);
            if (more && !XEXP(1)) {
                if constexpr (MAP) {
                    if (nx.first) {  // the next chunk starts middle nx.M = (this one) + 1: its rows were prefetched
#pragma unroll
                        for (int t = 0; t < NO; ++t) {
                            cr_o[t] = nr_o[t];
                            cr_s[t] = nr_s[t];
                        }
#pragma unroll
                        for (int t = 0; t < NI; ++t) cr_i[t] = nr_i[t];
                        put_map(nx.M);  // read by nx's store-out, after S(t + 1)
                        fetch_map(min(nx.M + 1, mlast), nr_o, nr_s, nr_i);
                    }
                }
                dma_rows(LOUT, 0, nx.M, nx.ch);
                dma_rows(LSELF, 2, nx.M, nx.ch);
                if (nx.first) dma_diag(nx.M);
            }
            if constexpr (MAP) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            // The out / self rows of chunk t + 1 are first read after W(t): with early_in they stay in flight across
            // S(t) and the store-out, and only the in-source pieces issued after S(t) may still be in flight at W(t)
            if (!p.early_in) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            XSTAMP(ci, 2);
            asm volatile("s_barrier" ::: "memory");  // S(t): in-phase done; in-region free
            XSTAMP(ci, 3);
            if (more && !XEXP(2)) dma_rows(LIN, 1, nx.M, nx.ch);
            if (XEXP(2)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            else wait_all_but_in<C::NII>(lw);
            asm volatile("s_barrier" ::: "memory");  // W(t): chunk t's results have left the partial buffer
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            XSTAMP(ci, 4);
            ++ci;
        }
        XSTAMP(XSTAMP_LAST, 7);
        return;
    }

    // ---------------- compute waves
    // Tile assignment: wave w owns, in both phases, the row tile m = w & 3 of the columns b (out) / a (in) =
    // 2 j + (w >> 2), j = 0..9, so every LDS address below is a per-lane base plus a compile-time offset in j and s.
    const int q4 = lane >> 4, fl = lane & 15;
    const int mw = wave & 3, wb = wave >> 2;
    float Ao[XTPW][XS], Ai[XTPW][XS];  // A fragments of this wave's out / in tiles (middle-resident)
    // A fragments of the next middle are prefetched where the registers are free: Ao after the last chunk's
    // out-phase (consumed by the next middle's first out-phase), Ai before its first chunk's out-phase
    // MAP: wave-uniform base + a 32-bit lane offset formed at each load, so no 64-bit per-lane pointer stays live (one
    // was spilled, and its reload's vmcnt(0) waited for the chunk's Z stores at every middle change); the plain kernel
    // keeps the pointer form, under which its registers allocate best (measured: the opaque form cost it ~7 us)
    auto load_W = [&](float (&W)[XTPW][XS], int M, int region) {
        if constexpr (MAP) {
            const char* pm = reinterpret_cast<const char*>(p.plan + (int64_t)M * XMB + region);
            const uint32_t lo = (uint32_t)opaque((lane + (wb * 4 + mw) * XS * 64) * 4);
#pragma unroll
            for (int j = 0; j < XTPW; ++j)
#pragma unroll
                for (int s = 0; s < XS; ++s)
                    W[j][s] = *reinterpret_cast<const float*>(pm + lo + (uint32_t)(((2 * j * 4) * XS + s) * 256));
        } else {
            const float* pm = p.plan + (int64_t)M * XMB + region + lane;
#pragma unroll
            for (int j = 0; j < XTPW; ++j)
#pragma unroll
                for (int s = 0; s < XS; ++s) W[j][s] = pm[(((2 * j + wb) * 4 + mw) * XS + s) * 64];
        }
    };
    auto load_Ao = [&](int M) { load_W(Ao, M, XPO); };
    auto load_Ai = [&](int M) { load_W(Ai, M, XPI); };
    // this lane's four accumulator rows i = 16 mw + 4 q4 + r: (k, a) in the out-phase, (k, b) in the in-phase. The
    // padding rows i = 60..63 repeat rows 56..59 (the plan holds their weights twice): their lanes compute the same
    // values and write them to the same places as the lanes of rows 56..59, so no lane needs a branch
    int rk[4], rv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        int i = 16 * mw + 4 * q4 + r;
        if (i >= 3 * XK) i -= 4;
        rk[r] = i / XK;
        rv[r] = i - rk[r] * XK;
    }
    // LDS byte offsets: sources [row][16 f] (RB-byte rows: 64 fp32, 32 bf16); partial [a][row k K + b][16 f] fp32
    const int src_lane = (q4 * XFC + fl) * ES;               // out: + (b * K + 4 s) * RB
    const int in_lane = (q4 * XCB * XFC + fl) * ES;          // in:  + (4 s * XCB + a) * RB
    int part_w[4], part_r[4], self_r[4], diag_r[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        part_w[r] = LPART + ((rv[r] * 3 * XK + rk[r] * XK + wb) * 16 + fl) * 4;  // out: a = rv, row k K + b; + 2 j * 64
        part_r[r] = LPART + ((wb * 3 * XK + rk[r] * XK + rv[r]) * 16 + fl) * 4;   // in: + 2 j * 60 * 64
        self_r[r] = LSELF + ((rv[r] * XK + wb) * XFC + fl) * ES;                  // out: (a = rv, b); + 2 j * RB
        diag_r[r] = LDIAG + ((rv[r] * XK + wb) * 3 + rk[r]) * 4;                   // + 2 j * 12
        part_w[r] = opaque(part_w[r]);
        part_r[r] = opaque(part_r[r]);
        self_r[r] = opaque(self_r[r]);
        diag_r[r] = opaque(diag_r[r]);
    }
    // store-out of a finished in-phase tile: lane l writes 16 B = features 4 (l & 3) .. + 3 of tile row l >> 2
    const int so_i = 16 * mw + (lane >> 2) - (16 * mw + (lane >> 2) >= 3 * XK ? 4 : 0);  // padding rows: as above
    const int so_k = so_i / XK, so_b = so_i - so_k * XK;
    const int so_lds = opaque(LPART + ((wb * 3 * XK + so_i) * 16 + 4 * (lane & 3)) * 4);  // + 2 j * 60 * 64
    const int64_t zstep = 2 * p.zsa * p.ldz;                                        // a -> a + 2
    if (g0 < g1) {
        load_Ao(chunk_at(g0).M);
        load_Ai(chunk_at(g0).M);
    }
    asm volatile("s_barrier" ::: "memory");  // S(-1)
    XSTAMP(XSTAMP_LAST, 6);
    [[maybe_unused]] int ci = 0;  // chunk slot of the diagnostics build's time stamps
#pragma unroll 1
    for (int g = g0; g < g1; ++g) {
        const Chunk cu = chunk_at(g);
        XSTAMP(ci, 0);
        const bool next_mid = g + 1 < g1 && (g + 1) % nchu == 0;  // the next chunk starts another middle
        // ---- out-phase: tiles (b = 2 j + wb, m = mw); hand-over of row (k, a) to the in-phase row k K + b of a.
        // Software-pipelined over tile pairs: the B fragments of pair j + 2 are read while pair j's MFMAs run.
        auto rd_out = [&](int j, float (&x)[2][XS]) {
#pragma unroll
            for (int s = 0; s < XS; ++s) {
                x[0][s] = lds_src<BF>(L + LOUT + src_lane + ((2 * j + wb) * XK + 4 * s) * RB);
                x[1][s] = lds_src<BF>(L + LOUT + src_lane + ((2 * j + 2 + wb) * XK + 4 * s) * RB);
            }
        };
        float xo[2][2][XS];
        rd_out(0, xo[0]);
#pragma unroll
        for (int j = 0; j < XTPW; j += 2) {
            float(&xc)[2][XS] = xo[(j >> 1) & 1];
            if (j + 2 < XTPW) rd_out(j + 2, xo[((j >> 1) + 1) & 1]);
            float w0[4], w1[4], s0[4], s1[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                w0[r] = *reinterpret_cast<const float*>(L + diag_r[r] + 2 * j * 12);
                w1[r] = *reinterpret_cast<const float*>(L + diag_r[r] + (2 * j + 2) * 12);
                s0[r] = lds_src<BF>(L + self_r[r] + 2 * j * RB);
                s1[r] = lds_src<BF>(L + self_r[r] + (2 * j + 2) * RB);
            }
            asm volatile("" ::: "memory");  // the reads above are issued before the MFMAs below
            f4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < XS; ++s) {
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(Ao[j][s], xc[0][s], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(Ao[j + 1][s], xc[1][s], acc1, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {  // + the diagonal term Wdiag_k[a, b] X[a.M.b, f]
                *reinterpret_cast<float*>(L + part_w[r] + 2 * j * 64) = __builtin_fmaf(w0[r], s0[r], acc0[r]);
                *reinterpret_cast<float*>(L + part_w[r] + (2 * j + 2) * 64) = __builtin_fmaf(w1[r], s1[r], acc1[r]);
            }
            asm volatile("" ::: "memory");
        }
        if (next_mid) load_Ao(cu.M + 1);
        XSTAMP(ci, 1);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // M(t)
        XSTAMP(ci, 2);
        // ---- in-phase: tiles (a = 2 j + wb, m = mw): rows (k, b); initial accumulators from the partial buffer; the
        // finished values go back into the partial buffer and leave it as 16-B row pieces
        const int M = cu.M;
        [[maybe_unused]] ET* zso = nullptr;
        if constexpr (!MAP)  // (the mapped kernel forms its store address after the in-phase: fewer live registers)
            zso = reinterpret_cast<ET*>(p.Z) + ((int64_t)wb * p.zsa + (M - p.m0) * p.zsm + so_b) * p.ldz +
                  (int64_t)so_k * p.F + cu.ch * XFC + 4 * (lane & 3);
        auto rd_in = [&](int j, float (&x)[2][XS]) {
#pragma unroll
            for (int s = 0; s < XS; ++s) {
                x[0][s] = lds_src<BF>(L + LIN + in_lane + (4 * s * XCB + 2 * j + wb) * RB);
                x[1][s] = lds_src<BF>(L + LIN + in_lane + (4 * s * XCB + 2 * j + 2 + wb) * RB);
            }
        };
        float xi[2][2][XS];
        rd_in(0, xi[0]);
#pragma unroll
        for (int j = 0; j < XTPW; j += 2) {
            float(&xc)[2][XS] = xi[(j >> 1) & 1];
            f4_t acc0, acc1;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                acc0[r] = *reinterpret_cast<const float*>(L + part_r[r] + 2 * j * 3 * XK * 64);
                acc1[r] = *reinterpret_cast<const float*>(L + part_r[r] + (2 * j + 2) * 3 * XK * 64);
            }
            if (j + 2 < XTPW) rd_in(j + 2, xi[((j >> 1) + 1) & 1]);
            asm volatile("" ::: "memory");  // the reads above are issued before the MFMAs below
#pragma unroll
            for (int s = 0; s < XS; ++s) {
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(Ai[j][s], xc[0][s], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(Ai[j + 1][s], xc[1][s], acc1, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                *reinterpret_cast<float*>(L + part_r[r] + 2 * j * 3 * XK * 64) = acc0[r];
                *reinterpret_cast<float*>(L + part_r[r] + (2 * j + 2) * 3 * XK * 64) = acc1[r];
            }
            asm volatile("" ::: "memory");
        }
        XSTAMP(ci, 3);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // S(t)
        XSTAMP(ci, 4);
        // ---- store-out of chunk t, in the next out-phase's shadow (the out/self DMA of the in-phase is done; only
        // the smaller in-source DMA shares the CU's memory pipeline with these stores): every row of the partial
        // buffer as 16-B pieces, then W(t) before the next out-phase overwrites it
        if constexpr (MAP) zso = reinterpret_cast<ET*>(p.Z) + (int64_t)so_k * p.F + cu.ch * XFC + 4 * (lane & 3);
#pragma unroll
        for (int j = 0; j < XTPW; j += 2) {
            const f4_t v0 = *reinterpret_cast<const f4_t*>(L + so_lds + 2 * j * 3 * XK * 64);
            const f4_t v1 = *reinterpret_cast<const f4_t*>(L + so_lds + (2 * j + 2) * 3 * XK * 64);
            if constexpr (MAP) {  // node rows of (a = 2 j + wb [+ 2], b = so_b) from the LDS row map; -1: not stored
                const int* mb = reinterpret_cast<const int*>(L + C::LMAP + (M & 1) * XR * 4) + wb * XK + so_b;
                const int r0 = mb[2 * j * XK], r1 = mb[(2 * j + 2) * XK];
                if constexpr (BF) {
                    if (r0 >= 0)
                        *reinterpret_cast<uint2*>(zso + (int64_t)r0 * p.ldz) =
                            make_uint2(pgbf::pack2(v0[0], v0[1]), pgbf::pack2(v0[2], v0[3]));
                    if (r1 >= 0)
                        *reinterpret_cast<uint2*>(zso + (int64_t)r1 * p.ldz) =
                            make_uint2(pgbf::pack2(v1[0], v1[1]), pgbf::pack2(v1[2], v1[3]));
                } else {
                    if (r0 >= 0) *reinterpret_cast<f4_t*>(zso + (int64_t)r0 * p.ldz) = v0;
                    if (r1 >= 0) *reinterpret_cast<f4_t*>(zso + (int64_t)r1 * p.ldz) = v1;
                }
            } else if (!XEXP(0)) {
                if constexpr (BF) {  // one rounding to bf16 (RNE), 8-B stores
                    *reinterpret_cast<uint2*>(zso + (int64_t)j * zstep) =
                        make_uint2(pgbf::pack2(v0[0], v0[1]), pgbf::pack2(v0[2], v0[3]));
                    *reinterpret_cast<uint2*>(zso + (int64_t)(j + 1) * zstep) =
                        make_uint2(pgbf::pack2(v1[0], v1[1]), pgbf::pack2(v1[2], v1[3]));
                } else {
                    *reinterpret_cast<f4_t*>(zso + (int64_t)j * zstep) = v0;
                    *reinterpret_cast<f4_t*>(zso + (int64_t)(j + 1) * zstep) = v1;
                }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // W(t)
        XSTAMP(ci, 5);
        ++ci;
        if (next_mid) load_Ai(cu.M + 1);
    }
    XSTAMP(XSTAMP_LAST, 7);
}

// ---------------------------------------------------------------------------------------------------------
// Transposed middle-tile kernel: the backward of the forward above for the symmetric n-gram matrices (A_k^T = A_k; the
// autograd of protgram_directgcn.py:101-112), with G_k = G[:, kF:(k+1)F]:
//   dX[a.M.b, f] (+)= sum_k ( sum_c Wout_k[a,b,c] G_k[M.b.c, f] + sum_c Win_k[a,b,c] G_k[c.a.M, f]
//                             [+ Wdiag_k[a,b] G_k[a.M.b, f]] )
// fp32 (pg_spmm3t_ngram_mid_offdiag_f32): WITHOUT the bracketed diagonal term. The out-sources of middle M are the rows
// with prefix M, its in-sources the rows with suffix M and its own rows those with middle M -- three disjoint sets, so
// the diagonal term is a THIRD read of every G row (the 4x4-block kernel's 1,057 MB per launch), and at fp32 one
// slice's own rows (25.6 KB) do not fit beside the ring; the caller adds it (NgramPlan.diag3).
// bf16 (pg_spmm3t_ngram_mid_bf16: bf16 G and dX rows, fp32 weights and sums, dX rounded once): the full product. Half-
// size rows leave room for slice k's own rows in the out-sub-phase's slot beside its out-sources; they are added
// after that slice's out-MFMAs with the middle's diagonal weights (LDS, loaded at each middle change).
//
// Per (middle, 16-feature chunk) six sub-phases, one slice G_k each:
//   out k = 0, 1, 2: tiles (b, m), rows a = 16 m + 0..15 (20 valid), K-dim (k, c): 5 MFMA k-steps per slice, the
//                    accumulators kept across the three slices and handed over as P[a][b][16 f] (LDS) after k = 2;
//   in  k = 0, 1, 2: tiles (a, m), rows b, started from P after k = 0's barrier; the finished rows go back to P and
//                    leave for HBM (16-B pieces) in the next chunk's first sub-phase.
// Every wave computes AND issues the LDS-DMA (no loader waves): one slice's source rows per sub-phase (out: 400 rows,
// in: 420 with the pad rows; 64-B row chunks fp32, 32-B bf16) into a ring of four slots, three sub-phases ahead, one
// barrier per sub-phase. Wave w owns the row tile m = w & 1 of the columns b (out) / a (in) = (w >> 1) + 4 j, j = 0..4;
// its A fragments, gathered from the forward plan (rows (k, a) -> a, K-dim c -> (k, c)), stay in registers per middle:
// 75 out + 75 in per lane (8 waves, 2 per SIMD: up to 256 VGPRs), reloaded at a middle change.
// The four slots and P are separate LDS objects, and the sub-phase loop is unrolled by 12 (= lcm of 6 sub-phases per
// chunk and 4 slots), so every slot a DMA writes and every slot a read uses is known at compile time.
constexpr int T2_SLOT = 27 * 1024;                     // ring slot: fp32 one slice's in-sources (420 rows x 64 B);
                                                       // bf16 out-sources (13 KiB) + own rows (13 KiB) of a slice
constexpr int T2_NOUT = XR * 64 / 1024;                // fp32: 25 wave-instructions of out-source pieces per slice
constexpr int T2_NIN = (XK * XCB * 64 + 1023) / 1024;  // 27 of in-source pieces (the last one partly padding)
template <bool BF>
struct T2L {
    static constexpr int ES = BF ? 2 : 4;                       // bytes per G / dX element
    static constexpr int RB = XFC * ES;                         // bytes per row chunk
    static constexpr int PPR = RB / 16, EPP = 16 / ES;          // 16-B pieces per row chunk, elements per piece
    static constexpr int NO = (XR * RB + 1023) / 1024;          // wave-instructions per out / own-row / stage slice
    static constexpr int NI = (XK * XCB * RB + 1023) / 1024;    // per in slice
    static constexpr int SELF = NO * 1024;                      // bf16: own rows after the out-sources in the slot
};
static_assert(T2L<true>::NO == 13 && T2L<true>::NI == 14 && 2 * T2L<true>::SELF <= T2_SLOT, "bf16 slot");
static_assert(T2L<false>::NO == T2_NOUT && T2L<false>::NI == T2_NIN, "fp32 slot");
constexpr int T2_PB = XFC, T2_PA = XK * T2_PB;        // P[a][b][16 f] (dwords; the 2-way conflicts of its 40 ops per
                                                       // wave and chunk cost less than the padding's LDS)
constexpr int T2_TPW = 5;                              // tiles per wave per sub-phase
static_assert(T2_NIN * 1024 <= T2_SLOT && T2_NOUT * 1024 <= T2_SLOT && T2_NIN <= 32 && T2_NOUT <= 32, "ring slot");
static_assert(4 * T2_SLOT + 2 * XR * 64 <= 163840, "LDS: four slots, P and the accumulate stage");

// s_waitcnt vmcnt(min(n, 23)) for a wave-uniform n (a smaller bound than needed only waits longer)
__device__ __forceinline__ void vm_wait(int n) {
    switch (n < 0 ? 0 : n) {
#define PG_VMW(k)                                              \
    case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); \
        break;
        PG_VMW(0) PG_VMW(1) PG_VMW(2) PG_VMW(3) PG_VMW(4) PG_VMW(5) PG_VMW(6) PG_VMW(7) PG_VMW(8) PG_VMW(9)
        PG_VMW(10) PG_VMW(11) PG_VMW(12) PG_VMW(13) PG_VMW(14) PG_VMW(15) PG_VMW(16) PG_VMW(17) PG_VMW(18)
        PG_VMW(19) PG_VMW(20) PG_VMW(21) PG_VMW(22)
#undef PG_VMW
        default: asm volatile("s_waitcnt vmcnt(23)" ::: "memory"); break;
    }
}

template <int V>
using ic = std::integral_constant<int, V>;

// LDS-DMA piece (16 B per lane -> LDS byte address lds + 16 lane) in inline asm: hidden from the compiler's wait
// bookkeeping, which otherwise drains every DMA in flight (vmcnt(0)) before LDS reads it cannot tell apart from them
// (at control-flow joins); the kernel counts these operations itself (vm_wait). M0 saved and restored in the statement.
__device__ __forceinline__ void glds16_asm(const float* src, uint32_t lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds)
                 : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const float* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)p;
}

template <bool BF>
__global__ __launch_bounds__(512) void ngram_midt2_kernel(XP p, int accumulate) {
    using C = T2L<BF>;
    constexpr int ES = C::ES, RB = C::RB, PPR = C::PPR, EPP = C::EPP;
    using ET = std::conditional_t<BF, uint16_t, float>;
    __shared__ __attribute__((aligned(16))) float S0[T2_SLOT / 4];
    __shared__ __attribute__((aligned(16))) float S1[T2_SLOT / 4];
    __shared__ __attribute__((aligned(16))) float S2[T2_SLOT / 4];
    __shared__ __attribute__((aligned(16))) float S3[T2_SLOT / 4];
    __shared__ __attribute__((aligned(16))) float Pb[XK * T2_PA];
    __shared__ __attribute__((aligned(16))) float SX[C::NO * 256];  // accumulate: the chunk's dX rows (LDS-DMA, whole instructions)
    __shared__ __attribute__((aligned(16))) float Dg[BF ? XR * 3 : 4];  // bf16: the middle's diagonal weights [a][b][k]
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // the forward's chunk ranges and workgroup pairs (see ngram_mid_kernel)
    const int64_t lb = pg::xcd_logical_block(blockIdx.x, gridDim.x, p.remap != 0);
    const int half = p.cstride == 2 ? (int)(lb & 1) : 0;
    const int64_t lu = p.cstride == 2 ? lb >> 1 : lb, nu = p.cstride == 2 ? gridDim.x >> 1 : gridDim.x;
    const int g0 = (int)(lu * p.chunks / nu), g1 = (int)((lu + 1) * p.chunks / nu);
    if (g0 >= g1) return;
    const int nchu = p.nch / p.cstride;
    const int nc = g1 - g0;  // chunks of this workgroup, sub-phases u = 6 c + j
    const int U = 6 * nc;
    auto mid_of = [&](int c) { return (int)p.m0 + (g0 + c) / nchu; };
    auto ch_of = [&](int c) { return ((g0 + c) % nchu) * p.cstride + half; };
    const int q = lane >> 4, fl = lane & 15;
    const int mt = wave & 1, grp = wave >> 1;
    const int64_t ldg = p.ldx;
    const ET* __restrict__ G = reinterpret_cast<const ET*>(p.X);

    // LDS-DMA: wave-instruction it = wave + 8 t of a slice (piece it * 64 + lane, lane-linear in the slot); the per-lane
    // element offsets do not depend on the middle, chunk or slice; < 2^32 (the host checks n_rows * ldg): 32-bit per
    // lane, added to a wave-uniform base. Pieces past a slice's last row read a valid row into the slot's padding.
    uint32_t off_o[4], off_i[4], off_s[4], off_x[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int pc = (wave + 8 * t) * 64 + lane, rl = pc / PPR, qq = (pc % PPR) * EPP;
        const int ro = rl < XR ? rl : 0;
        off_o[t] = (uint32_t)ro * (uint32_t)ldg + qq;                              // out: row M K^2 + rl (= M.b.c)
        const int c = rl / XCB, a = rl - c * XCB;                                  // in: row c.a.M; pad pieces: row M
        off_i[t] = (a >= XK || c >= XK) ? qq
                                        : (uint32_t)(c * (uint32_t)p.Kn1 + a * (uint32_t)p.Kn2) * (uint32_t)ldg + qq;
        const int sa = ro / XK, sb = ro - sa * XK;                                 // own: row a.M.b (bf16)
        off_s[t] = (uint32_t)(sa * (uint32_t)p.Kn1 + sb) * (uint32_t)ldg + qq;
        off_x[t] = (uint32_t)(sa * (uint32_t)p.zsa + sb) * (uint32_t)p.ldz + qq;   // accumulate: dX row a.M.b
    }
    const int n_out = (C::NO - wave + 7) / 8, n_in = (C::NI - wave + 7) / 8;      // this wave's instructions per slice
    auto dma_x = [&](int c) {
        const ET* base = reinterpret_cast<const ET*>(p.Z) + (int64_t)(mid_of(c) - p.m0) * p.zsm * p.ldz + ch_of(c) * XFC;
#pragma unroll
        for (int t = 0; t < 4; ++t)
            if (t < n_out) glds16_asm(reinterpret_cast<const float*>(base + off_x[t]), lds_addr(SX) + (wave + 8 * t) * 1024);
    };
    auto slot = [&](auto sc) -> float* {
        constexpr int S = decltype(sc)::value;
        if constexpr (S == 0) return S0;
        else if constexpr (S == 1) return S1;
        else if constexpr (S == 2) return S2;
        else return S3;
    };
    auto dma = [&](float* dst, int c, int j) {  // sub-phase (chunk c, j): slice k = j mod 3 of the out / in sources
        const int M = mid_of(c), k = j < 3 ? j : j - 3;
        const ET* base = G + (int64_t)k * p.F + ch_of(c) * XFC;
        if (j < 3) {
#pragma unroll
            for (int t = 0; t < 4; ++t)
                if (t < n_out)
                    glds16_asm(reinterpret_cast<const float*>(base + (int64_t)M * XR * ldg + off_o[t]),
                               lds_addr(dst) + (wave + 8 * t) * 1024);
            if constexpr (BF) {  // the slice's own rows a.M.b beside them
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    if (t < n_out)
                        glds16_asm(reinterpret_cast<const float*>(base + (int64_t)M * XK * ldg + off_s[t]),
                                   lds_addr(dst) + C::SELF + (wave + 8 * t) * 1024);
            }
        } else {
#pragma unroll
            for (int t = 0; t < 4; ++t)
                if (t < n_in)
                    glds16_asm(reinterpret_cast<const float*>(base + (int64_t)M * ldg + off_i[t]),
                               lds_addr(dst) + (wave + 8 * t) * 1024);
        }
    };
    const int n_dma_out = (BF ? 2 : 1) * n_out;  // pieces of an out-sub-phase's DMA (bf16: + the own rows)
    // A fragments: Wo[j][5 k + s] (tile b = grp + 4 j, m = mt): lane holds A[a = 16 mt + fl][c = 4 s + q] of slice k
    // = Wout_k[a, b, c], in the forward plan at out fragment (b, row (k, a) = 20 k + a, c). Wi likewise with (a, b)
    // exchanged (tile a = grp + 4 j, rows b = 16 mt + fl). Rows past 19 load row 19's weights: an MFMA row only feeds
    // its own accumulator row, and those rows are never handed over or stored.
    float Wo[T2_TPW][15], Wi[T2_TPW][15];
    const int rrc = min(16 * mt + fl, XK - 1);
    auto gather = [&](auto kc, auto inc, int M) {
        constexpr int k = decltype(kc)::value;
        constexpr bool IN = decltype(inc)::value != 0;
        const int i_f = XK * k + rrc;
        const char* pm = reinterpret_cast<const char*>(p.plan + (int64_t)M * XMB + (IN ? XPI : XPO));  // wave-uniform
        // per-lane byte offset, recomputed at every gather (opaque: not hoisted into 25 live copies per slice)
        const uint32_t lo = (uint32_t)opaque(((q << 4) + (i_f & 15) + ((grp * 4 + (i_f >> 4)) * XS) * 64) * 4);
#pragma unroll
        for (int j = 0; j < T2_TPW; ++j)
#pragma unroll
            for (int s = 0; s < XS; ++s) {
                const float v = *reinterpret_cast<const float*>(pm + lo + (uint32_t)((16 * j * XS + s) * 256));
                if constexpr (IN) Wi[j][5 * k + s] = v;
                else Wo[j][5 * k + s] = v;
            }
    };

    f4_t acc[T2_TPW];
    const bool prow = mt == 0 || q == 0;  // accumulator rows 16 mt + 4 q + r < 20
    const int p_out = opaque((((16 * mt + 4 * q) * T2_PA + grp * T2_PB + fl) * 4));  // P[a][b]: + (r T2_PA + 4 j T2_PB) 4
    const int p_in = opaque(((grp * T2_PA + (16 * mt + 4 * q) * T2_PB + fl) * 4));   // P[a][b]: + (4 j T2_PA + r T2_PB) 4
    const int b_out = opaque(((grp * XK + q) * XFC + fl) * ES);  // out-source (b = grp + 4j, c = 4 s + q): + (4 j K + 4 s) RB
    const int b_in = opaque(((q * XCB + grp) * XFC + fl) * ES);  // in-source (c = 4 s + q, a = grp + 4j): + (4 s XCB + 4 j) RB
    // bf16 own-row term: own row (a = 16 mt + 4 q + r, b = grp + 4 j) of the slot's second half, + (r K + 4 j) RB; its
    // diagonal weight Dg[(a K + b) 3 + k], + ((r K + 4 j) 3 + k) 4
    [[maybe_unused]] const int b_self = opaque(C::SELF + (((16 * mt + 4 * q) * XK + grp) * XFC + fl) * ES);
    [[maybe_unused]] const int d_self = opaque((((16 * mt + 4 * q) * XK + grp) * 3) * 4);
    char* const P8 = reinterpret_cast<char*>(Pb);
    auto out_sub = [&](const float* sl, auto kc) {
        constexpr int k = decltype(kc)::value;
        const char* sb = reinterpret_cast<const char*>(sl) + b_out;
        if constexpr (k == 0) {
#pragma unroll
            for (int j = 0; j < T2_TPW; ++j) acc[j] = f4_t{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int s = 0; s < XS; ++s) {
            float bv[T2_TPW];
#pragma unroll
            for (int j = 0; j < T2_TPW; ++j) bv[j] = lds_src<BF>(sb + (4 * j * XK + 4 * s) * RB);
#pragma unroll
            for (int j = 0; j < T2_TPW; ++j)
                acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(Wo[j][5 * k + s], bv[j], acc[j], 0, 0, 0);
        }
        if constexpr (BF) {  // + Wdiag_k[a, b] G_k[a.M.b, f] (rows a < 20)
            if (prow) {
                const char* ss = reinterpret_cast<const char*>(sl) + b_self;
                const char* dd = reinterpret_cast<const char*>(Dg) + d_self;
#pragma unroll
                for (int j = 0; j < T2_TPW; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        acc[j][r] = __builtin_fmaf(*reinterpret_cast<const float*>(dd + ((r * XK + 4 * j) * 3 + k) * 4),
                                                   lds_src<true>(ss + (r * XK + 4 * j) * RB), acc[j][r]);
            }
        }
        if constexpr (k == 2) {
            if (prow) {
#pragma unroll
                for (int j = 0; j < T2_TPW; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        *reinterpret_cast<float*>(P8 + p_out + (r * T2_PA + 4 * j * T2_PB) * 4) = acc[j][r];
            }
        }
    };
    auto in_sub = [&](const float* sl, auto kc) {
        constexpr int k = decltype(kc)::value;
        const char* sb = reinterpret_cast<const char*>(sl) + b_in;
        if constexpr (k == 0) {
#pragma unroll
            for (int j = 0; j < T2_TPW; ++j) {
                acc[j] = f4_t{0.f, 0.f, 0.f, 0.f};
                if (prow)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        acc[j][r] = *reinterpret_cast<const float*>(P8 + p_in + (4 * j * T2_PA + r * T2_PB) * 4);
            }
        }
#pragma unroll
        for (int s = 0; s < XS; ++s) {
            float bv[T2_TPW];
#pragma unroll
            for (int j = 0; j < T2_TPW; ++j) bv[j] = lds_src<BF>(sb + (4 * s * XCB + 4 * j) * RB);
#pragma unroll
            for (int j = 0; j < T2_TPW; ++j)
                acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(Wi[j][5 * k + s], bv[j], acc[j], 0, 0, 0);
        }
        if constexpr (k == 2) {
            if (prow) {
#pragma unroll
                for (int j = 0; j < T2_TPW; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        *reinterpret_cast<float*>(P8 + p_in + (4 * j * T2_PA + r * T2_PB) * 4) = acc[j][r];
            }
        }
    };
    // store-out of chunk c: P's 400 rows as 1,600 16-B pieces over the 512 threads (wave 0: 4, the others 3), plus the
    // staged dX rows when accumulating
    const int n_st = wave == 0 ? 4 : 3;  // vector-memory operations it issues
    auto store_out = [&](int c) {
        const int M = mid_of(c);
        ET* dx = reinterpret_cast<ET*>(p.Z) + (int64_t)(M - p.m0) * p.zsm * p.ldz + ch_of(c) * XFC;
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) {
            const int pc = tid + 512 * tt;
            if (tt < 3 || wave == 0) {  // pc < 1,600
                const int row = pc >> 2, a = row / XK, b = row - a * XK, q4 = pc & 3;
                f4_t v = *reinterpret_cast<const f4_t*>(P8 + (a * T2_PA + b * T2_PB + 4 * q4) * 4);
                ET* dst = dx + ((int64_t)a * p.zsa + b) * p.ldz + 4 * q4;
                if constexpr (BF) {  // fp32 sums, one rounding (RNE)
                    if (accumulate) {
                        const uint2 o = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(SX) + pc * 8);
                        v[0] += pgbf::lo(o.x);
                        v[1] += pgbf::hi(o.x);
                        v[2] += pgbf::lo(o.y);
                        v[3] += pgbf::hi(o.y);
                    }
                    *reinterpret_cast<uint2*>(dst) = make_uint2(pgbf::pack2(v[0], v[1]), pgbf::pack2(v[2], v[3]));
                } else {
                    if (accumulate) v += *reinterpret_cast<const f4_t*>(reinterpret_cast<const char*>(SX) + pc * 16);
                    *reinterpret_cast<f4_t*>(dst) = v;
                }
            }
        }
    };
    // bf16: the middle's diagonal weights into Dg (1,200 floats = 300 16-B pieces; plain loads, waited for by the caller)
    auto load_diag = [&](int M) {
        if constexpr (BF) {
            if (tid < XR * 3 / 4)
                reinterpret_cast<float4*>(Dg)[tid] = reinterpret_cast<const float4*>(p.plan + (int64_t)M * XMB + XPD)[tid];
        }
    };

    // prologue: the first middle's weights and the first three sub-phases' slices, all landed
    {
        const int M = mid_of(0);
        gather(ic<0>{}, ic<0>{}, M);
        gather(ic<1>{}, ic<0>{}, M);
        gather(ic<2>{}, ic<0>{}, M);
        gather(ic<0>{}, ic<1>{}, M);
        gather(ic<1>{}, ic<1>{}, M);
        gather(ic<2>{}, ic<1>{}, M);
        load_diag(M);
        dma(S0, 0, 0);
        dma(S1, 0, 1);
        dma(S2, 0, 2);
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the weights (hipcc sees this wait) and the DMA
    }  // (Dg is published by the first sub-phase's barrier)
    // vector-memory operations per sub-phase block, in issue order: [accumulate stage pieces] [DMA of sub-phase u + 3]
    // [stores, weights]; blk = all of them, aft = those after the DMA
    int blk[4] = {0, 0, 0, 0}, aft[4] = {0, 0, 0, 0};
    auto sub = [&](auto jjc, int u) {
        constexpr int JJ = decltype(jjc)::value, S = JJ % 4, J = JJ % 6;
        const int c = u / 6;
        // this wave's pieces of sub-phase u were issued in block u - 3 (and the stage pieces of chunk c - 1 before
        // them); wait for them, then for everyone's
        vm_wait(aft[(S + 1) % 4] + blk[(S + 2) % 4] + blk[(S + 3) % 4]);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        int n = 0, o = 0;
        if constexpr (J == 3) {  // stage this chunk's dX rows (read at the next chunk's store-out)
            if (accumulate) {
                dma_x(c);
                n += n_out;
            }
        }
        // slot (S + 3) % 4 was read by sub-phase u - 1, which every wave has finished: sub-phase u + 3's slice
        if (u + 3 < U) {
            dma(slot(ic<(S + 3) % 4>{}), (u + 3) / 6, (J + 3) % 6);
            n += (J + 3) % 6 < 3 ? n_dma_out : n_in;
        }
        asm volatile("" ::: "memory");  // nothing below moves above the DMA
        if constexpr (J == 0) {
            if (c > 0) {
                store_out(c - 1);
                o += n_st;
                const int M = mid_of(c);
                if (mid_of(c - 1) != M) {  // a new middle: its weights (the previous middle's last use was u - 1),
                    // waited for here (vmcnt(0), which hipcc's bookkeeping sees): one drain per middle change
                    gather(ic<0>{}, ic<0>{}, M);
                    gather(ic<1>{}, ic<0>{}, M);
                    gather(ic<2>{}, ic<0>{}, M);
                    gather(ic<0>{}, ic<1>{}, M);
                    gather(ic<1>{}, ic<1>{}, M);
                    gather(ic<2>{}, ic<1>{}, M);
                    if constexpr (BF) {  // the new middle's diagonal weights (the old ones' last use was u - 1)
                        load_diag(M);
                        __builtin_amdgcn_s_waitcnt(0x0F70);
                        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // uniform branch
                    } else {
                        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
                    }
                }
            }
        }
        asm volatile("" ::: "memory");
        blk[S] = n + o;
        aft[S] = o;
        if constexpr (J < 3) out_sub(slot(ic<S>{}), ic<J>{});
        else in_sub(slot(ic<S>{}), ic<J - 3>{});
    };
#pragma unroll 1
    for (int u0 = 0; u0 < U; u0 += 12) {
        sub(ic<0>{}, u0);
        sub(ic<1>{}, u0 + 1);
        sub(ic<2>{}, u0 + 2);
        sub(ic<3>{}, u0 + 3);
        sub(ic<4>{}, u0 + 4);
        sub(ic<5>{}, u0 + 5);
        if (u0 + 6 >= U) break;
        sub(ic<6>{}, u0 + 6);
        sub(ic<7>{}, u0 + 7);
        sub(ic<8>{}, u0 + 8);
        sub(ic<9>{}, u0 + 9);
        sub(ic<10>{}, u0 + 10);
        sub(ic<11>{}, u0 + 11);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");  // the last chunk's rows in P (and SX)
    store_out(nc - 1);
}

// ---------------------------------------------------------------------------------------------------------
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
                if (rr >= 3 * K - 4) W[off + 4] = w3[k];  // rows 56..59 again as the padding rows 60..63
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

template <bool BF, bool MAP>
int mid_go(unsigned grid, hipStream_t s, const XP& p, const char* name) {
    constexpr int lds = MAP ? ML<BF>::LBYTES_MAP : ML<BF>::LBYTES;
    static bool attr_set = false;  // the kernel's dynamic LDS exceeds the 64 KiB default (set once; idempotent)
    if (!attr_set) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(ngram_mid_kernel<BF, MAP>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
            return pg::set_error(PG_ERR_HIP, "%s: cannot raise the LDS limit", name);
        attr_set = true;
    }
    hipLaunchKernelGGL((ngram_mid_kernel<BF, MAP>), dim3(grid), dim3(XTHREADS), lds, s, p);
    return pg::check_launch(name);
}

// Plan of a MAPPED graph (pg_ngram_mplan_map_f32): node i sits at grid row ginv[i] (-1: off the grid). Each CSR entry
// (i <- j) with both ends on the grid goes to its slot as in ngram_mplan_kernel; every other entry -- an end off the
// grid, or no out / in / diagonal slot -- is marked resid[e] = 1 and left to the residual CSR pass.
__global__ __launch_bounds__(256) void ngram_mplan_map_kernel(int64_t Kn1, int64_t n_nodes, const int64_t* rowptr,
                                                              const int4* edges, const int* ginv, float* plan,
                                                              uint8_t* resid) {
    const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (v >= n_nodes) return;
    const int K = XK;
    const int64_t i = ginv[v];
    for (int64_t e = rowptr[v]; e < rowptr[v + 1]; ++e) {
        const int4 rec = edges[e];
        const int64_t j = i < 0 ? -1 : ginv[rec.x];
        if (j < 0) {
            resid[e] = 1;
            continue;
        }
        const int a = (int)(i / Kn1), b = (int)(i % K);
        const int64_t M = (i % Kn1) / K, suffix = i % Kn1, prefix = i / K;
        int type, c;
        if (j / K == suffix) {
            type = 0;
            c = (int)(j % K);
        } else if (j % Kn1 == prefix) {
            type = 1;
            c = (int)(j / Kn1);
        } else if (j == i) {
            type = 2;
            c = 0;
        } else {
            resid[e] = 1;
            continue;
        }
        resid[e] = 0;
        float* W = plan + M * XMB;
        const float w3[3] = {__int_as_float(rec.y), __int_as_float(rec.z), __int_as_float(rec.w)};
        for (int k = 0; k < 3; ++k) {
            int64_t off;
            if (type == 2) {
                off = XPD + ((int64_t)(a * K + b) * 3 + k);
            } else {
                const int grp = type == 0 ? b : a;
                const int rr = k * K + (type == 0 ? a : b);
                const int m = rr >> 4, li = rr & 15;
                const int s = c >> 2, lk = c & 3;
                off = (type == 0 ? XPO : XPI) + ((int64_t)((grp * 4 + m) * XS + s) * 64 + lk * 16 + li);
                if (rr >= 3 * K - 4) W[off + 4] = w3[k];
            }
            W[off] = w3[k];
        }
    }
}

// Residual pass of a mapped graph (pg_spmm3_resid_f32): LPR lanes per listed row (64 / LPR rows per wave; LPR = 16
// for F <= 64, 32 for F <= 128, else 64), all of its residual entries, the three aggregates in fp32 (lane q: float4
// columns q, q + LPR, ...); the row's Z slices are overwritten (a node off the grid) or added to (a grid node: bit 31
// of its list entry). Compact CSR: entries of list position i at [rowptr[i], rowptr[i + 1]), so the row id and the
// entry range load in parallel (no dependent rowptr read).
__global__ __launch_bounds__(256) void ngram_resid_kernel(int64_t n_list, const int64_t* rowptr, const int* rows,
                                                          const int4* edges, const float* X, int64_t ldx, int F,
                                                          float* Z, int64_t ldz, int lpr) {
    const int lane = threadIdx.x & 63;
    const int64_t i = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * (64 / lpr) + lane / lpr;
    if (i >= n_list) return;
    const int code = rows[i];
    const bool add = code < 0;
    const int64_t row = code & 0x7fffffff;
    const int64_t e0 = rowptr[i], e1 = rowptr[i + 1];
    const int F4 = F >> 2;
    for (int q = lane % lpr; q < F4; q += lpr) {
        f4_t a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0;
        int64_t e = e0;
        for (; e + 4 <= e1; e += 4) {  // four gathers in flight
            int4 r[4];
            f4_t x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) r[u] = edges[e + u];
#pragma unroll
            for (int u = 0; u < 4; ++u) x[u] = *reinterpret_cast<const f4_t*>(X + (int64_t)r[u].x * ldx + 4 * q);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                a0 += __int_as_float(r[u].y) * x[u];
                a1 += __int_as_float(r[u].z) * x[u];
                a2 += __int_as_float(r[u].w) * x[u];
            }
        }
        for (; e < e1; ++e) {
            const int4 r = edges[e];
            const f4_t x = *reinterpret_cast<const f4_t*>(X + (int64_t)r.x * ldx + 4 * q);
            a0 += __int_as_float(r.y) * x;
            a1 += __int_as_float(r.z) * x;
            a2 += __int_as_float(r.w) * x;
        }
        f4_t* z = reinterpret_cast<f4_t*>(Z + row * ldz) + q;
        if (add) {
            a0 += z[0];
            a1 += z[F4];
            a2 += z[2 * F4];
        }
        z[0] = a0;
        z[F4] = a1;
        z[2 * F4] = a2;
    }
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

// bf: X and Z are bf16 rows (the bf16 kernel); ldx / ldz in elements; gmap: the mapped kernel (n_rows = the grid's K^n)
static int mid_launch(int K, int n, int64_t n_rows, const float* plan, const void* X, int64_t ldx, int64_t F,
                      int64_t m_begin, int64_t m_end, bool middle_major, const pg_layer_args_t* gates, void* Z,
                      int64_t ldz, uint32_t flags, unsigned long long* stamps, bool bf, void* stream,
                      const int* gmap = nullptr) {
    const char* name = bf ? "pg_spmm3_ngram_mid_bf16" : "pg_spmm3_ngram_mid_f32";
    int64_t Kn1 = 0, Kn2 = 0;
    PG_REQUIRE(mid_shape(K, n, n_rows, Kn1, Kn2), "bad n-gram shape (K must be %d, n_rows = K^n)", XK);
    if (m_end < 0) m_end = Kn2;
    PG_REQUIRE(0 <= m_begin && m_begin <= m_end && m_end <= Kn2, "middle range [%lld, %lld) outside [0, %lld)",
               (long long)m_begin, (long long)m_end, (long long)Kn2);
    if (m_begin == m_end) return PG_OK;
    PG_REQUIRE(plan && X && Z, "null pointer");
    PG_REQUIRE(ldz >= 3 * F && ldx >= F, "leading dimensions too small");
    if (gates) return pg::set_error(PG_ERR_UNSUPPORTED, "%s: no gated store (the dense kernel gates)", name);
    if (F <= 0 || F % XFC) return pg::set_error(PG_ERR_UNSUPPORTED, "%s: F must be a multiple of %d", name, XFC);
    const int64_t es = bf ? 2 : 4;
    // LDS-DMA pieces of 16 B from every X row; Z stores of 16 B (fp32) / 8 B (bf16)
    const bool z_ok = bf ? ((reinterpret_cast<uintptr_t>(Z) & 7) == 0 && (ldz * es) % 8 == 0)
                         : (pg::aligned16(Z) && (ldz * es) % 16 == 0);
    if (!pg::aligned16(X) || !pg::aligned16(plan) || (ldx * es) % 16 || !z_ok)
        return pg::set_error(PG_ERR_UNSUPPORTED, "%s: needs 16-B aligned X rows and aligned Z rows", name);
    PG_REQUIRE(Kn2 * (F / XFC) < (int64_t(1) << 30), "too many column chunks");
    PG_REQUIRE(!(bf && stamps), "time stamps: fp32 kernel only");
    PG_REQUIRE(!gmap || (!middle_major && m_begin == 0 && m_end == Kn2 && n_rows < (int64_t(1) << 31) && !stamps),
               "the mapped kernel covers the whole grid (< 2^31 rows)");
    XP p{};
    p.gmap = gmap;
    p.Kn1 = Kn1;
    p.Kn2 = Kn2;
    p.m0 = m_begin;
    p.zsa = middle_major ? XK : Kn1;
    p.zsm = middle_major ? XR : XK;
    p.plan = plan;
    p.X = X;
    p.ldx = ldx;
    p.Z = Z;
    p.ldz = ldz;
    p.F = (int)F;
    p.nch = (int)(F / XFC);
    p.remap = (flags & PG_FLAG_NO_XCD_REMAP) ? 0 : 1;
    const int64_t cap = grid_cap();
    const int64_t total = (m_end - m_begin) * p.nch;
    // workgroup pairs on odd / even chunks (even chunk count, an even grid, and the XCD-contiguous block order that
    // keeps a pair on one XCD)
    p.cstride = (p.nch % 2 == 0 && p.remap && total >= 2 && !(flags & PG_FLAG_MID_NO_PAIRS)) ? 2 : 1;
    p.chunks = (int)(total / p.cstride);
    p.stamps = stamps;
    p.early_in = (flags & PG_FLAG_MID_LOADER_SYNC) ? 0 : 1;
    p.exp = stamps ? (int)((flags >> 24) & 15u) : 0;
    unsigned grid = (unsigned)(total < cap ? total : cap);
    if (p.cstride == 2) grid &= ~1u;
    hipStream_t s = (hipStream_t)stream;
    if (gmap) return bf ? mid_go<true, true>(grid, s, p, name) : mid_go<false, true>(grid, s, p, name);
    return bf ? mid_go<true, false>(grid, s, p, name) : mid_go<false, false>(grid, s, p, name);
}

int pg_spmm3_ngram_mid_f32(int K, int n, int64_t n_rows, const float* plan, const float* X, int64_t ldx, int64_t F,
                           const pg_layer_args_t* gates, float* Z, int64_t ldz, uint32_t flags, void* stream) {
    return mid_launch(K, n, n_rows, plan, X, ldx, F, 0, -1, false, gates, Z, ldz, flags, nullptr, false, stream);
}

int pg_ngram_mplan_map_f32(int K, int n, int64_t n_nodes, const int64_t* rowptr, const pg_edge3_t* edges,
                           const int32_t* ginv, float* plan, int64_t plan_floats, uint8_t* resid, void* stream) {
    int64_t Kn1 = 0, Kn2 = 0, grid = 1;
    for (int t = 0; t < n && grid < (int64_t(1) << 40); ++t) grid *= K;
    PG_REQUIRE(mid_shape(K, n, grid, Kn1, Kn2), "the grid must be K^n with K = %d (K=%d, n=%d)", XK, K, n);
    PG_REQUIRE(grid < (int64_t(1) << 31), "grid of %lld rows: the mapped kernel takes < 2^31", (long long)grid);
    PG_REQUIRE(plan_floats >= Kn2 * XMB, "plan buffer too small");
    PG_REQUIRE(n_nodes >= 0 && (n_nodes == 0 || (rowptr && edges && ginv && plan && resid)), "null pointer");
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(plan, 0, sizeof(float) * plan_floats, s) != hipSuccess)
        return pg::set_error(PG_ERR_HIP, "pg_ngram_mplan_map_f32: memset failed");
    if (n_nodes == 0) return PG_OK;
    hipLaunchKernelGGL(ngram_mplan_map_kernel, dim3((unsigned)((n_nodes + 255) / 256)), dim3(256), 0, s, Kn1, n_nodes,
                       rowptr, reinterpret_cast<const int4*>(edges), ginv, plan, resid);
    return pg::check_launch("pg_ngram_mplan_map_f32");
}

int pg_spmm3_ngram_mid_map_f32(int K, int n, const float* plan, const int32_t* gmap, const float* X, int64_t ldx,
                               int64_t F, float* Z, int64_t ldz, uint32_t flags, void* stream) {
    int64_t grid = 1;
    for (int t = 0; t < n && grid < (int64_t(1) << 40); ++t) grid *= K;
    PG_REQUIRE(gmap != nullptr, "null row map");
    return mid_launch(K, n, grid, plan, X, ldx, F, 0, -1, false, nullptr, Z, ldz, flags, nullptr, false, stream, gmap);
}

int pg_spmm3_resid_f32(int64_t n_list, const int64_t* rowptr, const int32_t* rows, const pg_edge3_t* edges,
                       const float* X, int64_t ldx, int64_t F, float* Z, int64_t ldz, uint32_t flags, void* stream) {
    (void)flags;
    PG_REQUIRE(n_list >= 0 && n_list < (int64_t(1) << 31), "bad list length");
    if (n_list == 0) return PG_OK;
    PG_REQUIRE(rowptr && rows && edges && X && Z, "null pointer");
    PG_REQUIRE(F > 0 && F % 4 == 0 && F < (1 << 20), "F must be a positive multiple of 4");
    PG_REQUIRE(ldx >= F && ldz >= 3 * F, "leading dimensions too small");
    if (!pg::aligned16(X) || !pg::aligned16(Z) || ldx % 4 || ldz % 4)
        return pg::set_error(PG_ERR_UNSUPPORTED, "pg_spmm3_resid_f32: needs 16-B aligned rows");
    const int lpr = F <= 64 ? 16 : (F <= 128 ? 32 : 64);  // lanes per row: every lane has a float4 column
    const int64_t per_block = 4 * (64 / lpr);
    hipLaunchKernelGGL(ngram_resid_kernel, dim3((unsigned)((n_list + per_block - 1) / per_block)), dim3(256), 0,
                       (hipStream_t)stream, n_list, rowptr, rows, reinterpret_cast<const int4*>(edges), X, ldx, (int)F,
                       Z, ldz, lpr);
    return pg::check_launch("pg_spmm3_resid_f32");
}

int pg_spmm3_ngram_mid_rows_f32(int K, int n, int64_t n_rows, const float* plan, const float* X, int64_t ldx, int64_t F,
                                int64_t m_begin, int64_t m_end, float* Z, int64_t ldz, uint32_t flags, void* stream) {
    return mid_launch(K, n, n_rows, plan, X, ldx, F, m_begin, m_end, true, nullptr, Z, ldz, flags, nullptr, false,
                      stream);
}

int pg_spmm3_ngram_mid_bf16(int K, int n, int64_t n_rows, const float* plan, const uint16_t* X, int64_t ldx, int64_t F,
                            uint16_t* Z, int64_t ldz, uint32_t flags, void* stream) {
    return mid_launch(K, n, n_rows, plan, X, ldx, F, 0, -1, false, nullptr, Z, ldz, flags, nullptr, true, stream);
}

int pg_spmm3_ngram_mid_rows_bf16(int K, int n, int64_t n_rows, const float* plan, const uint16_t* X, int64_t ldx,
                                 int64_t F, int64_t m_begin, int64_t m_end, uint16_t* Z, int64_t ldz, uint32_t flags,
                                 void* stream) {
    return mid_launch(K, n, n_rows, plan, X, ldx, F, m_begin, m_end, true, nullptr, Z, ldz, flags, nullptr, true,
                      stream);
}

}  // extern "C"

// the transposed middle-tile launch (fp32: off-diagonal part; bf16: the full product)
static int midt_launch(int K, int n, int64_t n_rows, const float* plan, const void* G, int64_t ldg, int64_t F, void* dX,
                       int64_t lddx, int accumulate, uint32_t flags, void* stream, bool bf) {
    const char* name = bf ? "pg_spmm3t_ngram_mid_bf16" : "pg_spmm3t_ngram_mid_offdiag_f32";
    int64_t Kn1 = 0, Kn2 = 0;
    PG_REQUIRE(mid_shape(K, n, n_rows, Kn1, Kn2), "bad n-gram shape (K must be %d, n_rows = K^n)", XK);
    PG_REQUIRE(plan && G && dX, "null pointer");
    PG_REQUIRE(ldg >= 3 * F && lddx >= F, "leading dimensions too small");
    if (F <= 0 || F % XFC) return pg::set_error(PG_ERR_UNSUPPORTED, "%s: F must be a multiple of %d", name, XFC);
    const int64_t es = bf ? 2 : 4;
    if (!pg::aligned16(G) || !pg::aligned16(dX) || !pg::aligned16(plan) || (ldg * es) % 16 || (lddx * es) % 16)
        return pg::set_error(PG_ERR_UNSUPPORTED, "%s: needs 16-B aligned G and dX rows", name);
    PG_REQUIRE(Kn2 * (F / XFC) < (int64_t(1) << 28), "too many column chunks");
    if (n_rows * ldg >= (int64_t(1) << 32) || n_rows * lddx >= (int64_t(1) << 32))
        return pg::set_error(PG_ERR_UNSUPPORTED, "%s: 32-bit per-lane element offsets", name);
    XP p{};
    p.Kn1 = Kn1;
    p.Kn2 = Kn2;
    p.m0 = 0;
    p.zsa = Kn1;
    p.zsm = XK;
    p.plan = plan;
    p.X = G;
    p.ldx = ldg;
    p.Z = dX;
    p.ldz = lddx;
    p.F = (int)F;
    p.nch = (int)(F / XFC);
    p.remap = (flags & PG_FLAG_NO_XCD_REMAP) ? 0 : 1;
    const int64_t total = Kn2 * p.nch;
    p.cstride = (p.nch % 2 == 0 && p.remap && total >= 2 && !(flags & PG_FLAG_MID_NO_PAIRS)) ? 2 : 1;
    p.chunks = (int)(total / p.cstride);
    const int64_t cap = grid_cap();
    unsigned grid = (unsigned)(total < cap ? total : cap);
    if (p.cstride == 2) grid &= ~1u;
    const int acc = accumulate ? 1 : 0;
    if (bf) hipLaunchKernelGGL(ngram_midt2_kernel<true>, dim3(grid), dim3(512), 0, (hipStream_t)stream, p, acc);
    else hipLaunchKernelGGL(ngram_midt2_kernel<false>, dim3(grid), dim3(512), 0, (hipStream_t)stream, p, acc);
    return pg::check_launch(name);
}

extern "C" {

int pg_spmm3t_ngram_mid_offdiag_f32(int K, int n, int64_t n_rows, const float* plan, const float* G, int64_t ldg,
                                    int64_t F, float* dX, int64_t lddx, int accumulate, uint32_t flags, void* stream) {
    return midt_launch(K, n, n_rows, plan, G, ldg, F, dX, lddx, accumulate, flags, stream, false);
}

int pg_spmm3t_ngram_mid_bf16(int K, int n, int64_t n_rows, const float* plan, const uint16_t* G, int64_t ldg, int64_t F,
                             uint16_t* dX, int64_t lddx, int accumulate, uint32_t flags, void* stream) {
    return midt_launch(K, n, n_rows, plan, G, ldg, F, dX, lddx, accumulate, flags, stream, true);
}

#ifdef PG_MID_STAMPS
// diagnostics library only (tools/mid_stamps.py): the same launch with per-block time stamps
int pg_mid_stamped(int K, int n, int64_t n_rows, const float* plan, const float* X, int64_t ldx, int64_t F, float* Z,
                   int64_t ldz, uint32_t flags, unsigned long long* stamps, void* stream) {
    return mid_launch(K, n, n_rows, plan, X, ldx, F, 0, -1, false, nullptr, Z, ldz, flags, stamps, false, stream);
}
#endif
}  // extern "C"
