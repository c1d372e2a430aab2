// LDS-staged tiled variant of the fused three-adjacency SpMM (same result as pg_spmm3_f32, bit for bit).
//
// Why: pg_spmm3_f32 gathers one F-wide source row per pattern entry from L2 (~41 per destination row at
// 4-gram); it runs at the chip's L2->CU gather rate while >90% of those rows are L2 hits. In an n-gram
// graph the rows that share an (n-1)-prefix share their in-neighbours and the rows that share an
// (n-1)-suffix share their out-neighbours, so a K x L tile of the (prefix x suffix) grid needs only
// 20K + 20L + KL distinct source rows for 41KL entries (4.6x fewer at K=4, L=8). The host builds such
// tiles once per graph (graph.py build_tiles: per tile the sorted unique source rows + entries re-indexed
// to LDS slots, each row's entries kept in CSR order).
//
// Kernel: one workgroup per (tile, FC-wide feature chunk). Phase 1 gathers the tile's unique source-row
// chunks into LDS (every lane's loads issued before any LDS write). Phase 2: each row group of FC/4
// lanes accumulates one destination row from LDS -- same separately rounded mul/add sequence in the
// same order as the reference's scatter_add_ -- and writes its three output chunks.
#include "pg_common.h"

namespace {

struct TiledP {
    const int32_t* tile_rowptr;
    const int32_t* tile_rows;
    const int64_t* erow_ptr;
    const int4* entries;
    const int32_t* tile_uptr;
    const int32_t* tile_ucols;
    int64_t n_tiles;
    const float* X;
    int64_t ldx;
    int F;
    float* Z;
    int64_t ldz;
    int remap;
};

__device__ __forceinline__ float fb(int v) { return __int_as_float(v); }
__device__ __forceinline__ float4 axpy4(float4 acc, float w, float4 x) {
    acc.x = __fadd_rn(acc.x, __fmul_rn(w, x.x));
    acc.y = __fadd_rn(acc.y, __fmul_rn(w, x.y));
    acc.z = __fadd_rn(acc.z, __fmul_rn(w, x.z));
    acc.w = __fadd_rn(acc.w, __fmul_rn(w, x.w));
    return acc;
}

template <int FC, int UMAX, int EMAX, int U>
__global__ __launch_bounds__(256) void spmm3_tiled_kernel(TiledP p) {
    constexpr int LPR = FC / 4;           // lanes per row chunk (one float4 each)
    constexpr int GROUPS = 256 / LPR;     // row groups per block
    constexpr int SLD = FC + 4;           // padded LDS row (floats)
    constexpr int PASSES = (UMAX + GROUPS - 1) / GROUPS;
    constexpr int EPASSES = (EMAX + 255) / 256;
    __shared__ __attribute__((aligned(16))) float Xs[UMAX * SLD];
    __shared__ __attribute__((aligned(16))) int4 Rs[EMAX];  // the tile's entry records

    const int nchunk = p.F / FC;
    const int64_t lb = pg::xcd_logical_block(blockIdx.x, gridDim.x, p.remap != 0);
    const int64_t tile = lb / nchunk;
    const int chunk = (int)(lb % nchunk);
    const int grp = threadIdx.x / LPR, t = threadIdx.x % LPR;
    const int fo = chunk * FC + 4 * t;  // feature offset of this lane

    // phase 1: stage the unique source-row chunks and the tile's entry records (all loads in flight
    // before the first LDS write)
    const int u0 = p.tile_uptr[tile];
    const int nu = p.tile_uptr[tile + 1] - u0;
    const int r0 = p.tile_rowptr[tile];
    const int nr = p.tile_rowptr[tile + 1] - r0;
    const int64_t E0 = p.erow_ptr[r0];
    const int ne = (int)(p.erow_ptr[r0 + nr] - E0);
    {
        int4 rv[EPASSES];
#pragma unroll
        for (int k = 0; k < EPASSES; ++k) {
            const int i = threadIdx.x + 256 * k;
            rv[k] = i < ne ? p.entries[E0 + i] : make_int4(0, 0, 0, 0);
        }
        float4 v[PASSES];
#pragma unroll
        for (int k = 0; k < PASSES; ++k) {
            const int slot = grp + k * GROUPS;
            v[k] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (slot < nu) {
                const int64_t col = p.tile_ucols[u0 + slot];
                v[k] = *reinterpret_cast<const float4*>(p.X + col * p.ldx + fo);
            }
        }
#pragma unroll
        for (int k = 0; k < PASSES; ++k) {
            const int slot = grp + k * GROUPS;
            if (slot < nu) *reinterpret_cast<float4*>(&Xs[slot * SLD + 4 * t]) = v[k];
        }
#pragma unroll
        for (int k = 0; k < EPASSES; ++k) {
            const int i = threadIdx.x + 256 * k;
            if (i < ne) Rs[i] = rv[k];
        }
    }
    __syncthreads();

    // phase 2: destination rows of the tile, from LDS only
    for (int ri = grp; ri < nr; ri += GROUPS) {
        const int64_t pos = r0 + ri;
        const int64_t row = p.tile_rows[pos];
        const int e0 = (int)(p.erow_ptr[pos] - E0), e1 = (int)(p.erow_ptr[pos + 1] - E0);
        float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0, a2 = a0;
        int e = e0;
        for (; e + U <= e1; e += U) {
            int4 r[U];
#pragma unroll
            for (int u = 0; u < U; ++u) r[u] = Rs[e + u];
            float4 xv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) xv[u] = *reinterpret_cast<const float4*>(&Xs[r[u].x * SLD + 4 * t]);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                a0 = axpy4(a0, fb(r[u].y), xv[u]);
                a1 = axpy4(a1, fb(r[u].z), xv[u]);
                a2 = axpy4(a2, fb(r[u].w), xv[u]);
            }
        }
        for (; e < e1; ++e) {
            const int4 r = Rs[e];
            const float4 xv = *reinterpret_cast<const float4*>(&Xs[r.x * SLD + 4 * t]);
            a0 = axpy4(a0, fb(r.y), xv);
            a1 = axpy4(a1, fb(r.z), xv);
            a2 = axpy4(a2, fb(r.w), xv);
        }
        float* z = p.Z + row * p.ldz + fo;
        *reinterpret_cast<float4*>(z) = a0;
        *reinterpret_cast<float4*>(z + p.F) = a1;
        *reinterpret_cast<float4*>(z + 2 * p.F) = a2;
    }
}

template <int FC, int UMAX, int EMAX>
void launch(const TiledP& p, uint32_t flags, hipStream_t s) {
    const int64_t nb = p.n_tiles * (p.F / FC);
    if (flags & PG_FLAG_UNROLL4)
        hipLaunchKernelGGL((spmm3_tiled_kernel<FC, UMAX, EMAX, 4>), dim3((unsigned)nb), dim3(256), 0, s, p);
    else
        hipLaunchKernelGGL((spmm3_tiled_kernel<FC, UMAX, EMAX, 8>), dim3((unsigned)nb), dim3(256), 0, s, p);
}

}  // namespace

extern "C" int pg_spmm3_tiled_f32(const pg_tiles_t* tl, const float* X, int64_t ldx, int64_t F, float* Z, int64_t ldz,
                                  uint32_t flags, void* stream) {
    PG_REQUIRE(tl != nullptr, "null tiles");
    if (tl->n_tiles == 0) return PG_OK;
    PG_REQUIRE(tl->n_tiles > 0 && tl->tile_rowptr && tl->tile_rows && tl->erow_ptr && tl->entries && tl->tile_uptr &&
                   tl->tile_ucols,
               "incomplete tiles");
    PG_REQUIRE(X && Z && F > 0 && ldx >= F && ldz >= 3 * F, "bad X/Z");
    PG_REQUIRE(F % 32 == 0 && ldx % 4 == 0 && ldz % 4 == 0 && pg::aligned16(X) && pg::aligned16(Z),
               "tiled kernel needs F % 32 == 0 and 16-B aligned rows");
    const bool wide = (flags & PG_FLAG_TILED_FC64) && F % 64 == 0;
    const int64_t umax = wide ? 192 : 320;
    if (tl->max_ucols > umax || tl->max_entries > 1344)
        return pg::set_error(PG_ERR_UNSUPPORTED, "tile stages %d source rows / %d entries (> %lld / 1344)",
                             tl->max_ucols, tl->max_entries, (long long)umax);
    TiledP p{tl->tile_rowptr, tl->tile_rows, tl->erow_ptr, reinterpret_cast<const int4*>(tl->entries), tl->tile_uptr,
             tl->tile_ucols, tl->n_tiles, X, ldx, (int)F, Z, ldz, (flags & PG_FLAG_NO_XCD_REMAP) ? 0 : 1};
    hipStream_t s = (hipStream_t)stream;
    if (wide) launch<64, 192, 1344>(p, flags, s);
    else launch<32, 320, 1344>(p, flags, s);
    return pg::check_launch("pg_spmm3_tiled_f32");
}

// ------------------------------------------------------------------------------------------------
// v3: full-width rows. One workgroup per tile of at most RPB = 256/LPR rows (one row group of LPR = F/4
// lanes per row, F in {64, 128, 256}); phase 1 stages the tile's unique source rows (<= UMAX) whole,
// LPR lanes x 16 B = one contiguous row per row-group instruction (the access shape the feature gathers
// already have), with the slot's column index broadcast inside the group by __shfl (LDS crossbar, not
// the L1 data path). Phase 2: each row group reads its records through a private LDS window (as
// pg_spmm.hip variant C) and its source rows from the staged tile. Same per-row order: bit-exact.
// ------------------------------------------------------------------------------------------------
namespace {

template <int LPR, int UMAX, int U>
__global__ __launch_bounds__(256) void spmm3_tiled_full_kernel(TiledP p) {
    constexpr int RPB = 256 / LPR;
    constexpr int PASSES = (UMAX + RPB - 1) / RPB;  // staged rows per row group
    static_assert(PASSES <= LPR, "one column index per lane");
    __shared__ __attribute__((aligned(16))) float4 Xs[UMAX * LPR];
    __shared__ __attribute__((aligned(16))) int4 win[RPB][LPR];

    const int64_t tile = pg::xcd_logical_block(blockIdx.x, gridDim.x, p.remap != 0);
    const int grp = threadIdx.x / LPR, t = threadIdx.x % LPR;
    const int u0 = p.tile_uptr[tile];
    const int nu = p.tile_uptr[tile + 1] - u0;
    const int r0 = p.tile_rowptr[tile];
    const int nr = p.tile_rowptr[tile + 1] - r0;
    const float4* __restrict__ X4 = reinterpret_cast<const float4*>(p.X);
    const int64_t ldx4 = p.ldx >> 2;

    // this group's row and its first record window (in flight during phase 1)
    const bool live = grp < nr;
    int64_t row = 0, e0 = 0, e1 = 0;
    if (live) {
        row = p.tile_rows[r0 + grp];
        e0 = p.erow_ptr[r0 + grp];
        e1 = p.erow_ptr[r0 + grp + 1];
    }
    int4 nxt = (e0 + t < e1) ? p.entries[e0 + t] : make_int4(0, 0, 0, 0);

    // phase 1: row group g stages slots g, g + RPB, ...; lane k of the group fetches the k-th slot's
    // column index, then the group loads each slot's row (LPR x 16 B contiguous)
    {
        const int myslot = grp + RPB * t;
        const int mycol = (t < PASSES && myslot < nu) ? p.tile_ucols[u0 + myslot] : 0;
        float4 v[PASSES];
#pragma unroll
        for (int k = 0; k < PASSES; ++k) {
            const int col = __shfl(mycol, k, LPR);
            const int slot = grp + RPB * k;
            v[k] = slot < nu ? X4[(int64_t)col * ldx4 + t] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int k = 0; k < PASSES; ++k) {
            const int slot = grp + RPB * k;
            if (slot < nu) Xs[slot * LPR + t] = v[k];
        }
    }
    __syncthreads();
    if (!live) return;

    // phase 2
    float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0, a2 = a0;
    int4* mywin = win[grp];
    for (int64_t w0 = e0; w0 < e1; w0 += LPR) {
        __builtin_amdgcn_wave_barrier();
        mywin[t] = nxt;
        __builtin_amdgcn_wave_barrier();
        if (w0 + LPR + t < e1) nxt = p.entries[w0 + LPR + t];
        const int n = (int)((e1 - w0) < LPR ? (e1 - w0) : LPR);
        int j = 0;
        for (; j + U <= n; j += U) {
            int4 r[U];
            float4 xv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) r[u] = mywin[j + u];
#pragma unroll
            for (int u = 0; u < U; ++u) xv[u] = Xs[r[u].x * LPR + t];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                a0 = axpy4(a0, fb(r[u].y), xv[u]);
                a1 = axpy4(a1, fb(r[u].z), xv[u]);
                a2 = axpy4(a2, fb(r[u].w), xv[u]);
            }
        }
        for (; j < n; ++j) {
            const int4 r = mywin[j];
            const float4 xv = Xs[r.x * LPR + t];
            a0 = axpy4(a0, fb(r.y), xv);
            a1 = axpy4(a1, fb(r.z), xv);
            a2 = axpy4(a2, fb(r.w), xv);
        }
    }
    float4* z = reinterpret_cast<float4*>(p.Z + row * p.ldz) + t;
    z[0] = a0;
    z[LPR] = a1;
    z[2 * LPR] = a2;
}

}  // namespace

extern "C" int pg_spmm3_tiled_rows_f32(const pg_tiles_t* tl, const float* X, int64_t ldx, int64_t F, float* Z,
                                       int64_t ldz, uint32_t flags, void* stream) {
    PG_REQUIRE(tl != nullptr, "null tiles");
    if (tl->n_tiles == 0) return PG_OK;
    PG_REQUIRE(tl->tile_rowptr && tl->tile_rows && tl->erow_ptr && tl->entries && tl->tile_uptr && tl->tile_ucols,
               "incomplete tiles");
    PG_REQUIRE(X && Z && ldx >= F && ldz >= 3 * F && ldx % 4 == 0 && ldz % 4 == 0 && pg::aligned16(X) &&
                   pg::aligned16(Z),
               "bad X/Z");
    TiledP p{tl->tile_rowptr, tl->tile_rows, tl->erow_ptr, reinterpret_cast<const int4*>(tl->entries), tl->tile_uptr,
             tl->tile_ucols, tl->n_tiles, X, ldx, (int)F, Z, ldz, (flags & PG_FLAG_NO_XCD_REMAP) ? 0 : 1};
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid((unsigned)tl->n_tiles);
    // capacities: F=128 -> 8 rows, 128 staged rows (64 KiB); F=64 -> 16 rows, 192 (48 KiB); F=256 -> 4, 64
    if (F == 128 && tl->max_rows <= 8 && tl->max_ucols <= 128) {
        hipLaunchKernelGGL((spmm3_tiled_full_kernel<32, 128, 4>), grid, dim3(256), 0, s, p);
    } else if (F == 64 && tl->max_rows <= 16 && tl->max_ucols <= 192) {
        hipLaunchKernelGGL((spmm3_tiled_full_kernel<16, 192, 4>), grid, dim3(256), 0, s, p);
    } else if (F == 256 && tl->max_rows <= 4 && tl->max_ucols <= 64) {
        hipLaunchKernelGGL((spmm3_tiled_full_kernel<64, 64, 4>), grid, dim3(256), 0, s, p);
    } else {
        return pg::set_error(PG_ERR_UNSUPPORTED, "tiles (rows %d, staged %d) do not fit F=%lld", tl->max_rows,
                             tl->max_ucols, (long long)F);
    }
    return pg::check_launch("pg_spmm3_tiled_rows_f32");
}
