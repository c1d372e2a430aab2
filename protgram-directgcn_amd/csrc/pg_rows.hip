// Row gather / scatter by an index list (the multi-GPU exchange's data movement, shard.py): the rows a rank sends
// are gathered from its output, the rows it receives are scattered into the global-layout input of the next layer.
// Byte-generic (fp32 and bf16 rows alike). 16-B rows pieces when the rows and strides allow it (half a wave per
// 512-B row: coalesced 16-B loads and stores), 4-B pieces otherwise. An index outside [0, n_rows) of the indexed
// side is an error detected on the host only if the caller checks it; the product's index lists are built from the
// partition's closed form (shard.middle_partition) and checked there.
#include "pg_bf16_util.h"
#include "pg_common.h"

namespace {

// out[i, f] = sum over entries e in [rowptr[i], rowptr[i + 1]) of src_e[f], in entry order, in fp32: idx[e] >= 0 is
// row idx[e] of A (fp32), idx[e] < 0 row -1 - idx[e] of B (fp32 or bf16). One thread per (row, 4 features).
template <bool BBF, bool OBF>
__global__ __launch_bounds__(256) void gather_sum_kernel(const float* A, int64_t lda, const void* B, int64_t ldb,
                                                         const int64_t* rowptr, const int32_t* idx, int64_t n, int q4,
                                                         void* out, int64_t ldo) {
    const int64_t total = n * q4;
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
        const int64_t i = t / q4;
        const int q = (int)(t - i * q4);
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        const int64_t e1 = rowptr[i + 1];
        // entries in batches of 4: the index loads, then the row loads, are issued together (not one dependent
        // pair per entry); the adds keep the entry order
        for (int64_t e = rowptr[i]; e < e1; e += 4) {
            int32_t v[4];
            float4 x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = e + u < e1 ? idx[e + u] : 0;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (e + u < e1) {
                    if (v[u] >= 0) {
                        x[u] = *reinterpret_cast<const float4*>(A + (int64_t)v[u] * lda + 4 * q);
                    } else if constexpr (BBF) {
                        x[u] = pgbf::unpack4(*reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(B) +
                                                                          (int64_t)(-1 - v[u]) * ldb + 4 * q));
                    } else {
                        x[u] = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(B) +
                                                                (int64_t)(-1 - v[u]) * ldb + 4 * q);
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (e + u < e1) {
                    acc.x += x[u].x;
                    acc.y += x[u].y;
                    acc.z += x[u].z;
                    acc.w += x[u].w;
                }
            }
        }
        if constexpr (OBF)
            *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) + i * ldo + 4 * q) = pgbf::pack4(acc);
        else
            *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + i * ldo + 4 * q) = acc;
    }
}

template <typename T, bool SCATTER>
__global__ __launch_bounds__(256) void rows_kernel(const char* src, int64_t ld_src, char* dst, int64_t ld_dst,
                                                   const int64_t* idx, int64_t n, int64_t pieces) {
    const int64_t total = n * pieces;
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
        const int64_t i = t / pieces, q = t - i * pieces;
        const int64_t j = idx[i];
        const int64_t si = SCATTER ? i : j, di = SCATTER ? j : i;
        const T v = *reinterpret_cast<const T*>(src + si * ld_src + q * (int64_t)sizeof(T));
        *reinterpret_cast<T*>(dst + di * ld_dst + q * (int64_t)sizeof(T)) = v;
    }
}

template <bool SCATTER>
int rows_launch(const void* src, int64_t ld_src, void* dst, int64_t ld_dst, const int64_t* idx, int64_t n,
                int64_t row_bytes, void* stream, const char* name) {
    PG_REQUIRE(n >= 0 && row_bytes >= 0, "%s: negative size", name);
    if (n == 0 || row_bytes == 0) return PG_OK;
    PG_REQUIRE(src && dst && idx, "%s: null pointer", name);
    PG_REQUIRE(ld_src >= row_bytes && ld_dst >= row_bytes, "%s: row stride smaller than the row", name);
    PG_REQUIRE(row_bytes % 4 == 0 && ld_src % 4 == 0 && ld_dst % 4 == 0, "%s: rows must be whole 4-B words", name);
    hipStream_t s = (hipStream_t)stream;
    const bool v16 = row_bytes % 16 == 0 && ld_src % 16 == 0 && ld_dst % 16 == 0 && pg::aligned16(src) &&
                     pg::aligned16(dst);
    const int64_t pieces = v16 ? row_bytes / 16 : row_bytes / 4;
    const int64_t blocks = (n * pieces + 255) / 256;
    const unsigned grid = (unsigned)(blocks < 65536 ? blocks : 65536);
    if (v16)
        hipLaunchKernelGGL((rows_kernel<uint4, SCATTER>), dim3(grid), dim3(256), 0, s, (const char*)src, ld_src,
                           (char*)dst, ld_dst, idx, n, pieces);
    else
        hipLaunchKernelGGL((rows_kernel<uint32_t, SCATTER>), dim3(grid), dim3(256), 0, s, (const char*)src, ld_src,
                           (char*)dst, ld_dst, idx, n, pieces);
    return pg::check_launch(name);
}

}  // namespace

extern "C" {

int pg_rows_gather(const void* src, int64_t ld_src, const int64_t* idx, int64_t n, int64_t row_bytes, void* dst,
                   int64_t ld_dst, void* stream) {
    return rows_launch<false>(src, ld_src, dst, ld_dst, idx, n, row_bytes, stream, "pg_rows_gather");
}

int pg_rows_scatter(const void* src, int64_t ld_src, const int64_t* idx, int64_t n, int64_t row_bytes, void* dst,
                    int64_t ld_dst, void* stream) {
    return rows_launch<true>(src, ld_src, dst, ld_dst, idx, n, row_bytes, stream, "pg_rows_scatter");
}

// out [n_out, F] (fp32 or bf16) = per row the fp32 sum of its entries' rows of A (fp32; idx >= 0) and B (fp32 or
// bf16; idx < 0: row -1 - idx), in entry order (the middle partition's backward: the scatter kernel's parts of a row
// plus the rows received for it, shard.py)
int pg_rows_gather_sum(const float* A, int64_t lda, const void* B, int64_t ldb, int b_bf16, const int64_t* rowptr,
                       const int32_t* idx, int64_t n_out, int64_t F, void* out, int64_t ldo, int out_bf16,
                       void* stream) {
    const char* name = "pg_rows_gather_sum";
    PG_REQUIRE(n_out >= 0 && F >= 0, "%s: negative size", name);
    if (n_out == 0 || F == 0) return PG_OK;
    PG_REQUIRE(rowptr && idx && out, "%s: null pointer", name);
    PG_REQUIRE(F % 4 == 0, "%s: F = %lld must be a multiple of 4", name, (long long)F);
    PG_REQUIRE(lda >= F && ldb >= F && ldo >= F && lda % 4 == 0 && ldb % 4 == 0 && ldo % 4 == 0,
               "%s: row strides must be >= F and multiples of 4", name);
    PG_REQUIRE((!A || pg::aligned16(A)) && (!B || (reinterpret_cast<uintptr_t>(B) & (b_bf16 ? 7u : 15u)) == 0) &&
                   (reinterpret_cast<uintptr_t>(out) & (out_bf16 ? 7u : 15u)) == 0,
               "%s: misaligned base pointer", name);
    const int q4 = (int)(F / 4);
    const int64_t blocks = (n_out * q4 + 255) / 256;
    const dim3 grid((unsigned)(blocks < 65536 ? blocks : 65536));
    hipStream_t s = (hipStream_t)stream;
    if (b_bf16 && out_bf16)
        hipLaunchKernelGGL((gather_sum_kernel<true, true>), grid, dim3(256), 0, s, A, lda, B, ldb, rowptr, idx, n_out, q4, out, ldo);
    else if (b_bf16)
        hipLaunchKernelGGL((gather_sum_kernel<true, false>), grid, dim3(256), 0, s, A, lda, B, ldb, rowptr, idx, n_out, q4, out, ldo);
    else if (out_bf16)
        hipLaunchKernelGGL((gather_sum_kernel<false, true>), grid, dim3(256), 0, s, A, lda, B, ldb, rowptr, idx, n_out, q4, out, ldo);
    else
        hipLaunchKernelGGL((gather_sum_kernel<false, false>), grid, dim3(256), 0, s, A, lda, B, ldb, rowptr, idx, n_out, q4, out, ldo);
    return pg::check_launch(name);
}

}  // extern "C"
