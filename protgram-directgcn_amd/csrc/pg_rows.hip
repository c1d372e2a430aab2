// Row gather / scatter by an index list (the multi-GPU exchange's data movement, shard.py): the rows a rank sends
// are gathered from its output, the rows it receives are scattered into the global-layout input of the next layer.
// Byte-generic (fp32 and bf16 rows alike). 16-B rows pieces when the rows and strides allow it (half a wave per
// 512-B row: coalesced 16-B loads and stores), 4-B pieces otherwise. An index outside [0, n_rows) of the indexed
// side is an error detected on the host only if the caller checks it; the product's index lists are built from the
// partition's closed form (shard.middle_partition) and checked there.
#include "pg_common.h"

namespace {

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

}  // extern "C"
