// n-gram transition producer: the window / transition extraction of
// src/pipeline/data_builder.py:38-54 (_extract_ngrams_from_sequence_tuple, _extract_edges_from_sequence_tuple)
// as integer keys on the GPU. A window of n characters maps to key = sum_j code(c_j) * K^(n-1-j) with an
// order-preserving code (code = rank of the character among the characters present), so the numeric order of
// keys is the sorted-string order the reference uses for node ids (data_builder.py:171-175). Byte work,
// HBM-bound: one block per sequence, threads stride its positions (neighbouring windows share bytes in L1).
#include "pg_common.h"

namespace {

__global__ __launch_bounds__(256) void ngram_keys_kernel(int64_t nseq, const int64_t* offsets, const uint8_t* bytes,
                                                         const int32_t* lut, int n, int64_t K, int64_t* keys,
                                                         int64_t* next_keys) {
    for (int64_t sq = blockIdx.x; sq < nseq; sq += gridDim.x) {
        const int64_t beg = offsets[sq], end = offsets[sq + 1];
        for (int64_t p = beg + threadIdx.x; p < end; p += blockDim.x) {
            int64_t key = -1, nxt = -1;
            if (p + n <= end) {
                key = 0;
                for (int j = 0; j < n; ++j) key = key * K + lut[bytes[p + j]];
                if (p + n + 1 <= end) {  // the window starting at p+1 lies in the same sequence
                    nxt = 0;
                    for (int j = 1; j <= n; ++j) nxt = nxt * K + lut[bytes[p + j]];
                }
            }
            keys[p] = key;
            next_keys[p] = nxt;
        }
    }
}

}  // namespace

extern "C" int pg_ngram_keys(int64_t nseq, const int64_t* offsets, const uint8_t* bytes, const int32_t* lut, int n,
                             int64_t K, int64_t* keys, int64_t* next_keys, void* stream) {
    PG_REQUIRE(nseq >= 0 && n >= 1 && K >= 1, "bad arguments nseq=%lld n=%d K=%lld", (long long)nseq, n, (long long)K);
    if (nseq == 0) return PG_OK;
    PG_REQUIRE(offsets && bytes && lut && keys && next_keys, "null pointer");
    // K^n must fit a signed 64-bit key
    double bits = 0;
    for (int j = 0; j < n; ++j) bits += __builtin_log2((double)K);
    PG_REQUIRE(bits < 62.5, "K^n = %lld^%d does not fit a 64-bit key", (long long)K, n);
    const unsigned nb = (unsigned)(nseq < 65536 ? nseq : 65536);
    hipLaunchKernelGGL(ngram_keys_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, nseq, offsets, bytes, lut, n, K,
                       keys, next_keys);
    return pg::check_launch("pg_ngram_keys");
}
