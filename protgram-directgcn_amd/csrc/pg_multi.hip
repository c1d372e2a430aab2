// Multi-tensor helpers for the training step: the reference trainer's L2 term
// l2_lambda * sum_p ||p||^2 over ALL parameters (protgram_directgcn_trainer.py:96, :136) costs one norm, one
// pow and one add per parameter forward and as many backward -- ~110 small launches per step for the
// 2-layer model, several of them over the N x F `constant` tensors. Here:
//   pg_multi_sqsum_f32 -- sum_t sum_i x_t[i]^2 over a list of tensors in one launch (fixed-order two-level
//                         reduction: deterministic), the L2 value;
//   pg_multi_axpy_f32  -- y_t += alpha * x_t for every tensor of a list in one launch (the L2 gradient
//                         2*lambda*p added to p.grad).
// A list is a device array of pg_tensor_desc_t; work is split into fixed 64K-element chunks.
#include "pg_common.h"

namespace {

constexpr int64_t CHUNK = 65536;

__global__ __launch_bounds__(256) void sqsum_chunks_kernel(int ntens, const pg_tensor_desc_t* d,
                                                           const int64_t* chunk_ptr, float* partial) {
    // block b handles chunk b (a chunk never spans tensors); partial[b] = sum of squares of that chunk
    const int64_t b = blockIdx.x;
    int lo = 0, hi = ntens;  // tensor of chunk b: chunk_ptr[t] <= b < chunk_ptr[t+1]
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (chunk_ptr[mid] <= b) lo = mid;
        else hi = mid;
    }
    const pg_tensor_desc_t t = d[lo];
    const int64_t beg = (b - chunk_ptr[lo]) * CHUNK;
    const int64_t end = min(beg + CHUNK, t.numel);
    float s = 0.f;
    for (int64_t i = beg + threadIdx.x; i < end; i += 256) {
        const float v = t.x[i];
        s += v * v;
    }
    __shared__ float red[256];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[b] = red[0];
}

__global__ __launch_bounds__(256) void sum_partials_kernel(int64_t n, const float* partial, float* out) {
    __shared__ float red[256];
    float s = 0.f;
    for (int64_t i = threadIdx.x; i < n; i += 256) s += partial[i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[0] = red[0];
}

__global__ __launch_bounds__(256) void axpy_chunks_kernel(int ntens, const pg_tensor_desc_t* d, const int64_t* chunk_ptr,
                                                          float alpha, const float* alpha_scale) {
    if (alpha_scale) alpha *= alpha_scale[0];
    const int64_t b = blockIdx.x;
    int lo = 0, hi = ntens;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (chunk_ptr[mid] <= b) lo = mid;
        else hi = mid;
    }
    const pg_tensor_desc_t t = d[lo];
    const int64_t beg = (b - chunk_ptr[lo]) * CHUNK;
    const int64_t end = min(beg + CHUNK, t.numel);
    for (int64_t i = beg + threadIdx.x; i < end; i += 256) t.y[i] += alpha * t.x[i];
}

}  // namespace

extern "C" {

int64_t pg_multi_chunks(int64_t numel) { return (numel + CHUNK - 1) / CHUNK; }

int pg_multi_sqsum_f32(int ntens, const pg_tensor_desc_t* descs, const int64_t* chunk_ptr, int64_t nchunks,
                       float* partial, float* out, void* stream) {
    PG_REQUIRE(ntens >= 0 && nchunks >= 0 && out, "bad arguments");
    hipStream_t s = (hipStream_t)stream;
    if (nchunks > 0) {
        PG_REQUIRE(descs && chunk_ptr && partial, "null pointer");
        hipLaunchKernelGGL(sqsum_chunks_kernel, dim3((unsigned)nchunks), dim3(256), 0, s, ntens, descs, chunk_ptr, partial);
    }
    hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, s, nchunks, (const float*)partial, out);
    return pg::check_launch("pg_multi_sqsum_f32");
}

int pg_multi_axpy_f32(int ntens, const pg_tensor_desc_t* descs, const int64_t* chunk_ptr, int64_t nchunks, float alpha,
                      const float* alpha_scale, void* stream) {
    PG_REQUIRE(ntens >= 0 && nchunks >= 0, "bad arguments");
    if (nchunks == 0) return PG_OK;
    PG_REQUIRE(descs && chunk_ptr, "null pointer");
    hipLaunchKernelGGL(axpy_chunks_kernel, dim3((unsigned)nchunks), dim3(256), 0, (hipStream_t)stream, ntens, descs,
                       chunk_ptr, alpha, alpha_scale);
    return pg::check_launch("pg_multi_axpy_f32");
}

}  // extern "C"
