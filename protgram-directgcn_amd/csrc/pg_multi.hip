// Multi-tensor helpers for the training step: the reference trainer's L2 term
// l2_lambda * sum_p ||p||^2 over ALL parameters (protgram_directgcn_trainer.py:96, :136) costs one norm, one
// pow and one add per parameter forward and as many backward -- ~110 small launches per step for the
// 2-layer model, several of them over the N x F `constant` tensors. Here:
//   pg_multi_sqsum_f32 -- sum_t sum_i x_t[i]^2 over a list of tensors in one launch (fixed-order two-level
//                         reduction: deterministic), the L2 value;
//   pg_multi_axpy_f32  -- y_t += alpha * x_t for every tensor of a list in one launch (the L2 gradient
//                         2*lambda*p added to p.grad);
//   pg_adam_f32        -- Adam over the list in one launch, optionally with the L2 value of the pre-update
//                         parameters as per-chunk partials (pg_multi_sum_f32 adds them in fixed order).
// A list is a device array of pg_tensor_desc_t; work is split into fixed 16K-element chunks.
#include "pg_bf16_util.h"
#include "pg_common.h"

namespace {

// 16K elements per chunk (one 256-thread block each): a 16M-element parameter list gives ~1000 blocks, four per
// CU, whose loads overlap (at 64K, one block of four waves per CU walked its chunk one latency at a time: Adam over
// config 5's per-node state took 2x its bytes' time)
constexpr int64_t CHUNK = 16384;

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
    if ((reinterpret_cast<uintptr_t>(t.x) & 15) == 0) {  // float4 body (chunks start at multiples of 16K)
        const int64_t end4 = beg + ((end - beg) & ~int64_t(3));
        const float4* x4 = reinterpret_cast<const float4*>(t.x);
        for (int64_t i = beg / 4 + threadIdx.x; i < end4 / 4; i += 256) {
            const float4 v = x4[i];
            s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
        }
        for (int64_t i = end4 + threadIdx.x; i < end; i += 256) s += t.x[i] * t.x[i];
    } else {
        for (int64_t i = beg + threadIdx.x; i < end; i += 256) {
            const float v = t.x[i];
            s += v * v;
        }
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
    if (((reinterpret_cast<uintptr_t>(t.x) | reinterpret_cast<uintptr_t>(t.y)) & 15) == 0) {
        const int64_t end4 = beg + ((end - beg) & ~int64_t(3));
        const float4* x4 = reinterpret_cast<const float4*>(t.x);
        float4* y4 = reinterpret_cast<float4*>(t.y);
        for (int64_t i = beg / 4 + threadIdx.x; i < end4 / 4; i += 256) {
            const float4 xv = x4[i];
            float4 yv = y4[i];
            yv.x += alpha * xv.x;
            yv.y += alpha * xv.y;
            yv.z += alpha * xv.z;
            yv.w += alpha * xv.w;
            y4[i] = yv;
        }
        for (int64_t i = end4 + threadIdx.x; i < end; i += 256) t.y[i] += alpha * t.x[i];
    } else {
        for (int64_t i = beg + threadIdx.x; i < end; i += 256) t.y[i] += alpha * t.x[i];
    }
}

// Adam (torch.optim.Adam, foreach path, amsgrad = maximize = False) for every parameter of a list in one launch:
//   g  = grad * inv_scale (+ weight_decay * p)
//   m  = lerp(m, g, 1 - beta1) ; v = v * beta2 + (1 - beta2) * g * g
//   p += (-lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps),   bc_k = 1 - beta_k^t  (t = step + 1, in double)
// hyper (optional): device double[2] = {lr, weight_decay}, read at run time instead of the by-value lr (and added to
// the by-value weight_decay, the trainer's folded L2 gradient 2*l2_lambda): a HIP-graph replay then follows a
// learning-rate schedule written into it between replays (ReduceLROnPlateau, protgram_directgcn_trainer.py:84,102).
// Skipped when *found_inf != 0 (GradScaler's device-side flag; no host sync). sq_partial (optional): chunk b's
// sum of p^2 BEFORE the update into sq_partial[b] -- the trainer's L2 value from the pass that reads p anyway
// (computed on skipped steps too, as the reference's loss includes it).
__device__ __forceinline__ float block_sum256(float s) {
    __shared__ float red[256];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    return red[0];
}

__global__ __launch_bounds__(256) void adam_kernel(int ntens, const pg_adam_desc_t* d, const int64_t* chunk_ptr,
                                                   double lr, double beta1, double beta2, float eps, float weight_decay,
                                                   const float* step, const float* grad_scale, const float* found_inf,
                                                   float* sq_partial, const double* hyper, double wd_extra) {
    const bool skip = found_inf && found_inf[0] != 0.f;
    if (skip && !sq_partial) return;
    const int64_t b = blockIdx.x;
    int lo = 0, hi = ntens;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (chunk_ptr[mid] <= b) lo = mid;
        else hi = mid;
    }
    const pg_adam_desc_t t = d[lo];
    if (hyper) {  // the same double arithmetic the host does for the by-value form: bit-identical updates
        lr = hyper[0];
        weight_decay = (float)(hyper[1] + wd_extra);
    }
    const double tt = (double)step[0] + 1.0;
    const double bc1 = 1.0 - pow(beta1, tt), bc2 = 1.0 - pow(beta2, tt);
    const float step_size = (float)((lr / bc1) * -1.0);
    const float bc2s = (float)sqrt(bc2);
    const float w1 = (float)(1.0 - beta1), b2 = (float)beta2, w2 = (float)(1.0 - beta2);
    const float inv = grad_scale ? (float)(1.0 / (double)grad_scale[0]) : 1.f;
    const int64_t beg = (b - chunk_ptr[lo]) * CHUNK;
    const int64_t end = min(beg + CHUNK, t.numel);
    auto upd = [&](float g, float& p, float& m, float& v) {
        if (grad_scale) g = g * inv;
        if (weight_decay != 0.f) g = g + weight_decay * p;
        m = (w1 < 0.5f) ? m + w1 * (g - m) : g - (g - m) * (1.f - w1);  // at::lerp
        v = v * b2;
        v = v + w2 * g * g;
        const float denom = sqrtf(v) / bc2s + eps;
        p = p + step_size * (m / denom);
    };
    // 16-B accesses when all four arrays allow it (the same per-element arithmetic), scalar tail
    // a bf16 gradient (gtype 1: the bf16 dense backward's dpre, the per-node constant's gradient) is widened
    // exactly -- the same fp32 values as its fp32 copy -- and read in 8-B pieces of four
    const bool gbf = t.gtype == 1;
    const float* gf = static_cast<const float*>(t.g);
    const uint16_t* gb = static_cast<const uint16_t*>(t.g);
    const bool vec = ((reinterpret_cast<uintptr_t>(t.g) & (gbf ? 7 : 15)) |
                      ((reinterpret_cast<uintptr_t>(t.p) | reinterpret_cast<uintptr_t>(t.m) |
                        reinterpret_cast<uintptr_t>(t.v)) & 15)) == 0;
    int64_t i0 = beg;
    float sq = 0.f;
    if (skip) {  // L2 value only
        for (int64_t i = beg + threadIdx.x; i < end; i += 256) sq += t.p[i] * t.p[i];
        sq = block_sum256(sq);
        if (threadIdx.x == 0) sq_partial[b] = sq;
        return;
    }
    if (vec) {
        const int64_t n4 = (end - beg) >> 2;
// Non-temporal loads / stores of the streams (each byte touched once per step; PG_ADAM_NT=0 builds the cached form):
// 0.652 -> 0.582 ms over config 5's 123M parameters, the same bits (tools/r06_adam_probe.py, profiles/r06_ab_adam_nt.txt)
#ifndef PG_ADAM_NT
#define PG_ADAM_NT 1
#endif
        typedef float f4v __attribute__((ext_vector_type(4)));
        auto ld = [](const float* q) {
            if (PG_ADAM_NT) {
                const f4v x = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(q));
                return make_float4(x.x, x.y, x.z, x.w);
            }
            return *reinterpret_cast<const float4*>(q);
        };
        auto st = [](float* q, float4 x) {
            if (PG_ADAM_NT) {
                const f4v y = {x.x, x.y, x.z, x.w};
                __builtin_nontemporal_store(y, reinterpret_cast<f4v*>(q));
            } else {
                *reinterpret_cast<float4*>(q) = x;
            }
        };
        for (int64_t k = threadIdx.x; k < n4; k += 256) {
            const int64_t i = beg + 4 * k;
            // (the bf16 gradient keeps the cached load: non-temporal 8-B loads measured 0.62 against 0.58 ms)
            const float4 g = gbf ? pgbf::unpack4(*reinterpret_cast<const uint2*>(gb + i)) : ld(gf + i);
            float4 p = ld(t.p + i);
            float4 m = ld(t.m + i);
            float4 v = ld(t.v + i);
            sq += p.x * p.x + p.y * p.y + p.z * p.z + p.w * p.w;
            upd(g.x, p.x, m.x, v.x);
            upd(g.y, p.y, m.y, v.y);
            upd(g.z, p.z, m.z, v.z);
            upd(g.w, p.w, m.w, v.w);
            st(t.p + i, p);
            st(t.m + i, m);
            st(t.v + i, v);
        }
        i0 = beg + 4 * n4;
    }
    for (int64_t i = i0 + threadIdx.x; i < end; i += 256) {
        float p = t.p[i], m = t.m[i], v = t.v[i];
        sq += p * p;
        upd(gbf ? __uint_as_float((uint32_t)gb[i] << 16) : gf[i], p, m, v);
        t.p[i] = p;
        t.m[i] = m;
        t.v[i] = v;
    }
    if (sq_partial) {
        sq = block_sum256(sq);
        if (threadIdx.x == 0) sq_partial[b] = sq;
    }
}

__global__ void adam_step_kernel(float* step, const float* found_inf) {
    if (!(found_inf && found_inf[0] != 0.f)) step[0] += 1.f;
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

int pg_multi_sum_f32(int64_t n, const float* x, float* out, void* stream) {
    PG_REQUIRE(n >= 0 && out && (n == 0 || x), "bad arguments");
    hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, n, x, out);
    return pg::check_launch("pg_multi_sum_f32");
}

int pg_adam_f32(int ntens, const pg_adam_desc_t* descs, const int64_t* chunk_ptr, int64_t nchunks, double lr,
                double beta1, double beta2, double eps, double weight_decay, float* step, const float* grad_scale,
                const float* found_inf, float* sq_partial, const double* hyper, void* stream) {
    PG_REQUIRE(ntens >= 0 && nchunks >= 0 && step, "bad arguments");
    PG_REQUIRE(beta1 >= 0 && beta1 < 1 && beta2 >= 0 && beta2 < 1 && lr >= 0 && eps >= 0, "bad hyper-parameters");
    hipStream_t s = (hipStream_t)stream;
    if (nchunks > 0) {
        PG_REQUIRE(descs && chunk_ptr, "null pointer");
        hipLaunchKernelGGL(adam_kernel, dim3((unsigned)nchunks), dim3(256), 0, s, ntens, descs, chunk_ptr, lr, beta1, beta2,
                           (float)eps, hyper ? 0.f : (float)weight_decay, (const float*)step, grad_scale, found_inf,
                           sq_partial, hyper, weight_decay);
    }
    hipLaunchKernelGGL(adam_step_kernel, dim3(1), dim3(1), 0, s, step, found_inf);
    return pg::check_launch("pg_adam_f32");
}

}  // extern "C"

