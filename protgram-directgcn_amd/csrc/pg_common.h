// Shared helpers for the C-ABI entry points: thread-local error message, argument checks, launch
// error capture. Every entry point returns PG_OK or a negative code (include/pg_directgcn.h).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "pg_directgcn.h"

namespace pg {

int set_error(int code, const char* fmt, ...);
void clear_error();

// XCD-contiguous logical block index. The dispatcher deals workgroups round-robin over the 8 XCDs
// (blocks b and b+8 share an XCD, MI355X_MICROARCH.md "Workgroup dispatch"); remapping gives each
// XCD one contiguous range of row blocks so the rows that share neighbour lists share an L2.
// Speed only: any placement gives identical results. Bijective for any grid size.
__device__ __forceinline__ int64_t xcd_logical_block(int64_t b, int64_t nb, bool remap) {
    if (!remap || nb < 16) return b;
    const int64_t q = nb >> 3, r = nb & 7;
    const int64_t x = b & 7, i = b >> 3;
    return x * q + (x < r ? x : r) + i;
}

// Correctly rounded fp32 square root. hipcc lowers sqrtf and __fsqrt_rn on gfx950 to v_sqrt_f32 (faithful,
// not correctly rounded: 19.5M of the 131M 5-gram propagation weights came out 1 ulp below the IEEE value).
// One residual step picks the correctly rounded one of the approximation and its two neighbours (the rule of
// the device libraries' correctly rounded sqrt; checked exhaustively against exact rational arithmetic on
// 60k cases); tiny inputs are scaled by an exact power of two first so the residuals stay normal.
__device__ __forceinline__ float sqrt_rn(float x) {
    if (!(x > 0.0f) || x == __builtin_inff()) return __builtin_sqrtf(x);  // 0, negative, NaN, inf
    const bool tiny = x < 0x1p-96f;
    const float xs = tiny ? x * 0x1p64f : x;
    float y = __builtin_sqrtf(xs);
    const int yi = __float_as_int(y);
    const float ym = __int_as_float(yi - 1), yp = __int_as_float(yi + 1);
    const float vm = __builtin_fmaf(-ym, y, xs), vp = __builtin_fmaf(-yp, y, xs);
    y = vm <= 0.0f ? ym : y;
    y = vp > 0.0f ? yp : y;
    return tiny ? y * 0x1p-32f : y;
}

// Layer-output dropout fused into the dense epilogue (the F.dropout after every layer, protgram_directgcn.py:216):
// element e = m * F_out + j of the layer output is kept when (drop_hash(seed, e) >> 8) >= thr, thr = p * 2^24
// rounded, and a kept element is scaled by 1 / (1 - p). Counter-based (murmur3's 32-bit finalizer of the index
// mixed with the device seed): nothing is stored, and the backward needs no draw at all (act_grad).
__device__ __forceinline__ uint32_t drop_hash(uint64_t seed, uint32_t e) {
    uint32_t x = (e * 0x9E3779B1u + (uint32_t)seed) ^ (uint32_t)(seed >> 32);
    x ^= x >> 16;
    x *= 0x85EBCA6Bu;
    x ^= x >> 13;
    x *= 0xC2B2AE35u;
    x ^= x >> 16;
    return x;
}

// Gradient through the layer's leaky_relu (slope) and, when ds != 0, the fused dropout after it (scale ds = 1/(1-p)),
// from the stored layer output y: a kept element of a leaky_relu output is nonzero (its sign is the pre-activation's),
// a dropped one is 0. ds == 0: leaky_relu' alone, y > 0 ? d : d * slope. (An exactly-zero pre-activation that was kept
// reads as dropped: its gradient is 0 instead of d * ds * slope.)
__device__ __forceinline__ float act_grad(float d, float y, float slope, float ds) {
    if (ds == 0.f) return y > 0.f ? d : d * slope;
    const float e = d * ds;
    return y > 0.f ? e : (y < 0.f ? e * slope : 0.f);
}

// Host side of the fused dropout: threshold and scale from args->drop_p (0 <= p < 1; p == 0: off). Fused dropout
// needs the activation (act_grad recovers the mask from the sign of the output) and, in the forward, a device seed.
inline int drop_params(const pg_layer_args_t* a, uint32_t& thr, float& scale, bool need_seed = true) {
    thr = 0;
    scale = 0.f;
    if (a->drop_p == 0.f) return PG_OK;
    if (!(a->drop_p > 0.f && a->drop_p < 1.f) || !a->act || (need_seed && !a->drop_seed))
        return set_error(PG_ERR_ARG, "fused dropout needs 0 <= drop_p < 1, act and drop_seed (drop_p = %g)",
                         (double)a->drop_p);
    thr = (uint32_t)((double)a->drop_p * 16777216.0 + 0.5);
    scale = (float)(1.0 / (1.0 - (double)a->drop_p));
    return PG_OK;
}

inline int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(PG_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
    return PG_OK;
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

}  // namespace pg

#define PG_REQUIRE(cond, ...)                                         \
    do {                                                              \
        if (!(cond)) return ::pg::set_error(PG_ERR_ARG, __VA_ARGS__); \
    } while (0)
