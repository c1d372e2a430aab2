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
