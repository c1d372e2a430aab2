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
