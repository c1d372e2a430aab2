// bf16 helpers shared by the bf16-mode kernels: bit-level conversions (round-to-nearest-even, as
// c10::BFloat16) and the 32x32x16 bf16 MFMA operand type.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace pgbf {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ uint32_t f2bf(float f) {  // c10::BFloat16 round_to_nearest_even
    const uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0u;
    return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ uint32_t pack2(float a, float b) { return f2bf(a) | (f2bf(b) << 16); }
__device__ __forceinline__ void unpack8(uint4 v, float (&f)[8]) {
    f[0] = lo(v.x); f[1] = hi(v.x); f[2] = lo(v.y); f[3] = hi(v.y);
    f[4] = lo(v.z); f[5] = hi(v.z); f[6] = lo(v.w); f[7] = hi(v.w);
}
__device__ __forceinline__ uint4 pack8(const float (&f)[8]) {
    return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}
__device__ __forceinline__ float4 unpack4(uint2 v) { return make_float4(lo(v.x), hi(v.x), lo(v.y), hi(v.y)); }
__device__ __forceinline__ uint2 pack4(float4 f) { return make_uint2(pack2(f.x, f.y), pack2(f.z, f.w)); }

}  // namespace pgbf
