// Exact three-way bf16 splitting of fp32 operands for the split-bf16 MFMA kernels (pg_dense.hip forward,
// pg_dense_bwd.hip weight gradient). A float v splits exactly into v0 + v1 + v2 with v0 = bf16(v),
// v1 = bf16(v - v0), v2 = v - v0 - v1 (round-to-nearest-even at each step; both subtractions are exact in fp32 and
// v2 has at most 8 significant bits, so it is a bf16). A product a*w is then the six bf16 products a_i w_j with
// i + j <= 2 (the dropped a1 w2, a2 w1, a2 w2 are below 2^-24 |a w|), accumulated in fp32 by
// v_mfma_f32_16x16x32_bf16.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace pgx3 {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

// bf16 pair (RNE, v_cvt_pk_bf16_f32) and the two values it represents, back in fp32
__device__ __forceinline__ uint32_t bf2(float a, float b, float& fa, float& fb) {
    const uint32_t u = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{a, b}, bf16x2_t));
    fa = __uint_as_float(u << 16);
    fb = __uint_as_float(u & 0xffff0000u);
    return u;
}
// exact three-way split of 8 fp32 values into three bf16x8 operands
__device__ __forceinline__ void split8(const float (&v)[8], uint4& s0, uint4& s1, uint4& s2) {
    uint32_t w0[4], w1[4], w2[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        float a = v[2 * i], b = v[2 * i + 1], fa, fb;
        w0[i] = bf2(a, b, fa, fb);
        a -= fa;
        b -= fb;
        w1[i] = bf2(a, b, fa, fb);
        a -= fa;
        b -= fb;
        w2[i] = bf2(a, b, fa, fb);
    }
    s0 = make_uint4(w0[0], w0[1], w0[2], w0[3]);
    s1 = make_uint4(w1[0], w1[1], w1[2], w1[3]);
    s2 = make_uint4(w2[0], w2[1], w2[2], w2[3]);
}
__device__ __forceinline__ f32x4_t mfma_bf(uint4 a, uint4 b, f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                   0, 0, 0);
}
// the six products of a split pair, small terms first (the order of every split-bf16 kernel here)
__device__ __forceinline__ f32x4_t mfma_x3(uint4 a0, uint4 a1, uint4 a2, uint4 b0, uint4 b1, uint4 b2, f32x4_t c) {
    c = mfma_bf(a2, b0, c);
    c = mfma_bf(a1, b1, c);
    c = mfma_bf(a0, b2, c);
    c = mfma_bf(a1, b0, c);
    c = mfma_bf(a0, b1, c);
    c = mfma_bf(a0, b0, c);
    return c;
}

}  // namespace pgx3
