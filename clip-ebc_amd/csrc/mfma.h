// MFMA fragment helpers for gfx950 (CDNA4).
//
// Every operand is handled as an "8-element fragment": for the 16x16x32 f16/bf16 MFMA, lane l
// holds A[m = l&15][k = 8*(l>>4) + j] and B[k = 8*(l>>4) + j][n = l&15], j = 0..7.  The exact-f32
// path (parity mode) issues eight v_mfma_f32_16x16x4_f32, the j-th on element j of the same
// fragments (k index permuted consistently on both operands, so the product is unchanged), which
// lets one tiling/LDS layout serve f32, f16 and bf16.
// C/D layout (all dtypes): acc[i] = C[row = 4*(l>>4) + i][col = l&15].
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

namespace ebc {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

#define EBC_LDS(p) ((__attribute__((address_space(3))) void*)(p))

struct EF32 {
    using T = float;
    using Frag = f32x8;
    static constexpr int BYTES = 4;
    __device__ static inline float to(T v) { return v; }
    __device__ static inline T from(float v) { return v; }
};
struct EF16 {
    using T = _Float16;
    using Frag = f16x8;
    static constexpr int BYTES = 2;
    __device__ static inline float to(T v) { return (float)v; }
    __device__ static inline T from(float v) { return (T)v; }
};
struct EBF16 {
    using T = __bf16;
    using Frag = bf16x8;
    static constexpr int BYTES = 2;
    __device__ static inline float to(T v) { return (float)v; }
    __device__ static inline T from(float v) { return (T)v; }
};

__device__ __forceinline__ f32x4 mma(const f16x8& a, const f16x8& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mma(const bf16x8& a, const bf16x8& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mma(const f32x8& a, const f32x8& b, f32x4 c) {
#pragma unroll
    for (int j = 0; j < 8; ++j) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], c, 0, 0, 0);
    return c;
}

// 8 contiguous elements at p (16-B aligned for 16-bit, 32-B for f32) -> fragment
template <class E> __device__ __forceinline__ typename E::Frag load8(const typename E::T* p);
template <> __device__ __forceinline__ f16x8 load8<EF16>(const _Float16* p) {
    return __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4*>(p));
}
template <> __device__ __forceinline__ bf16x8 load8<EBF16>(const __bf16* p) {
    return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(p));
}
template <> __device__ __forceinline__ f32x8 load8<EF32>(const float* p) {
    const float4 a = reinterpret_cast<const float4*>(p)[0];
    const float4 b = reinterpret_cast<const float4*>(p)[1];
    f32x8 r = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    return r;
}

// 8 elements from float registers (rounded to the element type)
template <class E> __device__ __forceinline__ typename E::Frag pack8(const float* v) {
    typename E::Frag r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = E::from(v[j]);
    return r;
}

// "Column" fragment for a B operand stored row-major [k][n] in LDS with row stride `ld` elements:
// lane l gets X[r(j)][n0 + (l&15)] where r(j) = r0 + 4*(l>>4) + j for j < 4 and
// r0 + 16 + 4*(l>>4) + (j-4) for j >= 4 (the k permutation matching an accumulator-as-A operand).
// 16-bit: two ds_read_b64_tr_b16 (lane 4q+p of each 16-lane group addresses row q, cols 4p..4p+3).
template <class E> __device__ __forceinline__ typename E::Frag load_colfrag(const typename E::T* lds, int ld, int r0, int n0);
template <> __device__ __forceinline__ f32x8 load_colfrag<EF32>(const float* lds, int ld, int r0, int n0) {
    const int l = threadIdx.x & 63, g = l >> 4, c = n0 + (l & 15);
    f32x8 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        r[j] = lds[(r0 + 4 * g + j) * ld + c];
        r[j + 4] = lds[(r0 + 16 + 4 * g + j) * ld + c];
    }
    return r;
}
template <class E16> __device__ __forceinline__ typename E16::Frag load_colfrag16(const typename E16::T* lds, int ld, int r0, int n0) {
    const int l = threadIdx.x & 63, g = l >> 4, w = l & 15, q = w >> 2, p = w & 3;
    const typename E16::T* a0 = lds + (r0 + 4 * g + q) * ld + n0 + 4 * p;
    const typename E16::T* a1 = a0 + 16 * ld;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a0));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a1));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(typename E16::Frag, v);
}
template <> __device__ __forceinline__ f16x8 load_colfrag<EF16>(const _Float16* lds, int ld, int r0, int n0) {
    return load_colfrag16<EF16>(lds, ld, r0, n0);
}
template <> __device__ __forceinline__ bf16x8 load_colfrag<EBF16>(const __bf16* lds, int ld, int r0, int n0) {
    return load_colfrag16<EBF16>(lds, ld, r0, n0);
}

// Bijective XCD-aware remap of a 1-D workgroup id (cdna_hip_programming.md §5 "XCD swizzle")
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    if (nwg <= 8) return orig;
    const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

}  // namespace ebc
