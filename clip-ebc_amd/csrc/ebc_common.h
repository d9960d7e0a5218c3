// Shared helpers for the CLIP-EBC gfx950 kernels (CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include "../../include/ebc_hip.h"

#define EBC_WAVE 64

#define EBC_CHECK_LAUNCH()                                   \
    do {                                                     \
        hipError_t _e = hipGetLastError();                   \
        if (_e != hipSuccess) return EBC_E_LAUNCH;           \
    } while (0)

namespace ebc {

// A kernel that asks for more than 64 KiB of dynamic LDS must be opted in with hipFuncSetAttribute, and the attribute
// is held per device: set it once per (kernel, device) for the device the launch stream belongs to (a process may
// drive several devices from one thread).  `bytes` must be the kernel's largest request.
template <auto KERNEL>
inline bool ensure_lds(int bytes, hipStream_t st)
{
    if (bytes <= 64 * 1024) return true;
    static unsigned long long done = 0;          // bit d: set on device d (benign race: setting twice is harmless)
    int dev = 0;
    if (hipStreamGetDevice(st, &dev) != hipSuccess || dev < 0 || dev >= 64) return false;
    const unsigned long long bit = 1ull << dev;
    if (__atomic_load_n(&done, __ATOMIC_RELAXED) & bit) return true;
    int cur = dev;
    if (hipGetDevice(&cur) != hipSuccess) return false;
    if (cur != dev && hipSetDevice(dev) != hipSuccess) return false;
    const hipError_t e = hipFuncSetAttribute((const void*)KERNEL, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (cur != dev) (void)hipSetDevice(cur);
    if (e != hipSuccess) return false;
    __atomic_fetch_or(&done, bit, __ATOMIC_RELAXED);
    return true;
}

// Wave-wide reductions on DPP (VALU lane moves) instead of __shfl_xor, which hipcc lowers to six
// ds_bpermute LDS round trips each followed by lgkmcnt(0): quad xor-1 / xor-2, row half-mirror and
// row mirror leave every lane with its 16-lane row's total, row_bcast:15 / row_bcast:31 fold the
// four rows into lane 63, and readlane broadcasts it (the result is wave-uniform).  Every lane of
// the wave must be active.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
template <int CTRL, int ROWS>
__device__ __forceinline__ float dpp_rows(float v, float old) {  // rows outside ROWS keep `old`
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old), __builtin_bit_cast(int, v),
                                                                 CTRL, ROWS, 0xF, false));
}
__device__ __forceinline__ float wave_sum(float v) {
    v += dpp_mov<0xB1>(v);
    v += dpp_mov<0x4E>(v);
    v += dpp_mov<0x141>(v);
    v += dpp_mov<0x140>(v);
    v += dpp_rows<0x142, 0xA>(v, 0.f);
    v += dpp_rows<0x143, 0xC>(v, 0.f);
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}

__device__ __forceinline__ float wave_max(float v) {
    v = fmaxf(v, dpp_mov<0xB1>(v));
    v = fmaxf(v, dpp_mov<0x4E>(v));
    v = fmaxf(v, dpp_mov<0x141>(v));
    v = fmaxf(v, dpp_mov<0x140>(v));
    v = fmaxf(v, dpp_rows<0x142, 0xA>(v, -INFINITY));
    v = fmaxf(v, dpp_rows<0x143, 0xC>(v, -INFINITY));
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}

__device__ __forceinline__ int wave_or(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o, 64);
    return v;
}

// Block-wide sum; `scratch` holds >= blockDim/64 floats.  Result broadcast to every thread.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    v = wave_sum(v);
    __syncthreads();
    if (lane == 0) scratch[w] = v;
    __syncthreads();
    float r = 0.f;
    for (int i = 0; i < nw; ++i) r += scratch[i];
    return r;
}

__device__ __forceinline__ double block_sum_d(double v, double* scratch) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    __syncthreads();
    if (lane == 0) scratch[w] = v;
    __syncthreads();
    double r = 0.0;
    for (int i = 0; i < nw; ++i) r += scratch[i];
    return r;
}

__device__ __forceinline__ int block_or(int v, int* scratch) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    v = wave_or(v);
    __syncthreads();
    if (lane == 0) scratch[w] = v;
    __syncthreads();
    int r = 0;
    for (int i = 0; i < nw; ++i) r |= scratch[i];
    return r;
}

__device__ __forceinline__ float sgnf(float x) { return (x > 0.f) ? 1.f : ((x < 0.f) ? -1.f : 0.f); }

template <typename T> __device__ __forceinline__ float to_f32(T v);
template <> __device__ __forceinline__ float to_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f32<__half>(__half v) { return __half2float(v); }
template <> __device__ __forceinline__ float to_f32<__hip_bfloat16>(__hip_bfloat16 v) { return __bfloat162float(v); }

template <typename T> __device__ __forceinline__ T from_f32(float v);
template <> __device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ __half from_f32<__half>(float v) { return __float2half(v); }
template <> __device__ __forceinline__ __hip_bfloat16 from_f32<__hip_bfloat16>(float v) { return __float2bfloat16(v); }

}  // namespace ebc
