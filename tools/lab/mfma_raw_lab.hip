// MFMA -> VALU read-after-write lab (experiment harness, not product code; r06).
//
// The failing r03 ordering of the long-attention forward (tools/lab/attn_long_max_lab.diff) ends a non-masked key tile's
// MFMA pair in a branch over the tail mask: on the taken path the first VALU read of the product's accumulator (the
// tile maximum, v_max_f32) follows the second v_mfma_f32_16x16x32_f16 by 7 instructions.  The rows that
// come out non-finite have a running maximum of 1e3..3e3 (tools/dbg/long_max_dump.py with an end-of-kernel dump): values
// no score of those inputs reaches, i.e. bits of the accumulator registers' previous contents.  This lab issues the same
// instruction on fixed registers (accumulator zeroed first) and reads its result k wait states later (k x s_nop 0,
// k = 0..16), against a read 16 states later, and prints per k how many of the 256 results differ.
//   build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/lab/mfma_raw_lab.hip -o tools/lab/bin/mfma_raw_lab
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int K> __global__ void rd_kernel(const unsigned* __restrict__ a, const unsigned* __restrict__ b, float* __restrict__ d);
template <> __global__ void rd_kernel<0>(const unsigned* __restrict__ a, const unsigned* __restrict__ b,
                                         float* __restrict__ d)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[4 * l], a1 = a[4 * l + 1], a2 = a[4 * l + 2], a3 = a[4 * l + 3];
    const unsigned b0 = b[4 * l], b1 = b[4 * l + 1], b2 = b[4 * l + 2], b3 = b[4 * l + 3];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
        "v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[50:53], v[44:47], v[22:25], 0\n"
        ""
        "v_max_f32 %0, v50, v50\n v_max_f32 %1, v51, v51\n v_max_f32 %2, v52, v52\n v_max_f32 %3, v53, v53\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3)
        : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v50", "v51", "v52", "v53");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void rd_kernel<1>(const unsigned* __restrict__ a, const unsigned* __restrict__ b,
                                         float* __restrict__ d)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[4 * l], a1 = a[4 * l + 1], a2 = a[4 * l + 2], a3 = a[4 * l + 3];
    const unsigned b0 = b[4 * l], b1 = b[4 * l + 1], b2 = b[4 * l + 2], b3 = b[4 * l + 3];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
        "v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[50:53], v[44:47], v[22:25], 0\n"
        "s_nop 0\n"
        "v_max_f32 %0, v50, v50\n v_max_f32 %1, v51, v51\n v_max_f32 %2, v52, v52\n v_max_f32 %3, v53, v53\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3)
        : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v50", "v51", "v52", "v53");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void rd_kernel<2>(const unsigned* __restrict__ a, const unsigned* __restrict__ b,
                                         float* __restrict__ d)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[4 * l], a1 = a[4 * l + 1], a2 = a[4 * l + 2], a3 = a[4 * l + 3];
    const unsigned b0 = b[4 * l], b1 = b[4 * l + 1], b2 = b[4 * l + 2], b3 = b[4 * l + 3];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
        "v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[50:53], v[44:47], v[22:25], 0\n"
        "s_nop 0\ns_nop 0\n"
        "v_max_f32 %0, v50, v50\n v_max_f32 %1, v51, v51\n v_max_f32 %2, v52, v52\n v_max_f32 %3, v53, v53\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3)
        : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v50", "v51", "v52", "v53");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void rd_kernel<3>(const unsigned* __restrict__ a, const unsigned* __restrict__ b,
                                         float* __restrict__ d)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[4 * l], a1 = a[4 * l + 1], a2 = a[4 * l + 2], a3 = a[4 * l + 3];
    const unsigned b0 = b[4 * l], b1 = b[4 * l + 1], b2 = b[4 * l + 2], b3 = b[4 * l + 3];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
        "v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[50:53], v[44:47], v[22:25], 0\n"
        "s_nop 0\ns_nop 0\ns_nop 0\n"
        "v_max_f32 %0, v50, v50\n v_max_f32 %1, v51, v51\n v_max_f32 %2, v52, v52\n v_max_f32 %3, v53, v53\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3)
        : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v50", "v51", "v52", "v53");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void rd_kernel<4>(const unsigned* __restrict__ a, const unsigned* __restrict__ b,
                                         float* __restrict__ d)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[4 * l], a1 = a[4 * l + 1], a2 = a[4 * l + 2], a3 = a[4 * l + 3];
    const unsigned b0 = b[4 * l], b1 = b[4 * l + 1], b2 = b[4 * l + 2], b3 = b[4 * l + 3];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
        "v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[50:53], v[44:47], v[22:25], 0\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_max_f32 %0, v50, v50\n v_max_f32 %1, v51, v51\n v_max_f32 %2, v52, v52\n v_max_f32 %3, v53, v53\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3)
        : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v50", "v51", "v52", "v53");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void rd_kernel<5>(const unsigned* __restrict__ a, const unsigned* __restrict__ b,
                                         float* __restrict__ d)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[4 * l], a1 = a[4 * l + 1], a2 = a[4 * l + 2], a3 = a[4 * l + 3];
    const unsigned b0 = b[4 * l], b1 = b[4 * l + 1], b2 = b[4 * l + 2], b3 = b[4 * l + 3];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
        "v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[50:53], v[44:47], v[22:25], 0\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_max_f32 %0, v50, v50\n v_max_f32 %1, v51, v51\n v_max_f32 %2, v52, v52\n v_max_f32 %3, v53, v53\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3)
        : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v50", "v51", "v52", "v53");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void rd_kernel<6>(const unsigned* __restrict__ a, const unsigned* __restrict__ b,
                                         float* __restrict__ d)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[4 * l], a1 = a[4 * l + 1], a2 = a[4 * l + 2], a3 = a[4 * l + 3];
    const unsigned b0 = b[4 * l], b1 = b[4 * l + 1], b2 = b[4 * l + 2], b3 = b[4 * l + 3];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
        "v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[50:53], v[44:47], v[22:25], 0\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_max_f32 %0, v50, v50\n v_max_f32 %1, v51, v51\n v_max_f32 %2, v52, v52\n v_max_f32 %3, v53, v53\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3)
        : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v50", "v51", "v52", "v53");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void rd_kernel<7>(const unsigned* __restrict__ a, const unsigned* __restrict__ b,
                                         float* __restrict__ d)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[4 * l], a1 = a[4 * l + 1], a2 = a[4 * l + 2], a3 = a[4 * l + 3];
    const unsigned b0 = b[4 * l], b1 = b[4 * l + 1], b2 = b[4 * l + 2], b3 = b[4 * l + 3];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
        "v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[50:53], v[44:47], v[22:25], 0\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_max_f32 %0, v50, v50\n v_max_f32 %1, v51, v51\n v_max_f32 %2, v52, v52\n v_max_f32 %3, v53, v53\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3)
        : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v50", "v51", "v52", "v53");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void rd_kernel<8>(const unsigned* __restrict__ a, const unsigned* __restrict__ b,
                                         float* __restrict__ d)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[4 * l], a1 = a[4 * l + 1], a2 = a[4 * l + 2], a3 = a[4 * l + 3];
    const unsigned b0 = b[4 * l], b1 = b[4 * l + 1], b2 = b[4 * l + 2], b3 = b[4 * l + 3];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
        "v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[50:53], v[44:47], v[22:25], 0\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_max_f32 %0, v50, v50\n v_max_f32 %1, v51, v51\n v_max_f32 %2, v52, v52\n v_max_f32 %3, v53, v53\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3)
        : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v50", "v51", "v52", "v53");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void rd_kernel<9>(const unsigned* __restrict__ a, const unsigned* __restrict__ b,
                                         float* __restrict__ d)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[4 * l], a1 = a[4 * l + 1], a2 = a[4 * l + 2], a3 = a[4 * l + 3];
    const unsigned b0 = b[4 * l], b1 = b[4 * l + 1], b2 = b[4 * l + 2], b3 = b[4 * l + 3];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
        "v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[50:53], v[44:47], v[22:25], 0\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_max_f32 %0, v50, v50\n v_max_f32 %1, v51, v51\n v_max_f32 %2, v52, v52\n v_max_f32 %3, v53, v53\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3)
        : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v50", "v51", "v52", "v53");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void rd_kernel<10>(const unsigned* __restrict__ a, const unsigned* __restrict__ b,
                                         float* __restrict__ d)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[4 * l], a1 = a[4 * l + 1], a2 = a[4 * l + 2], a3 = a[4 * l + 3];
    const unsigned b0 = b[4 * l], b1 = b[4 * l + 1], b2 = b[4 * l + 2], b3 = b[4 * l + 3];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
        "v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[50:53], v[44:47], v[22:25], 0\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_max_f32 %0, v50, v50\n v_max_f32 %1, v51, v51\n v_max_f32 %2, v52, v52\n v_max_f32 %3, v53, v53\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3)
        : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v50", "v51", "v52", "v53");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void rd_kernel<11>(const unsigned* __restrict__ a, const unsigned* __restrict__ b,
                                         float* __restrict__ d)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[4 * l], a1 = a[4 * l + 1], a2 = a[4 * l + 2], a3 = a[4 * l + 3];
    const unsigned b0 = b[4 * l], b1 = b[4 * l + 1], b2 = b[4 * l + 2], b3 = b[4 * l + 3];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
        "v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[50:53], v[44:47], v[22:25], 0\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_max_f32 %0, v50, v50\n v_max_f32 %1, v51, v51\n v_max_f32 %2, v52, v52\n v_max_f32 %3, v53, v53\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3)
        : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v50", "v51", "v52", "v53");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void rd_kernel<12>(const unsigned* __restrict__ a, const unsigned* __restrict__ b,
                                         float* __restrict__ d)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[4 * l], a1 = a[4 * l + 1], a2 = a[4 * l + 2], a3 = a[4 * l + 3];
    const unsigned b0 = b[4 * l], b1 = b[4 * l + 1], b2 = b[4 * l + 2], b3 = b[4 * l + 3];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
        "v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[50:53], v[44:47], v[22:25], 0\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_max_f32 %0, v50, v50\n v_max_f32 %1, v51, v51\n v_max_f32 %2, v52, v52\n v_max_f32 %3, v53, v53\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3)
        : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v50", "v51", "v52", "v53");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void rd_kernel<16>(const unsigned* __restrict__ a, const unsigned* __restrict__ b,
                                         float* __restrict__ d)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[4 * l], a1 = a[4 * l + 1], a2 = a[4 * l + 2], a3 = a[4 * l + 3];
    const unsigned b0 = b[4 * l], b1 = b[4 * l + 1], b2 = b[4 * l + 2], b3 = b[4 * l + 3];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
        "v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[50:53], v[44:47], v[22:25], 0\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_max_f32 %0, v50, v50\n v_max_f32 %1, v51, v51\n v_max_f32 %2, v52, v52\n v_max_f32 %3, v53, v53\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3)
        : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v50", "v51", "v52", "v53");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}

static unsigned short f2h(float f)
{
    _Float16 h = (_Float16)f;
    unsigned short u;
    memcpy(&u, &h, 2);
    return u;
}

template <int K> void run(const unsigned* da, const unsigned* db, float* dd, std::vector<float>& out)
{
    hipLaunchKernelGGL(rd_kernel<K>, dim3(1), dim3(64), 0, 0, da, db, dd);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(out.data(), dd, out.size() * 4, hipMemcpyDeviceToHost));
}

int main()
{
    const int n = 256;
    std::vector<unsigned> ha(n), hb(n);
    srand(11);
    for (int i = 0; i < n; ++i) {
        auto r = [] { return (float)rand() / (float)RAND_MAX * 2.f - 1.f; };
        ha[i] = f2h(r()) | ((unsigned)f2h(r()) << 16);
        hb[i] = f2h(r()) | ((unsigned)f2h(r()) << 16);
    }
    unsigned *da, *db;
    float* dd;
    CK(hipMalloc(&da, n * 4)); CK(hipMalloc(&db, n * 4)); CK(hipMalloc(&dd, n * 4));
    CK(hipMemcpy(da, ha.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, hb.data(), n * 4, hipMemcpyHostToDevice));
    std::vector<float> ref(n), out(n);
    run<16>(da, db, dd, ref);
    auto report = [&](int k, const std::vector<float>& o) {
        int bad = 0, zero = 0;
        for (int i = 0; i < n; ++i) { bad += o[i] != ref[i]; zero += o[i] == 0.f && ref[i] != 0.f; }
        printf("read %2d wait states after the MFMA: %3d of %d results differ from the 16-state read (%d read the zeroed accumulator)\n",
               k, bad, n, zero);
    };
    run<0>(da, db, dd, out); report(0, out);
    run<1>(da, db, dd, out); report(1, out);
    run<2>(da, db, dd, out); report(2, out);
    run<3>(da, db, dd, out); report(3, out);
    run<4>(da, db, dd, out); report(4, out);
    run<5>(da, db, dd, out); report(5, out);
    run<6>(da, db, dd, out); report(6, out);
    run<7>(da, db, dd, out); report(7, out);
    run<8>(da, db, dd, out); report(8, out);
    run<9>(da, db, dd, out); report(9, out);
    run<10>(da, db, dd, out); report(10, out);
    run<11>(da, db, dd, out); report(11, out);
    run<12>(da, db, dd, out); report(12, out);
    run<16>(da, db, dd, out); report(16, out);
    return 0;
}
