// MFMA accumulation-pair lab (experiment harness, not product code; r06).
//
// The exact register pattern of the failing r03 long-attention ordering (tools/lab/attn_long_max_lab.diff, ISA in
// DESIGN.md 6e): a key tile's two chained products, the first with its destination PARTIALLY over its own A operand,
//     v_mfma_f32_16x16x32_f16 v[46:49], v[44:47], v[22:25], 0
//     (4 instructions)
//     v_mfma_f32_16x16x32_f16 v[46:49], v[52:55], v[18:21], v[46:49]
//     (7 instructions: the taken branch over the tail mask)
//     v_max_f32 ..., v47, v47
// run on fixed registers with the gaps varied, against the same pair on a disjoint accumulator with long gaps.
//   build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/lab/mfma_pair_lab.hip -o tools/lab/bin/mfma_pair_lab
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int V> __global__ void seq_kernel(const unsigned* __restrict__ a, const unsigned* __restrict__ b, float* __restrict__ d);
template <> __global__ void seq_kernel<0>(const unsigned* __restrict__ a, const unsigned* __restrict__ b, float* __restrict__ d)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[8 * l], a1 = a[8 * l + 1], a2 = a[8 * l + 2], a3 = a[8 * l + 3];
    const unsigned a4 = a[8 * l + 4], a5 = a[8 * l + 5], a6 = a[8 * l + 6], a7 = a[8 * l + 7];
    const unsigned b0 = b[8 * l], b1 = b[8 * l + 1], b2 = b[8 * l + 2], b3 = b[8 * l + 3];
    const unsigned b4 = b[8 * l + 4], b5 = b[8 * l + 5], b6 = b[8 * l + 6], b7 = b[8 * l + 7];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v52, %8\n v_mov_b32 v53, %9\n v_mov_b32 v54, %10\n v_mov_b32 v55, %11\n"
        "v_mov_b32 v22, %12\n v_mov_b32 v23, %13\n v_mov_b32 v24, %14\n v_mov_b32 v25, %15\n"
        "v_mov_b32 v18, %16\n v_mov_b32 v19, %17\n v_mov_b32 v20, %18\n v_mov_b32 v21, %19\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[58:61], v[44:47], v[22:25], 0\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_mfma_f32_16x16x32_f16 v[58:61], v[52:55], v[18:21], v[58:61]\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_max_f32 %0, v58, v58\n v_max_f32 %1, v59, v59\n v_max_f32 %2, v60, v60\n v_max_f32 %3, v61, v61\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7),
          "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(b4), "v"(b5), "v"(b6), "v"(b7)
        : "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v48", "v49",
          "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void seq_kernel<1>(const unsigned* __restrict__ a, const unsigned* __restrict__ b, float* __restrict__ d)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[8 * l], a1 = a[8 * l + 1], a2 = a[8 * l + 2], a3 = a[8 * l + 3];
    const unsigned a4 = a[8 * l + 4], a5 = a[8 * l + 5], a6 = a[8 * l + 6], a7 = a[8 * l + 7];
    const unsigned b0 = b[8 * l], b1 = b[8 * l + 1], b2 = b[8 * l + 2], b3 = b[8 * l + 3];
    const unsigned b4 = b[8 * l + 4], b5 = b[8 * l + 5], b6 = b[8 * l + 6], b7 = b[8 * l + 7];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v52, %8\n v_mov_b32 v53, %9\n v_mov_b32 v54, %10\n v_mov_b32 v55, %11\n"
        "v_mov_b32 v22, %12\n v_mov_b32 v23, %13\n v_mov_b32 v24, %14\n v_mov_b32 v25, %15\n"
        "v_mov_b32 v18, %16\n v_mov_b32 v19, %17\n v_mov_b32 v20, %18\n v_mov_b32 v21, %19\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[46:49], v[44:47], v[22:25], 0\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_mfma_f32_16x16x32_f16 v[46:49], v[52:55], v[18:21], v[46:49]\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_max_f32 %0, v46, v46\n v_max_f32 %1, v47, v47\n v_max_f32 %2, v48, v48\n v_max_f32 %3, v49, v49\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7),
          "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(b4), "v"(b5), "v"(b6), "v"(b7)
        : "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v48", "v49",
          "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void seq_kernel<2>(const unsigned* __restrict__ a, const unsigned* __restrict__ b, float* __restrict__ d)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[8 * l], a1 = a[8 * l + 1], a2 = a[8 * l + 2], a3 = a[8 * l + 3];
    const unsigned a4 = a[8 * l + 4], a5 = a[8 * l + 5], a6 = a[8 * l + 6], a7 = a[8 * l + 7];
    const unsigned b0 = b[8 * l], b1 = b[8 * l + 1], b2 = b[8 * l + 2], b3 = b[8 * l + 3];
    const unsigned b4 = b[8 * l + 4], b5 = b[8 * l + 5], b6 = b[8 * l + 6], b7 = b[8 * l + 7];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v52, %8\n v_mov_b32 v53, %9\n v_mov_b32 v54, %10\n v_mov_b32 v55, %11\n"
        "v_mov_b32 v22, %12\n v_mov_b32 v23, %13\n v_mov_b32 v24, %14\n v_mov_b32 v25, %15\n"
        "v_mov_b32 v18, %16\n v_mov_b32 v19, %17\n v_mov_b32 v20, %18\n v_mov_b32 v21, %19\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[46:49], v[44:47], v[22:25], 0\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_mfma_f32_16x16x32_f16 v[46:49], v[52:55], v[18:21], v[46:49]\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_max_f32 %0, v46, v46\n v_max_f32 %1, v47, v47\n v_max_f32 %2, v48, v48\n v_max_f32 %3, v49, v49\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7),
          "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(b4), "v"(b5), "v"(b6), "v"(b7)
        : "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v48", "v49",
          "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void seq_kernel<3>(const unsigned* __restrict__ a, const unsigned* __restrict__ b, float* __restrict__ d)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[8 * l], a1 = a[8 * l + 1], a2 = a[8 * l + 2], a3 = a[8 * l + 3];
    const unsigned a4 = a[8 * l + 4], a5 = a[8 * l + 5], a6 = a[8 * l + 6], a7 = a[8 * l + 7];
    const unsigned b0 = b[8 * l], b1 = b[8 * l + 1], b2 = b[8 * l + 2], b3 = b[8 * l + 3];
    const unsigned b4 = b[8 * l + 4], b5 = b[8 * l + 5], b6 = b[8 * l + 6], b7 = b[8 * l + 7];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v52, %8\n v_mov_b32 v53, %9\n v_mov_b32 v54, %10\n v_mov_b32 v55, %11\n"
        "v_mov_b32 v22, %12\n v_mov_b32 v23, %13\n v_mov_b32 v24, %14\n v_mov_b32 v25, %15\n"
        "v_mov_b32 v18, %16\n v_mov_b32 v19, %17\n v_mov_b32 v20, %18\n v_mov_b32 v21, %19\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[46:49], v[44:47], v[22:25], 0\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_mfma_f32_16x16x32_f16 v[46:49], v[52:55], v[18:21], v[46:49]\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_max_f32 %0, v46, v46\n v_max_f32 %1, v47, v47\n v_max_f32 %2, v48, v48\n v_max_f32 %3, v49, v49\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7),
          "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(b4), "v"(b5), "v"(b6), "v"(b7)
        : "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v48", "v49",
          "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void seq_kernel<4>(const unsigned* __restrict__ a, const unsigned* __restrict__ b, float* __restrict__ d)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[8 * l], a1 = a[8 * l + 1], a2 = a[8 * l + 2], a3 = a[8 * l + 3];
    const unsigned a4 = a[8 * l + 4], a5 = a[8 * l + 5], a6 = a[8 * l + 6], a7 = a[8 * l + 7];
    const unsigned b0 = b[8 * l], b1 = b[8 * l + 1], b2 = b[8 * l + 2], b3 = b[8 * l + 3];
    const unsigned b4 = b[8 * l + 4], b5 = b[8 * l + 5], b6 = b[8 * l + 6], b7 = b[8 * l + 7];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v52, %8\n v_mov_b32 v53, %9\n v_mov_b32 v54, %10\n v_mov_b32 v55, %11\n"
        "v_mov_b32 v22, %12\n v_mov_b32 v23, %13\n v_mov_b32 v24, %14\n v_mov_b32 v25, %15\n"
        "v_mov_b32 v18, %16\n v_mov_b32 v19, %17\n v_mov_b32 v20, %18\n v_mov_b32 v21, %19\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[58:61], v[44:47], v[22:25], 0\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_mfma_f32_16x16x32_f16 v[58:61], v[52:55], v[18:21], v[58:61]\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_max_f32 %0, v58, v58\n v_max_f32 %1, v59, v59\n v_max_f32 %2, v60, v60\n v_max_f32 %3, v61, v61\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7),
          "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(b4), "v"(b5), "v"(b6), "v"(b7)
        : "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v48", "v49",
          "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void seq_kernel<5>(const unsigned* __restrict__ a, const unsigned* __restrict__ b, float* __restrict__ d)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[8 * l], a1 = a[8 * l + 1], a2 = a[8 * l + 2], a3 = a[8 * l + 3];
    const unsigned a4 = a[8 * l + 4], a5 = a[8 * l + 5], a6 = a[8 * l + 6], a7 = a[8 * l + 7];
    const unsigned b0 = b[8 * l], b1 = b[8 * l + 1], b2 = b[8 * l + 2], b3 = b[8 * l + 3];
    const unsigned b4 = b[8 * l + 4], b5 = b[8 * l + 5], b6 = b[8 * l + 6], b7 = b[8 * l + 7];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v52, %8\n v_mov_b32 v53, %9\n v_mov_b32 v54, %10\n v_mov_b32 v55, %11\n"
        "v_mov_b32 v22, %12\n v_mov_b32 v23, %13\n v_mov_b32 v24, %14\n v_mov_b32 v25, %15\n"
        "v_mov_b32 v18, %16\n v_mov_b32 v19, %17\n v_mov_b32 v20, %18\n v_mov_b32 v21, %19\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[46:49], v[44:47], v[22:25], 0\n"
        ""
        "v_mfma_f32_16x16x32_f16 v[46:49], v[52:55], v[18:21], v[46:49]\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_max_f32 %0, v46, v46\n v_max_f32 %1, v47, v47\n v_max_f32 %2, v48, v48\n v_max_f32 %3, v49, v49\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7),
          "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(b4), "v"(b5), "v"(b6), "v"(b7)
        : "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v48", "v49",
          "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void seq_kernel<6>(const unsigned* __restrict__ a, const unsigned* __restrict__ b, float* __restrict__ d)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[8 * l], a1 = a[8 * l + 1], a2 = a[8 * l + 2], a3 = a[8 * l + 3];
    const unsigned a4 = a[8 * l + 4], a5 = a[8 * l + 5], a6 = a[8 * l + 6], a7 = a[8 * l + 7];
    const unsigned b0 = b[8 * l], b1 = b[8 * l + 1], b2 = b[8 * l + 2], b3 = b[8 * l + 3];
    const unsigned b4 = b[8 * l + 4], b5 = b[8 * l + 5], b6 = b[8 * l + 6], b7 = b[8 * l + 7];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v52, %8\n v_mov_b32 v53, %9\n v_mov_b32 v54, %10\n v_mov_b32 v55, %11\n"
        "v_mov_b32 v22, %12\n v_mov_b32 v23, %13\n v_mov_b32 v24, %14\n v_mov_b32 v25, %15\n"
        "v_mov_b32 v18, %16\n v_mov_b32 v19, %17\n v_mov_b32 v20, %18\n v_mov_b32 v21, %19\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[58:61], v[44:47], v[22:25], 0\n"
        ""
        "v_mfma_f32_16x16x32_f16 v[58:61], v[52:55], v[18:21], v[58:61]\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_max_f32 %0, v58, v58\n v_max_f32 %1, v59, v59\n v_max_f32 %2, v60, v60\n v_max_f32 %3, v61, v61\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7),
          "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(b4), "v"(b5), "v"(b6), "v"(b7)
        : "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v48", "v49",
          "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void seq_kernel<7>(const unsigned* __restrict__ a, const unsigned* __restrict__ b, float* __restrict__ d)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[8 * l], a1 = a[8 * l + 1], a2 = a[8 * l + 2], a3 = a[8 * l + 3];
    const unsigned a4 = a[8 * l + 4], a5 = a[8 * l + 5], a6 = a[8 * l + 6], a7 = a[8 * l + 7];
    const unsigned b0 = b[8 * l], b1 = b[8 * l + 1], b2 = b[8 * l + 2], b3 = b[8 * l + 3];
    const unsigned b4 = b[8 * l + 4], b5 = b[8 * l + 5], b6 = b[8 * l + 6], b7 = b[8 * l + 7];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v52, %8\n v_mov_b32 v53, %9\n v_mov_b32 v54, %10\n v_mov_b32 v55, %11\n"
        "v_mov_b32 v22, %12\n v_mov_b32 v23, %13\n v_mov_b32 v24, %14\n v_mov_b32 v25, %15\n"
        "v_mov_b32 v18, %16\n v_mov_b32 v19, %17\n v_mov_b32 v20, %18\n v_mov_b32 v21, %19\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[46:49], v[44:47], v[22:25], 0\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_mfma_f32_16x16x32_f16 v[46:49], v[52:55], v[18:21], v[46:49]\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_max_f32 %0, v46, v46\n v_max_f32 %1, v47, v47\n v_max_f32 %2, v48, v48\n v_max_f32 %3, v49, v49\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7),
          "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(b4), "v"(b5), "v"(b6), "v"(b7)
        : "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v48", "v49",
          "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}

static unsigned short f2h(float f)
{
    _Float16 h = (_Float16)f;
    unsigned short u;
    memcpy(&u, &h, 2);
    return u;
}

template <int V> void run(const unsigned* da, const unsigned* db, float* dd, std::vector<float>& out)
{
    hipLaunchKernelGGL(seq_kernel<V>, dim3(1), dim3(64), 0, 0, da, db, dd);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(out.data(), dd, out.size() * 4, hipMemcpyDeviceToHost));
}

int main()
{
    const int n = 512;
    std::vector<unsigned> ha(n), hb(n);
    srand(13);
    for (int i = 0; i < n; ++i) {
        auto r = [] { return (float)rand() / (float)RAND_MAX * 2.f - 1.f; };
        ha[i] = f2h(r()) | ((unsigned)f2h(r()) << 16);
        hb[i] = f2h(r()) | ((unsigned)f2h(r()) << 16);
    }
    unsigned *da, *db;
    float* dd;
    CK(hipMalloc(&da, n * 4)); CK(hipMalloc(&db, n * 4)); CK(hipMalloc(&dd, 256 * 4));
    CK(hipMemcpy(da, ha.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, hb.data(), n * 4, hipMemcpyHostToDevice));
    std::vector<float> ref(256), out(256);
    run<0>(da, db, dd, ref);
    auto report = [&](const char* name, const std::vector<float>& o) {
        int bad = 0;
        double mx = 0;
        for (int i = 0; i < 256; ++i) if (o[i] != ref[i]) { ++bad; mx = std::max(mx, (double)std::fabs(o[i])); }
        printf("%-58s: %3d of 256 results differ from the reference (largest wrong |value| %.4g)\n", name, bad, mx);
    };
    run<0>(da, db, dd, out); report("reference: dst v[58:61] (disjoint), 16 / 16 states", out);
    run<1>(da, db, dd, out); report("failing build: dst v[46:49] over A v[44:47], 4 / 7 states", out);
    run<2>(da, db, dd, out); report("dst v[46:49] over A, 4 / 16 states", out);
    run<3>(da, db, dd, out); report("dst v[46:49] over A, 16 / 7 states", out);
    run<4>(da, db, dd, out); report("disjoint dst v[58:61], 4 / 7 states", out);
    run<5>(da, db, dd, out); report("dst v[46:49] over A, 0 / 7 states", out);
    run<6>(da, db, dd, out); report("disjoint dst v[58:61], 0 / 7 states", out);
    run<7>(da, db, dd, out); report("dst v[46:49] over A, 4 / 4 states", out);
    return 0;
}
