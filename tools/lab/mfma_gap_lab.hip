// MFMA result wait-state lab, by instruction kind (experiment harness, not product code; r06).
//
// tools/lab/mfma_raw_lab.hip: a VALU read of a v_mfma_f32_16x16x32_f16 result needs >= 7 s_nop wait states.  The
// failing r03 long-attention build reads the accumulator 7 instructions after the MFMA on the path that
// branches over the tail mask: s_add, 3 x v_or, v_mov, s_cmp, a taken s_cbranch -- 7 by the compiler's count, since
// every instruction counts as a wait state.  Here the same read follows each kind of 7-instruction gap: the failing
// path itself (taken and not taken), SALU-only, VALU-only, s_nop-only, a taken branch.
//   build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/lab/mfma_gap_lab.hip -o tools/lab/bin/mfma_gap_lab
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int V> __global__ void gap_kernel(const unsigned* __restrict__ a, const unsigned* __restrict__ b, float* __restrict__ d, int flag);
template <> __global__ void gap_kernel<0>(const unsigned* __restrict__ a, const unsigned* __restrict__ b, float* __restrict__ d, int flag)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[4 * l], a1 = a[4 * l + 1], a2 = a[4 * l + 2], a3 = a[4 * l + 3];
    const unsigned b0 = b[4 * l], b1 = b[4 * l + 1], b2 = b[4 * l + 2], b3 = b[4 * l + 3];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
        "v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n"
        "s_mov_b32 s90, %12\n s_mov_b32 s91, 0\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[50:53], v[44:47], v[22:25], 0\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_max_f32 %0, v51, v51\n v_max_f32 %1, v50, v50\n v_max_f32 %2, v53, v53\n v_max_f32 %3, v52, v52\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3), "s"(flag)
        : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v50", "v51", "v52", "v53", "v60", "v61", "v62", "v63",
          "s90", "s91", "scc");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void gap_kernel<1>(const unsigned* __restrict__ a, const unsigned* __restrict__ b, float* __restrict__ d, int flag)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[4 * l], a1 = a[4 * l + 1], a2 = a[4 * l + 2], a3 = a[4 * l + 3];
    const unsigned b0 = b[4 * l], b1 = b[4 * l + 1], b2 = b[4 * l + 2], b3 = b[4 * l + 3];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
        "v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n"
        "s_mov_b32 s90, %12\n s_mov_b32 s91, 0\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[50:53], v[44:47], v[22:25], 0\n"
        "s_add_i32 s91, s91, 1\n v_or_b32 v60, 1, v22\n v_or_b32 v61, 2, v22\n v_or_b32 v62, 3, v22\n v_mov_b32 v63, 0\n s_cmp_lg_u32 s90, 0\n s_cbranch_scc1 1f\n s_nop 0\n 1:\n"
        "v_max_f32 %0, v51, v51\n v_max_f32 %1, v50, v50\n v_max_f32 %2, v53, v53\n v_max_f32 %3, v52, v52\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3), "s"(flag)
        : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v50", "v51", "v52", "v53", "v60", "v61", "v62", "v63",
          "s90", "s91", "scc");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void gap_kernel<2>(const unsigned* __restrict__ a, const unsigned* __restrict__ b, float* __restrict__ d, int flag)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[4 * l], a1 = a[4 * l + 1], a2 = a[4 * l + 2], a3 = a[4 * l + 3];
    const unsigned b0 = b[4 * l], b1 = b[4 * l + 1], b2 = b[4 * l + 2], b3 = b[4 * l + 3];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
        "v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n"
        "s_mov_b32 s90, %12\n s_mov_b32 s91, 0\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[50:53], v[44:47], v[22:25], 0\n"
        "s_add_i32 s91, s91, 1\n v_or_b32 v60, 1, v22\n v_or_b32 v61, 2, v22\n v_or_b32 v62, 3, v22\n v_mov_b32 v63, 0\n s_cmp_eq_u32 s90, 0\n s_cbranch_scc1 1f\n s_nop 0\n 1:\n"
        "v_max_f32 %0, v51, v51\n v_max_f32 %1, v50, v50\n v_max_f32 %2, v53, v53\n v_max_f32 %3, v52, v52\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3), "s"(flag)
        : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v50", "v51", "v52", "v53", "v60", "v61", "v62", "v63",
          "s90", "s91", "scc");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void gap_kernel<3>(const unsigned* __restrict__ a, const unsigned* __restrict__ b, float* __restrict__ d, int flag)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[4 * l], a1 = a[4 * l + 1], a2 = a[4 * l + 2], a3 = a[4 * l + 3];
    const unsigned b0 = b[4 * l], b1 = b[4 * l + 1], b2 = b[4 * l + 2], b3 = b[4 * l + 3];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
        "v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n"
        "s_mov_b32 s90, %12\n s_mov_b32 s91, 0\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[50:53], v[44:47], v[22:25], 0\n"
        "s_add_i32 s91, s91, 1\ns_add_i32 s91, s91, 1\ns_add_i32 s91, s91, 1\ns_add_i32 s91, s91, 1\ns_add_i32 s91, s91, 1\ns_add_i32 s91, s91, 1\ns_add_i32 s91, s91, 1\n"
        "v_max_f32 %0, v51, v51\n v_max_f32 %1, v50, v50\n v_max_f32 %2, v53, v53\n v_max_f32 %3, v52, v52\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3), "s"(flag)
        : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v50", "v51", "v52", "v53", "v60", "v61", "v62", "v63",
          "s90", "s91", "scc");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void gap_kernel<4>(const unsigned* __restrict__ a, const unsigned* __restrict__ b, float* __restrict__ d, int flag)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[4 * l], a1 = a[4 * l + 1], a2 = a[4 * l + 2], a3 = a[4 * l + 3];
    const unsigned b0 = b[4 * l], b1 = b[4 * l + 1], b2 = b[4 * l + 2], b3 = b[4 * l + 3];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
        "v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n"
        "s_mov_b32 s90, %12\n s_mov_b32 s91, 0\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[50:53], v[44:47], v[22:25], 0\n"
        "v_or_b32 v60, 1, v22\nv_or_b32 v60, 1, v22\nv_or_b32 v60, 1, v22\nv_or_b32 v60, 1, v22\nv_or_b32 v60, 1, v22\nv_or_b32 v60, 1, v22\nv_or_b32 v60, 1, v22\n"
        "v_max_f32 %0, v51, v51\n v_max_f32 %1, v50, v50\n v_max_f32 %2, v53, v53\n v_max_f32 %3, v52, v52\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3), "s"(flag)
        : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v50", "v51", "v52", "v53", "v60", "v61", "v62", "v63",
          "s90", "s91", "scc");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void gap_kernel<5>(const unsigned* __restrict__ a, const unsigned* __restrict__ b, float* __restrict__ d, int flag)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[4 * l], a1 = a[4 * l + 1], a2 = a[4 * l + 2], a3 = a[4 * l + 3];
    const unsigned b0 = b[4 * l], b1 = b[4 * l + 1], b2 = b[4 * l + 2], b3 = b[4 * l + 3];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
        "v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n"
        "s_mov_b32 s90, %12\n s_mov_b32 s91, 0\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[50:53], v[44:47], v[22:25], 0\n"
        "s_add_i32 s91, s91, 1\n v_or_b32 v60, 1, v22\n v_or_b32 v61, 2, v22\n v_or_b32 v62, 3, v22\n v_mov_b32 v63, 0\n s_cmp_lg_u32 s90, 0\n s_nop 0\n"
        "v_max_f32 %0, v51, v51\n v_max_f32 %1, v50, v50\n v_max_f32 %2, v53, v53\n v_max_f32 %3, v52, v52\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3), "s"(flag)
        : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v50", "v51", "v52", "v53", "v60", "v61", "v62", "v63",
          "s90", "s91", "scc");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void gap_kernel<6>(const unsigned* __restrict__ a, const unsigned* __restrict__ b, float* __restrict__ d, int flag)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[4 * l], a1 = a[4 * l + 1], a2 = a[4 * l + 2], a3 = a[4 * l + 3];
    const unsigned b0 = b[4 * l], b1 = b[4 * l + 1], b2 = b[4 * l + 2], b3 = b[4 * l + 3];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
        "v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n"
        "s_mov_b32 s90, %12\n s_mov_b32 s91, 0\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[50:53], v[44:47], v[22:25], 0\n"
        "s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_max_f32 %0, v51, v51\n v_max_f32 %1, v50, v50\n v_max_f32 %2, v53, v53\n v_max_f32 %3, v52, v52\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3), "s"(flag)
        : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v50", "v51", "v52", "v53", "v60", "v61", "v62", "v63",
          "s90", "s91", "scc");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}
template <> __global__ void gap_kernel<7>(const unsigned* __restrict__ a, const unsigned* __restrict__ b, float* __restrict__ d, int flag)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[4 * l], a1 = a[4 * l + 1], a2 = a[4 * l + 2], a3 = a[4 * l + 3];
    const unsigned b0 = b[4 * l], b1 = b[4 * l + 1], b2 = b[4 * l + 2], b3 = b[4 * l + 3];
    float r0, r1, r2, r3;
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
        "v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n"
        "s_mov_b32 s90, %12\n s_mov_b32 s91, 0\n"
        "s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[50:53], v[44:47], v[22:25], 0\n"
        "s_cmp_lg_u32 s90, 0\n s_cbranch_scc1 1f\n s_nop 0\n 1:\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\ns_nop 0\n"
        "v_max_f32 %0, v51, v51\n v_max_f32 %1, v50, v50\n v_max_f32 %2, v53, v53\n v_max_f32 %3, v52, v52\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3), "s"(flag)
        : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v50", "v51", "v52", "v53", "v60", "v61", "v62", "v63",
          "s90", "s91", "scc");
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}

// contention: 8 waves a workgroup (2 a SIMD), every wave runs the tested sequence right after a barrier while its SIMD
// partner also issues MFMAs (the attention workgroups' situation); BUSY > 0: the odd waves first issue BUSY more
// back-to-back MFMAs on other registers
template <int V, int BUSY>
__global__ __launch_bounds__(512) void gap_contended(const unsigned* __restrict__ a, const unsigned* __restrict__ b,
                                                      float* __restrict__ d, int flag)
{
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned a0 = a[4 * l], a1 = a[4 * l + 1], a2 = a[4 * l + 2], a3 = a[4 * l + 3];
    const unsigned b0 = b[4 * l], b1 = b[4 * l + 1], b2 = b[4 * l + 2], b3 = b[4 * l + 3];
    float r0, r1, r2, r3;
    __syncthreads();
    if (BUSY > 0 && (w & 1)) {
        asm volatile(
            "v_mov_b32 v100, %0\n v_mov_b32 v101, %1\n v_mov_b32 v102, %2\n v_mov_b32 v103, %3\n"
            ".rept %4\n v_mfma_f32_16x16x32_f16 v[104:107], v[100:103], v[100:103], v[104:107]\n .endr\n s_nop 7\n s_nop 7\n"
            :: "v"(a0), "v"(a1), "v"(b0), "v"(b1), "n"(BUSY) : "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107");
    }
    asm volatile(
        "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
        "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
        "v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n"
        "s_mov_b32 s90, %12\n s_mov_b32 s91, 0\n"
        "v_mfma_f32_16x16x32_f16 v[50:53], v[44:47], v[22:25], 0\n"
        "s_add_i32 s91, s91, 1\n v_or_b32 v60, 1, v22\n v_or_b32 v61, 2, v22\n v_or_b32 v62, 3, v22\n v_mov_b32 v63, 0\n"
        "s_cmp_lg_u32 s90, 0\n s_cbranch_scc1 1f\n s_nop 0\n 1:\n"
        "v_max_f32 %0, v51, v51\n v_max_f32 %1, v50, v50\n v_max_f32 %2, v53, v53\n v_max_f32 %3, v52, v52\n"
        "s_nop 7\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3), "s"(flag)
        : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v50", "v51", "v52", "v53", "v60", "v61", "v62", "v63",
          "s90", "s91", "scc");
    float* o = d + (size_t)w * 256;
    o[4 * l] = r0; o[4 * l + 1] = r1; o[4 * l + 2] = r2; o[4 * l + 3] = r3;
}
template <int BUSY> void run_cont(const unsigned* da, const unsigned* db, float* dd, const std::vector<float>& ref, const char* name)
{
    hipLaunchKernelGGL((gap_contended<1, BUSY>), dim3(1), dim3(512), 0, 0, da, db, dd, 1);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    std::vector<float> o(8 * 256);
    CK(hipMemcpy(o.data(), dd, o.size() * 4, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int w = 0; w < 8; ++w)
        for (int i = 0; i < 256; ++i) bad += o[w * 256 + i] != ref[i];
    printf("%-62s: %4d of %d results stale\n", name, bad, 8 * 256);
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
    hipLaunchKernelGGL(gap_kernel<V>, dim3(1), dim3(64), 0, 0, da, db, dd, 1);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(out.data(), dd, out.size() * 4, hipMemcpyDeviceToHost));
}

int main()
{
    const int n = 256;
    std::vector<unsigned> ha(n), hb(n);
    srand(17);
    for (int i = 0; i < n; ++i) {
        auto r = [] { return (float)rand() / (float)RAND_MAX * 2.f - 1.f; };
        ha[i] = f2h(r()) | ((unsigned)f2h(r()) << 16);
        hb[i] = f2h(r()) | ((unsigned)f2h(r()) << 16);
    }
    unsigned *da, *db;
    float* dd;
    CK(hipMalloc(&da, n * 4)); CK(hipMalloc(&db, n * 4)); CK(hipMalloc(&dd, 8 * n * 4));
    CK(hipMemcpy(da, ha.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, hb.data(), n * 4, hipMemcpyHostToDevice));
    std::vector<float> ref(n), out(n);
    run<0>(da, db, dd, ref);
    auto report = [&](const char* name, const std::vector<float>& o) {
        int bad = 0;
        for (int i = 0; i < n; ++i) bad += o[i] != ref[i];
        printf("%-62s: %3d of %d results stale\n", name, bad, n);
    };
    run<0>(da, db, dd, out); report("16 x s_nop 0 (reference)", out);
    run<1>(da, db, dd, out); report("failing path: s_add, 3 v_or, v_mov, s_cmp, taken s_cbranch", out);
    run<2>(da, db, dd, out); report("same, branch not taken (falls through + s_nop 0)", out);
    run<3>(da, db, dd, out); report("7 SALU (s_add)", out);
    run<4>(da, db, dd, out); report("7 VALU (v_or)", out);
    run<5>(da, db, dd, out); report("4 VALU + 3 SALU", out);
    run<6>(da, db, dd, out); report("7 s_nop 0", out);
    run<7>(da, db, dd, out); report("taken s_cbranch right after the MFMA + 6 s_nop 0", out);
    for (int rep = 0; rep < 3; ++rep) {
        run_cont<0>(da, db, dd, ref, "failing path, 8 waves (2 a SIMD), all running it");
        run_cont<8>(da, db, dd, ref, "failing path, odd waves issue 8 MFMAs first");
        run_cont<32>(da, db, dd, ref, "failing path, odd waves issue 32 MFMAs first");
    }
    return 0;
}
