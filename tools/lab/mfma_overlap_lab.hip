// MFMA operand-overlap lab (experiment harness, not product code; r06).
//
// The failing r03 ordering of the long-attention forward (tools/lab/attn_long_max_lab.diff, f16, L = 257: 1046 of 6168
// rows non-finite, tools/dbg/long_max_dump.py) is the only build of that kernel whose ISA holds an MFMA whose destination
// PARTIALLY overlaps its A operand:
//     v_mfma_f32_16x16x32_f16 v[46:49], v[44:47], v[22:25], 0        (the first product of a key tile, C = 0)
// (the passing ordering's MFMAs overlap their A operand fully -- dst == A -- or not at all; tools/dbg/mfma_overlap_scan.py).
// This lab runs that exact instruction on fixed registers, one wave, random f16 operands, against the same product with
// a disjoint destination, plus the other overlap shapes the compiler emits (full A overlap, lower-half A overlap, B
// overlap, a C operand shifted by two registers as the GEMM instances have it), and prints the elements that differ.
//   build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/lab/mfma_overlap_lab.hip -o tools/lab/bin/mfma_overlap_lab
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

// operands per lane: a[4] / b[4] (packed f16 pairs), c[4] f32; result d[4]
template <int V>
__global__ void overlap_kernel(const unsigned* __restrict__ a, const unsigned* __restrict__ b, const float* __restrict__ c,
                               float* __restrict__ d, int reps)
{
    const int l = threadIdx.x;
    const unsigned a0 = a[4 * l], a1 = a[4 * l + 1], a2 = a[4 * l + 2], a3 = a[4 * l + 3];
    const unsigned b0 = b[4 * l], b1 = b[4 * l + 1], b2 = b[4 * l + 2], b3 = b[4 * l + 3];
    const float c0 = c[4 * l], c1 = c[4 * l + 1], c2 = c[4 * l + 2], c3 = c[4 * l + 3];
    float r0 = 0.f, r1 = 0.f, r2 = 0.f, r3 = 0.f;
    for (int it = 0; it < reps; ++it) {
        if constexpr (V == 0) {        // reference: disjoint destination
            asm volatile(
                "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
                "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
                "s_nop 4\n"
                "v_mfma_f32_16x16x32_f16 v[50:53], v[44:47], v[22:25], 0\n"
                "s_nop 7\n s_nop 7\n s_nop 7\n"
                "v_mov_b32 %0, v50\n v_mov_b32 %1, v51\n v_mov_b32 %2, v52\n v_mov_b32 %3, v53\n"
                : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
                : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3)
                : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53");
        } else if constexpr (V == 1) { // the failing build's instruction: dst v[46:49] over A's upper half
            asm volatile(
                "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
                "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
                "s_nop 4\n"
                "v_mfma_f32_16x16x32_f16 v[46:49], v[44:47], v[22:25], 0\n"
                "s_nop 7\n s_nop 7\n s_nop 7\n"
                "v_mov_b32 %0, v46\n v_mov_b32 %1, v47\n v_mov_b32 %2, v48\n v_mov_b32 %3, v49\n"
                : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
                : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3)
                : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53");
        } else if constexpr (V == 2) { // full A overlap (the passing builds' form)
            asm volatile(
                "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
                "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
                "s_nop 4\n"
                "v_mfma_f32_16x16x32_f16 v[44:47], v[44:47], v[22:25], 0\n"
                "s_nop 7\n s_nop 7\n s_nop 7\n"
                "v_mov_b32 %0, v44\n v_mov_b32 %1, v45\n v_mov_b32 %2, v46\n v_mov_b32 %3, v47\n"
                : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
                : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3)
                : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53");
        } else if constexpr (V == 3) { // dst over A's lower half
            asm volatile(
                "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
                "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
                "s_nop 4\n"
                "v_mfma_f32_16x16x32_f16 v[42:45], v[44:47], v[22:25], 0\n"
                "s_nop 7\n s_nop 7\n s_nop 7\n"
                "v_mov_b32 %0, v42\n v_mov_b32 %1, v43\n v_mov_b32 %2, v44\n v_mov_b32 %3, v45\n"
                : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
                : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3)
                : "v22", "v23", "v24", "v25", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53");
        } else if constexpr (V == 4) { // dst over B's upper half
            asm volatile(
                "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
                "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
                "s_nop 4\n"
                "v_mfma_f32_16x16x32_f16 v[24:27], v[44:47], v[22:25], 0\n"
                "s_nop 7\n s_nop 7\n s_nop 7\n"
                "v_mov_b32 %0, v24\n v_mov_b32 %1, v25\n v_mov_b32 %2, v26\n v_mov_b32 %3, v27\n"
                : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
                : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3)
                : "v22", "v23", "v24", "v25", "v26", "v27", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53");
        } else if constexpr (V == 5) { // C shifted by two registers under dst (the GEMM instances' form), vs disjoint C
            asm volatile(
                "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
                "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
                "v_mov_b32 v60, %12\n v_mov_b32 v61, %13\n v_mov_b32 v62, %14\n v_mov_b32 v63, %15\n"
                "s_nop 4\n"
                "v_mfma_f32_16x16x32_f16 v[58:61], v[44:47], v[22:25], v[60:63]\n"
                "s_nop 7\n s_nop 7\n s_nop 7\n"
                "v_mov_b32 %0, v58\n v_mov_b32 %1, v59\n v_mov_b32 %2, v60\n v_mov_b32 %3, v61\n"
                : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
                : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(c0), "v"(c1), "v"(c2), "v"(c3)
                : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v58", "v59", "v60", "v61", "v62", "v63");
        } else {                       // V == 6: the reference for V == 5 (C disjoint)
            asm volatile(
                "v_mov_b32 v44, %4\n v_mov_b32 v45, %5\n v_mov_b32 v46, %6\n v_mov_b32 v47, %7\n"
                "v_mov_b32 v22, %8\n v_mov_b32 v23, %9\n v_mov_b32 v24, %10\n v_mov_b32 v25, %11\n"
                "v_mov_b32 v60, %12\n v_mov_b32 v61, %13\n v_mov_b32 v62, %14\n v_mov_b32 v63, %15\n"
                "s_nop 4\n"
                "v_mfma_f32_16x16x32_f16 v[52:55], v[44:47], v[22:25], v[60:63]\n"
                "s_nop 7\n s_nop 7\n s_nop 7\n"
                "v_mov_b32 %0, v52\n v_mov_b32 %1, v53\n v_mov_b32 %2, v54\n v_mov_b32 %3, v55\n"
                : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
                : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(c0), "v"(c1), "v"(c2), "v"(c3)
                : "v22", "v23", "v24", "v25", "v44", "v45", "v46", "v47", "v52", "v53", "v54", "v55", "v60", "v61", "v62", "v63");
        }
    }
    d[4 * l] = r0; d[4 * l + 1] = r1; d[4 * l + 2] = r2; d[4 * l + 3] = r3;
}

static unsigned short f2h(float f)
{
    _Float16 h = (_Float16)f;
    unsigned short u;
    memcpy(&u, &h, 2);
    return u;
}

int main()
{
    const int n = 64 * 4;
    std::vector<unsigned> ha(n), hb(n);
    std::vector<float> hc(n);
    srand(7);
    for (int i = 0; i < n; ++i) {
        auto r = [] { return (float)rand() / RAND_MAX * 2.f - 1.f; };
        ha[i] = f2h(r()) | ((unsigned)f2h(r()) << 16);
        hb[i] = f2h(r()) | ((unsigned)f2h(r()) << 16);
        hc[i] = r();
    }
    unsigned *da, *db;
    float *dc, *dd;
    CK(hipMalloc(&da, n * 4)); CK(hipMalloc(&db, n * 4)); CK(hipMalloc(&dc, n * 4)); CK(hipMalloc(&dd, n * 4));
    CK(hipMemcpy(da, ha.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, hb.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dc, hc.data(), n * 4, hipMemcpyHostToDevice));
    std::vector<std::vector<float>> out(7, std::vector<float>(n));
    const char* names[7] = {"disjoint dst (reference)", "dst v[46:49] over A v[44:47] upper half (failing build)",
                            "dst == A v[44:47] (full overlap)", "dst v[42:45] over A lower half", "dst v[24:27] over B upper half",
                            "dst v[58:61] over C v[60:63] (C shifted)", "disjoint dst, same C (reference for C)"};
    auto run = [&](int v) {
        switch (v) {
            case 0: hipLaunchKernelGGL(overlap_kernel<0>, dim3(1), dim3(64), 0, 0, da, db, dc, dd, 1); break;
            case 1: hipLaunchKernelGGL(overlap_kernel<1>, dim3(1), dim3(64), 0, 0, da, db, dc, dd, 1); break;
            case 2: hipLaunchKernelGGL(overlap_kernel<2>, dim3(1), dim3(64), 0, 0, da, db, dc, dd, 1); break;
            case 3: hipLaunchKernelGGL(overlap_kernel<3>, dim3(1), dim3(64), 0, 0, da, db, dc, dd, 1); break;
            case 4: hipLaunchKernelGGL(overlap_kernel<4>, dim3(1), dim3(64), 0, 0, da, db, dc, dd, 1); break;
            case 5: hipLaunchKernelGGL(overlap_kernel<5>, dim3(1), dim3(64), 0, 0, da, db, dc, dd, 1); break;
            default: hipLaunchKernelGGL(overlap_kernel<6>, dim3(1), dim3(64), 0, 0, da, db, dc, dd, 1); break;
        }
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(out[v].data(), dd, n * 4, hipMemcpyDeviceToHost));
    };
    for (int v = 0; v < 7; ++v) run(v);
    for (int v = 1; v < 7; ++v) {
        const int ref = v == 5 ? 6 : 0;
        if (v == 6) continue;
        int bad = 0;
        double maxd = 0;
        for (int i = 0; i < n; ++i)
            if (out[v][i] != out[ref][i] && !(std::isnan(out[v][i]) && std::isnan(out[ref][i]))) {
                ++bad;
                maxd = std::max(maxd, (double)std::fabs(out[v][i] - out[ref][i]));
            }
        printf("%-58s: %3d of %d result elements differ from the disjoint form (max |diff| %.4g)\n", names[v], bad, n, maxd);
        for (int i = 0, shown = 0; i < n && shown < 6; ++i)
            if (out[v][i] != out[ref][i]) {
                printf("    lane %2d elem %d: %.6g vs %.6g\n", i / 4, i % 4, out[v][i], out[ref][i]);
                ++shown;
            }
    }
    return 0;
}
