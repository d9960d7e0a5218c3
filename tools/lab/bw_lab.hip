// Per-CU L2 -> CU ingest rate by load path (experiment, not product code).
//
// Question: is the ~70 GB/s-per-CU fill that bounds the N = 768 GEMM tiles a limit of
// the LDS-DMA path (global_load_lds_dwordx4) or of the CU's vector-memory path as a whole?  Every workgroup
// streams 1-KiB pieces (one wave-instruction each) of an L2-resident buffer:
//   mode 0  LDS-DMA only             (global_load_lds_dwordx4 into an LDS ring)
//   mode 1  VGPR loads only          (global_load_dwordx4, values folded into a checksum)
//   mode 2  half the waves each way  (same total bytes)
// usage: bw_lab [span_kib] [waves] [inflight]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int MODE, int IF>
__global__ __launch_bounds__(1024) void bw_kernel(const char* __restrict__ src, unsigned span, int iters, unsigned* sink)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const bool dma = MODE == 0 || (MODE == 2 && (wave & 1) == 0);
    unsigned acc = 0;
    unsigned off = (blockIdx.x * 37u + wave * 5u) * 1024u % span;
    for (int it = 0; it < iters; ++it) {
        if (MODE == 3) {
            // continuous stream: two groups of IF pieces alternate ring halves, the older group waited for by count
#pragma unroll
            for (int p = 0; p < IF; ++p) {
                const char* g = src + (off + p * 1024u) % span + lane * 16;
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                                 (__attribute__((address_space(3))) void*)(smem + ((wave * 2 + (it & 1)) * IF + p) * 1024), 16, 0, 0);
            }
            asm volatile("s_waitcnt vmcnt(%0)" :: "n"(IF) : "memory");
        } else if (dma) {
#pragma unroll
            for (int p = 0; p < IF; ++p) {
                const char* g = src + (off + p * 1024u) % span + lane * 16;
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                                 (__attribute__((address_space(3))) void*)(smem + (wave * IF + p) * 1024), 16, 0, 0);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            uint4 v[IF];
#pragma unroll
            for (int p = 0; p < IF; ++p) v[p] = *reinterpret_cast<const uint4*>(src + (off + p * 1024u) % span + lane * 16);
#pragma unroll
            for (int p = 0; p < IF; ++p) acc ^= v[p].x ^ v[p].y ^ v[p].z ^ v[p].w;
        }
        off = (off + IF * 1024u * nw) % span;
    }
    if (acc == 0x12345678u) sink[0] = acc;
    if (dma && lane == 0 && smem[wave] == 0x7f) sink[1] = 1;
}

template <int MODE, int IF>
float run(const char* src, unsigned span, int waves, int iters, unsigned* sink, int blocks)
{
    const int lds = waves * IF * 1024 * (MODE == 3 ? 2 : 1);
    CK(hipFuncSetAttribute((const void*)bw_kernel<MODE, IF>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((bw_kernel<MODE, IF>), dim3(blocks), dim3(64 * waves), lds, 0, src, span, iters, sink);
    CK(hipEventRecord(a));
    const int reps = 10;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((bw_kernel<MODE, IF>), dim3(blocks), dim3(64 * waves), lds, 0, src, span, iters, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double bytes = (double)blocks * waves * iters * IF * 1024.0;
    return (float)(bytes / (ms / reps * 1e-3) / 1e9);
}

int main(int argc, char** argv)
{
    const unsigned span = (argc > 1 ? atoi(argv[1]) : 2048) * 1024u;
    char* src;
    unsigned* sink;
    CK(hipMalloc(&src, span));
    CK(hipMalloc(&sink, 64));
    std::vector<unsigned char> h(span);
    for (unsigned i = 0; i < span; ++i) h[i] = (unsigned char)(i * 2654435761u >> 13);
    CK(hipMemcpy(src, h.data(), span, hipMemcpyHostToDevice));
    const int blocks = 256, iters = 400;
    printf("span %u KiB, %d blocks; GB/s per CU (chip TB/s)\n", span / 1024, blocks);
    for (int waves : {4, 8, 12, 16}) {
        for (int round = 0; round < 2; ++round) {
            float a = run<3, 4>(src, span, waves, iters * 2, sink, blocks);
            float b = waves <= 8 ? run<3, 8>(src, span, waves, iters, sink, blocks) : 0.f;
            float c = waves <= 4 ? run<3, 16>(src, span, waves, iters / 2, sink, blocks) : 0.f;
            printf("waves %d  stream IF4 %.1f  IF8 %.1f  IF16 %.1f\n", waves, a / blocks, b / blocks, c / blocks);
        }
    }
    for (int waves : {4, 8}) {
        for (int round = 0; round < 2; ++round) {
            float r[9];
            r[0] = run<0, 8>(src, span, waves, iters, sink, blocks);
            r[1] = run<1, 8>(src, span, waves, iters, sink, blocks);
            r[2] = run<2, 8>(src, span, waves, iters, sink, blocks);
            r[3] = run<0, 16>(src, span, waves, iters / 2, sink, blocks);
            r[4] = run<1, 16>(src, span, waves, iters / 2, sink, blocks);
            r[5] = run<2, 16>(src, span, waves, iters / 2, sink, blocks);
            printf("waves %d  IF8: dma %.1f  vgpr %.1f  mix %.1f | IF16: dma %.1f  vgpr %.1f  mix %.1f   (chip TB/s dma8 %.1f)\n",
                   waves, r[0] / blocks, r[1] / blocks, r[2] / blocks, r[3] / blocks, r[4] / blocks, r[5] / blocks, r[0] / 1000);
        }
    }
    return 0;
}
