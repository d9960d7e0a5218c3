// LayerNorm-forward lab (experiment harness, not product code): ln_1 / ln_2 of the 16-crop ViT-B/16 + VPT(32)
// step (M = 16 x 229 = 3664 rows of 768 f32 -> fp16 + row mean / rstd), timed under rocprofv3 --kernel-trace:
//   prod     vit_misc.hip's ln_fwd_kernel<_Float16, 3> (one row per wave, 4 waves per workgroup)
//   r2       two rows per wave (6 row loads in flight per lane)
//   w1       one row per wave, one wave per workgroup (3664 workgroups)
//   copy     the floor: the same bytes (f32 row in, fp16 row out) with no statistics
// each after a producer kernel that rewrites x (as the residual GEMM's epilogue does in the step) and also
// back to back (x still in the XCD's L2 from the previous launch).  Distinct template tags give every
// (variant, case) its own kernel name in the trace.  Outputs of r2 / w1 are compared bitwise with prod.
//   build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/lab/ln_lab.hip -o tools/lab/bin/ln_lab
//   run:   rocprofv3 --kernel-trace --stats -d DIR -o run -- tools/lab/bin/ln_lab [reps]
#include "../../clip-ebc_amd/csrc/vit_misc.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

namespace ebc {
bool probe_on() { return false; }
int probe_start(int, int, int, int, int, int, int, int, hipStream_t) { return -1; }
void probe_stop(int, hipStream_t) {}
}  // namespace ebc

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int D = 768, NV = 3;

template <int TAG>
__global__ __launch_bounds__(256) void produce_kernel(float* x, size_t n, unsigned seed)
{
    // grid-stride over float4 in a different row -> workgroup order than the LayerNorm (as a GEMM epilogue)
    const size_t n4 = n / 4;
    for (size_t i = (size_t)(gridDim.x - 1 - blockIdx.x) * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
        const float f = (float)(h & 0xffff) / 16384.0f - 2.0f;
        reinterpret_cast<float4*>(x)[i] = make_float4(f, f * 0.5f + 0.1f, -f, f * 0.25f - 0.3f);
    }
}

template <int TAG>
__global__ __launch_bounds__(256) void ln_prod(const float* x, const float* g, const float* b, _Float16* out, float* mean,
                                               float* rstd, int M)
{
    // the product kernel's body, instantiated under its own name
    constexpr int DD = 256 * NV;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (r >= M) return;
    const float* xr = x + (size_t)r * DD;
    float4 v[NV], gb[2 * NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = *reinterpret_cast<const float4*>(xr + 4 * lane + 256 * i);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        gb[2 * i] = *reinterpret_cast<const float4*>(g + 4 * lane + 256 * i);
        gb[2 * i + 1] = *reinterpret_cast<const float4*>(b + 4 * lane + 256 * i);
    }
    float mu, rs;
    ln_row<NV>(v, gb, mu, rs);
#pragma unroll
    for (int i = 0; i < NV; ++i) st4<_Float16>(out + (size_t)r * DD + 4 * lane + 256 * i, v[i]);
    if (lane == 0) { mean[r] = mu; rstd[r] = rs; }
}

template <int TAG, int RPW, int WPB>
__global__ __launch_bounds__(64 * WPB) void ln_multi(const float* x, const float* g, const float* b, _Float16* out,
                                                     float* mean, float* rstd, int M)
{
    const int r0 = (blockIdx.x * WPB + (threadIdx.x >> 6)) * RPW, lane = threadIdx.x & 63;
    float4 v[RPW][NV], gb[2 * NV];
#pragma unroll
    for (int k = 0; k < RPW; ++k)
        if (r0 + k < M)
#pragma unroll
            for (int i = 0; i < NV; ++i) v[k][i] = *reinterpret_cast<const float4*>(x + (size_t)(r0 + k) * D + 4 * lane + 256 * i);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        gb[2 * i] = *reinterpret_cast<const float4*>(g + 4 * lane + 256 * i);
        gb[2 * i + 1] = *reinterpret_cast<const float4*>(b + 4 * lane + 256 * i);
    }
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
        if (r0 + k >= M) break;
        float mu, rs;
        ln_row<NV>(v[k], gb, mu, rs);
#pragma unroll
        for (int i = 0; i < NV; ++i) st4<_Float16>(out + (size_t)(r0 + k) * D + 4 * lane + 256 * i, v[k][i]);
        if (lane == 0) { mean[r0 + k] = mu; rstd[r0 + k] = rs; }
    }
}

template <int TAG>
__global__ __launch_bounds__(256) void copy_floor(const float* x, _Float16* out, int M)
{
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (r >= M) return;
    float4 v[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = *reinterpret_cast<const float4*>(x + (size_t)r * D + 4 * lane + 256 * i);
#pragma unroll
    for (int i = 0; i < NV; ++i) st4<_Float16>(out + (size_t)r * D + 4 * lane + 256 * i, v[i]);
}

int main(int argc, char** argv)
{
    const int reps = argc > 1 ? atoi(argv[1]) : 50;
    const int M = 16 * 229;
    float *x, *g, *b, *mean, *rstd;
    _Float16 *o0, *o1;
    CK(hipMalloc(&x, (size_t)M * D * 4));
    CK(hipMalloc(&g, D * 4));
    CK(hipMalloc(&b, D * 4));
    CK(hipMalloc(&mean, M * 4));
    CK(hipMalloc(&rstd, M * 4));
    CK(hipMalloc(&o0, (size_t)M * D * 2));
    CK(hipMalloc(&o1, (size_t)M * D * 2));
    std::vector<float> hg(D), hb(D);
    for (int i = 0; i < D; ++i) { hg[i] = 1.0f + 0.001f * i; hb[i] = 0.01f * (i % 7); }
    CK(hipMemcpy(g, hg.data(), D * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(b, hb.data(), D * 4, hipMemcpyHostToDevice));
    const size_t n = (size_t)M * D;
    const dim3 pg(2048);
    hipLaunchKernelGGL(produce_kernel<0>, pg, dim3(256), 0, 0, x, n, 7u);
    // bitwise checks against the product body
    std::vector<unsigned short> ref(n), got(n);
    hipLaunchKernelGGL(ln_prod<0>, dim3((M + 3) / 4), dim3(256), 0, 0, x, g, b, o0, mean, rstd, M);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(ref.data(), o0, n * 2, hipMemcpyDeviceToHost));
    auto check = [&](const char* name) {
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got.data(), o1, n * 2, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 0; i < n; ++i) bad += ref[i] != got[i];
        printf("%-6s vs prod: %zu of %zu differ\n", name, bad, n);
    };
    hipLaunchKernelGGL((ln_multi<0, 2, 4>), dim3((M + 7) / 8), dim3(256), 0, 0, x, g, b, o1, mean, rstd, M);
    check("r2");
    hipLaunchKernelGGL((ln_multi<0, 1, 1>), dim3(M), dim3(64), 0, 0, x, g, b, o1, mean, rstd, M);
    check("w1");
    for (int i = 0; i < reps; ++i) {
        // after a producer
        hipLaunchKernelGGL(produce_kernel<1>, pg, dim3(256), 0, 0, x, n, 7u);
        hipLaunchKernelGGL(ln_prod<1>, dim3((M + 3) / 4), dim3(256), 0, 0, x, g, b, o0, mean, rstd, M);
        hipLaunchKernelGGL(produce_kernel<2>, pg, dim3(256), 0, 0, x, n, 7u);
        hipLaunchKernelGGL((ln_multi<2, 2, 4>), dim3((M + 7) / 8), dim3(256), 0, 0, x, g, b, o1, mean, rstd, M);
        hipLaunchKernelGGL(produce_kernel<3>, pg, dim3(256), 0, 0, x, n, 7u);
        hipLaunchKernelGGL((ln_multi<3, 1, 1>), dim3(M), dim3(64), 0, 0, x, g, b, o1, mean, rstd, M);
        hipLaunchKernelGGL(produce_kernel<4>, pg, dim3(256), 0, 0, x, n, 7u);
        hipLaunchKernelGGL(copy_floor<4>, dim3((M + 3) / 4), dim3(256), 0, 0, x, o1, M);
        hipLaunchKernelGGL(produce_kernel<5>, pg, dim3(256), 0, 0, x, n, 7u);
        hipLaunchKernelGGL((ln_multi<5, 1, 2>), dim3((M + 1) / 2), dim3(128), 0, 0, x, g, b, o1, mean, rstd, M);
    }
    for (int i = 0; i < reps; ++i) {
        // back to back
        hipLaunchKernelGGL(ln_prod<10>, dim3((M + 3) / 4), dim3(256), 0, 0, x, g, b, o0, mean, rstd, M);
        hipLaunchKernelGGL(ln_prod<10>, dim3((M + 3) / 4), dim3(256), 0, 0, x, g, b, o0, mean, rstd, M);
        hipLaunchKernelGGL((ln_multi<12, 2, 4>), dim3((M + 7) / 8), dim3(256), 0, 0, x, g, b, o1, mean, rstd, M);
        hipLaunchKernelGGL((ln_multi<12, 2, 4>), dim3((M + 7) / 8), dim3(256), 0, 0, x, g, b, o1, mean, rstd, M);
        hipLaunchKernelGGL(copy_floor<14>, dim3((M + 3) / 4), dim3(256), 0, 0, x, o1, M);
        hipLaunchKernelGGL(copy_floor<14>, dim3((M + 3) / 4), dim3(256), 0, 0, x, o1, M);
    }
    CK(hipDeviceSynchronize());
    printf("bytes per launch: %.2f MB (f32 in) + %.2f MB (fp16 out)\n", n * 4 / 1e6, n * 2 / 1e6);
    return 0;
}
