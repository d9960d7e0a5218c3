// LayerNorm-fold lab (experiment harness, not product code): the encoder's c_fc (+QuickGELU) and QKV products at
// 16 crops (M = 16 x 229) timed as plain products (EPI_GELU / EPI_STORE) and as LayerNorm-folded ones (EPI_LN_GELU /
// EPI_LN reading 16 row partials per row), on a normalised-like A and on a raw-residual-like A, interleaved rounds in
// one process.  Separates the cost of the fold from operand effects (profiles/r04t_lnfold_lab_*.txt were taken on the
// first form, register loads of the partials, with isolation switches since removed; the tree's form stages them
// into LDS by DMA).
//   build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1 -DEBC_GEMM_LAB \
//          tools/lab/lnfold_lab.hip -o tools/lab/bin/lnfold_lab
//   run:   lnfold_lab [rounds] [reps]
#include "../../clip-ebc_amd/csrc/gemm.hip"

#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

namespace ebc {
bool probe_on() { return false; }
int probe_start(int, int, int, int, int, int, int, int, hipStream_t) { return -1; }
void probe_stop(int, hipStream_t) {}
}  // namespace ebc

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

// x = scale * u + shift (u uniform in [-1, 1)), per element hashed
__global__ void fill_f16(_Float16* p, size_t n, unsigned seed, float scale, float shift)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
        p[i] = (_Float16)(((h & 0xffff) / 32768.0f - 1.0f) * scale + shift);
    }
}
__global__ void fill_f32(float* p, size_t n, unsigned seed)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2246822519u ^ seed;
        h ^= h >> 13; h *= 2654435761u; h ^= h >> 16;
        p[i] = (h & 0xffff) / 32768.0f - 1.0f;
    }
}
// row partials of A [M][K] (16 per row, 48 columns each) as the residual products write them
__global__ void partials(const _Float16* A, float2* rp, int M, int K, int parts)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M * parts) return;
    const int m = i / parts, p = i % parts, w = K / parts;
    float s = 0.f, q = 0.f;
    for (int k = p * w; k < (p + 1) * w; ++k) { const float v = (float)A[(size_t)m * K + k]; s += v; q += v * v; }
    rp[i] = float2{s, q};
}
__global__ void rowsum(const _Float16* W, float* out, int N, int K)
{
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    float s = 0.f;
    for (int k = 0; k < K; ++k) s += (float)W[(size_t)n * K + k];
    out[n] = s;
}

template <class T> T* dalloc(size_t n) { T* p; CK(hipMalloc(&p, n * sizeof(T))); return p; }

int main(int argc, char** argv)
{
    const int rounds = argc > 1 ? atoi(argv[1]) : 3, reps = argc > 2 ? atoi(argv[2]) : 30;
    const int M = 16 * 229, K = 768, P = 16;
    _Float16* An = dalloc<_Float16>((size_t)M * K);
    _Float16* Ar = dalloc<_Float16>((size_t)M * K);
    _Float16* W = dalloc<_Float16>((size_t)3072 * K);
    _Float16* C = dalloc<_Float16>((size_t)M * 3072);
    _Float16* Aux = dalloc<_Float16>((size_t)M * 3072);
    float* bias = dalloc<float>(3072);
    float* lnw = dalloc<float>(3072);
    float2* rp = dalloc<float2>((size_t)M * P);
    float* mean = dalloc<float>(M);
    float* rstd = dalloc<float>(M);
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, An, (size_t)M * K, 1u, 1.7f, 0.f);
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, Ar, (size_t)M * K, 7u, 0.6f, 0.05f);
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, W, (size_t)3072 * K, 2u, 0.03f, 0.f);
    hipLaunchKernelGGL(fill_f32, dim3(64), dim3(256), 0, 0, bias, (size_t)3072, 4u);
    hipLaunchKernelGGL(partials, dim3((M * P + 255) / 256), dim3(256), 0, 0, Ar, rp, M, K, P);
    hipLaunchKernelGGL(rowsum, dim3(12), dim3(256), 0, 0, W, lnw, 3072, K);
    CK(hipDeviceSynchronize());

    auto args = [&](const _Float16* A, int N, void* aux) {
        GemmArgs g{A, W, C, bias, nullptr, aux, M, N, K};
        g.kslice = K;
        return g;
    };
    auto lnargs = [&](int N, void* aux) {
        GemmArgs g = args(Ar, N, aux);
        g.lnp = reinterpret_cast<const float*>(rp); g.lnparts = P; g.lnw = lnw; g.ln_mean = mean; g.ln_rstd = rstd;
        return g;
    };
    struct V { std::string name; std::function<int()> fn; };
    std::vector<V> vs = {
        {"c_fc GELU  A=norm", [&] { return launch_gemm_k<EF16, _Float16, EPI_GELU, 256, 192, 2, 4, 2, 128, 0, false, 0>(args(An, 3072, Aux), 0); }},
        {"c_fc GELU  A=raw ", [&] { return launch_gemm_k<EF16, _Float16, EPI_GELU, 256, 192, 2, 4, 2, 128, 0, false, 0>(args(Ar, 3072, Aux), 0); }},
        {"c_fc LN_GELU A=raw", [&] { return launch_gemm_k<EF16, _Float16, EPI_LN_GELU, 256, 192, 2, 4, 2, 128, 0, false, 0>(lnargs(3072, Aux), 0); }},
        {"QKV STORE  A=norm", [&] { return launch_gemm_k<EF16, _Float16, EPI_STORE, 192, 192, 2, 4, 2, 128, 0, false, 0>(args(An, 2304, nullptr), 0); }},
        {"QKV STORE  A=raw ", [&] { return launch_gemm_k<EF16, _Float16, EPI_STORE, 192, 192, 2, 4, 2, 128, 0, false, 0>(args(Ar, 2304, nullptr), 0); }},
        {"QKV LN     A=raw ", [&] { return launch_gemm_k<EF16, _Float16, EPI_LN, 192, 192, 2, 4, 2, 128, 0, false, 0>(lnargs(2304, nullptr), 0); }},
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (auto& v : vs) if (v.fn() != 0) { printf("launch failed: %s\n", v.name.c_str()); return 1; }
    CK(hipDeviceSynchronize());
    for (int r = 0; r < rounds; ++r) {
        for (auto& v : vs) {
            for (int i = 0; i < 3; ++i) v.fn();
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < reps; ++i) v.fn();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("round %d  %-20s %8.2f us\n", r, v.name.c_str(), 1000.f * ms / reps);
        }
    }
    return 0;
}
