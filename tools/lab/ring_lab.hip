// Ring-depth lab (experiment harness, not product code): the encoder's c_fc (+QuickGELU, 256x192) and QKV (192x192)
// products at 16 crops (M = 16 x 229) with the r04 ring (128-B K rows = 64-deep k-tiles, 2 stages: one k-tile in
// flight) against deeper rings: 64-B rows, 4 stages (3 k-tiles of 32 in flight), 128-B rows, 3 stages.  Timed warm (back to
// back) and cold (a 768 MB sweep before each launch evicts L2 and the Infinity Cache, as the step's weights are),
// interleaved rounds in one process; every variant's output compared bitwise with the first.
//   build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1 -DEBC_GEMM_LAB \
//          tools/lab/ring_lab.hip -o tools/lab/bin/ring_lab
//   run:   ring_lab [rounds] [reps]
#include "../../clip-ebc_amd/csrc/gemm.hip"

#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

namespace ebc {
bool probe_on() { return false; }
int probe_start(int, int, int, int, int, int, int, int, hipStream_t) { return -1; }
void probe_stop(int, hipStream_t) {}
}  // namespace ebc

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void fill_f16(_Float16* p, size_t n, unsigned seed, float scale)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
        p[i] = (_Float16)(((h & 0xffff) / 32768.0f - 1.0f) * scale);
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
__global__ __launch_bounds__(256) void sweep(uint4* p, size_t n16)
{
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) p[i] = make_uint4(i, 0, 0, 0);
}

// gemm.hip group_rows (outside the lab part of the file)
static int lab_group_rows(int M, int N, int bm, int bn) {
    const long ntm = (M + bm - 1) / bm, ntn = N / bn;
    if (ntn < 12) return 0;
    const double C = (double)(ntm * ntn) / 8.0;
    const int gm = (int)(sqrt(C * bn / bm) + 0.5);
    return gm > 1 && gm < ntm ? gm : 0;
}

template <class T> T* dalloc(size_t n) { T* p; CK(hipMalloc(&p, n * sizeof(T))); return p; }

using Fn = std::function<int(const GemmArgs&)>;
template <int EPI, int BM, int BN, int S, int WGM, int WGN, int ROWB>
Fn var() { return [](const GemmArgs& g) { return launch_gemm_k<EF16, _Float16, EPI, BM, BN, S, WGM, WGN, ROWB, 0, false, 0>(g, 0); }; }

int main(int argc, char** argv)
{
    const int rounds = argc > 1 ? atoi(argv[1]) : 3, reps = argc > 2 ? atoi(argv[2]) : 20;
    const int M = 16 * 229, K = 768;
    _Float16* A = dalloc<_Float16>((size_t)M * K);
    _Float16* W = dalloc<_Float16>((size_t)3072 * K);
    _Float16* C0 = dalloc<_Float16>((size_t)M * 3072);
    _Float16* C1 = dalloc<_Float16>((size_t)M * 3072);
    _Float16* Aux = dalloc<_Float16>((size_t)M * 3072);
    float* bias = dalloc<float>(3072);
    const size_t sweep_bytes = (size_t)768 << 20;
    uint4* junk = dalloc<uint4>(sweep_bytes / 16);
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, A, (size_t)M * K, 1u, 1.7f);
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, W, (size_t)3072 * K, 2u, 0.03f);
    hipLaunchKernelGGL(fill_f32, dim3(64), dim3(256), 0, 0, bias, (size_t)3072, 4u);
    CK(hipDeviceSynchronize());

    struct V { std::string name; int N, epi; Fn fn; int gm = 0; };
    std::vector<V> vs = {
        {"c_fc 256x192 R128 S2", 3072, EPI_GELU, var<EPI_GELU, 256, 192, 2, 4, 2, 128>()},
        {"c_fc 256x192 R64 S4", 3072, EPI_GELU, var<EPI_GELU, 256, 192, 4, 4, 2, 64>()},
        {"c_fc 256x256 R128 S2", 3072, EPI_GELU, var<EPI_GELU, 256, 256, 2, 4, 2, 128>()},
        {"QKV 192x192 R128 S2", 2304, EPI_STORE, var<EPI_STORE, 192, 192, 2, 4, 2, 128>()},
        {"QKV 192x192 R128 S3", 2304, EPI_STORE, var<EPI_STORE, 192, 192, 3, 4, 2, 128>()},
        {"QKV 192x192 R64 S4", 2304, EPI_STORE, var<EPI_STORE, 192, 192, 4, 4, 2, 64>()},
        {"QKV 256x192 R128 S2", 2304, EPI_STORE, var<EPI_STORE, 256, 192, 2, 4, 2, 128>()},
    };
    // tile order as gemm.hip's group_rows for each variant's tile
    const int tiles_bm[] = {256, 256, 256, 192, 192, 192, 256}, tiles_bn[] = {192, 192, 256, 192, 192, 192, 192};
    for (size_t i = 0; i < vs.size(); ++i) vs[i].gm = lab_group_rows(M, vs[i].N, tiles_bm[i], tiles_bn[i]);
    auto args = [&](const V& v, _Float16* C) {
        GemmArgs g{A, W, C, bias, nullptr, v.epi == EPI_GELU ? Aux : nullptr, M, v.N, K};
        g.kslice = K;
        g.group_m = v.gm;
        return g;
    };
    // bitwise check against the first variant of the same N
    std::vector<_Float16> ref((size_t)M * 3072), got((size_t)M * 3072);
    for (size_t i = 0; i < vs.size(); ++i) {
        const bool first = i == 0 || vs[i].N != vs[i - 1].N;
        if (vs[i].fn(args(vs[i], first ? C0 : C1))) { printf("launch failed: %s\n", vs[i].name.c_str()); return 1; }
        CK(hipDeviceSynchronize());
        if (!first) {
            CK(hipMemcpy(ref.data(), C0, (size_t)M * vs[i].N * 2, hipMemcpyDeviceToHost));
            CK(hipMemcpy(got.data(), C1, (size_t)M * vs[i].N * 2, hipMemcpyDeviceToHost));
            size_t bad = 0;
            for (size_t e = 0; e < (size_t)M * vs[i].N; ++e) bad += memcmp(&ref[e], &got[e], 2) != 0;
            printf("%-22s vs first: %zu of %zu elements differ\n", vs[i].name.c_str(), bad, (size_t)M * vs[i].N);
        }
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; ++r) {
        for (auto& v : vs) {
            const GemmArgs g = args(v, C1);
            for (int i = 0; i < 3; ++i) v.fn(g);
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < reps; ++i) v.fn(g);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float warm;
            CK(hipEventElapsedTime(&warm, e0, e1));
            float cold = 0;
            for (int i = 0; i < reps; ++i) {
                hipLaunchKernelGGL(sweep, dim3(4096), dim3(256), 0, 0, junk, sweep_bytes / 16);
                CK(hipEventRecord(e0, 0));
                v.fn(g);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float t;
                CK(hipEventElapsedTime(&t, e0, e1));
                cold += t;
            }
            const double tf = 2.0 * M * v.N * K / 1e12;
            printf("r%d %-22s warm %7.2f us (%5.0f TF/s)  cold %7.2f us (%5.0f TF/s)\n", r, v.name.c_str(), 1e3 * warm / reps,
                   tf / (warm / reps * 1e-3), 1e3 * cold / reps, tf / (cold / reps * 1e-3));
        }
    }
    return 0;
}
