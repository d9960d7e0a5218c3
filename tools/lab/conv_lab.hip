// Decoder 3x3-conv weight-gradient lab (experiment harness, not product code): the MODE 2 implicit GEMM of
// gemm.hip at the 16-crop decoder shape (dW [768][6912] f32 = dz^T [768][K] . x^T-images, K = 16 x 14 x 64
// interior pixel rows), by tile, split count and split reduction (last arriver vs partials + reduce launch).
// Interleaved rounds in one process; every variant compared with the unsplit 256x192 result.
//   build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1 -DEBC_GEMM_LAB \
//          tools/lab/conv_lab.hip -o tools/lab/bin/conv_lab
#include "../../clip-ebc_amd/csrc/gemm.hip"

#include <cmath>
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

constexpr size_t GEMM_CNT_BYTES = 16 * 1024;     // gemm.hip's split-K counter block
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part, float* __restrict__ C, long MN,
                                                            int splits)
{
    const long e = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
    if (e >= MN) return;
    float4 acc = *reinterpret_cast<const float4*>(part + e);
    for (int sp = 1; sp < splits; ++sp) {
        const float4 v = *reinterpret_cast<const float4*>(part + (size_t)sp * MN + e);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    *reinterpret_cast<float4*>(C + e) = acc;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void fill_f16(_Float16* p, size_t n, unsigned seed, float scale)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
        p[i] = (_Float16)(((h & 0xffff) / 32768.0f - 1.0f) * scale);
    }
}

template <int BM_, int BN_, int S_, int WGM_, int WGN_> struct Tl {
    static constexpr int BM = BM_, BN = BN_, S = S_, WGM = WGM_, WGN = WGN_;
};
using T256x192 = Tl<256, 192, 2, 4, 2>;
using T256x256 = Tl<256, 256, 2, 4, 2>;
using T128x192 = Tl<128, 192, 3, 2, 2>;

int main(int argc, char** argv)
{
    const int rounds = argc > 1 ? atoi(argv[1]) : 3, reps = argc > 2 ? atoi(argv[2]) : 10;
    // decoder geometry at 16 crops (decoder.hip make_geo: B 16, H = W = 28, C 768)
    const int B = 16, H = 28, W = 28, C = 768, N = 768;
    const int Hp = H + 2, Wp = 32, G = 64, bk = 64, kpi = (H * Wp + bk - 1) / bk;
    const long Q = (long)B * Hp * Wp, Qs = ((G + Q + bk + Wp + 63) / 64) * 64;
    const int M = N, NN = 9 * C, K = B * kpi * bk;
    _Float16 *dzT, *xT3;
    CK(hipMalloc(&dzT, (size_t)M * Qs * 2));
    CK(hipMalloc(&xT3, (size_t)3 * C * Qs * 2));
    float *out0, *out1, *part;
    CK(hipMalloc(&out0, (size_t)M * NN * 4));
    CK(hipMalloc(&out1, (size_t)M * NN * 4));
    const size_t pbytes = (size_t)8 * M * NN * 4;
    CK(hipMalloc(&part, GEMM_CNT_BYTES + pbytes));
    CK(hipMemset(part, 0, GEMM_CNT_BYTES + pbytes));
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, dzT, (size_t)M * Qs, 11u, 1.0f);
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, xT3, (size_t)3 * C * Qs, 12u, 1.0f);
    CK(hipDeviceSynchronize());

    auto args = [&](float* out, int splits, bool partials) {
        GemmArgs g{dzT, xT3, out, nullptr, nullptr, nullptr, M, NN, K};
        g.cH = H; g.cW = W; g.cC = C; g.cHp = Hp; g.cWp = Wp; g.kpi = kpi; g.cQs = Qs; g.cG = G;
        g.splits = splits; g.kslice = K / splits;
        g.cnt = splits > 1 && !partials ? reinterpret_cast<int*>(part) : nullptr;
        g.part = splits > 1 ? reinterpret_cast<float*>(reinterpret_cast<char*>(part) + GEMM_CNT_BYTES) : nullptr;
        return g;
    };
    struct V { std::string name; std::function<void(float*)> fn; };
    auto tile = [&](auto bm_bn_s, int splits, bool partials) {
        using TT = decltype(bm_bn_s);
        return [&, splits, partials](float* out) {
            GemmArgs g = args(out, splits, partials);
            int rc;
            if (splits > 1)
                rc = launch_gemm_k<EF16, float, EPI_STORE, TT::BM, TT::BN, TT::S, TT::WGM, TT::WGN, 128, 2, true>(g, 0);
            else
                rc = launch_gemm_k<EF16, float, EPI_STORE, TT::BM, TT::BN, TT::S, TT::WGM, TT::WGN, 128, 2, false>(g, 0);
            if (rc) { printf("launch rc %d\n", rc); exit(1); }
            if (splits > 1 && partials) {
                hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)(((long)M * NN / 4 + 255) / 256)), dim3(256), 0, 0,
                                   g.part, out, (long)M * NN, splits);
            }
        };
    };
    std::vector<V> vars = {
        {"256x192 s1", tile(T256x192{}, 1, false)},
        {"256x192 s2 last-arriver", tile(T256x192{}, 2, false)},
        {"256x192 s2 partials+reduce", tile(T256x192{}, 2, true)},
        {"256x192 s4 partials+reduce", tile(T256x192{}, 4, true)},
        {"256x256 s2 partials+reduce", tile(T256x256{}, 2, true)},
        {"256x192 s7 partials+reduce", tile(T256x192{}, 7, true)},
        {"128x192 s1", tile(T128x192{}, 1, false)},
        {"128x192 s2 partials+reduce", tile(T128x192{}, 2, true)},
    };
    std::vector<float> ref((size_t)M * NN), got((size_t)M * NN);
    for (size_t v = 0; v < vars.size(); ++v) {
        float* o = v == 0 ? out0 : out1;
        CK(hipMemset(o, 0, (size_t)M * NN * 4));
        vars[v].fn(o);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(v == 0 ? ref.data() : got.data(), o, (size_t)M * NN * 4, hipMemcpyDeviceToHost));
        if (v) {
            double num = 0, den = 0;
            for (size_t i = 0; i < ref.size(); ++i) { num += (got[i] - ref[i]) * (double)(got[i] - ref[i]); den += (double)ref[i] * ref[i]; }
            printf("%-30s rel-L2 vs s1: %.2e\n", vars[v].name.c_str(), std::sqrt(num / den));
        }
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const double tf = 2.0 * M * NN * K / 1e12;
    for (int r = 0; r < rounds; ++r)
        for (auto& v : vars) {
            v.fn(out1);
            CK(hipEventRecord(e0));
            for (int i = 0; i < reps; ++i) v.fn(out1);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("r%d %-30s %8.2f us  %7.1f TF/s\n", r, v.name.c_str(), ms / reps * 1e3, tf / (ms / reps * 1e-3));
        }
    return 0;
}
