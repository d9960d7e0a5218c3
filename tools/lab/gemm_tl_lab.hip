// GEMM timeline lab (experiment harness, not product code): per-workgroup phase stamps of gemm.hip's kernel templates at
// the ViT-B/16 16-crop shapes (M = 16 x 229): entry, first k-tile landed, K loop done, epilogue issued, epilogue's
// memory operations retired (s_memrealtime, 100 MHz), plus the shader clock over the workgroup (s_memtime) and its
// XCC / CU.  Answers where a launch's time goes: start skew, prologue, K loop, epilogue, store drain.
//   build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1 -DEBC_GEMM_LAB \
//          tools/lab/gemm_tl_lab.hip -o tools/lab/bin/gemm_tl_lab
//   run:   gemm_tl_lab [reps]
#include <hip/hip_runtime.h>

__device__ unsigned long long* g_tl = nullptr;          // [tile][8]
__device__ __forceinline__ void tl_stamp(int phase, int tile)
{
    if (threadIdx.x != 0 || g_tl == nullptr) return;
    unsigned long long* p = g_tl + (size_t)tile * 8;
    if (phase == 3) {
        p[3] = __builtin_amdgcn_s_memrealtime();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        p[4] = __builtin_amdgcn_s_memrealtime();
        p[6] = __builtin_amdgcn_s_memtime();
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        p[7] = ((unsigned long long)xcc << 32) | hw;
    } else {
        p[phase] = __builtin_amdgcn_s_memrealtime();
        if (phase == 0) p[5] = __builtin_amdgcn_s_memtime();
    }
}
#define EBC_GEMM_STAMP(phase, tile) tl_stamp(phase, tile)

#include "../../clip-ebc_amd/csrc/gemm.hip"

#include <algorithm>
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
template <class T> T* dalloc(size_t n) { T* p; CK(hipMalloc(&p, n * sizeof(T))); return p; }

struct Variant {
    std::string name;
    int N, K;
    std::function<int(GemmArgs&)> fn;      // fills the operands it needs, launches
    int ntiles;
};

static double pct(std::vector<double> v, double q)
{
    std::sort(v.begin(), v.end());
    return v[std::min(v.size() - 1, (size_t)(q * (v.size() - 1) + 0.5))];
}

int main(int argc, char** argv)
{
    const int reps = argc > 1 ? atoi(argv[1]) : 5;
    const int M = 16 * 229;
    _Float16* A = dalloc<_Float16>((size_t)M * 3072);
    _Float16* W = dalloc<_Float16>((size_t)3072 * 3072);
    _Float16* Cfc = dalloc<_Float16>((size_t)M * 3072);
    _Float16* Afc = dalloc<_Float16>((size_t)M * 3072);
    float* R = dalloc<float>((size_t)M * 768);
    float* bias = dalloc<float>(3072);
    void* C = dalloc<float>((size_t)M * 3072);
    unsigned long long* tl = dalloc<unsigned long long>(4096 * 8);
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, A, (size_t)M * 3072, 1u, 1.0f);
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, W, (size_t)3072 * 3072, 2u, 0.03f);
    hipLaunchKernelGGL(fill_f32, dim3(1024), dim3(256), 0, 0, R, (size_t)M * 768, 3u);
    hipLaunchKernelGGL(fill_f32, dim3(64), dim3(256), 0, 0, bias, (size_t)3072, 4u);
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, Cfc, (size_t)M * 3072, 5u, 1.0f);
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, Afc, (size_t)M * 3072, 6u, 1.0f);
    CK(hipDeviceSynchronize());
    auto nt = [&](int bm, int bn, int N) { return ((M + bm - 1) / bm) * (N / bn); };

    std::vector<Variant> vars;
    vars.push_back({"c_fc GELU 256x192", 3072, 768, [&](GemmArgs& g) {
        g.A = A; g.aux = Afc; g.C = Cfc;
        return launch_gemm_k<EF16, _Float16, EPI_GELU, 256, 192, 2, 4, 2, 128, 0, false, 0>(g, 0); }, nt(256, 192, 3072)});
    vars.push_back({"GELU' 256x192", 3072, 768, [&](GemmArgs& g) {
        g.A = A; g.aux = Afc; g.C = C;
        return launch_gemm_k<EF16, _Float16, EPI_GELU_BWD, 256, 192, 2, 4, 2, 128, 0, false, 0>(g, 0); }, nt(256, 192, 3072)});
    vars.push_back({"QKV 192x192", 2304, 768, [&](GemmArgs& g) {
        g.A = A; g.C = C;
        return launch_gemm_k<EF16, _Float16, EPI_STORE, 192, 192, 2, 4, 2, 128, 0, false, 0>(g, 0); }, nt(192, 192, 2304)});
    vars.push_back({"c_proj+res S4+4L", 768, 3072, [&](GemmArgs& g) {
        g.A = Cfc; g.resid = R; g.C = C;
        return launch_gemm_k<EF16, float, EPI_RESID, 128, 96, 4, 2, 2, 128, 0, false, 4>(g, 0); }, nt(128, 96, 768)});
    vars.push_back({"c_proj store S4+4L", 768, 3072, [&](GemmArgs& g) {
        g.A = Cfc; g.C = C;
        return launch_gemm_k<EF16, _Float16, EPI_STORE, 128, 96, 4, 2, 2, 128, 0, false, 4>(g, 0); }, nt(128, 96, 768)});
    vars.push_back({"dH store K2304 S4+4L", 768, 2304, [&](GemmArgs& g) {
        g.A = Cfc; g.C = C;
        return launch_gemm_k<EF16, _Float16, EPI_STORE, 128, 96, 4, 2, 2, 128, 0, false, 4>(g, 0); }, nt(128, 96, 768)});
    vars.push_back({"out+res S3+4L", 768, 768, [&](GemmArgs& g) {
        g.A = A; g.resid = R; g.C = C;
        return launch_gemm_k<EF16, float, EPI_RESID, 128, 96, 3, 2, 2, 128, 0, false, 4>(g, 0); }, nt(128, 96, 768)});
    vars.push_back({"dO store S3+4L", 768, 768, [&](GemmArgs& g) {
        g.A = A; g.C = C;
        return launch_gemm_k<EF16, _Float16, EPI_STORE, 128, 96, 3, 2, 2, 128, 0, false, 4>(g, 0); }, nt(128, 96, 768)});

    // r06: 256-B K rows (BK = 128), 2 stages: half the k-tiles (barriers) of the 128-B rings at the same LDS
    vars.push_back({"c_proj+res R256 S2+4L", 768, 3072, [&](GemmArgs& g) {
        g.A = Cfc; g.resid = R; g.C = C;
        return launch_gemm_k<EF16, float, EPI_RESID, 128, 96, 2, 2, 2, 256, 0, false, 4>(g, 0); }, nt(128, 96, 768)});
    vars.push_back({"c_proj store R256 S2+4L", 768, 3072, [&](GemmArgs& g) {
        g.A = Cfc; g.C = C;
        return launch_gemm_k<EF16, _Float16, EPI_STORE, 128, 96, 2, 2, 2, 256, 0, false, 4>(g, 0); }, nt(128, 96, 768)});
    vars.push_back({"dH K2304 R256 S2+4L", 768, 2304, [&](GemmArgs& g) {
        g.A = Cfc; g.C = C;
        return launch_gemm_k<EF16, _Float16, EPI_STORE, 128, 96, 2, 2, 2, 256, 0, false, 4>(g, 0); }, nt(128, 96, 768)});
    vars.push_back({"out+res R256 S2+4L", 768, 768, [&](GemmArgs& g) {
        g.A = A; g.resid = R; g.C = C;
        return launch_gemm_k<EF16, float, EPI_RESID, 128, 96, 2, 2, 2, 256, 0, false, 4>(g, 0); }, nt(128, 96, 768)});
    vars.push_back({"dO store R256 S2+4L", 768, 768, [&](GemmArgs& g) {
        g.A = A; g.C = C;
        return launch_gemm_k<EF16, _Float16, EPI_STORE, 128, 96, 2, 2, 2, 256, 0, false, 4>(g, 0); }, nt(128, 96, 768)});
    vars.push_back({"c_proj store R256 S2", 768, 3072, [&](GemmArgs& g) {
        g.A = Cfc; g.C = C;
        return launch_gemm_k<EF16, _Float16, EPI_STORE, 128, 96, 2, 2, 2, 256, 0, false, 0>(g, 0); }, nt(128, 96, 768)});
    vars.push_back({"QKV R256 128x192 S2", 2304, 768, [&](GemmArgs& g) {
        g.A = A; g.C = C;
        return launch_gemm_k<EF16, _Float16, EPI_STORE, 128, 192, 2, 2, 4, 256, 0, false, 0>(g, 0); }, nt(128, 192, 2304)});

    GemmArgs gfc{A, W, Cfc, bias, nullptr, Afc, M, 3072, 768};
    gfc.kslice = 768;
    auto cfc = [&]() { return launch_gemm_k<EF16, _Float16, EPI_GELU, 256, 192, 2, 4, 2, 128, 0, false, 0>(gfc, 0); };
    unsigned long long* null = nullptr;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<unsigned long long> h(4096 * 8);
    for (auto& v : vars) {
        GemmArgs g{A, W, C, bias, nullptr, nullptr, M, v.N, v.K};
        g.kslice = v.K;
        // event time of the launch without stamps (after the c_fc product, as in the step)
        float ev = 0;
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_tl), &null, sizeof(null)));
        for (int i = 0; i < reps + 2; ++i) {
            cfc();
            CK(hipEventRecord(e0));
            if (v.fn(g)) { printf("%s: launch error\n", v.name.c_str()); return 1; }
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (i >= 2) ev += t / reps;
        }
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_tl), &tl, sizeof(tl)));
        std::vector<double> pro, kl, epi, drn, st, en, ghz;
        double span = 0;
        for (int i = 0; i < reps; ++i) {
            cfc();
            CK(hipMemset(tl, 0, 4096 * 8 * 8));
            v.fn(g);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h.data(), tl, h.size() * 8, hipMemcpyDeviceToHost));
            unsigned long long t0 = ~0ull, t4 = 0;
            for (int t = 0; t < v.ntiles; ++t) { t0 = std::min(t0, h[t * 8]); t4 = std::max(t4, h[t * 8 + 4]); }
            span += (t4 - t0) * 0.01 / reps;
            for (int t = 0; t < v.ntiles; ++t) {
                const unsigned long long* p = &h[t * 8];
                st.push_back((p[0] - t0) * 0.01);
                pro.push_back((p[1] - p[0]) * 0.01);
                kl.push_back((p[2] - p[1]) * 0.01);
                epi.push_back((p[3] - p[2]) * 0.01);
                drn.push_back((p[4] - p[3]) * 0.01);
                en.push_back((p[4] - t0) * 0.01);
                if (p[4] > p[0]) ghz.push_back((double)(p[6] - p[5]) / ((p[4] - p[0]) * 10.0));   // cycles / ns
            }
        }
        printf("%-22s tiles %4d  event %6.2f us  stamped span %6.2f us  clock %.2f GHz\n", v.name.c_str(), v.ntiles,
               ev * 1e3, span, pct(ghz, 0.5));
        auto row = [](const char* n, const std::vector<double>& x) {
            printf("    %-10s p10 %6.2f  p50 %6.2f  p90 %6.2f  max %6.2f us\n", n, pct(x, 0.1), pct(x, 0.5), pct(x, 0.9), pct(x, 1.0));
        };
        row("start", st); row("prologue", pro); row("k-loop", kl); row("epilogue", epi); row("drain", drn); row("end", en);
    }
    // one stamped launch per variant: the per-tile table (tile, xcc, cu, phases relative to the launch's first entry)
    if (argc > 2) {
        for (auto& v : vars) {
            GemmArgs g{A, W, C, bias, nullptr, nullptr, M, v.N, v.K};
            g.kslice = v.K;
            cfc();
            CK(hipMemset(tl, 0, 4096 * 8 * 8));
            v.fn(g);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h.data(), tl, h.size() * 8, hipMemcpyDeviceToHost));
            unsigned long long t0 = ~0ull;
            for (int t = 0; t < v.ntiles; ++t) t0 = std::min(t0, h[t * 8]);
            printf("# %s: tile xcc cu start first_tile kloop_end epi_end drain_end (us)\n", v.name.c_str());
            for (int t = 0; t < v.ntiles; ++t) {
                const unsigned long long* p = &h[t * 8];
                const unsigned hw = (unsigned)p[7];
                printf("%d %u %u %.2f %.2f %.2f %.2f %.2f\n", t, (unsigned)(p[7] >> 32), (hw >> 8) & 15, (p[0] - t0) * 0.01,
                       (p[1] - t0) * 0.01, (p[2] - t0) * 0.01, (p[3] - t0) * 0.01, (p[4] - t0) * 0.01);
            }
        }
    }
    return 0;
}
