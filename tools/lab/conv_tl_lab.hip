// Decoder conv timeline lab (experiment harness, not product code): per-workgroup phase stamps (tools/lab/gemm_tl_lab.hip's
// hook) of the product's 3x3-conv launches at the 16-crop decoder shape (B 16, 28 x 28, C = N = 768) through gemm.hip's own
// dispatch (ebc::conv_gemm: tile, stream-K plan and split exactly as the step runs them): the forward with BN statistics,
// the data gradient, and the weight gradient.  A stream-K workgroup's two segments are stamped separately.
//   build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1 tools/lab/conv_tl_lab.hip \
//          -o tools/lab/bin/conv_tl_lab
//   run:   conv_tl_lab [reps] [crops]
#include <hip/hip_runtime.h>

__device__ unsigned long long* g_tl = nullptr;          // [2 * workgroup + segment][8]
__device__ __forceinline__ void tl_stamp(int phase, int /*tile*/)
{
    __shared__ int seg;
    if (threadIdx.x != 0 || g_tl == nullptr) return;
    if (phase == 0) seg = g_tl[(size_t)blockIdx.x * 16] != 0;
    unsigned long long* p = g_tl + ((size_t)blockIdx.x * 2 + seg) * 8;
    if (phase == 3) {
        p[3] = __builtin_amdgcn_s_memrealtime();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        p[4] = __builtin_amdgcn_s_memrealtime();
        p[6] = __builtin_amdgcn_s_memtime();
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
static double pct(std::vector<double> v, double q)
{
    if (v.empty()) return 0;
    std::sort(v.begin(), v.end());
    return v[std::min(v.size() - 1, (size_t)(q * (v.size() - 1) + 0.5))];
}

int main(int argc, char** argv)
{
    const int reps = argc > 1 ? atoi(argv[1]) : 5, B = argc > 2 ? atoi(argv[2]) : 16;
    const int H = 28, W = 28, C = 768, N = 768;
    const int Hp = H + 2, Wp = 32, HWp = H * W, M1 = B * H * W;
    const long Q = (long)B * Hp * Wp, Kq = (long)B * HWp, Pimg = (long)(H + 2) * W;
    const long Qs = ((std::max(Kq, (long)(B + 2) * Pimg + HWp + 2L * W + 64) + 63) / 64) * 64;
    _Float16 *xpad, *wk, *dzT, *xT3, *z, *gy, *y;
    float* dw;
    CK(hipMalloc(&xpad, (size_t)Q * C * 2));
    CK(hipMalloc(&wk, (size_t)N * 9 * C * 2));
    CK(hipMalloc(&z, (size_t)M1 * N * 2));
    CK(hipMalloc(&gy, (size_t)M1 * N * 2));
    CK(hipMalloc(&y, (size_t)M1 * N * 2));
    CK(hipMalloc(&dzT, (size_t)N * Qs * 2));
    CK(hipMalloc(&xT3, (size_t)3 * C * Qs * 2));
    CK(hipMalloc(&dw, (size_t)N * 9 * C * 4));
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, xpad, (size_t)Q * C, 11u, 1.0f);
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, wk, (size_t)N * 9 * C, 12u, 0.05f);
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, dzT, (size_t)N * Qs, 13u, 1.0f);
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, xT3, (size_t)3 * C * Qs, 14u, 1.0f);
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, gy, (size_t)M1 * N, 15u, 1.0f);
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, y, (size_t)M1 * N, 16u, 1.0f);
    ebc::ConvGeom g1{H, W, C, Hp, Wp, HWp, Qs, Pimg, B};
    size_t wsb = std::max({ebc::conv_gemm_workspace_bytes(EBC_F16, 1, M1, N, 9 * C),
                           ebc::conv_gemm_workspace_bytes(EBC_F16, 2, N, 9 * C, (int)Kq)});
    char* ws;
    CK(hipMalloc(&ws, wsb));
    CK(hipMemset(ws, 0, wsb));
    unsigned long long* tl;
    const int SLOTS = 2 * 4096;
    CK(hipMalloc(&tl, (size_t)SLOTS * 8 * 8));
    CK(hipDeviceSynchronize());

    struct Var { std::string name; std::function<int()> fn; double flop; };
    int tiles = 0;
    std::vector<Var> vars = {
        {"conv fwd + BN stats", [&] { return ebc::conv_gemm(EBC_F16, 1, 4, xpad, wk, z, g1, M1, N, 9 * C, ws, wsb, &tiles, 0, nullptr, nullptr); },
         2.0 * M1 * N * 9.0 * C},
        {"conv dgrad + relu grad", [&] { return ebc::conv_gemm(EBC_F16, 1, 5, xpad, wk, z, g1, M1, N, 9 * C, ws, wsb, nullptr, 0, gy, y); },
         2.0 * M1 * N * 9.0 * C},
        {"conv dgrad store", [&] { return ebc::conv_gemm(EBC_F16, 1, 0, xpad, wk, z, g1, M1, N, 9 * C, ws, wsb, nullptr, 0, nullptr, nullptr); },
         2.0 * M1 * N * 9.0 * C},
        {"conv wgrad", [&] { return ebc::conv_gemm(EBC_F16, 2, 0, dzT, xT3, dw, g1, N, 9 * C, (int)Kq, ws, wsb, nullptr, 0, nullptr, nullptr); },
         2.0 * N * 9.0 * C * (double)Kq},
    };
    unsigned long long* null = nullptr;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<unsigned long long> h((size_t)SLOTS * 8);
    for (auto& v : vars) {
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_tl), &null, sizeof(null)));
        float ev = 0;
        for (int i = 0; i < reps + 2; ++i) {
            CK(hipEventRecord(e0));
            if (v.fn()) { printf("%s: launch error\n", v.name.c_str()); return 1; }
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (i >= 2) ev += t / reps;
        }
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_tl), &tl, sizeof(tl)));
        std::vector<double> st, pro, kl, epi, drn, en, ghz;
        double span = 0;
        int segs = 0;
        for (int i = 0; i < reps; ++i) {
            CK(hipMemset(tl, 0, (size_t)SLOTS * 8 * 8));
            v.fn();
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h.data(), tl, h.size() * 8, hipMemcpyDeviceToHost));
            unsigned long long t0 = ~0ull, t4 = 0;
            for (int s = 0; s < SLOTS; ++s) if (h[s * 8]) { t0 = std::min(t0, h[s * 8]); t4 = std::max(t4, h[s * 8 + 4]); }
            span += (t4 - t0) * 0.01 / reps;
            segs = 0;
            for (int s = 0; s < SLOTS; ++s) {
                const unsigned long long* p = &h[(size_t)s * 8];
                if (!p[0] || !p[4]) continue;
                ++segs;
                st.push_back((p[0] - t0) * 0.01);
                pro.push_back((p[1] - p[0]) * 0.01);
                kl.push_back((p[2] - p[1]) * 0.01);
                epi.push_back((p[3] - p[2]) * 0.01);
                drn.push_back((p[4] - p[3]) * 0.01);
                en.push_back((p[4] - t0) * 0.01);
                if (p[4] > p[0]) ghz.push_back((double)(p[6] - p[5]) / ((p[4] - p[0]) * 10.0));
            }
        }
        printf("%-24s segments %4d  event %7.2f us (%6.1f TF/s)  stamped span %7.2f us  clock %.2f GHz\n", v.name.c_str(), segs,
               ev * 1e3, v.flop / 1e12 / (ev * 1e-3), span, pct(ghz, 0.5));
        auto row = [](const char* n, const std::vector<double>& x) {
            printf("    %-10s p10 %7.2f  p50 %7.2f  p90 %7.2f  max %7.2f us\n", n, pct(x, 0.1), pct(x, 0.5), pct(x, 0.9), pct(x, 1.0));
        };
        row("start", st); row("prologue", pro); row("k-loop", kl); row("epilogue", epi); row("drain", drn); row("end", en);
    }
    return 0;
}
