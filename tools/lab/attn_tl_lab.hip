// Attention timeline lab (experiment harness, not product code): per-workgroup phase stamps of the product's attention
// forward and one-workgroup backward at the ViT-B/16 + VPT(32) shape (L 229, 12 heads, B crops) through attention.hip's
// own dispatch: entry (0), operands staged in LDS after the barrier (1), each wave's end (2).  Per launch: HIP-event time,
// the stamped span (first entry to last wave end), and percentiles of the start skew, the staging phase (1 - 0) and the
// compute phase (last wave end - 1).  No weight touch (touch = none), so the phases are the kernel's own.
//   build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/lab/attn_tl_lab.hip -o tools/lab/bin/attn_tl_lab
//   run:   attn_tl_lab [reps] [crops]
#include <hip/hip_runtime.h>

__device__ unsigned long long* g_atl = nullptr;        // [workgroup][18]: 0 entry, 1 staged, 2 + w wave w's end
__device__ __forceinline__ void atl_stamp(int phase)
{
    if (g_atl == nullptr || (threadIdx.x & 63) != 0) return;
    unsigned long long* p = g_atl + (size_t)(blockIdx.x + gridDim.x * blockIdx.y) * 18;
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    if (phase < 2) { if (threadIdx.x == 0) p[phase] = t; }
    else p[2 + (threadIdx.x >> 6)] = t;
}
#define EBC_ATTN_STAMP(phase) atl_stamp(phase)

#include "../../clip-ebc_amd/csrc/attention.hip"

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

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

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
    const int L = 229, H = 12, D = H * 64, D3 = 3 * D;
    _Float16 *qkv, *out, *dout, *dqkv;
    float *lse, *delta;
    CK(hipMalloc(&qkv, (size_t)B * L * D3 * 2));
    CK(hipMalloc(&out, (size_t)B * L * D * 2));
    CK(hipMalloc(&dout, (size_t)B * L * D * 2));
    CK(hipMalloc(&dqkv, (size_t)B * L * D3 * 2));
    CK(hipMalloc(&lse, (size_t)B * H * L * 4));
    CK(hipMalloc(&delta, (size_t)B * H * L * 4));
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, qkv, (size_t)B * L * D3, 11u, 1.5f);
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, dout, (size_t)B * L * D, 12u, 1.0f);
    CK(hipDeviceSynchronize());
    const int SLOTS = 4096;
    unsigned long long* tl;
    CK(hipMalloc(&tl, (size_t)SLOTS * 18 * 8));
    struct Var { std::string name; std::function<int()> fn; };
    std::vector<Var> vars = {
        {"attn fwd", [&] { return ebc::attention_fwd(EBC_F16, qkv, out, lse, B, L, H, 0, nullptr); }},
        {"attn bwd (one workgroup)", [&] { return ebc::attention_bwd(EBC_F16, qkv, dout, out, lse, delta, dqkv, B, L, H, 0, 0, nullptr); }},
    };
    unsigned long long* null = nullptr;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<unsigned long long> h((size_t)SLOTS * 18);
    for (auto& v : vars) {
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_atl), &null, sizeof(null)));
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
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_atl), &tl, sizeof(tl)));
        std::vector<double> st, stage, comp, wend;
        double span = 0;
        int wgs = 0;
        for (int i = 0; i < reps; ++i) {
            CK(hipMemset(tl, 0, (size_t)SLOTS * 18 * 8));
            v.fn();
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h.data(), tl, h.size() * 8, hipMemcpyDeviceToHost));
            unsigned long long t0 = ~0ull, tend = 0;
            for (int s = 0; s < SLOTS; ++s) if (h[(size_t)s * 18]) t0 = std::min(t0, h[(size_t)s * 18]);
            wgs = 0;
            for (int s = 0; s < SLOTS; ++s) {
                const unsigned long long* p = &h[(size_t)s * 18];
                if (!p[0]) continue;
                ++wgs;
                unsigned long long last = 0;
                for (int w = 0; w < 16; ++w) last = std::max(last, p[2 + w]);
                tend = std::max(tend, last);
                st.push_back((p[0] - t0) * 0.01);
                stage.push_back((p[1] - p[0]) * 0.01);
                comp.push_back((last - p[1]) * 0.01);
                wend.push_back((last - t0) * 0.01);
            }
            span += (tend - t0) * 0.01 / reps;
        }
        printf("%-26s B %2d  workgroups %4d  event %7.2f us  stamped span %7.2f us\n", v.name.c_str(), B, wgs, ev * 1e3, span);
        auto line = [&](const char* nm, const std::vector<double>& x) {
            printf("    %-10s p10 %7.2f  p50 %7.2f  p90 %7.2f  max %7.2f us\n", nm, pct(x, 0.1), pct(x, 0.5), pct(x, 0.9), pct(x, 1.0));
        };
        line("start", st);
        line("staging", stage);
        line("compute", comp);
        line("end", wend);
    }
    return 0;
}
