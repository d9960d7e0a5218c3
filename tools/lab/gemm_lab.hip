// GEMM variant lab (experiment harness, not product code): times gemm.hip's kernel templates directly at the
// ViT-B/16 16-crop shapes (M = 16 x 229), interleaved rounds in one process (cdna_hip_programming.md §5.4 rule
// 24), outputs of every variant compared bitwise with the first variant of its shape.
//   build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1 -DEBC_GEMM_LAB \
//          tools/lab/gemm_lab.hip -o tools/lab/bin/gemm_lab
//   run:   gemm_lab [rounds] [reps]
#include "../../clip-ebc_amd/csrc/gemm.hip"

#include <cmath>
#include <cstdio>
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

// read a buffer once (16 B a lane) so its lines are on-die (Infinity Cache) when the next kernel needs them
__global__ __launch_bounds__(256) void touch_kernel(const uint4* __restrict__ p, size_t n16, unsigned* sink)
{
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.w;
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

template <class T> T* dalloc(size_t n) { T* p; CK(hipMalloc(&p, n * sizeof(T))); return p; }

struct Variant { std::string name; std::function<int(const GemmArgs&)> fn; };

using std::string;
template <class TO, int EPI, int S, int NLW>
Variant v128x96(const char* nm) {
    return {nm, [](const GemmArgs& g) { return launch_gemm_k<EF16, TO, EPI, 128, 96, S, 2, 2, 128, 0, false, NLW>(g, 0); }};
}

// split-K over `splits` workgroups per tile with the in-kernel last-arriver sum (gemm_nt_kernel SPL path); the
// counters + partials live in one workspace (counters zero on entry, re-armed by the kernel)
static void* g_splitws = nullptr;
constexpr size_t LAB_CNT_BYTES = 16 * 1024;
template <class TO, int EPI, int BM, int BN, int S, int WGM, int WGN>
Variant vsplit(const char* nm, int splits) {
    return {nm, [splits](const GemmArgs& g0) {
        GemmArgs g = g0;
        g.splits = splits;
        g.kslice = g.K / splits;
        g.cnt = reinterpret_cast<int*>(g_splitws);
        g.part = reinterpret_cast<float*>(reinterpret_cast<char*>(g_splitws) + LAB_CNT_BYTES);
        return launch_gemm_k<EF16, TO, EPI, BM, BN, S, WGM, WGN, 128, 0, true, 0>(g, 0);
    }};
}

int main(int argc, char** argv)
{
    const int rounds = argc > 1 ? atoi(argv[1]) : 3, reps = argc > 2 ? atoi(argv[2]) : 30;
    const int M = 16 * 229;
    _Float16* A = dalloc<_Float16>((size_t)M * 3072);
    _Float16* W = dalloc<_Float16>((size_t)3072 * 3072);
    _Float16* Cfc = dalloc<_Float16>((size_t)M * 3072);
    _Float16* Afc = dalloc<_Float16>((size_t)M * 3072);
    float* R = dalloc<float>((size_t)M * 768);
    float* bias = dalloc<float>(3072);
    void* C0 = dalloc<float>((size_t)M * 3072);
    void* C1 = dalloc<float>((size_t)M * 3072);
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, A, (size_t)M * 3072, 1u, 1.0f);
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, W, (size_t)3072 * 3072, 2u, 0.03f);
    hipLaunchKernelGGL(fill_f32, dim3(1024), dim3(256), 0, 0, R, (size_t)M * 768, 3u);
    hipLaunchKernelGGL(fill_f32, dim3(64), dim3(256), 0, 0, bias, (size_t)3072, 4u);
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, Cfc, (size_t)M * 3072, 5u, 1.0f);
    CK(hipDeviceSynchronize());

    struct Shape { const char* name; int N, K, epi; bool f32; std::vector<Variant> vars; };
    std::vector<Shape> shapes;
    shapes.push_back({"c_proj+res K3072", 768, 3072, EPI_RESID, true,
                      {v128x96<float, EPI_RESID, 3, 0>("128x96 S3 4w"), v128x96<float, EPI_RESID, 4, 4>("128x96 S4 4w+4L")}});
    shapes.push_back({"dH2 store K3072", 768, 3072, EPI_STORE, false,
                      {v128x96<_Float16, EPI_STORE, 3, 0>("128x96 S3 4w"), v128x96<_Float16, EPI_STORE, 4, 4>("128x96 S4 4w+4L")}});
    shapes.push_back({"out+res K768", 768, 768, EPI_RESID, true,
                      {v128x96<float, EPI_RESID, 3, 0>("128x96 S3 4w"), v128x96<float, EPI_RESID, 3, 4>("128x96 S3 4w+4L")}});
    // r03 split-K A/B: the in-kernel last-arriver sum at the N = 768 shapes
    CK(hipMalloc(&g_splitws, LAB_CNT_BYTES + ((size_t)64 << 20)));
    CK(hipMemset(g_splitws, 0, LAB_CNT_BYTES + ((size_t)64 << 20)));
    shapes.push_back({"split c_proj K3072", 768, 3072, EPI_RESID, true,
                      {v128x96<float, EPI_RESID, 4, 4>("128x96 S4 4w+4L"),
                       vsplit<float, EPI_RESID, 128, 192, 3, 2, 2>("128x192 S3 s2", 2),
                       vsplit<float, EPI_RESID, 128, 96, 2, 2, 2>("128x96 S2 s2", 2),
                       vsplit<float, EPI_RESID, 256, 192, 2, 4, 2>("256x192 S2 s4", 4),
                       vsplit<float, EPI_RESID, 256, 192, 2, 4, 2>("256x192 S2 s2", 2)}});
    shapes.push_back({"split out K768", 768, 768, EPI_RESID, true,
                      {v128x96<float, EPI_RESID, 3, 4>("128x96 S3 4w+4L"),
                       v128x96<float, EPI_RESID, 3, 0>("128x96 S3 4w"),
                       vsplit<float, EPI_RESID, 128, 96, 3, 2, 2>("128x96 S3 s1(SPL)", 1),
                       vsplit<float, EPI_RESID, 128, 192, 3, 2, 2>("128x192 S3 s2", 2),
                       vsplit<float, EPI_RESID, 128, 96, 2, 2, 2>("128x96 S2 s2", 2),
                       vsplit<float, EPI_RESID, 256, 192, 2, 4, 2>("256x192 S2 s4", 4)}});

    // in-step emulation: the c_fc + GELU product (writes 2 x 22.5 MB) runs right before each timed launch; the
    // K = 3072 products read its output as their A operand, as c_proj does in the step
    GemmArgs gfc{A, W, Cfc, bias, nullptr, Afc, M, 3072, 768};
    gfc.kslice = 768;
    auto cfc = [&]() { return launch_gemm_k<EF16, _Float16, EPI_GELU, 256, 192, 2, 4, 2, 128, 0, false, 0>(gfc, 0); };

    hipEvent_t e0, e1, e2;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&e2));
    for (auto& sh : shapes) {
        GemmArgs g{sh.K == 3072 ? (void*)Cfc : (void*)A, W, C0, bias, sh.epi == EPI_RESID ? R : nullptr, nullptr, M, sh.N, sh.K};
        g.kslice = sh.K;
        const size_t outb = (size_t)M * sh.N * (sh.f32 ? 4 : 2);
        // correctness: every variant bitwise equal to the first
        std::vector<char> ref(outb), got(outb);
        for (size_t v = 0; v < sh.vars.size(); ++v) {
            g.C = v == 0 ? C0 : C1;
            CK(hipMemset(g.C, 0, outb));
            if (sh.vars[v].fn(g)) { printf("%s %s: launch error\n", sh.name, sh.vars[v].name.c_str()); return 1; }
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(v == 0 ? ref.data() : got.data(), g.C, outb, hipMemcpyDeviceToHost));
            if (v > 0) {
                size_t bad = 0;
                for (size_t i = 0; i < outb; ++i) bad += ref[i] != got[i];
                double num = 0, den = 0;
                if (sh.f32) {
                    const float* a = reinterpret_cast<const float*>(ref.data());
                    const float* b = reinterpret_cast<const float*>(got.data());
                    for (size_t i = 0; i < outb / 4; ++i) { num += (double)(a[i] - b[i]) * (a[i] - b[i]); den += (double)a[i] * a[i]; }
                }
                printf("%-18s %-18s bitwise vs %s: %s (%zu bytes differ, rel-L2 %.2e)\n", sh.name, sh.vars[v].name.c_str(),
                       sh.vars[0].name.c_str(), bad ? "DIFFERENT" : "identical", bad, den > 0 ? sqrt(num / den) : 0.0);
            }
        }
        g.C = C1;
        const double tf = 2.0 * M * sh.N * sh.K / 1e12;
        for (int r = 0; r < rounds; ++r) {
            for (auto& v : sh.vars) {
                // alone: back-to-back launches
                for (int w = 0; w < 3; ++w) v.fn(g);
                CK(hipEventRecord(e0));
                for (int i = 0; i < reps; ++i) v.fn(g);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float alone = 0;
                CK(hipEventElapsedTime(&alone, e0, e1));
                alone /= reps;
                // after the c_fc product
                float inst = 0;
                for (int i = 0; i < reps; ++i) {
                    cfc();
                    CK(hipEventRecord(e0));
                    v.fn(g);
                    CK(hipEventRecord(e1));
                    CK(hipEventSynchronize(e1));
                    float t;
                    CK(hipEventElapsedTime(&t, e0, e1));
                    inst += t;
                }
                inst /= reps;
                printf("%s r%d %-18s %-18s alone %7.2f us (%6.1f TF/s)   after c_fc %7.2f us (%6.1f TF/s)\n", EBC_STORE_NT ? "nt" : "plain", r, sh.name,
                       v.name.c_str(), alone * 1e3, tf / (alone * 1e-3), inst * 1e3, tf / (inst * 1e-3));
            }
        }
    }
    // ---- the MLP pair as the step runs it: 12 layers, each with its own weights, c_fc output and residual, so
    // c_proj's operands are as cold as in the step; per variant of c_proj's tile order (group_m) and ring
    {
        const int NL = 12;
        std::vector<_Float16*> Wfc(NL), Wpr(NL), G(NL), Ax(NL);
        std::vector<float*> X1(NL), Xn(NL);
        for (int l = 0; l < NL; ++l) {
            Wfc[l] = dalloc<_Float16>((size_t)3072 * 768); Wpr[l] = dalloc<_Float16>((size_t)768 * 3072);
            G[l] = dalloc<_Float16>((size_t)M * 3072); Ax[l] = dalloc<_Float16>((size_t)M * 3072);
            X1[l] = dalloc<float>((size_t)M * 768); Xn[l] = dalloc<float>((size_t)M * 768);
            hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, Wfc[l], (size_t)3072 * 768, 100u + l, 0.03f);
            hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, Wpr[l], (size_t)3072 * 768, 200u + l, 0.02f);
            hipLaunchKernelGGL(fill_f32, dim3(1024), dim3(256), 0, 0, X1[l], (size_t)M * 768, 300u + l);
        }
        CK(hipDeviceSynchronize());
        struct PV { const char* name; int gm; std::function<int(const GemmArgs&)> fn; int share = 0; int pf = 0; };
        hipStream_t side;
        CK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
        hipEvent_t fork;
        CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
        unsigned* sink;
        CK(hipMalloc(&sink, 64));
        // share: 1 = every layer uses layer 0's c_proj weight (warm W), 2 = layer 0's residual (warm X1), 4 = both
        auto S4L = [](const GemmArgs& g) { return launch_gemm_k<EF16, float, EPI_RESID, 128, 96, 4, 2, 2, 128, 0, false, 4>(g, 0); };
        std::vector<PV> pv = {
            {"S4+4L warm W", 0, S4L, 1},
            {"S4+4L warm X1", 0, S4L, 2},
            {"S4+4L warm W+X1", 0, S4L, 3},
            {"S4+4L touch W (side, 64 WG)", 0, S4L, 0, 64},
            {"S4+4L touch W (side, 256 WG)", 0, S4L, 0, 256},
            {"S4+4L rowmajor", 0, [](const GemmArgs& g) { return launch_gemm_k<EF16, float, EPI_RESID, 128, 96, 4, 2, 2, 128, 0, false, 4>(g, 0); }},
            {"S4+4L group_m 3", 3, [](const GemmArgs& g) { return launch_gemm_k<EF16, float, EPI_RESID, 128, 96, 4, 2, 2, 128, 0, false, 4>(g, 0); }},
            {"S4+4L group_m 5", 5, [](const GemmArgs& g) { return launch_gemm_k<EF16, float, EPI_RESID, 128, 96, 4, 2, 2, 128, 0, false, 4>(g, 0); }},
            {"S4+4L group_m 8", 8, [](const GemmArgs& g) { return launch_gemm_k<EF16, float, EPI_RESID, 128, 96, 4, 2, 2, 128, 0, false, 4>(g, 0); }},
            {"S3 4w rowmajor", 0, [](const GemmArgs& g) { return launch_gemm_k<EF16, float, EPI_RESID, 128, 96, 3, 2, 2, 128, 0, false, 0>(g, 0); }},
        };
        std::vector<hipEvent_t> ev(2 * NL);
        for (auto& evx : ev) CK(hipEventCreate(&evx));
        for (int r = 0; r < rounds; ++r)
            for (auto& v : pv) {
                float tot = 0, fc = 0;
                for (int it = 0; it < 3; ++it)
                    for (int l = 0; l < NL; ++l) {
                        GemmArgs a{A, Wfc[l], G[l], bias, nullptr, Ax[l], M, 3072, 768};
                        a.kslice = 768;
                        GemmArgs b{G[l], Wpr[(v.share & 1) ? 0 : l], Xn[l], bias, X1[(v.share & 2) ? 0 : l], nullptr, M, 768, 3072};
                        b.kslice = 3072;
                        b.group_m = v.gm;
                        if (v.pf) {                     // prefetch c_proj's weight on a side stream beside c_fc
                            CK(hipEventRecord(fork, 0));
                            CK(hipStreamWaitEvent(side, fork, 0));
                            hipLaunchKernelGGL(touch_kernel, dim3(v.pf), dim3(256), 0, side,
                                               reinterpret_cast<const uint4*>(Wpr[l]), (size_t)768 * 3072 * 2 / 16, sink);
                        }
                        CK(hipEventRecord(ev[2 * l]));
                        launch_gemm_k<EF16, _Float16, EPI_GELU, 256, 192, 2, 4, 2, 128, 0, false, 0>(a, 0);
                        CK(hipEventRecord(ev[2 * l + 1]));
                        v.fn(b);
                        CK(hipEventRecord(e2));
                        CK(hipEventSynchronize(e2));
                        float t1 = 0, t2 = 0;
                        CK(hipEventElapsedTime(&t1, ev[2 * l], ev[2 * l + 1]));
                        CK(hipEventElapsedTime(&t2, ev[2 * l + 1], e2));
                        if (it > 0) { fc += t1; tot += t2; }
                    }
                printf("%s r%d mlp-seq c_proj %-16s %7.2f us   (c_fc %7.2f us)\n", EBC_STORE_NT ? "nt" : "plain", r, v.name,
                       tot / (2 * NL) * 1e3, fc / (2 * NL) * 1e3);
            }
    }
    for (int r = 0; r < rounds; ++r) {
        for (int w = 0; w < 3; ++w) cfc();
        CK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) cfc();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float t = 0;
        CK(hipEventElapsedTime(&t, e0, e1));
        printf("%s r%d c_fc+gelu 256x192 alone %7.2f us\n", EBC_STORE_NT ? "nt" : "plain", r, t / reps * 1e3);
    }
    return 0;
}
