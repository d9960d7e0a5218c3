// Decoder 3x3-conv lab (experiment harness, not product code), 16-crop decoder shape (B 16, 28 x 28, C = N = 768):
//   mode 1  the implicit-GEMM conv (M = 12544, N = 768, K = 9 x 768) by tile: 256x192 (196 tiles = 77 % of the 256
//           CUs), 224x192 (224 tiles, 88 %), 160x256 (237 tiles, 93 %); store and BN-statistics epilogues
//   mode 2  the weight gradient over the interior pixels (K = 16 x 784 = 12544) by tile and split
//   sk      stream-K: 256 workgroups share all tiles' k-tiles (gemm.hip sk_plan)
// Interleaved rounds in one process; every variant compared with the first one of its mode.
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

struct V { std::string name; int mode; size_t outn; std::function<void(void*)> fn; double flop; };

int main(int argc, char** argv)
{
    const int rounds = argc > 1 ? atoi(argv[1]) : 3, reps = argc > 2 ? atoi(argv[2]) : 10;
    const int B = argc > 3 ? atoi(argv[3]) : 16, H = 28, W = 28, C = 768, N = 768;      // crops (16 or 32)
    const int Hp = H + 2, Wp = 32, HWp = H * W, M1 = B * H * W;
    const long Q = (long)B * Hp * Wp, Kq = (long)B * HWp, Pimg = (long)(H + 2) * W;
    const long Qs = ((std::max(Kq, (long)(B + 2) * Pimg + HWp + 2L * W + 64) + 63) / 64) * 64;
    _Float16 *xpad, *wk, *dzT, *xT3, *z;
    float *dw, *stats;
    CK(hipMalloc(&xpad, (size_t)Q * C * 2));
    CK(hipMalloc(&wk, (size_t)N * 9 * C * 2));
    CK(hipMalloc(&z, (size_t)2 * M1 * N * 2));
    CK(hipMalloc(&dzT, (size_t)N * Qs * 2));
    CK(hipMalloc(&xT3, (size_t)3 * C * Qs * 2));
    CK(hipMalloc(&dw, (size_t)2 * N * 9 * C * 4));
    char* ws;
    const size_t wsb = GEMM_CNT_BYTES + std::max((size_t)8 * N * 9 * C * 4, (size_t)2 * 256 * 256 * 192 * 4);
    CK(hipMalloc(&ws, wsb));
    CK(hipMemset(ws, 0, wsb));
    CK(hipMalloc(&stats, (size_t)128 * 2 * N * 4));
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, xpad, (size_t)Q * C, 11u, 1.0f);
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, wk, (size_t)N * 9 * C, 12u, 0.05f);
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, dzT, (size_t)N * Qs, 13u, 1.0f);
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, xT3, (size_t)3 * C * Qs, 14u, 1.0f);
    CK(hipDeviceSynchronize());

    auto sk_args = [&](GemmArgs& g, int tiles, int nk) {
        g.sk_total = (long)tiles * nk; g.sk_nk = nk; g.sk_grid = 256;
        g.cnt = reinterpret_cast<int*>(ws);
        g.part = reinterpret_cast<float*>(ws + GEMM_CNT_BYTES);
    };
    auto conv = [&](auto tl, int epi, bool sk = false) {
        using TT = decltype(tl);
        return [&, epi, sk](void* out) {
            GemmArgs g{xpad, wk, out, nullptr, nullptr, nullptr, M1, N, 9 * C};
            g.cH = H; g.cW = W; g.cC = C; g.cHp = Hp; g.cWp = Wp;
            g.splits = 1; g.kslice = 9 * C; g.stats = stats;
            const int T = ((M1 + TT::BM - 1) / TT::BM) * (N / TT::BN), dp = T / 256 * 256;
            if (sk && dp) {           // whole waves as a plain launch first (gemm.hip sk_plan)
                GemmArgs d = g;
                d.ntile = dp;
                const int rc = epi == EPI_STATS
                    ? launch_gemm_k<EF16, _Float16, EPI_STATS, TT::BM, TT::BN, TT::S, TT::WGM, TT::WGN, 128, 1, false>(d, 0)
                    : launch_gemm_k<EF16, _Float16, EPI_STORE, TT::BM, TT::BN, TT::S, TT::WGM, TT::WGN, 128, 1, false>(d, 0);
                if (rc) { printf("launch rc %d\n", rc); exit(1); }
                g.tile0 = dp;
            }
            if (sk) sk_args(g, T - dp, 9 * C / 64);
            const int rc = sk
                ? (epi == EPI_STATS
                   ? launch_gemm_k<EF16, _Float16, EPI_STATS, TT::BM, TT::BN, TT::S, TT::WGM, TT::WGN, 128, 1, true>(g, 0)
                   : launch_gemm_k<EF16, _Float16, EPI_STORE, TT::BM, TT::BN, TT::S, TT::WGM, TT::WGN, 128, 1, true>(g, 0))
                : epi == EPI_STATS
                ? launch_gemm_k<EF16, _Float16, EPI_STATS, TT::BM, TT::BN, TT::S, TT::WGM, TT::WGN, 128, 1, false>(g, 0)
                : launch_gemm_k<EF16, _Float16, EPI_STORE, TT::BM, TT::BN, TT::S, TT::WGM, TT::WGN, 128, 1, false>(g, 0);
            if (rc) { printf("launch rc %d\n", rc); exit(1); }
        };
    };
    auto wgrad = [&](auto tl, int splits) {
        using TT = decltype(tl);
        return [&, splits](void* out) {
            GemmArgs g{dzT, xT3, out, nullptr, nullptr, nullptr, N, 9 * C, (int)Kq};
            g.cH = H; g.cW = W; g.cC = C; g.cHp = Hp; g.cWp = Wp;
            g.cHWp = HWp; g.cQs = Qs; g.cPimg = Pimg;
            g.splits = splits > 0 ? splits : 1; g.kslice = (int)Kq / g.splits;
            g.cnt = splits > 1 ? reinterpret_cast<int*>(ws) : nullptr;
            g.part = splits > 1 ? reinterpret_cast<float*>(ws + GEMM_CNT_BYTES) : nullptr;
            if (splits == 0) sk_args(g, (N / TT::BM) * (9 * C / TT::BN), (int)Kq / 64);     // stream-K
            const int rc = splits != 1
                ? launch_gemm_k<EF16, float, EPI_STORE, TT::BM, TT::BN, TT::S, TT::WGM, TT::WGN, 128, 2, true>(g, 0)
                : launch_gemm_k<EF16, float, EPI_STORE, TT::BM, TT::BN, TT::S, TT::WGM, TT::WGN, 128, 2, false>(g, 0);
            if (rc) { printf("launch rc %d\n", rc); exit(1); }
        };
    };
    const double f1 = 2.0 * M1 * N * 9.0 * C, f2 = 2.0 * N * 9.0 * C * (double)(B * H * W);
    const size_t n1 = (size_t)M1 * N, n2 = (size_t)N * 9 * C;
    std::vector<V> vars = {
        {"conv 256x192 store", 1, n1, conv(Tl<256, 192, 2, 4, 2>{}, EPI_STORE), f1},
        {"conv 256x192 store sk", 1, n1, conv(Tl<256, 192, 2, 4, 2>{}, EPI_STORE, true), f1},
        {"conv 224x192 store", 1, n1, conv(Tl<224, 192, 2, 2, 4>{}, EPI_STORE), f1},
        {"conv 256x192 stats", 1, n1, conv(Tl<256, 192, 2, 4, 2>{}, EPI_STATS), f1},
        {"conv 256x192 stats sk", 1, n1, conv(Tl<256, 192, 2, 4, 2>{}, EPI_STATS, true), f1},
        {"wgrad 256x192 s2", 2, n2, wgrad(Tl<256, 192, 2, 4, 2>{}, 2), f2},
        {"wgrad 256x192 sk", 2, n2, wgrad(Tl<256, 192, 2, 4, 2>{}, 0), f2},
    };
    std::vector<float> ref, got;
    std::vector<_Float16> refh, goth;
    for (size_t v = 0; v < vars.size(); ++v) {
        const bool first = v == 0 || vars[v].mode != vars[v - 1].mode;
        void* o = vars[v].mode == 1 ? (void*)(z + (first ? 0 : n1)) : (void*)(dw + (first ? 0 : n2));
        vars[v].fn(o);
        CK(hipDeviceSynchronize());
        double num = 0, den = 0;
        if (vars[v].mode == 1) {
            (first ? refh : goth).resize(n1);
            CK(hipMemcpy(first ? refh.data() : goth.data(), o, n1 * 2, hipMemcpyDeviceToHost));
            if (!first) for (size_t i = 0; i < n1; ++i) { const double d = (double)goth[i] - (double)refh[i]; num += d * d; den += (double)refh[i] * refh[i]; }
        } else {
            (first ? ref : got).resize(n2);
            CK(hipMemcpy(first ? ref.data() : got.data(), o, n2 * 4, hipMemcpyDeviceToHost));
            if (!first) for (size_t i = 0; i < n2; ++i) { const double d = (double)got[i] - ref[i]; num += d * d; den += (double)ref[i] * ref[i]; }
        }
        if (!first) printf("%-24s rel-L2 vs %s: %.2e\n", vars[v].name.c_str(), vars[v].mode == 1 ? "256x192 store" : "256x192 s2",
                           std::sqrt(num / den));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; ++r)
        for (auto& v : vars) {
            void* o = v.mode == 1 ? (void*)(z + n1) : (void*)(dw + n2);
            v.fn(o);
            CK(hipEventRecord(e0));
            for (int i = 0; i < reps; ++i) v.fn(o);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("r%d %-24s %8.2f us  %7.1f TF/s\n", r, v.name.c_str(), ms / reps * 1e3, v.flop / 1e12 / (ms / reps * 1e-3));
        }
    return 0;
}
