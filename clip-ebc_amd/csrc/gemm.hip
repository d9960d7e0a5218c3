// MFMA GEMM with fused epilogues for the CLIP ViT-B/16 encoder (gfx950).
//
//   C[M,N] = A[M,K] . B[N,K]^T      (both operands K-contiguous: nn.Linear weight layout)
//
// Reference ops replaced (models/clip/_clip/blocks.py:22-42 via nn.MultiheadAttention /
// nn.Linear, models/clip/_clip/image_encoder.py:141 conv1 as im2col-GEMM, models/clip/model.py:91-95
// projection):  QKV in-proj (+bias), out-proj (+bias +residual), MLP c_fc (+bias, QuickGELU),
// c_proj (+bias +residual), and their dX-only backward products (GELU' fused).
//
// Structure: 256 threads = 4 waves (2x2), wave tile (BM/2)x(BN/2) of 16x16 MFMA sub-tiles, a
// 128-byte K slab per stage (BK = 64 for 16-bit, 32 for f32) staged global->LDS by
// global_load_lds_dwordx4 (LDS-DMA), double-buffered, XOR-swizzled on the source address so the
// ds_read_b128 fragment reads are bank-conflict free; XCD-aware bijective tile remap.
// The MFMA is issued "swapped" (weights as the A operand) so each lane ends with 4 consecutive
// output columns of one row: vector epilogue loads/stores.
#include "ebc_common.h"
#include "mfma.h"

using namespace ebc;

namespace {

enum { EPI_STORE = 0, EPI_GELU = 1, EPI_RESID = 2, EPI_GELU_BWD = 3 };

struct GemmArgs {
    const void* A; const void* B; void* C;
    const float* bias;      // [N] or null
    const float* resid;     // [M,N] f32 (EPI_RESID), may alias C
    void* aux;              // [M,N] element type: GELU pre-activation (written by EPI_GELU, read by EPI_GELU_BWD)
    int M, N, K;
};

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ float quick_gelu(float a) { return a / (1.0f + expf(-1.702f * a)); }
__device__ __forceinline__ float quick_gelu_grad(float a) {
    const float s = 1.0f / (1.0f + expf(-1.702f * a));
    return s + 1.702f * a * s * (1.0f - s);
}

template <class TO> __device__ __forceinline__ void store4(TO* p, const float* v);
template <> __device__ __forceinline__ void store4<float>(float* p, const float* v) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
template <> __device__ __forceinline__ void store4<_Float16>(_Float16* p, const float* v) {
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    h4 r = {(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]};
    *reinterpret_cast<h4*>(p) = r;
}
template <> __device__ __forceinline__ void store4<__bf16>(__bf16* p, const float* v) {
    typedef __bf16 b4 __attribute__((ext_vector_type(4)));
    b4 r = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
    *reinterpret_cast<b4*>(p) = r;
}
template <class T> __device__ __forceinline__ void load4(const T* p, float* v) {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (float)p[i];
}
template <> __device__ __forceinline__ void load4<float>(const float* p, float* v) {
    const float4 x = *reinterpret_cast<const float4*>(p);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
}

template <class E, class TO, int EPI, int BM, int BN>
__global__ __launch_bounds__(256) void gemm_nt_kernel(GemmArgs g)
{
    using T = typename E::T;
    constexpr int EB = E::BYTES;
    constexpr int BK = 128 / EB;                 // elements per 128-B slab row
    constexpr int WM = BM / 2, WN = BN / 2;
    constexpr int TM = WM / 16, TN = WN / 16;
    constexpr int ROWS = BM + BN;                // slab rows per stage (A rows then B rows)
    constexpr int STAGE = ROWS * 128;            // bytes
    constexpr int NLD = ROWS / 32;               // glds wave-instructions per wave per stage
    static_assert(ROWS % 32 == 0, "stage rows");

    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int ntn = g.N / BN, ntm = (g.M + BM - 1) / BM;
    const int wg = xcd_remap(blockIdx.x, ntm * ntn);
    const int tm = wg / ntn, tn = wg % ntn;
    const int m0 = tm * BM, n0 = tn * BN;

    const T* A = reinterpret_cast<const T*>(g.A);
    const T* Bw = reinterpret_cast<const T*>(g.B);
    const int K = g.K, nk = K / BK;

    // per-lane source rows for the LDS-DMA staging (fixed across k)
    const T* src[NLD];
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
        const int row = (wave * NLD + i) * 8 + (lane >> 3);
        const int slot = lane & 7;
        const int c = slot ^ swz(row);
        const T* base;
        if (row < BM) {
            int gr = m0 + row;
            gr = gr < g.M ? gr : g.M - 1;           // clamp: rows >= M are computed, never stored
            base = A + (size_t)gr * K;
        } else {
            base = Bw + (size_t)(n0 + row - BM) * K;
        }
        src[i] = base + c * (16 / EB);
    }
    auto stage = [&](int buf, int kt) {
        char* dst = smem + buf * STAGE;
#pragma unroll
        for (int i = 0; i < NLD; ++i) {
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)(src[i] + (size_t)kt * BK),
                EBC_LDS(dst + (wave * NLD + i) * 1024), 16, 0, 0);
        }
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

    stage(0, 0);
    __syncthreads();
    const int fr = lane & 15, fg = lane >> 4;
    for (int kt = 0; kt < nk; ++kt) {
        if (kt + 1 < nk) stage((kt + 1) & 1, kt + 1);
        const char* sb = smem + (kt & 1) * STAGE;
#pragma unroll
        for (int kk = 0; kk < BK / 32; ++kk) {
            typename E::Frag af[TM], bf[TN];
            // element offset of this lane's 8 elements within the 128-B row: kk*32 + 8*fg
            const int e = kk * 32 + 8 * fg;
            const int ch = (e * EB) >> 4;             // first 16-B chunk
#pragma unroll
            for (int a = 0; a < TM; ++a) {
                const int row = wm * WM + a * 16 + fr;
                const char* rp = sb + row * 128;
                if constexpr (EB == 2) {
                    af[a] = __builtin_bit_cast(typename E::Frag, *reinterpret_cast<const uint4*>(rp + ((ch ^ swz(row)) << 4)));
                } else {
                    const float4 x0 = *reinterpret_cast<const float4*>(rp + ((ch ^ swz(row)) << 4));
                    const float4 x1 = *reinterpret_cast<const float4*>(rp + (((ch + 1) ^ swz(row)) << 4));
                    af[a] = typename E::Frag{x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
                }
            }
#pragma unroll
            for (int b = 0; b < TN; ++b) {
                const int row = BM + wn * WN + b * 16 + fr;
                const char* rp = sb + row * 128;
                if constexpr (EB == 2) {
                    bf[b] = __builtin_bit_cast(typename E::Frag, *reinterpret_cast<const uint4*>(rp + ((ch ^ swz(row)) << 4)));
                } else {
                    const float4 x0 = *reinterpret_cast<const float4*>(rp + ((ch ^ swz(row)) << 4));
                    const float4 x1 = *reinterpret_cast<const float4*>(rp + (((ch + 1) ^ swz(row)) << 4));
                    bf[b] = typename E::Frag{x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
                }
            }
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b) acc[a][b] = mma(bf[b], af[a], acc[a][b]);   // swapped: C^T tile
        }
        __syncthreads();
    }

    // epilogue: acc[a][b][i] = C[m = m0 + wm*WM + a*16 + fr][n = n0 + wn*WN + b*16 + 4*fg + i]
    TO* C = reinterpret_cast<TO*>(g.C);
#pragma unroll
    for (int a = 0; a < TM; ++a) {
        const int m = m0 + wm * WM + a * 16 + fr;
        if (m >= g.M) continue;
#pragma unroll
        for (int b = 0; b < TN; ++b) {
            const int n = n0 + wn * WN + b * 16 + 4 * fg;
            const size_t off = (size_t)m * g.N + n;
            float v[4] = {acc[a][b][0], acc[a][b][1], acc[a][b][2], acc[a][b][3]};
            if (g.bias) {
                const float4 bb = *reinterpret_cast<const float4*>(g.bias + n);
                v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
            }
            if constexpr (EPI == EPI_GELU) {
                if (g.aux) store4<T>(reinterpret_cast<T*>(g.aux) + off, v);
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] = quick_gelu(v[i]);
            } else if constexpr (EPI == EPI_GELU_BWD) {
                float pa[4];
                load4<T>(reinterpret_cast<const T*>(g.aux) + off, pa);
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] *= quick_gelu_grad(pa[i]);
            } else if constexpr (EPI == EPI_RESID) {
                float r[4];
                load4<float>(g.resid + off, r);
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] += r[i];
            }
            store4<TO>(C + off, v);
        }
    }
}

template <class E, class TO, int EPI, int BM, int BN>
int launch_gemm(const GemmArgs& g, hipStream_t st)
{
    constexpr int LDS = 2 * (BM + BN) * 128;
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute((const void*)gemm_nt_kernel<E, TO, EPI, BM, BN>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, LDS) != hipSuccess)
            return EBC_E_LAUNCH;
        attr = true;
    }
    const int nwg = ((g.M + BM - 1) / BM) * (g.N / BN);
    hipLaunchKernelGGL((gemm_nt_kernel<E, TO, EPI, BM, BN>), dim3(nwg), dim3(256), LDS, st, g);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

template <class E, class TO, int EPI>
int dispatch_tile(const GemmArgs& g, hipStream_t st)
{
    // enough workgroups to cover the 256 CUs: 128x128 when that gives >= 256 tiles, else 128x64
    const int t128 = ((g.M + 127) / 128) * (g.N / 128);
    if (g.N % 128 == 0 && t128 >= 256) return launch_gemm<E, TO, EPI, 128, 128>(g, st);
    if (g.N % 64 == 0) return launch_gemm<E, TO, EPI, 128, 64>(g, st);
    return EBC_E_UNSUPPORTED;
}

template <class E, int EPI>
int dispatch_out(const GemmArgs& g, int out_f32, hipStream_t st)
{
    if (out_f32) return dispatch_tile<E, float, EPI>(g, st);
    return dispatch_tile<E, typename E::T, EPI>(g, st);
}

template <class E>
int dispatch_epi(const GemmArgs& g, int epi, int out_f32, hipStream_t st)
{
    switch (epi) {
        case EPI_STORE: return dispatch_out<E, EPI_STORE>(g, out_f32, st);
        case EPI_GELU: return out_f32 ? EBC_E_UNSUPPORTED : dispatch_tile<E, typename E::T, EPI_GELU>(g, st);
        case EPI_RESID: return dispatch_tile<E, float, EPI_RESID>(g, st);
        case EPI_GELU_BWD: return out_f32 ? EBC_E_UNSUPPORTED : dispatch_tile<E, typename E::T, EPI_GELU_BWD>(g, st);
    }
    return EBC_E_ARG;
}

}  // namespace

namespace ebc {
int gemm_nt(int dtype, int epi, int out_f32, const void* A, const void* B, void* C, const float* bias,
            const float* resid, void* aux, int M, int N, int K, hipStream_t st)
{
    const int bk = dtype == EBC_F32 ? 32 : 64;
    if (M <= 0 || N <= 0 || K <= 0 || K % bk != 0 || N % 64 != 0 || !A || !B || !C) return EBC_E_ARG;
    if ((epi == EPI_RESID && !resid) || (epi == EPI_GELU_BWD && !aux)) return EBC_E_ARG;
    GemmArgs g{A, B, C, bias, resid, aux, M, N, K};
    switch (dtype) {
        case EBC_F32: return dispatch_epi<EF32>(g, epi, 0, st);   // element type is already f32
        case EBC_F16: return dispatch_epi<EF16>(g, epi, out_f32, st);
        case EBC_BF16: return dispatch_epi<EBF16>(g, epi, out_f32, st);
    }
    return EBC_E_ARG;
}
}  // namespace ebc

extern "C" int ebc_gemm(int dtype, int epilogue, int out_f32, const void* A, const void* B, void* C,
                        const float* bias, const float* resid, void* aux, int M, int N, int K,
                        ebc_stream_t stream)
{
    return ebc::gemm_nt(dtype, epilogue, out_f32, A, B, C, bias, resid, aux, M, N, K, (hipStream_t)stream);
}
