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
#include <algorithm>
#include <cmath>
#include <type_traits>

#include "ebc_common.h"
#include "mfma.h"
#include "kernels.h"

using namespace ebc;

// Phase stamps for tools/lab/gemm_tl_lab.hip (a per-workgroup timeline: entry, first k-tile landed, K loop done,
// epilogue issued); nothing in the library build
#ifndef EBC_GEMM_STAMP
#define EBC_GEMM_STAMP(phase, tile) ((void)0)
#endif
// Anatomy switches for the lab harnesses (tools/lab/*_tl_lab.hip, r06): the K loop without its MFMAs, without its
// LDS-DMA pieces (the fragments read stale LDS), and the segment ending right after the K loop (no epilogue, no
// split-K / stream-K hand-off); all 0 in the library build
#ifndef EBC_GEMM_LAB_NOMFMA
#define EBC_GEMM_LAB_NOMFMA 0
#endif
#ifndef EBC_GEMM_LAB_NOLOAD
#define EBC_GEMM_LAB_NOLOAD 0
#endif
#ifndef EBC_GEMM_LAB_NOEPI
#define EBC_GEMM_LAB_NOEPI 0
#endif

namespace {

constexpr int LN_PMAX = ebc::GEMM_LN_PMAX;   // EPI_LN: at most 16 row partials (N / BN * 2 of the producing product)
constexpr int LN_PMAX_B = ebc::GEMM_LN_PMAX_B;   // EPI_LN_BWD: at most 32
enum { EPI_STORE = 0, EPI_GELU = 1, EPI_RESID = 2, EPI_GELU_BWD = 3, EPI_STATS = 4, EPI_ADD_RELU_GRAD = 5, EPI_LN = 6,
       EPI_LN_GELU = 7, EPI_LN_BWD = 8 };
// row partials an LN-normalising epilogue reads (its LDS staging past the ring: BM rows of ln_pmax float2)
template <int EPI> constexpr int ln_pmax() {
    return EPI == EPI_LN_BWD ? LN_PMAX_B : (EPI == EPI_LN || EPI == EPI_LN_GELU) ? LN_PMAX : 0;
}

struct GemmArgs {
    const void* A; const void* B; void* C;
    const float* bias;      // [N] or null
    const float* resid;     // [M,N] f32 (EPI_RESID), may alias C
    void* aux;              // [M,N] element type: GELU pre-activation (written by EPI_GELU, read by EPI_GELU_BWD);
                            // EPI_ADD_RELU_GRAD: upstream gradient gy
    int M, N, K;
    // split-K: `splits` workgroups per output tile each take `kslice` of K; the last one to finish
    // (per-tile arrival counter `cnt`, re-armed to 0 by it) adds the others' f32 partials (`part`)
    int splits = 1, kslice = 0;
    float* part = nullptr;
    int* cnt = nullptr;
    // implicit-GEMM 3x3 convolutions (stride 1, pad 1; decoder BasicBlock, models/utils.py:254-303):
    //  MODE 1 (forward / data gradient): A row m = output pixel (b, y, x) of a [B][cHp][cWp][cC]
    //    zero-padded NHWC image, K = 9 taps x cC (tap-major), k-tile kt reads the row shifted by
    //    tap (ky, kx): ((ky-1)*cWp + kx-1) pixels;  B = weights [N][3][3][cC].
    //  MODE 2 (weight gradient): K runs over the interior pixels (column b*cHWp + r: pixel r < H*W of image b).
    //    A = dz^T [M][cQs]; B = three kx-shifted copies x^T [3][cC][cQs] of the row-padded input images
    //    (x_kx^T[c][b*cPimg + yp*cW + x] = x[b][yp-1][x+kx-1]); row n = (c, ky, kx) (the nn.Conv2d weight layout)
    //    starts at ky*cW, and a K chunk at column q = b*cHWp + r reads position b*cPimg + r of it.
    int cH = 0, cW = 0, cC = 0, cHp = 0, cWp = 0, cHWp = 0;
    long cQs = 0, cPimg = 0;
    float* stats = nullptr;  // EPI_STATS: [ceil(M/BM)][2][N] per-tile column sums / sums of squares
    int group_m = 0;         // > 1: tiles ordered in groups of group_m tile rows, column-major inside a group
    const void* aux2 = nullptr;   // EPI_ADD_RELU_GRAD: ReLU output y (mask y > 0): C = acc + gy * (y > 0)
    // a launch covers output tiles [tile0, tile0 + ntile) (ntile 0: through the last); split-K partials and
    // arrival counters are indexed from tile0
    int tile0 = 0, ntile = 0;
    // MODE 0 row-mapped A operand: A row of output row r = (r / a_rpg) * a_gstride + a_goff + r % a_rpg (a_rpg 0: r)
    int a_rpg = 0, a_gstride = 0, a_goff = 0;
    // stream-K (conv instances): the sk_grid workgroups share the sk_total = tiles x sk_nk k-tiles (0: off); the
    // partial slots (2 per workgroup) in `part`, the per-tile arrival counters in `cnt`
    long sk_total = 0;
    int sk_nk = 0, sk_grid = 0;
    // > 0: every workgroup's share is exactly sk_share k-tiles (R(w) = w * sk_share, the last one shorter), a multiple
    // chosen so that the shares start at few distinct k offsets inside their tiles: the workgroups on one XCD that start
    // at the same offset walk k together over tiles of one tile row (sk_plan)
    int sk_share = 0;
    // LayerNorm folded into the encoder GEMMs (vit.hip, 16-bit; r04): a RESID product may also write a compute-dtype
    // copy of its output rows (xh) and per-row partial sums / sums of squares of them (rpart [M][N / BN * WGN][2], one
    // pair per tile column and wave column); an EPI_LN / EPI_LN_GELU product normalises its rows from such partials
    // (lnp, lnparts) in the epilogue: out = rstd * (acc - mean * lnw[col]) + bias[col], its B operand being the weight
    // pre-scaled by gamma (W' = W diag(gamma)), lnw = W'.1 and bias = b + W beta; tile column 0 writes the row mean /
    // rstd (ln_mean, ln_rstd) for the LayerNorm backward
    void* xh = nullptr;
    float* rpart = nullptr;
    const float* lnp = nullptr;
    const float* lnw = nullptr;
    float* ln_mean = nullptr;
    float* ln_rstd = nullptr;
    int lnparts = 0;
    // ... and such a RESID product may replace the deep-VPT prompt rows of its output (rows r with 1 <= r % vrep_L <=
    // vrep_nv) by the next block's prompts: row r of crop b = r / vrep_L becomes vrep[b * vrep_bs + (r % vrep_L - 1) *
    // N ...] (copy, row partials and all), the next block's input exactly as the deep-VPT insertion defines it
    const float* vrep = nullptr;
    long vrep_bs = 0;
    int vrep_L = 1, vrep_nv = 0;
    // LayerNorm backward fold (kernels.h GemmLn, r05): GELU_BWD writes the row partials bpart [M][N / BN * WGN][2] of
    // sum dA s and sum dA (A - c) (s = lnb_s, c = lnb_c, staged per tile in LDS); EPI_LN_BWD reads them (lnp, lnparts),
    // the LayerNorm input rows lnx (f32) and the row mean / rstd (ln_mean / ln_rstd as inputs)
    const float* lnb_s = nullptr;
    const float* lnb_c = nullptr;
    float* bpart = nullptr;
    const float* lnx = nullptr;
    // algorithmic K the probe records (0: K).  MODE 2's K loop runs over padded image rows; its algorithmic K is
    // the interior pixel count B*H*W (bench.py counts 2*M*N*kalg FLOP)
    int kalg = 0;
};

// Slab rows are ROWB bytes (one BK-deep K slice): 128 (BK = 64 for 16-bit, 32 for f32) or 64
// (BK = 32, 16-bit: deeper rings for the 256-wide tiles).  The 16-B chunks of a row are XOR
// swizzled on the DMA source address so the ds_read_b128 fragment reads are conflict free
// (brute-force checked against the MI355X_MICROARCH.md §LDS lane groups).
template <int ROWB> __device__ __forceinline__ int swz_row(int row) {
    // 256-B rows (BK = 128, 16-bit): chunk ^ (row & 15) -- the 16 lanes of a ds_read_b128 lane group then read 4
    // aligned blocks of 4 chunks (c0, c0^4, c0^8, c0^12): all 64 banks
    if constexpr (ROWB == 256) return row & 15;
    if constexpr (ROWB == 128) return (row >> 1) & 7;
    else return (0x1320 >> (((row >> 2) & 3) * 4)) & 3;      // [0,2,3,1][(row >> 2) & 3]
}

// MODE 0 B-slab row -> output column within the tile.  The swapped MFMA leaves each lane 4
// consecutive columns (4*fg .. 4*fg+3) of one row per 16-column sub-tile; loading the B rows of a
// wave's WN columns in this order makes sub-tiles 2p and 2p+1 hold the 8 consecutive columns
// p*32 + 8*fg .. +7 of the lane's row (an odd last sub-tile keeps its own 4), so the epilogue stores
// straight from the accumulators in 16-B pieces (64 B per row per instruction), without staging the
// tile through LDS.
template <int WN, int TN> __device__ __forceinline__ int bcol(int s) {
    const int w = s / WN, l = s - w * WN, b = l >> 4, j = l & 15, fg = j >> 2, i = j & 3;
    const int c = ((TN & 1) && b == TN - 1) ? b * 16 + fg * 4 + i : (b >> 1) * 32 + fg * 8 + (b & 1) * 4 + i;
    return w * WN + c;
}

// QuickGELU x*sigmoid(1.702x) (blocks.py:17-19) with the hardware exp2 / reciprocal (1-ulp each):
// the IEEE expf + division forms cost ~25 VALU per element in the epilogue.
__device__ __forceinline__ float sigmoid1702(float a) {
    const float e = __builtin_amdgcn_exp2f(-1.702f * 1.4426950408889634f * a);
    return __builtin_amdgcn_rcpf(1.0f + e);
}
__device__ __forceinline__ float quick_gelu(float a) { return a * sigmoid1702(a); }
__device__ __forceinline__ float quick_gelu_grad(float a) {
    const float s = sigmoid1702(a);
    return s + 1.702f * a * s * (1.0f - s);
}

template <int I, int N, class F> __device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

// output stores (default cache policy: r02 measured nt operand loads 25-35 % slower, nt stores no faster)
template <class V> __device__ __forceinline__ void st_out(V* p, const V& v) { *p = v; }
template <class TO> __device__ __forceinline__ void store4(TO* p, const float* v);
template <> __device__ __forceinline__ void store4<float>(float* p, const float* v) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    st_out(reinterpret_cast<f4*>(p), f4{v[0], v[1], v[2], v[3]});
}
template <> __device__ __forceinline__ void store4<_Float16>(_Float16* p, const float* v) {
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    h4 r = {(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]};
    st_out(reinterpret_cast<h4*>(p), r);
}
template <> __device__ __forceinline__ void store4<__bf16>(__bf16* p, const float* v) {
    typedef __bf16 b4 __attribute__((ext_vector_type(4)));
    b4 r = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
    st_out(reinterpret_cast<b4*>(p), r);
}
template <class T> __device__ __forceinline__ void load4(const T* p, float* v) {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (float)p[i];
}
template <> __device__ __forceinline__ void load4<float>(const float* p, float* v) {
    const float4 x = *reinterpret_cast<const float4*>(p);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
}

// 8 consecutive elements <-> float[8] (16 B for 16-bit types, 32 B for f32)
template <class TO> __device__ __forceinline__ void store8(TO* p, const float* v) {
    store4<TO>(p, v);
    store4<TO>(p + 4, v + 4);
}
template <> __device__ __forceinline__ void store8<_Float16>(_Float16* p, const float* v) {
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    h8 r = {(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3],
            (_Float16)v[4], (_Float16)v[5], (_Float16)v[6], (_Float16)v[7]};
    st_out(reinterpret_cast<h8*>(p), r);
}
template <> __device__ __forceinline__ void store8<__bf16>(__bf16* p, const float* v) {
    typedef __bf16 b8 __attribute__((ext_vector_type(8)));
    b8 r = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3], (__bf16)v[4], (__bf16)v[5], (__bf16)v[6], (__bf16)v[7]};
    st_out(reinterpret_cast<b8*>(p), r);
}
template <class T> __device__ __forceinline__ void load8f(const T* p, float* v) {
    typedef T t8 __attribute__((ext_vector_type(8)));
    const t8 x = *reinterpret_cast<const t8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)x[i];
}
template <> __device__ __forceinline__ void load8f<float>(const float* p, float* v) {
    load4<float>(p, v);
    load4<float>(p + 4, v + 4);
}

// Epilogue output stores with a cache-policy immediate.  STORE_POL != 0: buffer stores through a resource based at the
// tile's first output row (wave-uniform; 32-bit offsets inside the tile's rows), 16 = sc1 (write-through at the XCD
// L2), 2 = nt
#ifndef EBC_GEMM_STORE_POL
#define EBC_GEMM_STORE_POL 0
#endif
constexpr int STORE_POL = EBC_GEMM_STORE_POL;
// ... of the 16-bit outputs (C and the compute-dtype copies xh)
#ifndef EBC_GEMM_STORE_POL_H
#define EBC_GEMM_STORE_POL_H EBC_GEMM_STORE_POL
#endif
constexpr int STORE_POL_H = EBC_GEMM_STORE_POL_H;
// The MLP pre-activation the c_fc product saves for the backward (EPI_GELU / EPI_LN_GELU aux, 22.5 MB a layer at 16
// crops) is read again only by the GELU' product a whole forward later: written through (sc1) it does not sit dirty in
// the L2s at the launch's end, where a launch boundary pays ~B / 6 TB/s for B dirty bytes (MI355X_MICROARCH.md
// "boundary"; tools/lab/gemm_tl_lab.hip: c_fc with every store sc1 29.0 -> 26.8 us).  Same-box bench A/B (r06c, 4
// interleaved pairs): 3678 -> 3690 crops/s.  The f32 residual-stream outputs (RESID / LN_BWD C, read two or three
// launches later) written through as well measured 3 % SLOWER (3579): their readers still found them in the L2s.
#ifndef EBC_GEMM_AUX_POL
#define EBC_GEMM_AUX_POL 16
#endif
constexpr int AUX_POL = EBC_GEMM_AUX_POL;
template <class TO, int W, int POL = STORE_POL> __device__ __forceinline__ void pstore(TO* base, unsigned off, const float* v) {
    static_assert(W == 4 || W == 8, "4 or 8 elements");
    if constexpr (POL == 0) {
        if constexpr (W == 8) store8<TO>(base + off, v);
        else store4<TO>(base + off, v);
    } else {
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
        const unsigned bo = off * (unsigned)sizeof(TO);
        if constexpr (std::is_same<TO, float>::value) {
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                                                         __float_as_uint(v[3])}, rs, bo, 0, POL);
            if constexpr (W == 8)
                __builtin_amdgcn_raw_buffer_store_b128(u32x4{__float_as_uint(v[4]), __float_as_uint(v[5]), __float_as_uint(v[6]),
                                                             __float_as_uint(v[7])}, rs, bo + 16, 0, POL);
        } else {
            typedef TO tw __attribute__((ext_vector_type(W)));
            tw r;
#pragma unroll
            for (int i = 0; i < W; ++i) r[i] = (TO)v[i];
            if constexpr (W == 8) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, r), rs, bo, 0, POL);
            else __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, r), rs, bo, 0, POL);
        }
    }
}

// The epilogue stages the f32 tile through LDS in passes of EPR rows: all BM rows when they fit the
// ring's bytes (or 64 KiB), else halves, quarters, ... (never below one wave's WM rows).
template <int BM, int BN, int S, int ROWB, int WM> constexpr int ep_rows() {
    const int ring = S * (BM + BN) * ROWB;
    const int cap = ring > 64 * 1024 ? ring : 64 * 1024;
    int r = BM;
    while (r > WM && r * (BN + 4) * 4 > cap) r /= 2;
    return r;
}
template <int BM, int BN, int S, int ROWB, int WM> constexpr int gemm_lds_bytes() {
    const int ring = S * (BM + BN) * ROWB;
    const int ep = ep_rows<BM, BN, S, ROWB, WM>() * (BN + 4) * 4;
    return ring > ep ? ring : ep;
}

// s_waitcnt vmcnt(n * PER) with an immediate: n is wave-uniform and in [0, MAXN]
template <int PER, int MAXN>
__device__ __forceinline__ void wait_vmcnt(int n) {
    if constexpr (MAXN >= 3) { if (n >= 3) { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(3 * PER) : "memory"); return; } }
    if constexpr (MAXN >= 2) { if (n == 2) { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * PER) : "memory"); return; } }
    if constexpr (MAXN >= 1) { if (n == 1) { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(PER) : "memory"); return; } }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// SPL: the split-K epilogue paths are compiled in (only the instances a launch with g.splits > 1 runs: their
// partial loads / stores beside the accumulators made the register allocator spill every 8-wave tile's epilogue,
// 256x256: 150-430 registers, even on launches that never split)
// NLW > 0: NLW extra "loader" waves issue every LDS-DMA piece of the ring and the WGM x WGN compute waves only
// read fragments and issue MFMAs.  A wave's LDS-DMA issue rate bounds the per-CU fill (tools/lab/bw_lab.hip:
// 4 streaming waves ~105 GB/s, 8 or more ~130 GB/s = the L1 <-> L2 rate, against ~84 GB/s when the 4 compute
// waves also issue the loads between their MFMAs).
template <class E, class TO, int EPI, int BM, int BN, int S, int WGM, int WGN, int ROWB, int MODE, bool SPL, int NLW>
__global__ __launch_bounds__(64 * (WGM * WGN + NLW)) void gemm_nt_kernel(GemmArgs g)
{
    static_assert(S >= 2 && S <= 5, "stages");
    static_assert(NLW == 0 || (MODE == 0 && !SPL), "loader waves: MODE 0 split-free tiles (no block-wide epilogue barriers)");
    using T = typename E::T;
    constexpr int NW = WGM * WGN;                // compute waves per workgroup
    constexpr int NLDR = NLW ? NLW : NW;         // waves that issue the LDS-DMA pieces
    constexpr int EB = E::BYTES;
    constexpr int BK = ROWB / EB;                // K elements per slab row
    constexpr int WM = BM / WGM, WN = BN / WGN;  // wave tile
    constexpr int TM = WM / 16, TN = WN / 16;
    constexpr int ROWS = BM + BN;                // slab rows per stage (A rows then B rows)
    constexpr int STAGE = ROWS * ROWB;           // bytes
    constexpr int RPI = 1024 / ROWB;             // slab rows per LDS-DMA wave-instruction (1 KiB)
    constexpr int CPR = ROWB / 16;               // 16-B chunks per row
    // glds wave-instructions per wave per stage: NLDF full 1-KiB pieces (16-B lanes), plus, when the
    // rows do not divide, NT4 256-B pieces (4-B lanes; there is no 8-B LDS-DMA) per wave, e.g. 256x192
    // tiles of 64-B rows: 3 x 1 KiB + 2 x 256 B
    constexpr int NLDF = ROWS / (RPI * NLDR);
    constexpr int REMR = ROWS - NLDF * RPI * NLDR;
    constexpr int R4 = 256 / ROWB;               // rows per 256-B piece
    constexpr int NT4 = REMR / (NLDR * R4);
    constexpr bool TAIL = REMR != 0;
    constexpr int NLD = NLDF + NT4;
    static_assert(REMR == NT4 * NLDR * R4, "tail pieces");
    static_assert(WM % 16 == 0 && WN % 16 == 0, "tiling");
    static_assert(BK % 32 == 0, "k32 MFMA steps");

    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lw = NLW ? wave - NW : wave;       // index among the waves that issue the loads
    const int wm = wave / WGN, wn = wave % WGN;
    const int ntn = g.N / BN, ntm = (g.M + BM - 1) / BM;
    const int wg = xcd_remap(blockIdx.x, (int)gridDim.x);
    const T* A = reinterpret_cast<const T*>(g.A);
    const T* Bw = reinterpret_cast<const T*>(g.B);
    const int K = g.K;
    // Stream-K (the conv instances, g.sk_total > 0): workgroup w takes the contiguous share [R(w), R(w+1)) of the
    // launch's tiles' k-tiles (tile-major, R(w) = w * sk_total / grid; no more tiles than workgroups, so a share of
    // at most sk_nk k-tiles) and runs it as one segment per tile touched, at most two; a tile cut between workgroups
    // is finished by the last of its pieces to arrive.  Otherwise one segment: one tile, or one split-K slice of it.
    constexpr bool SKM = SPL && MODE != 0;
    const bool skr = SKM && g.sk_total > 0;
    // (32-bit: (sk_total + 1) * grid < 2^31, launch_gemm_k)
    const unsigned G = gridDim.x, skt = (unsigned)g.sk_total, sknk = (unsigned)g.sk_nk, shr = (unsigned)g.sk_share;
    const unsigned it_beg = !skr ? 0u : shr ? (unsigned)wg * shr : (unsigned)wg * skt / G;
    const unsigned it_end = !skr ? 0u : shr ? min((unsigned)(wg + 1) * shr, skt) : (unsigned)(wg + 1) * skt / G;
    if (skr && it_beg >= it_end) return;
    // a segment: k-tiles [it, it + nk) of one tile (always inlined: a loop over the segments, or a call per segment,
    // made the 8-wave tiles spill 60-230 registers)
    auto segment = [&](const unsigned it) __attribute__((always_inline)) -> int {
        int ltile, split = 0, nk, ktbase;
        if (skr) {
            ltile = (int)(it / sknk);
            ktbase = (int)(it - (unsigned)ltile * sknk);
            nk = (int)min(sknk - (unsigned)ktbase, it_end - it);
        } else {
            ltile = wg / g.splits;                    // a tile's splits are adjacent
            split = wg - ltile * g.splits;
            nk = g.kslice / BK;
            ktbase = split * nk;
        }
        const int tile = g.tile0 + ltile;
        int tm = tile / ntn, tn = tile % ntn;
        if (g.group_m > 1) {
            // each XCD's contiguous run of tiles (xcd_remap) then covers a group_m-tall block of tile rows and a
            // few tile columns instead of one or two whole tile rows: the B (weight) panels are fetched into
            // fewer XCD L2s (the wide-N products re-fetched B once per XCD)
            const int per = g.group_m * ntn, grp = tile / per, first = grp * g.group_m;
            const int gm = min(ntm - first, g.group_m), r = tile - grp * per;
            tm = first + r % gm;
            tn = r / gm;
        }
        const int m0 = tm * BM, n0 = tn * BN;
        EBC_GEMM_STAMP(0, tile);

        // per-lane source rows for the LDS-DMA staging (fixed across k; the k-tile offset is added by stage())
        const T* src[NLD];
        bool isa[NLD];
        // MODE 2: each piece's 16-B chunk index inside its row (the lane's K offset in the tile / (16 / EB)), 4 bits a
        // piece in one register (r04: a K offset per piece made the 256x192 weight-gradient tiles spill)
        unsigned cpk = 0;
#pragma unroll
        for (int i = 0; i < NLD; ++i) {
            const bool tail = TAIL && i >= NLDF;
            // full pieces: rows (wave*NLDF + i)*RPI + lane/CPR; tail piece j: 4-B lanes, rows
            // NLDF*RPI*NW + (wave*NT4 + j)*R4 + lane/(4*CPR)
            const int row = tail ? NLDF * RPI * NLDR + (lw * NT4 + (i - NLDF)) * R4 + lane / (4 * CPR)
                                 : (lw * NLDF + i) * RPI + lane / CPR;
            const int slot = tail ? (lane % (4 * CPR)) / 4 : lane % CPR;
            const int c = slot ^ swz_row<ROWB>(row);
            const T* base;
            isa[i] = row < BM;
            if (row < BM) {
                int gr = m0 + row;
                gr = gr < g.M ? gr : g.M - 1;           // clamp: rows >= M are computed, never stored
                if constexpr (MODE == 1) {
                    const int hw = g.cH * g.cW;
                    const int b = gr / hw, r = gr - b * hw, y = r / g.cW, x = r - y * g.cW;
                    base = A + ((size_t)(b * g.cHp + y + 1) * g.cWp + x + 1) * g.cC;
                } else if constexpr (MODE == 2) {
                    base = A + (size_t)gr * g.cQs;
                } else {
                    if (g.a_rpg) gr = (gr / g.a_rpg) * g.a_gstride + g.a_goff + gr % g.a_rpg;
                    base = A + (size_t)gr * K;
                }
            } else {
                const int n = n0 + (MODE == 0 ? bcol<WN, TN>(row - BM) : row - BM);
                if constexpr (MODE == 2) {
                    const int cc = n / 9, t = n - 9 * cc, ky = t / 3, kx = t - 3 * ky;   // nn.Conv2d [o][c][ky][kx]
                    base = Bw + (size_t)(kx * g.cC + cc) * g.cQs + (long)ky * g.cW;
                } else {
                    base = Bw + (size_t)n * K;
                }
            }
            const int ko = c * (16 / EB) + (tail ? (lane & 3) * (4 / EB) : 0);
            src[i] = base + ko;
            if constexpr (MODE == 2) cpk |= (unsigned)(ko / (16 / EB)) << (4 * i);
        }
        auto stage_pieces = [&](int buf, int kt) {
            if constexpr (EBC_GEMM_LAB_NOLOAD) return;
            const int ktg = ktbase + kt;
            long oa, ob;
            if constexpr (MODE == 1) {
                const int tpc = g.cC / BK;                // k-tiles per tap
                const int tap = ktg / tpc, ky = tap / 3, kx = tap - 3 * ky;
                oa = ((long)(ky - 1) * g.cWp + (kx - 1)) * g.cC + (long)(ktg - tap * tpc) * BK;
                ob = (long)ktg * BK;
            } else if constexpr (MODE == 2) {
                oa = ob = (long)ktg * BK;
            } else {
                oa = ob = (long)ktg * BK;
            }
            // MODE 2: a B chunk at K column q sits at position b * cPimg + (q - b * cHWp) of its x^T row (image b = q / cHWp).
            // cHWp >= 64 (conv_gemm), so a tile of BK <= 64 columns starting in image b0 (wave-uniform) ends in b0 or b0 + 1:
            // a lane's chunk is in b0 + 1 when its column offset reaches the boundary d (a multiple of the chunk width)
            int b0 = 0, dch = 0;
            long shift0 = 0, dP = 0;
            if constexpr (MODE == 2) {
                b0 = (int)((unsigned)ob / (unsigned)g.cHWp);        // 32-bit: K < 2^31
                dch = ((b0 + 1) * g.cHWp - (int)ob) / (16 / EB);
                dP = g.cPimg - g.cHWp;
                shift0 = ob + (long)b0 * dP;
            }
            auto piece = [&](int i) -> const T* {
                if constexpr (MODE == 2) {
                    if (isa[i]) return src[i] + oa;
                    const int c = (int)((cpk >> (4 * i)) & 15u);
                    return src[i] + shift0 + (c >= dch ? dP : 0);
                } else {
                    return src[i] + (isa[i] ? oa : ob);
                }
            };
            char* dst = smem + buf * STAGE;
#pragma unroll
            for (int i = 0; i < NLDF; ++i) {
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)piece(i),
                                                 EBC_LDS(dst + (lw * NLDF + i) * 1024), 16, 0, 0);
            }
#pragma unroll
            for (int j = 0; j < NT4; ++j) {
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)piece(NLDF + j),
                                                 EBC_LDS(dst + NLDF * NLDR * 1024 + (lw * NT4 + j) * 256), 4, 0, 0);
            }
        };
        // the compute waves stage the ring themselves unless loader waves do
        auto stage = [&](int buf, int kt) {
            if constexpr (NLW == 0) stage_pieces(buf, kt);
        };
        constexpr bool LNP = MODE == 0 && ln_pmax<EPI>() > 0;
        auto stage_stats = [&]() {
            // 1 KiB a wave-instruction (16 B a lane), the last rows' bytes clamped inside the buffer (rows >= M).
            // (Issued with the k-tiles 1..4 of the 2-stage rings instead, r04 measured no difference.)
            const char* base = reinterpret_cast<const char*>(g.lnp);
            const unsigned rowb = (unsigned)g.lnparts * 8u, total = (unsigned)g.M * rowb, b0 = (unsigned)m0 * rowb;
            const int chunks = (int)((BM * rowb) >> 10);
            for (int c = lw; c < chunks; c += NLDR) {
                unsigned o = b0 + (unsigned)c * 1024u + (unsigned)lane * 16u;
                o = o + 16u <= total ? o : total - 16u;
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(base + o),
                                                 EBC_LDS(smem + S * STAGE + c * 1024), 16, 0, 0);
            }
        };
        // GELU_BWD writing the LayerNorm-backward partials (g.bpart): s and c of the tile's BN columns into LDS past the
        // ring as stage_stats does (counted loads older than every ring piece), SCP 1-KiB pieces a vector, lanes past
        // the tile's columns clamped (they land in the padding)
        constexpr bool BPT = MODE == 0 && EPI == EPI_GELU_BWD;
        constexpr int SCP = (BN * 4 + 1023) / 1024;
        auto stage_sc = [&]() {
            for (int pc = lw; pc < 2 * SCP; pc += NLDR) {
                const float* vsrc = pc < SCP ? g.lnb_s : g.lnb_c;
                int o = (pc < SCP ? pc : pc - SCP) * 256 + lane * 4;       // float offset in the tile's columns
                o = o + 4 <= BN ? o : BN - 4;
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(vsrc + n0 + o),
                                                 EBC_LDS(smem + S * STAGE + pc * 1024), 16, 0, 0);
            }
        };

        f32x4 acc[TM][TN];
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

        // S-deep LDS ring + register double-buffered fragments.  Tiles kt+1 .. kt+S-1 are in flight
        // while tile kt is consumed; the wait is a counted vmcnt (LDS-DMA loads count on it) and the
        // barrier a raw s_barrier, so no vmcnt(0) drain happens in the K loop (cdna_hip_programming.md
        // §5 "Pipelining across barriers").  The next k32 step's ds_reads are issued before the current
        // step's MFMAs; at a tile boundary the wait+barrier sit before the last step's MFMAs so the
        // next tile's first fragments load underneath them.
        constexpr int KS = BK / 32;                   // k32 steps per tile
        // two fragment register sets (next step's reads under this step's MFMAs) unless the wave tile's
        // accumulators leave no room (2 waves/SIMD: 256 registers per lane in all)
        constexpr bool DB = TM * TN * 4 + 2 * (TM + TN) * (EB == 2 ? 4 : 8) <= 200;
        static_assert(!DB || KS % 2 == 0 || S % 2 == 0, "register-set alternation");
        const int fr = lane & 15, fg = lane >> 4;
        // Fragment addressing is lane-constant: every fragment row is 16-aligned + fr, so the XOR
        // swizzle term is swz_row(fr) for all of them.  Per lane one VGPR offset per (k32 step,
        // 16-B half); the wave's row block, the sub-tile and the stage buffer are immediates.
        const int xs = swz_row<ROWB>(fr);
        int loff[KS][EB == 2 ? 1 : 2];
#pragma unroll
        for (int kk = 0; kk < KS; ++kk)
#pragma unroll
            for (int c = 0; c < (EB == 2 ? 1 : 2); ++c) {
                const int ch = ((kk * 32 + 8 * fg) * EB >> 4) + c;
                loff[kk][c] = fr * ROWB + ((ch ^ xs) << 4);
            }
        const char* abase = smem + wm * WM * ROWB;
        const char* bbase = smem + (BM + wn * WN) * ROWB;
        auto load_frags = [&](auto bufc, int kk, typename E::Frag (&af)[TM], typename E::Frag (&bf)[TN]) {
            constexpr int buf = decltype(bufc)::value;
#pragma unroll
            for (int a = 0; a < TM; ++a) {
                const char* rp = abase + buf * STAGE + a * 16 * ROWB;
                if constexpr (EB == 2) {
                    af[a] = __builtin_bit_cast(typename E::Frag, *reinterpret_cast<const uint4*>(rp + loff[kk][0]));
                } else {
                    const float4 x0 = *reinterpret_cast<const float4*>(rp + loff[kk][0]);
                    const float4 x1 = *reinterpret_cast<const float4*>(rp + loff[kk][EB == 2 ? 0 : 1]);
                    af[a] = typename E::Frag{x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
                }
            }
#pragma unroll
            for (int b = 0; b < TN; ++b) {
                const char* rp = bbase + buf * STAGE + b * 16 * ROWB;
                if constexpr (EB == 2) {
                    bf[b] = __builtin_bit_cast(typename E::Frag, *reinterpret_cast<const uint4*>(rp + loff[kk][0]));
                } else {
                    const float4 x0 = *reinterpret_cast<const float4*>(rp + loff[kk][0]);
                    const float4 x1 = *reinterpret_cast<const float4*>(rp + loff[kk][EB == 2 ? 0 : 1]);
                    bf[b] = typename E::Frag{x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
                }
            }
        };
        // tile next_kt landed (count the later tiles still in flight): the issuing wave's counted vmcnt
        auto wait_tile = [&](int next_kt, auto tailc) {
            if constexpr (decltype(tailc)::value) {
                const int later = (nk - 1 - next_kt) < (S - 2) ? (nk - 1 - next_kt) : (S - 2);
                wait_vmcnt<NLD, S - 2>(later);
            } else {
                asm volatile("s_waitcnt vmcnt(%0)" :: "n"((S - 2) * NLD) : "memory");
            }
        };
        auto sync_tile = [&](int next_kt, auto tailc) {
            // tile next_kt landed, every wave done reading the buffer that the refill below overwrites.
            // Outside the tail S-2 later tiles are in flight.
            if constexpr (NLW == 0) wait_tile(next_kt, tailc);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        };
        if constexpr (NLW > 0) {
            if (wave >= NW) {
                // loader wave: the compute waves' ring schedule (one barrier per k-tile, the buffer of tile kt
                // refilled with tile kt + S right after the barrier that retires its reads), then exit
                if constexpr (LNP) stage_stats();
                if constexpr (BPT) { if (g.bpart) stage_sc(); }
                for (int s = 0; s < S - 1; ++s)
                    if (s < nk) stage_pieces(s, s);
                wait_tile(0, std::true_type{});
                __builtin_amdgcn_s_barrier();
                if (S - 1 < nk) stage_pieces(S - 1, S - 1);
                for (int kt = 0; kt + 1 < nk; ++kt) {
                    wait_tile(kt + 1, std::true_type{});
                    __builtin_amdgcn_s_barrier();
                    if (kt + S < nk) stage_pieces(kt % S, kt + S);
                }
                return nk;
            }
        }

        // 4-wave RESID tiles (one wave per SIMD: registers to spare): the f32 residual operand of the epilogue is
        // loaded before the ring fills, so its latency hides under the first tiles' instead of being paid after the
        // K loop (vmcnt retires loads in order: issued any later, a counted ring wait would block on it mid-loop)
        constexpr bool PREF = MODE == 0 && (EPI == EPI_RESID || EPI == EPI_LN_BWD) && NW == 4 && NW + NLW <= 8;
        // RESID: the residual row r, or (vrep) the prompt row replacing output row r -- an address select, no branch
        constexpr bool VREP = MODE == 0 && EPI == EPI_RESID && EB == 2;    // (gemm_nt_ln: 16-bit only)
        auto vrep_row = [&](int r) -> bool {
            if (!VREP || !g.vrep) return false;
            const int j = r % g.vrep_L - 1;
            return (unsigned)j < (unsigned)g.vrep_nv;
        };
        auto resid_row = [&](int r) -> const float* {
            if constexpr (!VREP) return g.resid + (size_t)r * g.N;
            const int b = r / g.vrep_L, j = r - b * g.vrep_L - 1;         // (vrep_L >= 1 when vrep is set)
            const float* pv = g.vrep + b * g.vrep_bs + (size_t)j * g.N;
            const float* pr = g.resid + (size_t)r * g.N;
            return g.vrep && (unsigned)j < (unsigned)g.vrep_nv ? pv : pr;
        };
        typedef float rp8_t __attribute__((ext_vector_type(8)));
        typedef float rp4_t __attribute__((ext_vector_type(4)));
        rp8_t rp8[PREF ? TM : 1][TN / 2 > 0 ? TN / 2 : 1];
        rp4_t rp4[PREF && (TN & 1) ? TM : 1];
        // 8-wave GELU' tiles (256 registers a wave): the first half of the rows' pre-activation operand the same way
        constexpr bool PREF_G = MODE == 0 && EPI == EPI_GELU_BWD && NW >= 8 && TM % 2 == 0 && (TN & 1) == 0;
        typedef T gp8_t __attribute__((ext_vector_type(8)));
        gp8_t gp8[PREF_G ? TM / 2 : 1][TN / 2 > 0 ? TN / 2 : 1];
        auto prefetch_g = [&]() {
            const int mb = m0 + wm * WM + (lane & 15), nb = n0 + wn * WN, fq = lane >> 4;
            const T* aux = reinterpret_cast<const T*>(g.aux);
#pragma unroll
            for (int a = 0; a < TM / 2; ++a) {
                const size_t ro = (size_t)min(mb + a * 16, g.M - 1) * g.N + nb;
#pragma unroll
                for (int q = 0; q < TN / 2; ++q) gp8[a][q] = *reinterpret_cast<const gp8_t*>(aux + ro + q * 32 + fq * 8);
            }
        };
        auto prefetch_r = [&]() {
            const int mb = m0 + wm * WM + (lane & 15), nb = n0 + wn * WN, fq = lane >> 4;
#pragma unroll
            for (int a = 0; a < TM; ++a) {
                const float* src = resid_row(min(mb + a * 16, g.M - 1)) + nb;
#pragma unroll
                for (int q = 0; q < TN / 2; ++q) rp8[a][q] = *reinterpret_cast<const rp8_t*>(src + q * 32 + fq * 8);
                if constexpr (TN & 1) rp4[a] = *reinterpret_cast<const rp4_t*>(src + (TN / 2) * 32 + fq * 4);
            }
        };
        // Where the epilogue prefetches are issued (r06, tools/lab/gemm_tl_lab.hip: issued ahead of the ring they delayed
        // tile 0 by 1.3-1.4 us -- GELU' prologue 2.9 vs 1.6 us for c_fc, RESID 3.2 vs 1.8 us for the plain product):
        //  * loader-wave tiles: the compute waves issue theirs after tile 0 has landed (their vmcnt counts no ring piece);
        //  * the 8-wave GELU' tiles (2-stage ring): right behind tile 0's pieces, which are then waited for with a vmcnt
        //    that leaves the NPF younger prefetch loads in flight (tile 1's wait, vmcnt(0), covers them);
        //  * 4-wave tiles without loader waves: ahead of the ring as before (later, every counted ring wait would have to
        //    count them).
#ifndef EBC_GEMM_PREF_LATE
#define EBC_GEMM_PREF_LATE 1
#endif
        constexpr bool LATE_G = EBC_GEMM_PREF_LATE && PREF_G && NLW == 0 && S == 2;
        constexpr bool LATE_R = EBC_GEMM_PREF_LATE && PREF && NLW > 0;
        constexpr int NPF = (TM / 2) * (TN / 2) * (int)sizeof(gp8_t) / 16;   // 16-B loads of prefetch_g
        if constexpr (PREF_G && !LATE_G) prefetch_g();
        if constexpr (PREF && !LATE_R) prefetch_r();
        // EPI_LN: the workgroup's rows' partials (gemm_nt_ln; lnparts float2 a row, rows m0 .. m0 + BM contiguous) are
        // copied by LDS-DMA into LDS past the ring ahead of tile 0 -- counted loads of the issuing waves, older than
        // every ring piece, so landed once tile 0 has -- and reduced in the epilogue.  (Register loads of them, 2-4 per
        // row and lane, duplicated across the wave columns, cost the products 2.5-4 us a launch in the start-up burst:
        // profiles/r04t_lnfold_lab_*.txt.)
        if constexpr (LNP && NLW == 0) stage_stats();
        if constexpr (BPT && NLW == 0) { if (g.bpart) stage_sc(); }
#pragma unroll
        for (int s = 0; s < S - 1; ++s)
            if (s < nk) stage(s, s);
        if constexpr (LATE_G) {
            prefetch_g();
            // tile 0 landed (its pieces are older than the NPF prefetch loads), every wave past the barrier
            asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NPF) : "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        } else {
            sync_tile(0, std::true_type{});
        }
        if constexpr (LATE_R) prefetch_r();
        EBC_GEMM_STAMP(1, tile);
        if (S - 1 < nk) stage(S - 1, S - 1);
        typename E::Frag a0[TM], b0[TN], a1[TM], b1[TN];
        load_frags(std::integral_constant<int, 0>{}, 0, a0, b0);
        auto mma_all = [&](typename E::Frag (&af)[TM], typename E::Frag (&bf)[TN]) {
            if constexpr (EBC_GEMM_LAB_NOMFMA) {          // keep the fragment reads: one VALU add each
#pragma unroll
                for (int a = 0; a < TM; ++a) acc[a][0][0] += (float)af[a][0];
#pragma unroll
                for (int b = 0; b < TN; ++b) acc[0][b][1] += (float)bf[b][0];
                return;
            }
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b) acc[a][b] = mma(bf[b], af[a], acc[a][b]);   // swapped: C^T tile
        };
        // step body: prefetch the fragments of the step after (kt, kk) into (an, bn), then MMA (ac, bc);
        // the K loop is unrolled by S so the stage buffer of every fragment load is a constant.
        // The main loop runs whole groups of S tiles that are followed by at least S more, so it has no
        // bounds tests (a branch-free body keeps the accumulators in place across the back edge);
        // the last one or two groups run the same body with the tests.
        auto step = [&](auto bufc, auto tailc, int kt, int kk, typename E::Frag (&ac)[TM], typename E::Frag (&bc)[TN],
                        typename E::Frag (&an)[TM], typename E::Frag (&bn)[TN]) {
            constexpr int buf = decltype(bufc)::value;
            constexpr bool tail = decltype(tailc)::value;
            if constexpr (!DB) mma_all(ac, bc);      // single fragment set: consume, then refill it
            if (kk + 1 < KS) {
                load_frags(bufc, kk + 1, an, bn);
            } else if (!tail || kt + 1 < nk) {
                sync_tile(kt + 1, tailc);
                if (!tail || kt + S < nk) stage(buf, kt + S);
                load_frags(std::integral_constant<int, (buf + 1) % S>{}, 0, an, bn);
            }
            if constexpr (!DB) {
                __builtin_amdgcn_sched_barrier(0);
                return;
            }
            mma_all(ac, bc);
            // keep the next step's fragment reads ahead of (interleaved with) this step's MFMAs and
            // stop the scheduler from sinking them next to their first use
            // (all of them within the first half of the MFMAs, two per MFMA)
            constexpr int NRD = (TM + TN) * (EB == 2 ? 1 : 2), NG = (NRD + 1) / 2;
            static_assert(NG <= TM * TN, "read/MFMA interleave");
            // (r05: 256x192 MODE 0 step 3692 -> 3710 crops/s same box, profiles/r05g_glds_interleave_ab.txt)
            constexpr int NV = NLW == 0 && NLD + NG <= TM * TN ? NLD : 0;
            if (!tail && kk + 1 == KS && NV > 0) {
                // tile boundary: the next tile's LDS-DMA pieces (stage above) spread over this step's MFMAs instead of
                // issued as one burst right after the barrier (both waves of a SIMD then stop issuing MFMAs at once)
                // (the fragment reads of the next buffer stay behind every piece: the compiler orders LDS-DMA writes
                // before later LDS reads)
                static_for<0, NV>([&](auto) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);             // MFMA
                    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);             // VMEM (LDS-DMA piece)
                });
                static_for<0, NG>([&](auto) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);             // MFMA
                    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);             // DS reads
                });
                __builtin_amdgcn_sched_group_barrier(0x008, TM * TN - NG - NV, 0);
                __builtin_amdgcn_sched_barrier(0);
                return;
            }
            static_for<0, NG>([&](auto) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                 // MFMA
                __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);                 // DS reads
            });
            __builtin_amdgcn_sched_group_barrier(0x008, TM * TN - NG, 0);
            __builtin_amdgcn_sched_barrier(0);
        };
        auto group = [&](int kt0, auto tailc) {
            static_for<0, S>([&](auto sc) {
                constexpr int s = decltype(sc)::value;
                const int kt = kt0 + s;
                if (!decltype(tailc)::value || kt < nk) {
                    if constexpr (!DB) {
                        static_for<0, KS>([&](auto kc) { step(sc, tailc, kt, decltype(kc)::value, a0, b0, a0, b0); });
                    } else if constexpr (KS % 2 == 0) {       // 128-B rows: 2 k32 steps a tile; 256-B rows: 4
                        static_for<0, KS / 2>([&](auto hc) {
                            constexpr int h = decltype(hc)::value;
                            step(sc, tailc, kt, 2 * h, a0, b0, a1, b1);
                            step(sc, tailc, kt, 2 * h + 1, a1, b1, a0, b0);
                        });
                    } else if constexpr ((s & 1) == 0) {
                        step(sc, tailc, kt, 0, a0, b0, a1, b1);
                    } else {
                        step(sc, tailc, kt, 0, a1, b1, a0, b0);
                    }
                }
            });
        };
        int kt0 = 0;
        for (; kt0 + 2 * S <= nk; kt0 += S) group(kt0, std::false_type{});
        for (; kt0 < nk; kt0 += S) group(kt0, std::true_type{});
        EBC_GEMM_STAMP(2, tile);
        if constexpr (EBC_GEMM_LAB_NOEPI) {
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b) asm volatile("" :: "v"(acc[a][b]));
            EBC_GEMM_STAMP(3, tile);
            return nk;
        }

        if (SPL && g.splits > 1 && g.cnt == nullptr) {
            // split-K without a last arriver (deep splits of the weight-gradient products): every split stores its
            // f32 partial row-major into part[split][M][N] (columns as the epilogue maps them), a separate launch
            // (splitk_reduce_kernel) sums the splits in split order -- deterministic, and the sum is spread over
            // the whole GPU instead of re-read through one CU
            float* P = g.part + (size_t)split * g.M * g.N;
            const int mb = m0 + wm * WM + fr;
#pragma unroll
            for (int a = 0; a < TM; ++a) {
                const int m = mb + a * 16;
                if (m >= g.M) break;
#pragma unroll
                for (int b = 0; b < TN; ++b) {
                    int n;
                    if constexpr (MODE == 0) {
                        constexpr int NP = TN / 2;
                        const int nb = n0 + wn * WN;
                        n = (b / 2 < NP) ? nb + (b / 2) * 32 + fg * 8 + (b & 1) * 4 : nb + NP * 32 + fg * 4;
                    } else {
                        n = n0 + wn * WN + b * 16 + 4 * fg;
                    }
                    *reinterpret_cast<f32x4*>(P + (size_t)m * g.N + n) = acc[a][b];
                }
            }
            return nk;
        }
        bool fin = true;                              // this segment ends its tile: run the epilogue
        if (SPL && (skr ? (ktbase != 0 || nk != g.sk_nk) : g.splits > 1)) {
            // split-K / a stream-K piece: publish this piece's f32 partial (lane-major: the reader has the same lane
            // map, so every access is a coalesced 16-B per lane), count the arrival; the last arriver sums the pieces
            // and runs the epilogue, the rest go on (stream-K) or exit.
            // MI355X_MICROARCH.md cross-CU hand-off, sc1 form: sc1 (write-through) 16-B stores, every wave's vmcnt(0), a
            // barrier, ONE agent-scope atomic add; the last adder's waves read with sc1 loads after a barrier.  No agent
            // fences (a buffer_wbl2 per workgroup costs ~microseconds).
            constexpr int PT = NW * TM * TN * 64;     // f32x4 per partial tile
            // partial slots: split-K, tile ltile's `splits` slots; stream-K, two per workgroup (2w: its first segment,
            // 2w + 1: its last), pieces p = 0.. of a tile are workgroups wf + p
            int mine, mypiece, wf = 0, np = g.splits;
            const unsigned i0 = (unsigned)ltile * sknk;
            if (skr) {
                // the workgroups whose shares touch this tile: the last w with R(w) <= i0 .. the last with R(w) < i0 + nk
                wf = shr ? (int)(i0 / shr) : (int)(((i0 + 1) * G - 1) / skt);
                np = (shr ? (int)((i0 + sknk - 1) / shr) : (int)(((i0 + sknk) * G - 1) / skt)) - wf + 1;
                mine = it == it_beg ? 2 * wg : 2 * wg + 1;
                mypiece = wg - wf;
            } else {
                mine = mypiece = split;
            }
            auto slot = [&](int piece) -> int {
                if (!skr) return piece;
                const int w = wf + piece;
                const unsigned rw = shr ? (unsigned)w * shr : (unsigned)w * skt / G;
                return piece == 0 && rw < i0 ? 2 * w + 1 : 2 * w;
            };
            // one buffer resource over the partials; aux 16 = sc1
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                reinterpret_cast<f32x4*>(g.part) + (skr ? 0 : (size_t)ltile * g.splits * PT), 0, 0x7fffffff, 0x00020000);
            typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b)
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[a][b]), rs,
                                                           ((mine * PT) + ((wave * TM + a) * TN + b) * 64 + lane) * 16, 0, 16);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            __shared__ int last;
            if (tid == 0) last = atomicAdd(&g.cnt[ltile], 1) == np - 1;
            __syncthreads();
            fin = last;
            if (fin) {
                // bit-reproducible sum whichever piece arrives last: two pieces add the other's partial (f32 addition
                // commutes); more re-read every partial, this one's too, in piece order.  Loaded in row-group chunks of
                // at most 64 registers: the whole partial at once (TM*TN*4 registers on top of the accumulators)
                // spilled the 256-wide tiles' epilogues (256x256: 150-430 registers)
                constexpr int PCH = [] { int c = TM; while (c > 1 && (TM % c || c * TN * 4 > 64)) --c; return c; }();
                auto add_partial = [&](int sp) {
                    static_for<0, TM / PCH>([&](auto cc) {
                        constexpr int a0 = decltype(cc)::value * PCH;
                        f32x4 t[PCH][TN];
#pragma unroll
                        for (int a = 0; a < PCH; ++a)
#pragma unroll
                            for (int b = 0; b < TN; ++b)
                                t[a][b] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                    rs, ((sp * PT) + ((wave * TM + a0 + a) * TN + b) * 64 + lane) * 16, 0, 16));
#pragma unroll
                        for (int a = 0; a < PCH; ++a)
#pragma unroll
                            for (int b = 0; b < TN; ++b) acc[a0 + a][b] += t[a][b];
                        // keep the next chunk's loads below this one's adds (a sched_barrier alone did not: the DAG
                        // scheduler hoisted all 32 loads of a 256x256 partial)
                        asm volatile("" ::: "memory");
                        __builtin_amdgcn_sched_barrier(0);
                    });
                };
                if (np == 2) {
                    add_partial(slot(1 - mypiece));
                } else {
#pragma unroll
                    for (int a = 0; a < TM; ++a)
#pragma unroll
                        for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
                    for (int p = 0; p < np; ++p) add_partial(slot(p));
                }
                if (tid == 0) atomicExch(&g.cnt[ltile], 0);   // re-armed for the next launch
            }
        }

        if (fin) {
            if constexpr (MODE == 0) {
                // direct epilogue (bcol above): lane (fr, fg) holds rows m0 + wm*WM + a*16 + fr and, per column
                // group q, 8 (a sub-tile pair) or 4 (odd last sub-tile) consecutive columns.  Operands
                // (resid / aux) are loaded for the whole wave tile first (row-clamped, unconditional), then each
                // group is finished and stored; rows >= M are never stored.
                static_assert(EPI <= EPI_GELU_BWD || EPI == EPI_LN || EPI == EPI_LN_GELU || EPI == EPI_LN_BWD,
                              "MODE 0 epilogues");
                constexpr bool LN = EPI == EPI_LN || EPI == EPI_LN_GELU, GE = EPI == EPI_GELU || EPI == EPI_LN_GELU;
                constexpr bool LNB = EPI == EPI_LN_BWD;
                TO* C = reinterpret_cast<TO*>(g.C);
                constexpr int NP = TN / 2, ODD = TN & 1;
                constexpr bool PRE = EPI == EPI_GELU_BWD || EPI == EPI_RESID || LNB;
                using PA = typename std::conditional<EPI == EPI_RESID || LNB, float, T>::type;
                typedef PA pa8 __attribute__((ext_vector_type(8)));
                typedef PA pa4 __attribute__((ext_vector_type(4)));
                const int mb = m0 + wm * WM + fr;
                const int nb = n0 + wn * WN;
                // 8-wave tiles run two waves per SIMD (256 registers each): their operands are loaded for half of the
                // row groups at a time (the whole wave tile at once spilled: GELU' 256x192, 27 registers), with a scheduling
            // fence per row group
                constexpr int PREG = PRE ? TM * (NP * (int)sizeof(pa8) + ODD * (int)sizeof(pa4)) / 4 : 0;
                constexpr int PH = (NW >= 8 && PREG > 24 && TM % 2 == 0) ? 2 : 1;
                constexpr int TMP = TM / PH;
                float bv[NP > 0 ? NP : 1][8], bo[4];
#pragma unroll
                for (int q = 0; q < NP; ++q) {
                    if (g.bias) load8f<float>(g.bias + nb + q * 32 + fg * 8, bv[q]);
                    else for (int i = 0; i < 8; ++i) bv[q][i] = 0.f;
                }
                if constexpr (ODD) {
                    if (g.bias) load4<float>(g.bias + nb + NP * 32 + fg * 4, bo);
                    else for (int i = 0; i < 4; ++i) bo[i] = 0.f;
                }
                // the row's 4 lanes (lanes fr + 16 fg) meet by lane swaps (same bits on all four)
                auto pair_sum = [](float x) {
                    const auto a1 = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
                    x = __uint_as_float(a1[0]) + __uint_as_float(a1[1]);
                    const auto a2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
                    return __uint_as_float(a2[0]) + __uint_as_float(a2[1]);
                };
                // LN: W'.1 of the lane's columns; each row's rstd and rstd * mean from its partials in LDS (stage_stats):
                // the row's 4 lanes read 16-B pairs q = fg, fg + 4 and meet by lane swaps, so every tile of a row sums in
                // the same order (same bits).  var = E[x^2] - mean^2 in f32 (|mean| / std <= 0.15 on the encoder's rows;
                // tests/test_gpu_model.py holds the error to the LayerNorm-launch path's)
                float lw[LN && NP > 0 ? NP : 1][8], lwo[4];
                float rsv[LN ? TM : 1], rsmuv[LN ? TM : 1];
                if constexpr (LN) {
#pragma unroll
                    for (int q = 0; q < NP; ++q) load8f<float>(g.lnw + nb + q * 32 + fg * 8, lw[q]);
                    if constexpr (ODD) load4<float>(g.lnw + nb + NP * 32 + fg * 4, lwo);
                    const char* st = smem + S * STAGE;
#pragma unroll
                    for (int a = 0; a < TM; ++a) {
                        const float4* pp = reinterpret_cast<const float4*>(st + (wm * WM + a * 16 + fr) * g.lnparts * 8);
                        float s1 = 0.f, s2 = 0.f;
#pragma unroll
                        for (int j = 0; j < ln_pmax<EPI>() / 8; ++j) {
                            const int q = fg + 4 * j;
                            const bool in = 2 * q < g.lnparts;
                            const float4 t = pp[in ? q : 0];
                            s1 += in ? t.x + t.z : 0.f;
                            s2 += in ? t.y + t.w : 0.f;
                        }
                        s1 = pair_sum(s1);
                        s2 = pair_sum(s2);
                        const float mean = s1 / (float)g.K;
                        const float var = fmaxf(s2 / (float)g.K - mean * mean, 0.f);
                        rsv[a] = 1.0f / sqrtf(var + 1e-5f);
                        rsmuv[a] = rsv[a] * mean;
                        const int m = mb + a * 16;
                        if (g.ln_mean && tn == 0 && wn == 0 && fg == 0 && m < g.M) { g.ln_mean[m] = mean; g.ln_rstd[m] = rsv[a]; }
                    }
                }
                // LN_BWD: per row rstd, mean(g) = sum g / N and mean(g xhat) = sum g xhat / N from the GELU' product's
                // partials in LDS (the row's 4 lanes read the pairs fg, fg + 4, .. and meet by lane swaps, as above),
                // the LayerNorm's mean / rstd from ln_mean / ln_rstd:  out = rstd (g - mean(g) - (x - mu) rstd mean(g
                // xhat)) + resid
                float kr[LNB ? TM : 1], ka[LNB ? TM : 1], km[LNB ? TM : 1], kb[LNB ? TM : 1];
                if constexpr (LNB) {
                    const char* st = smem + S * STAGE;
#pragma unroll
                    for (int a = 0; a < TM; ++a) {
                        const float4* pp = reinterpret_cast<const float4*>(st + (wm * WM + a * 16 + fr) * g.lnparts * 8);
                        float s1 = 0.f, s2 = 0.f;
#pragma unroll
                        for (int j = 0; j < ln_pmax<EPI>() / 8; ++j) {
                            const int q = fg + 4 * j;
                            const bool in = 2 * q < g.lnparts;
                            const float4 t = pp[in ? q : 0];
                            s1 += in ? t.x + t.z : 0.f;
                            s2 += in ? t.y + t.w : 0.f;
                        }
                        s1 = pair_sum(s1);
                        s2 = pair_sum(s2);
                        const int m = min(mb + a * 16, g.M - 1);
                        kr[a] = g.ln_rstd[m];
                        km[a] = g.ln_mean[m];
                        ka[a] = s1 / (float)g.N;
                        kb[a] = kr[a] * (s2 / (float)g.N);
                    }
                }
                // GELU_BWD with bpart: the lane's partial sums dA s and dA (A - c) of its row over its columns
                float bs1 = 0.f, bs2 = 0.f;
                auto bpt_add = [&](const float* v, int w, const auto& pre, int cl) {
                    const float* sl = reinterpret_cast<const float*>(smem + S * STAGE) + cl;
                    const float* cv = reinterpret_cast<const float*>(smem + S * STAGE + SCP * 1024) + cl;
                    for (int i = 0; i < w; ++i) {
                        bs1 = fmaf(v[i], sl[i], bs1);
                        bs2 = fmaf(v[i], (float)pre[i] - cv[i], bs2);
                    }
                };
                float rs = 1.f, rsmu = 0.f;
                float lr = 1.f, la = 0.f, lm = 0.f, lb = 0.f;    // LN_BWD: the row's constants
                bool vr = false;                     // RESID: the row is a replaced prompt row
                // RESID with rpart: the lane's partial sum / sum of squares of its row's output values
                float rsum = 0.f, rsq = 0.f;
                const size_t tb = (size_t)m0 * g.N;          // the tile's first output row (pstore bases)
                auto put = [&](auto* base, size_t off, const float* v, int w, auto polc) {
                    using TT = typename std::remove_pointer<decltype(base)>::type;
                    constexpr int POL = std::is_same<TT, float>::value ? decltype(polc)::value
                                        : (decltype(polc)::value == STORE_POL ? STORE_POL_H : decltype(polc)::value);
                    if (w == 8) pstore<TT, 8, POL>(base + tb, (unsigned)(off - tb), v);
                    else pstore<TT, 4, POL>(base + tb, (unsigned)(off - tb), v);
                };
                using PolC = std::integral_constant<int, STORE_POL>;
                using PolA = std::integral_constant<int, AUX_POL>;
                auto finish = [&](float* v, int w, const float* bias, const float* lwv, const auto& pre, size_t off,
                                  const auto& xs) {
                    if constexpr (LN) {
                        for (int i = 0; i < w; ++i) v[i] = fmaf(rs, v[i], -rsmu * lwv[i]);
                    }
                    for (int i = 0; i < w; ++i) v[i] += bias[i];
                    if constexpr (GE) {
                        if (g.aux) put(reinterpret_cast<T*>(g.aux), off, v, w, PolA{});
                        for (int i = 0; i < w; ++i) v[i] = quick_gelu(v[i]);
                    } else if constexpr (EPI == EPI_GELU_BWD) {
                        for (int i = 0; i < w; ++i) v[i] *= quick_gelu_grad((float)pre[i]);
                    } else if constexpr (LNB) {
                        for (int i = 0; i < w; ++i) v[i] = fmaf(lr, v[i] - la - (xs[i] - lm) * lb, (float)pre[i]);
                        put(reinterpret_cast<T*>(g.xh), off, v, w, PolC{});
                    } else if constexpr (EPI == EPI_RESID) {
                        for (int i = 0; i < w; ++i) v[i] = vr ? (float)pre[i] : v[i] + pre[i];
                        if (VREP && g.rpart) {
                            for (int i = 0; i < w; ++i) { rsum += v[i]; rsq = fmaf(v[i], v[i], rsq); }
                            put(reinterpret_cast<T*>(g.xh), off, v, w, PolC{});
                        }
                    }
                    put(C, off, v, w, PolC{});
                };
                static_for<0, PH>([&](auto phc) {
                    constexpr int a0 = decltype(phc)::value * TMP;
                    pa8 p8[PRE ? TMP : 1][NP > 0 ? NP : 1];
                    pa4 p4[PRE && ODD ? TMP : 1];
                    typedef float xv8 __attribute__((ext_vector_type(8)));
                    typedef float xv4 __attribute__((ext_vector_type(4)));
                    xv8 x8[LNB ? TMP : 1][NP > 0 ? NP : 1];
                    xv4 x4[LNB && ODD ? TMP : 1];
                    if constexpr (LNB) {
#pragma unroll
                        for (int a = 0; a < TMP; ++a) {
                            const float* sr = g.lnx + (size_t)min(mb + (a0 + a) * 16, g.M - 1) * g.N + nb;
#pragma unroll
                            for (int q = 0; q < NP; ++q) x8[a][q] = *reinterpret_cast<const xv8*>(sr + q * 32 + fg * 8);
                            if constexpr (ODD) x4[a] = *reinterpret_cast<const xv4*>(sr + NP * 32 + fg * 4);
                        }
                    }
                    if constexpr (PREF) {
#pragma unroll
                        for (int a = 0; a < TMP; ++a) {
#pragma unroll
                            for (int q = 0; q < NP; ++q) p8[a][q] = rp8[a0 + a][q];
                            if constexpr (ODD) p4[a] = rp4[a0 + a];
                        }
                    } else if constexpr (PREF_G && a0 == 0 && TMP == TM / 2) {
#pragma unroll
                        for (int a = 0; a < TMP; ++a)
#pragma unroll
                            for (int q = 0; q < NP; ++q) p8[a][q] = __builtin_convertvector(gp8[a][q], pa8);
                    } else if constexpr (PRE) {
                        const PA* src = (EPI == EPI_RESID || LNB) ? reinterpret_cast<const PA*>(g.resid)
                                                                   : reinterpret_cast<const PA*>(g.aux);
#pragma unroll
                        for (int a = 0; a < TMP; ++a) {
                            const int r = min(mb + (a0 + a) * 16, g.M - 1);
                            const PA* sr = src + (size_t)r * g.N + nb;
                            if constexpr (EPI == EPI_RESID) sr = reinterpret_cast<const PA*>(resid_row(r)) + nb;
#pragma unroll
                            for (int q = 0; q < NP; ++q) p8[a][q] = *reinterpret_cast<const pa8*>(sr + q * 32 + fg * 8);
                            if constexpr (ODD) p4[a] = *reinterpret_cast<const pa4*>(sr + NP * 32 + fg * 4);
                        }
                    }
#pragma unroll
                    for (int a = 0; a < TMP; ++a) {
                        const int m = mb + (a0 + a) * 16;
                        if (m >= g.M) break;                 // rows ascend with a (the 4 lanes of a row together)
                        const size_t ro = (size_t)m * g.N + nb;
                        if constexpr (LN) {
                            rs = rsv[a0 + a];
                            rsmu = rsmuv[a0 + a];
                        }
                        if constexpr (LNB) {
                            lr = kr[a0 + a]; la = ka[a0 + a]; lm = km[a0 + a]; lb = kb[a0 + a];
                        }
                        if constexpr (EPI == EPI_RESID) vr = vrep_row(m);
#pragma unroll
                        for (int q = 0; q < NP; ++q) {
                            float v[8] = {acc[a0 + a][2 * q][0], acc[a0 + a][2 * q][1], acc[a0 + a][2 * q][2], acc[a0 + a][2 * q][3],
                                          acc[a0 + a][2 * q + 1][0], acc[a0 + a][2 * q + 1][1], acc[a0 + a][2 * q + 1][2],
                                          acc[a0 + a][2 * q + 1][3]};
                            const float* lwq = LN ? lw[q] : nullptr;
                            if constexpr (PRE) finish(v, 8, bv[q], lwq, p8[a][q], ro + q * 32 + fg * 8, x8[LNB ? a : 0][q]);
                            else finish(v, 8, bv[q], lwq, 0, ro + q * 32 + fg * 8, 0);
                            if constexpr (BPT) { if (g.bpart) bpt_add(v, 8, p8[a][q], wn * WN + q * 32 + fg * 8); }
                        }
                        if constexpr (ODD) {
                            float v[4] = {acc[a0 + a][TN - 1][0], acc[a0 + a][TN - 1][1], acc[a0 + a][TN - 1][2], acc[a0 + a][TN - 1][3]};
                            if constexpr (PRE) finish(v, 4, bo, lwo, p4[a], ro + NP * 32 + fg * 4, x4[LNB ? a : 0]);
                            else finish(v, 4, bo, lwo, 0, ro + NP * 32 + fg * 4, 0);
                            if constexpr (BPT) { if (g.bpart) bpt_add(v, 4, p4[a], wn * WN + NP * 32 + fg * 4); }
                        }
                        if constexpr (BPT) {
                            if (g.bpart) {
                                // one partial pair per (tile column, wave column), as the RESID row partials
                                const float t1 = pair_sum(bs1), t2 = pair_sum(bs2);
                                if (fg == 0)
                                    reinterpret_cast<float2*>(g.bpart)[(size_t)m * (g.N / BN * WGN) + tn * WGN + wn] = float2{t1, t2};
                                bs1 = 0.f;
                                bs2 = 0.f;
                            }
                        }
                        if constexpr (EPI == EPI_RESID) {
                            if (VREP && g.rpart) {
                                // one partial per (tile column, wave column)
                                const float ts = pair_sum(rsum), tq = pair_sum(rsq);
                                if (fg == 0)
                                    reinterpret_cast<float2*>(g.rpart)[(size_t)m * (g.N / BN * WGN) + tn * WGN + wn] = float2{ts, tq};
                                rsum = 0.f;
                                rsq = 0.f;
                            }
                        }
                        if constexpr (NW >= 8) __builtin_amdgcn_sched_barrier(0);
                    }
                });
            } else {
            // epilogue: acc[a][b][i] = C[m = m0 + wm*WM + a*16 + fr][n = n0 + wn*WN + b*16 + 4*fg + i].
            // Staged through LDS in passes of EPR rows (row pitch BN+4 floats: conflict-free b128 writes),
            // then every thread finishes 8 consecutive columns of a row: coalesced 16-B loads of resid/aux
            // and 16-B (or 2x16-B) stores, 4-8x fewer store instructions than the fragment layout.
            TO* C = reinterpret_cast<TO*>(g.C);
            constexpr int EPR = ep_rows<BM, BN, S, ROWB, WM>();
            static_assert(EPR % WM == 0 && BM % EPR == 0, "epilogue passes");
            constexpr int EPL = BN + 4;
            constexpr int NT = 64 * NW;
            constexpr int C8 = BN / 8;
            float* ep = reinterpret_cast<float*>(smem);
            float col_s = 0.f, col_q = 0.f;               // EPI_STATS: column tid's sums over the tile's rows
            // Epilogue operands (resid / aux / aux2) of a pass are all loaded before the tile is staged through
            // LDS (unconditional, row-clamped loads: no per-element branch or vmcnt(0)), so their latency
            // hides under the staging stores and barriers instead of being paid per row chunk.
            constexpr bool PRE = EPI == EPI_GELU_BWD || EPI == EPI_RESID || EPI == EPI_ADD_RELU_GRAD;
            constexpr int NCH = EPR * C8;                // 8-column chunks per pass
            constexpr int NIT = (NCH + NT - 1) / NT;
            using PA = typename std::conditional<EPI == EPI_RESID, float, T>::type;
            typedef PA pa8 __attribute__((ext_vector_type(8)));
            typedef T t8v __attribute__((ext_vector_type(8)));
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            const size_t tb = (size_t)m0 * g.N;              // the tile's first output row (pstore bases)
#pragma unroll 1
            for (int pass = 0; pass < BM / EPR; ++pass) {
                pa8 pre[PRE ? NIT : 1];
                t8v pre2[EPI == EPI_ADD_RELU_GRAD ? NIT : 1];
                if constexpr (PRE) {
                    const PA* src = EPI == EPI_RESID ? reinterpret_cast<const PA*>(g.resid) : reinterpret_cast<const PA*>(g.aux);
#pragma unroll
                    for (int k = 0; k < NIT; ++k) {
                        const int c = min(tid + k * NT, NCH - 1), r = c / C8, col = (c % C8) * 8;
                        const int m = min(m0 + pass * EPR + r, g.M - 1);
                        const size_t off = (size_t)m * g.N + n0 + col;
                        pre[k] = *reinterpret_cast<const pa8*>(src + off);
                        if constexpr (EPI == EPI_ADD_RELU_GRAD)
                            pre2[k] = *reinterpret_cast<const t8v*>(reinterpret_cast<const T*>(g.aux2) + off);
                    }
                }
                __syncthreads();
                if ((wm * WM) / EPR == pass) {
#pragma unroll
                    for (int a = 0; a < TM; ++a)
#pragma unroll
                        for (int b = 0; b < TN; ++b)
                            *reinterpret_cast<float4*>(ep + (wm * WM - pass * EPR + a * 16 + fr) * EPL + wn * WN + b * 16 + 4 * fg) =
                                make_float4(acc[a][b][0], acc[a][b][1], acc[a][b][2], acc[a][b][3]);
                }
                __syncthreads();
#pragma unroll
                for (int k = 0; k < NIT; ++k) {
                    const int c = tid + k * NT;
                    if (NCH % NT != 0 && c >= NCH) break;
                    const int r = c / C8, col = (c % C8) * 8;
                    const int m = m0 + pass * EPR + r;
                    if (m >= g.M) continue;
                    const int n = n0 + col;
                    const size_t off = (size_t)m * g.N + n;
                    const float4 x0 = *reinterpret_cast<const float4*>(ep + r * EPL + col);
                    const float4 x1 = *reinterpret_cast<const float4*>(ep + r * EPL + col + 4);
                    float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
                    if (g.bias) {
                        const float4 b0 = *reinterpret_cast<const float4*>(g.bias + n);
                        const float4 b1 = *reinterpret_cast<const float4*>(g.bias + n + 4);
                        v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
                        v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
                    }
                    if constexpr (EPI == EPI_GELU) {
                        if (g.aux) pstore<T, 8, AUX_POL>(reinterpret_cast<T*>(g.aux) + tb, (unsigned)(off - tb), v);
#pragma unroll
                        for (int i = 0; i < 8; ++i) v[i] = quick_gelu(v[i]);
                    } else if constexpr (EPI == EPI_GELU_BWD) {
#pragma unroll
                        for (int i = 0; i < 8; ++i) v[i] *= quick_gelu_grad((float)pre[k][i]);
                    } else if constexpr (EPI == EPI_ADD_RELU_GRAD) {
                        // decoder: conv1's input gradient plus the residual branch's (models/utils.py:300-302)
#pragma unroll
                        for (int i = 0; i < 8; ++i) v[i] += (float)pre2[k][i] > 0.f ? (float)pre[k][i] : 0.f;
                    } else if constexpr (EPI == EPI_RESID) {
#pragma unroll
                        for (int i = 0; i < 8; ++i) v[i] += pre[k][i];
                    }
                    pstore<TO, 8>(C + tb, (unsigned)(off - tb), v);
                }
                if constexpr (EPI == EPI_STATS) {
                    // BatchNorm batch statistics of the conv output (models/utils.py:254-303 bn1/bn2): per-tile
                    // column partials of sum and sum of squares, from the f32 accumulators (+ bias)
                    const int rows = min(EPR, g.M - (m0 + pass * EPR));
                    if (tid < BN) {
                        const float bc = g.bias ? g.bias[n0 + tid] : 0.f;
#pragma unroll 4
                        for (int r = 0; r < rows; ++r) {
                            const float x = ep[r * EPL + tid] + bc;
                            col_s += x;
                            col_q = fmaf(x, x, col_q);
                        }
                    }
                }
            }
            if constexpr (EPI == EPI_STATS) {
                if (tid < BN) {
                    g.stats[(size_t)tm * 2 * g.N + n0 + tid] = col_s;
                    g.stats[((size_t)tm * 2 + 1) * g.N + n0 + tid] = col_q;
                }
            }
            }   // staged epilogue (MODE 1 / 2)
        }   // fin
        EBC_GEMM_STAMP(3, tile);
        return nk;
    };
    const unsigned nk1 = (unsigned)segment(it_beg);
    if constexpr (SKM) {
        if (skr && it_beg + nk1 < it_end) {
            __syncthreads();     // every wave done with the ring and the epilogue's LDS before the next segment fills it
            segment(it_beg + nk1);
        }
    }
}

template <class E, class TO, int EPI, int BM, int BN, int S, int WGM, int WGN, int ROWB, int MODE, bool SPL, int NLW = 0>
int launch_gemm_k(const GemmArgs& g, hipStream_t st)
{
    constexpr int WM = BM / WGM;
    // EPI_LN / EPI_LN_BWD: the workgroup's row partials (BM rows of at most ln_pmax float2) past the ring; GELU_BWD:
    // the LayerNorm-backward fold's s / c column vectors (2 x 1-KiB-rounded)
    constexpr bool LNE = MODE == 0 && ln_pmax<EPI>() > 0;
    constexpr int RING = S * (BM + BN) * ROWB, LNB0 = LNE ? RING + BM * ln_pmax<EPI>() * 8 : 0;
    constexpr int BPB = MODE == 0 && EPI == EPI_GELU_BWD ? RING + 2 * ((BN * 4 + 1023) / 1024) * 1024 : 0;
    constexpr int LNB = LNB0 > BPB ? LNB0 : BPB;
    constexpr int LDS = gemm_lds_bytes<BM, BN, S, ROWB, WM>() > LNB ? gemm_lds_bytes<BM, BN, S, ROWB, WM>() : LNB;
    // (the LN_BWD instances of the 256-row tiles would need more: dispatch_tile never instantiates them)
    static_assert(LDS <= 160 * 1024, "LDS");
    {
    constexpr int BK = ROWB / E::BYTES;
    if (!ensure_lds<gemm_nt_kernel<E, TO, EPI, BM, BN, S, WGM, WGN, ROWB, MODE, SPL, NLW>>(LDS, st)) return EBC_E_LAUNCH;
    if (g.N % BN || g.kslice % BK || g.kslice * g.splits != g.K) return EBC_E_UNSUPPORTED;
    const int tiles = g.ntile ? g.ntile : ((g.M + BM - 1) / BM) * (g.N / BN) - g.tile0;
    if (tiles <= 0 || g.tile0 + tiles > ((g.M + BM - 1) / BM) * (g.N / BN)) return EBC_E_ARG;
    if (g.sk_total) {
        if (!SPL || MODE == 0 || g.splits != 1 || g.sk_nk * BK != g.K || (long)tiles * g.sk_nk != g.sk_total ||
            g.sk_grid < tiles || g.sk_grid > g.sk_total || (g.sk_total + 1) * g.sk_grid >= (1L << 31) || !g.cnt ||
            !g.part || tiles > 4096 ||
            (g.sk_share && (g.sk_share > g.sk_nk || (long)g.sk_grid != (g.sk_total + g.sk_share - 1) / g.sk_share)))
            return EBC_E_ARG;
    }
    const int nwg = g.sk_total ? g.sk_grid : tiles * g.splits;
    const int pi = probe_on() ? probe_start(EBC_PROBE_GEMM, EPI, BM, BN, MODE, g.M, g.N, g.kalg ? g.kalg : g.K, st) : -1;
    hipLaunchKernelGGL((gemm_nt_kernel<E, TO, EPI, BM, BN, S, WGM, WGN, ROWB, MODE, SPL, NLW>), dim3(nwg),
                       dim3(64 * (WGM * WGN + NLW)), LDS, st, g);
    probe_stop(pi, st);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
    }
}

// Split-K launches exist for the weight gradients (MODE 2, and MODE 0 f32 stores) and the conv GEMMs' tail tiles
// (MODE 1); every other product runs the split-free instance.
template <class E, class TO, int EPI, int BM, int BN, int S, int WGM = 2, int WGN = 2, int ROWB = 128, int MODE = 0, int NLW = 0>
int launch_gemm(const GemmArgs& g, hipStream_t st)
{
    if (g.splits > 1 || g.sk_total) {
        if constexpr (NLW == 0 && (MODE != 0 || EPI == EPI_STORE))
            return launch_gemm_k<E, TO, EPI, BM, BN, S, WGM, WGN, ROWB, MODE, true>(g, st);
        else return EBC_E_UNSUPPORTED;
    }
    return launch_gemm_k<E, TO, EPI, BM, BN, S, WGM, WGN, ROWB, MODE, false, NLW>(g, st);
}

}  // namespace
// tools/lab/gemm_lab.hip includes the kernel templates above without the dispatch and the C-ABI below
#ifndef EBC_GEMM_LAB
namespace {

// Tile configurations the heuristics below pick (the other shapes r01-r03 swept -- 256x128, 192x128, 128x192, 3- and
// 4-stage rings, 64-B K-row rings -- measured slower at every shape of this path; tools/lab/gemm_lab.hip times any):
//   1: 128x128/4w   2: 128x64/4w   3: 256x192/8w   4: 192x192/8w   5: 128x96/4w   7: 256x256/8w
//   (2-stage rings of 128-B K rows)   13: 128x96 S3 (conv weight gradients)
//   15: 128x96 S3 + 4 loader waves   16: 128x96 S4 + 4 loader waves   (r03, tools/lab/gemm_lab.hip)
// The L2 -> LDS fill rate per CU (~70 GB/s, MI355X_MICROARCH.md "gather into LDS") bounds a tile at
// BM*BN/(BM+BN) flop per byte, so the default takes the 256-wide tiles and splits K where the
// output has too few tiles to fill the 256 CUs.
struct TileCfg { int id, bm, bn; };
constexpr TileCfg CFGS[] = {{1, 128, 128}, {2, 128, 64}, {3, 256, 192}, {4, 192, 192}, {5, 128, 96}, {7, 256, 256},
                            {13, 128, 96}, {15, 128, 96}, {16, 128, 96}, {17, 224, 192}};
const TileCfg* find_cfg(int id) {
    for (const TileCfg& c : CFGS) if (c.id == id) return &c;
    return nullptr;
}

constexpr int NUM_CU = 256;
// split-K workspace: [0, GEMM_CNT_BYTES) per-tile arrival counters (zero on entry, left zero),
// then the f32 partial tiles
constexpr size_t GEMM_CNT_BYTES = 16 * 1024;

// heuristic tile choice for the 16-bit path; f32 (parity mode) always uses cfg 2
inline long ntiles(int M, int N, int bm, int bn) { return (long)((M + bm - 1) / bm) * (N / bn); }
int pick_cfg(int M, int N, int K, bool wide) {
    // Measured on MI355X at the ViT-B/16 shapes (M = 16 x 229; tools/gemm_bench.py, r01): the
    // 128x64 two-stage tile is best or within noise everywhere except the QKV projection (192x192,
    // 8 waves) and the long-K N = 768 products (128x96, 3 stages).  Split-K MODE 0 tiles (256x96, 256x256,
    // 256x128; r01-r03) were slower at every shape here (their epilogue and split fix-up dominate).
    if (!wide) return 2;
    // many-tile shapes (the sliding-window eval batch: M = 140 tiles x 229 tokens = 32060 rows; s5 sweep
    // tools/gpu72.sh): the 256-wide tiles win once they fill >= 1.5 waves of CUs -- qkv 161.6 -> 149.0 us,
    // out-proj 88.1 -> 66.4, c_fc 236.0 -> 205.7 (256x256), c_proj 250.8 -> 173.4
    if (N % 256 == 0 && N >= 3072 && K <= 1024 && ntiles(M, N, 256, 256) >= 384) return 7;
    // the ResNet-50 decoder's 2048-wide 1x1 convs and the 2048 -> 1024 projection (M = B*56*56 rows): no
    // 192- or 96-wide tile divides N; 256x256 keeps the L2 -> LDS fill below the MFMA rate
    if (N % 256 == 0 && N % 192 != 0 && N >= 1024 && ntiles(M, N, 256, 256) >= 384) return 7;
    if (N % 192 == 0 && ntiles(M, N, 256, 192) >= 384) return 3;
    if (N % 192 == 0 && N % 256 != 0 && K <= 1024 && ntiles(M, N, 192, 192) >= 128) return 4;
    // r01 sweep: MLP c_fc / GELU' (N = 3072, K = 768): 256x192 27.6 / 31.9 us vs 34.3 / 37.0 (128x64);
    // QKV (N = 2304): 192x192 20.1 us vs 23.3 (256x192)
    if (N % 192 == 0 && N >= 3072 && K <= 1024 && ntiles(M, N, 256, 192) >= 160) return 3;
    // (not for N <= 768: the projection's dX, N = 768 / K = 512 over 16*784 rows, is 17.4 us on 128x64
    // vs 24.3 us on 192x192, s5 sweep tools/gpu65.sh)
    if (N % 192 == 0 && N > 768 && K <= 1024 && ntiles(M, N, 192, 192) >= 128) return 4;
    // the 1x1 projection conv 768 -> 512 (f32 out, 16*784 rows): 128x128 18.9 us vs 23.3 us on 128x64
    if (N % 128 == 0 && N <= 512 && K <= 1024 && ntiles(M, N, 128, 128) >= 256) return 1;
    // decoder 3x3 convs as implicit GEMM (M = B*784, K = 9*768): one wave of 256x192 tiles
    if (N % 192 == 0 && K >= 4096 && ntiles(M, N, 256, 192) >= 160) return 3;
    // s5 re-sweep (tools/gpu63.sh): the N = 768, K = 768 products (out-proj + residual, its dX) are also
    // faster on 128x96 S3 than on 128x64: 13.6 -> 12.1 us / 9.1 -> 8.9 us
    // with more than one wave of 128x96 tiles (32 crops per GPU, SURVEY config 4: M = 7328) the 2-stage ring
    // wins: two workgroups fit a CU (56 KB of LDS instead of 84), s5 sweep tools/gpu78.sh: c_proj + residual
    // 51.5 -> 44.2 us, out-proj 21.9 -> 18.9, dH2 44.2 -> 37.8, dH 33.2 -> 29.5
    // r03 (tools/lab/gemm_lab.hip, interleaved, each launch right after the c_fc product as in the step): with 4
    // loader waves issuing the LDS-DMA pieces (gemm_nt_kernel NLW) the compute waves only read fragments and
    // issue MFMAs -- c_proj + residual 28.5 -> 26.6 us (4-stage ring), its dX 26.3 -> 24.0, dX of QKV 20.7 ->
    // 19.6, out-proj + residual 14.7 -> 14.2 (3 stages); 7 loader waves or a 5-stage ring gained nothing more.
    // More than one wave of tiles keeps the 2-stage 4-wave tile (two workgroups a CU).
    if (N % 96 == 0 && N < 2048 && K >= 768) return ntiles(M, N, 128, 96) > NUM_CU ? 5 : (K >= 2304 ? 16 : 15);
    return 2;
}
// Tile order for the wide-N products (>= 12 tile columns): with the row-major order each XCD's 1/8 of the
// tiles spans one or two whole tile rows, so every XCD fetches all of B (c_fc: 46 MB fetched for 10.4 MB
// of operands, PMC).  Grouping tile rows makes the XCD blocks squarer: the L2-miss bytes
// A*ntn*GM/C + B*ntm/GM (C = tiles per XCD) are minimal at GM = sqrt(C * BN / BM).
int group_rows(int M, int N, int bm, int bn, int splits) {
    const long ntm = (M + bm - 1) / bm, ntn = N / bn;
    if (ntn < 12 || splits > 1) return 0;
    const double C = (double)(ntm * ntn) / 8.0;
    const int gm = (int)(sqrt(C * bn / bm) + 0.5);
    return gm > 1 && gm < ntm ? gm : 0;
}
// the tile configuration a MODE 0 product runs
int select_cfg(bool sixteen, int M, int N, int K) { return pick_cfg(M, N, K, sixteen); }

template <class E, class TO, int EPI>
int dispatch_tile(GemmArgs g, void* /*ws*/, size_t /*ws_bytes*/, hipStream_t st)
{
    constexpr bool SIXTEEN = E::BYTES == 2;
    int cfg = select_cfg(SIXTEEN, g.M, g.N, g.K);
    // EPI_LN_BWD stages BM rows x 32 partial pairs past the ring: the 256-row tiles the many-tile shapes pick (M >= ~24k
    // rows, e.g. 30 crops of 448) would need 180 KB of LDS, so those shapes run the 128x96 tile (several waves of
    // tiles there).  The tile of this product is free: the partials' count comes from the GELU' product's tiling.
    if (EPI == EPI_LN_BWD && (cfg == 3 || cfg == 7)) cfg = 5;
    const TileCfg* c = find_cfg(cfg);
    g.splits = 1;
    g.kslice = g.K;
    g.group_m = group_rows(g.M, g.N, c->bm, c->bn, 1);
    switch (cfg) {
        case 1: return launch_gemm<E, TO, EPI, 128, 128, 2>(g, st);
        case 2: return launch_gemm<E, TO, EPI, 128, 64, 2>(g, st);
        case 4: return launch_gemm<E, TO, EPI, 192, 192, 2, 4, 2>(g, st);
        case 5: return launch_gemm<E, TO, EPI, 128, 96, 2>(g, st);
    }
    if constexpr (EPI != EPI_LN_BWD) {
        switch (cfg) {
            case 3: return launch_gemm<E, TO, EPI, 256, 192, 2, 4, 2>(g, st);
            case 7: return launch_gemm<E, TO, EPI, 256, 256, 2, 4, 2>(g, st);
        }
    }
    if constexpr (SIXTEEN) {
        switch (cfg) {
            case 15: return launch_gemm<E, TO, EPI, 128, 96, 3, 2, 2, 128, 0, 4>(g, st);
            case 16: return launch_gemm<E, TO, EPI, 128, 96, 4, 2, 2, 128, 0, 4>(g, st);
        }
    }
    return EBC_E_UNSUPPORTED;
}

template <class E, int EPI>
int dispatch_out(const GemmArgs& g, int out_f32, void* ws, size_t wsb, hipStream_t st)
{
    if (out_f32) return dispatch_tile<E, float, EPI>(g, ws, wsb, st);
    return dispatch_tile<E, typename E::T, EPI>(g, ws, wsb, st);
}

template <class E>
int dispatch_epi(const GemmArgs& g, int epi, int out_f32, void* ws, size_t wsb, hipStream_t st)
{
    switch (epi) {
        case EPI_STORE: return dispatch_out<E, EPI_STORE>(g, out_f32, ws, wsb, st);
        case EPI_GELU: return out_f32 ? EBC_E_UNSUPPORTED : dispatch_tile<E, typename E::T, EPI_GELU>(g, ws, wsb, st);
        case EPI_RESID: return out_f32 ? dispatch_tile<E, float, EPI_RESID>(g, ws, wsb, st)
                                       : dispatch_tile<E, typename E::T, EPI_RESID>(g, ws, wsb, st);
        case EPI_GELU_BWD: return out_f32 ? EBC_E_UNSUPPORTED : dispatch_tile<E, typename E::T, EPI_GELU_BWD>(g, ws, wsb, st);
        case EPI_LN:
            if constexpr (E::BYTES == 2) return out_f32 ? EBC_E_UNSUPPORTED : dispatch_tile<E, typename E::T, EPI_LN>(g, ws, wsb, st);
            return EBC_E_UNSUPPORTED;
        case EPI_LN_GELU:
            if constexpr (E::BYTES == 2) return out_f32 ? EBC_E_UNSUPPORTED : dispatch_tile<E, typename E::T, EPI_LN_GELU>(g, ws, wsb, st);
            return EBC_E_UNSUPPORTED;
        case EPI_LN_BWD:
            if constexpr (E::BYTES == 2) return out_f32 ? dispatch_tile<E, float, EPI_LN_BWD>(g, ws, wsb, st) : EBC_E_UNSUPPORTED;
            return EBC_E_UNSUPPORTED;
    }
    return EBC_E_ARG;
}

// implicit-GEMM 3x3 convolution tiles (MODE 1 / 2): 256x192 (8 waves) for the big decoder shapes,
// 128x96 / 128x64 otherwise; f32 (parity mode) 128x64
template <class E, class TO, int EPI, int MODE>
int launch_conv_tile(const GemmArgs& g, int cfg, hipStream_t st)
{
    if (cfg == 2) return launch_gemm<E, TO, EPI, 128, 64, 2, 2, 2, 128, MODE>(g, st);
    if constexpr (E::BYTES == 2) {
#if EBC_CONV_LAB_W4   // lab only (0 in the library): 4-wave conv tiles, one 128x96 / 112x96 wave tile a SIMD
        if (cfg == 3) return launch_gemm<E, TO, EPI, 256, 192, 2, 2, 2, 128, MODE>(g, st);
#else
        if (cfg == 3) return launch_gemm<E, TO, EPI, 256, 192, 2, 4, 2, 128, MODE>(g, st);
#endif
        if (cfg == 7) return launch_gemm<E, TO, EPI, 256, 256, 2, 4, 2, 128, MODE>(g, st);
        if (cfg == 13) return launch_gemm<E, TO, EPI, 128, 96, 3, 2, 2, 128, MODE>(g, st);
        if constexpr (MODE == 1) {
#if EBC_CONV_LAB_W4
            if (cfg == 17) return launch_gemm<E, TO, EPI, 224, 192, 2, 2, 2, 128, MODE>(g, st);
#else
            if (cfg == 17) return launch_gemm<E, TO, EPI, 224, 192, 2, 2, 4, 128, MODE>(g, st);
#endif
        }
    }
    return EBC_E_UNSUPPORTED;
}

// Weight-gradient products (MODE 2 conv dW, and ebc_gemm_wgrad's 1x1 dW): small outputs, long K (pixels).
// Tile and split-K are chosen on a cost model of the measured limits -- the L2 -> LDS fill (~70 GB/s per CU,
// MI355X_MICROARCH.md), ~8 TFLOP/s of MFMA per CU, whole waves of CUs -- plus the split's reduction: a
// last-arriver re-read through one CU for 2 splits, else f32 partials summed by a separate grid-wide launch.
// (r02: the RN50 encoder's 64 x 576 x 107520 conv dW ran one 256x192 tile x 8 splits: 267 us, 30 TFLOP/s.)
struct WPlan { int cfg, splits; bool partials; };
double wplan_cost(const TileCfg& c, int occ, int eb, int M, int N, int K, int s) {
    const long tiles = ntiles(M, N, c.bm, c.bn), wgs = tiles * s;
    const double ks = (double)K / s;
    const double fill = (double)(c.bm + c.bn) * ks * eb / 70e9, mma = 2.0 * c.bm * c.bn * ks / 8e12;
    const long slots = (long)NUM_CU * occ;
    const long rounds = (wgs + slots - 1) / slots;
    const int per_cu = (int)std::min<long>(occ, (wgs + NUM_CU - 1) / NUM_CU);
    double t = rounds * per_cu * std::max(fill, mma);
    if (s == 2) t += (double)c.bm * c.bn * 4 / 70e9;                       // last arriver re-reads one partial
    else if (s > 2) t += (double)(s + 1) * M * N * 4 / 4e12 + 4e-6;        // partials + reduce launch
    return t;
}
WPlan wgrad_plan(bool sixteen, bool conv, int M, int N, int K) {
    const int bk = sixteen ? 64 : 32, nk = K / bk, eb = sixteen ? 2 : 4;
    // (cfg, CUs' worth of LDS: workgroups per CU)
    static const int cand16_conv[][2] = {{3, 1}, {7, 1}, {13, 1}, {2, 3}};
    static const int cand16_gemm[][2] = {{7, 1}, {3, 1}, {1, 2}, {2, 3}};
    static const int cand32[][2] = {{2, 3}};
    const int (*cand)[2] = !sixteen ? cand32 : (conv ? cand16_conv : cand16_gemm);
    const int ncand = !sixteen ? 1 : 4;
    WPlan best{2, 1, false};
    double bt = 1e30;
    for (int i = 0; i < ncand; ++i) {
        const TileCfg* c = find_cfg(cand[i][0]);
        if (N % c->bn) continue;
        for (int sp = 1; sp <= 128; ++sp) {
            if (nk % sp || nk / sp < 8) continue;
            if (ntiles(M, N, c->bm, c->bn) * sp > 4L * NUM_CU) break;
            const double t = wplan_cost(*c, cand[i][1], eb, M, N, K, sp);
            if (t < bt * 0.98) { bt = t; best = WPlan{c->id, sp, sp > 2}; }
        }
    }
    return best;
}
size_t wplan_ws(const WPlan& w, int M, int N) {
    if (w.splits <= 1) return 0;
    const TileCfg* c = find_cfg(w.cfg);
    if (w.partials) return GEMM_CNT_BYTES + (size_t)w.splits * M * N * 4;
    return GEMM_CNT_BYTES + (size_t)w.splits * ntiles(M, N, c->bm, c->bn) * c->bm * c->bn * 4;
}
// C[e] = sum over splits of part[split][e] (split order), f32, 4 per thread
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
int splitk_reduce(const float* part, float* C, long MN, int splits, hipStream_t st) {
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((MN / 4 + 255) / 256)), dim3(256), 0, st, part, C, MN, splits);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

int conv_cfg(bool sixteen, int mode, int M, int N)
{
    if (!sixteen) return 2;
    // ResNet-50 decoder 3x3 conv (C = N = 2048, M = B*56*56): 256x256 tiles, several waves of them
    if (mode == 1 && N % 256 == 0 && N % 192 != 0 && ntiles(M, N, 256, 256) >= 256) return 7;
    // r01: 160x256 tiles (237 instead of 196 tiles at M = 16*784, N = 768) measured only 2-3 % faster on the
    // forward convs (their 80x64 wave tiles lose per-CU throughput), not kept
    // fewer 256x192 tiles than CUs (16 crops: 196): 224x192 tiles fill more of them (224), 131.8-136.6 vs 138.1-138.6 us
    // (store epilogue, interleaved, profiles/r04d_conv_lab_16crops.txt); more tiles than CUs keep 256x192 (stream-K)
    if (mode == 1 && N % 192 == 0 && ntiles(M, N, 256, 192) >= 160 && ntiles(M, N, 256, 192) < NUM_CU &&
        ntiles(M, N, 224, 192) <= NUM_CU)
        return 17;
    if (N % 192 == 0 && (mode == 2 || ntiles(M, N, 256, 192) >= 160)) return 3;
    return N % 96 == 0 ? 13 : 2;
}
// Stream-K for the implicit-GEMM convolutions (one 256-wide 8-wave workgroup per CU): when the launch's workgroups
// fill their last wave of CUs poorly, a grid of up to NUM_CU workgroups shares the k-tiles of the tiles past the
// last whole wave evenly (the whole waves run first as a plain launch of whole tiles, `dp`); a tile cut between
// workgroups is summed by the last piece to arrive (gemm_nt_kernel, SKM), at most 4 pieces a tile: the last piece
// re-reads the others' partials through one CU (the ResNet-50 decoder's 16 tail tiles of 288 k-tiles: 64
// workgroups, not 256 pieces of 18 k-tiles re-read 16-deep).  Where it is taken, measured (tools/lab/conv_lab.hip,
// interleaved, profiles/r04d_conv_lab_*.txt):
//   MODE 1 with more tiles than CUs: 32 crops, 392 256x192 tiles (1.53 waves): 244-248 us vs 266-278 plain
//     (fewer tiles than CUs, 16 crops' 196: 140-143 us vs 138-142 plain -- no gain, not taken)
//   MODE 2 up to 256 k-tiles a tile: the 16-crop weight gradient (108 tiles x 196 k-tiles): 140-143 us vs 144-152
//     on 2 splits (216 workgroups); 32 crops (392 k-tiles): 269-272 us vs 247-253 on 2 splits, not taken
//   MODE 2 shares aligned to few k offsets (r05, `share`): with R(w) = w * total / grid every workgroup starts at its own
//     offset inside its tile, so no two walk the same k-slice of a shared panel at the same time (r04 PMC: 968.7 MB per
//     launch beyond L2, hit rate 0.32).  A share of exactly `share` k-tiles, the multiple of nk / F (F distinct offsets)
//     nearest above total / NUM_CU: 108 tiles x 196 k-tiles -> 84 (F = 7, 252 workgroups); the workgroups w, w + 7,
//     w + 14, .. of one XCD then start at one offset, on tiles 3 apart in one tile row (one A panel).
struct SkPlan { int dp; long total; int nk, grid, share; };
int sk_share_for(long total, long nk) {
    const long lo = (total + NUM_CU - 1) / NUM_CU;
    int best = 0;
    long bestF = nk + 1;
    for (long s = lo; s <= lo + lo / 32 && s <= nk; ++s) {              // at most ~3 % over the even share
        long a = s, b = nk;
        while (b) { const long t = a % b; a = b; b = t; }                 // gcd(s, nk)
        if (nk / a < bestF) { bestF = nk / a; best = (int)s; }
    }
    return bestF <= 16 ? best : 0;
}
SkPlan sk_plan(int mode, int cfg, int M, int N, int K, int bk, long wgs) {
    if (cfg != 3 && cfg != 7) return SkPlan{0, 0, 0, 0, 0};
    const TileCfg* c = find_cfg(cfg);
    const long T = ntiles(M, N, c->bm, c->bn), nk = K / bk;
    const long waves = (wgs + NUM_CU - 1) / NUM_CU;
    const double fill = (double)wgs / (double)(waves * NUM_CU);
    const long dp = T / NUM_CU * NUM_CU, rest = T - dp;
    if (mode == 1 ? dp == 0 : nk > 256) return SkPlan{0, 0, 0, 0, 0};
    int grid = (int)std::min<long>(NUM_CU, rest * 4);
    if (fill >= 0.92 || rest == 0 || rest * nk < 16L * grid) return SkPlan{0, 0, 0, 0, 0};
    const int share = mode == 2 ? sk_share_for(rest * nk, nk) : 0;
    if (share) grid = (int)((rest * nk + share - 1) / share);
    return SkPlan{(int)dp, rest * nk, (int)nk, grid, share};
}
size_t sk_ws_bytes(int cfg, const SkPlan& p) {
    const TileCfg* c = find_cfg(cfg);
    return p.total ? (size_t)2 * p.grid * c->bm * c->bn * 4 : 0;
}
// conv workspace: [arrival counters][EPI_STATS per-tile-row partials (BM >= 128)][stream-K partials]
size_t conv_stats_bytes(int M, int N) { return (((size_t)((M + 127) / 128) * 2 * N * 4 + 255) / 256) * 256; }
int conv_splits(int cfg, int mode, int M, int N, int nk)
{
    if (mode != 2) return 1;
    const TileCfg* c = find_cfg(cfg);
    const long tiles = ntiles(M, N, c->bm, c->bn);
    int s = 1;
    while (tiles * (s + 1) <= NUM_CU * 6 / 5 && nk % (s + 1) == 0 && nk / (s + 1) >= 16) ++s;
    return s;
}

template <class E>
int dispatch_conv(GemmArgs g, int mode, int epi, void* ws, size_t wsb, hipStream_t st)
{
    constexpr bool SIXTEEN = E::BYTES == 2;
    const bool planned = mode == 2;
    const WPlan wp = planned ? wgrad_plan(SIXTEEN, true, g.M, g.N, g.K) : WPlan{0, 1, false};
    const int cfg = planned ? wp.cfg : conv_cfg(SIXTEEN, mode, g.M, g.N);
    const int BK = 128 / E::BYTES;
    const TileCfg* c = find_cfg(cfg);
    if (g.N % c->bn || g.K % BK) return EBC_E_UNSUPPORTED;
    if (planned && wp.partials) {
        if (!ws || wsb < wplan_ws(wp, g.M, g.N)) return EBC_E_ARG;
        g.part = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + GEMM_CNT_BYTES);
        g.cnt = nullptr;
        g.splits = wp.splits;
        g.kslice = g.K / wp.splits;
        EBC_TRY((launch_conv_tile<E, float, EPI_STORE, 2>(g, cfg, st)));
        return splitk_reduce(g.part, reinterpret_cast<float*>(g.C), (long)g.M * g.N, wp.splits, st);
    }
    int splits = planned ? wp.splits : conv_splits(cfg, mode, g.M, g.N, g.K / BK);
    using T = typename E::T;
    if (SIXTEEN) {
        const SkPlan sk = sk_plan(mode, cfg, g.M, g.N, g.K, BK, ntiles(g.M, g.N, c->bm, c->bn) * splits);
        const size_t off = GEMM_CNT_BYTES + (mode == 1 ? conv_stats_bytes(g.M, g.N) : 0);
        if (sk.total && ws && wsb >= off + sk_ws_bytes(cfg, sk)) {
            g.splits = 1;
            g.kslice = g.K;
            if (sk.dp) {
                GemmArgs d = g;
                d.ntile = sk.dp;
                if (mode == 1 && epi == EPI_STORE) EBC_TRY((launch_conv_tile<E, T, EPI_STORE, 1>(d, cfg, st)));
                else if (mode == 1 && epi == EPI_STATS) EBC_TRY((launch_conv_tile<E, T, EPI_STATS, 1>(d, cfg, st)));
                else if (mode == 1 && epi == EPI_ADD_RELU_GRAD) EBC_TRY((launch_conv_tile<E, T, EPI_ADD_RELU_GRAD, 1>(d, cfg, st)));
                else if (mode == 2 && epi == EPI_STORE) EBC_TRY((launch_conv_tile<E, float, EPI_STORE, 2>(d, cfg, st)));
                else return EBC_E_UNSUPPORTED;
                g.tile0 = sk.dp;
            }
            g.sk_total = sk.total;
            g.sk_nk = sk.nk;
            g.sk_grid = sk.grid;
            g.sk_share = sk.share;
            g.cnt = reinterpret_cast<int*>(ws);
            g.part = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + off);
            if (mode == 1 && epi == EPI_STORE) return launch_conv_tile<E, T, EPI_STORE, 1>(g, cfg, st);
            if (mode == 1 && epi == EPI_STATS) return launch_conv_tile<E, T, EPI_STATS, 1>(g, cfg, st);
            if (mode == 1 && epi == EPI_ADD_RELU_GRAD) return launch_conv_tile<E, T, EPI_ADD_RELU_GRAD, 1>(g, cfg, st);
            if (mode == 2 && epi == EPI_STORE) return launch_conv_tile<E, float, EPI_STORE, 2>(g, cfg, st);
            return EBC_E_UNSUPPORTED;
        }
    }
    if (splits > 1) {
        const size_t tiles = (size_t)ntiles(g.M, g.N, c->bm, c->bn);
        const size_t need = GEMM_CNT_BYTES + (size_t)splits * tiles * c->bm * c->bn * 4;
        if (!ws || wsb < need || tiles > GEMM_CNT_BYTES / 4) {
            splits = 1;
        } else {
            g.cnt = reinterpret_cast<int*>(ws);
            g.part = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + GEMM_CNT_BYTES);
        }
    }
    g.splits = splits;
    g.kslice = g.K / splits;
    if (mode == 1 && epi == EPI_STORE) return launch_conv_tile<E, T, EPI_STORE, 1>(g, cfg, st);
    if (mode == 1 && epi == EPI_STATS) return launch_conv_tile<E, T, EPI_STATS, 1>(g, cfg, st);
    if (mode == 1 && epi == EPI_ADD_RELU_GRAD) return launch_conv_tile<E, T, EPI_ADD_RELU_GRAD, 1>(g, cfg, st);
    if (mode == 2 && epi == EPI_STORE) return launch_conv_tile<E, float, EPI_STORE, 2>(g, cfg, st);
    return EBC_E_UNSUPPORTED;
}

}  // namespace

namespace ebc {
size_t conv_gemm_workspace_bytes(int dtype, int mode, int M, int N, int K)
{
    const bool sixteen = dtype != EBC_F32;
    size_t need = GEMM_CNT_BYTES;
    if (mode == 1) {
        need += conv_stats_bytes(M, N);                                // EPI_STATS partials (BM >= 128)
        if (sixteen) {
            const int cfg = conv_cfg(sixteen, mode, M, N);
            const TileCfg* c = find_cfg(cfg);
            need += sk_ws_bytes(cfg, sk_plan(mode, cfg, M, N, K, 64, ntiles(M, N, c->bm, c->bn)));
        }
    }
    if (mode == 2) {
        const WPlan wp = wgrad_plan(sixteen, true, M, N, K);
        size_t skb = 0;
        if (sixteen && !wp.partials) {
            const TileCfg* c = find_cfg(wp.cfg);
            skb = GEMM_CNT_BYTES + sk_ws_bytes(wp.cfg, sk_plan(2, wp.cfg, M, N, K, 64, ntiles(M, N, c->bm, c->bn) * wp.splits));
        }
        return std::max({need, wplan_ws(wp, M, N), skb});
    }
    const int cfg = conv_cfg(sixteen, mode, M, N);
    const TileCfg* c = find_cfg(cfg);
    const int bk = !sixteen ? 32 : 64;
    const int s = conv_splits(cfg, mode, M, N, K / bk);
    if (s > 1) need = std::max(need, GEMM_CNT_BYTES + (size_t)s * ntiles(M, N, c->bm, c->bn) * c->bm * c->bn * 4);
    return need;
}

int conv_gemm(int dtype, int mode, int epi, const void* A, const void* B, void* C, const ConvGeom& geo, int M, int N,
              int K, void* ws, size_t wsb, int* stats_tiles, hipStream_t st, const void* gy, const void* y)
{
    if (epi == EPI_ADD_RELU_GRAD && (!gy || !y)) return EBC_E_ARG;
    const int bk = dtype == EBC_F32 ? 32 : 64;
    if (M <= 0 || N <= 0 || K <= 0 || K % bk || N % 64 || !A || !B || !C || (mode != 1 && mode != 2)) return EBC_E_ARG;
    GemmArgs g{A, B, C, nullptr, nullptr, const_cast<void*>(gy), M, N, K};
    g.aux2 = y;
    g.cH = geo.H; g.cW = geo.W; g.cC = geo.C; g.cHp = geo.Hp; g.cWp = geo.Wp;
    if (mode == 1 && geo.C % bk) return EBC_E_UNSUPPORTED;
    if (mode == 2) {
        // a 16-B K chunk (8 16-bit / 4 f32 columns) must stay inside one image
        if (geo.HWp < 64 || geo.HWp % 8 || geo.Pimg < (long)geo.HWp || geo.Qs < (long)K) return EBC_E_ARG;
        g.cHWp = geo.HWp; g.cQs = geo.Qs; g.cPimg = geo.Pimg;
        g.kalg = geo.nimg * geo.H * geo.W;                                    // B * H * W interior pixels
    }
    if (epi == EPI_STATS) {
        if (!ws || wsb < conv_gemm_workspace_bytes(dtype, mode, M, N, K)) return EBC_E_ARG;
        g.stats = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + GEMM_CNT_BYTES);
        const TileCfg* c = find_cfg(conv_cfg(dtype != EBC_F32, mode, M, N));
        if (stats_tiles) *stats_tiles = (M + c->bm - 1) / c->bm;
    }
    switch (dtype) {
        case EBC_F32: return dispatch_conv<EF32>(g, mode, epi, ws, wsb, st);
        case EBC_F16: return dispatch_conv<EF16>(g, mode, epi, ws, wsb, st);
        case EBC_BF16: return dispatch_conv<EBF16>(g, mode, epi, ws, wsb, st);
    }
    return EBC_E_ARG;
}

size_t gemm_workspace_bytes(int, int, int, int)
{
    return 0;             // the MODE 0 products never split K (see pick_cfg), so they take no workspace
}

int gemm_nt(int dtype, int epi, int out_f32, const void* A, const void* B, void* C, const float* bias,
            const float* resid, void* aux, int M, int N, int K, hipStream_t st, void* ws, size_t ws_bytes,
            int a_rpg, int a_gstride, int a_goff)
{
    const int bk = dtype == EBC_F32 ? 32 : 64;
    if (M <= 0 || N <= 0 || K <= 0 || K % bk != 0 || N % 64 != 0 || !A || !B || !C) return EBC_E_ARG;
    if ((epi == EPI_RESID && !resid) || (epi == EPI_GELU_BWD && !aux)) return EBC_E_ARG;
    if (a_rpg < 0 || (a_rpg > 0 && (a_goff < 0 || a_goff + a_rpg > a_gstride || epi != EPI_STORE))) return EBC_E_ARG;
    GemmArgs g{A, B, C, bias, resid, aux, M, N, K};
    g.a_rpg = a_rpg; g.a_gstride = a_gstride; g.a_goff = a_goff;
    switch (dtype) {
        case EBC_F32: return dispatch_epi<EF32>(g, epi, 0, nullptr, 0, st);   // element type is already f32
        case EBC_F16: return dispatch_epi<EF16>(g, epi, out_f32, ws, ws_bytes, st);
        case EBC_BF16: return dispatch_epi<EBF16>(g, epi, out_f32, ws, ws_bytes, st);
    }
    return EBC_E_ARG;
}

bool gemm_ln_bwd_fold_pays(int dtype, int M, int N, int K)
{
    // The EPI_LN_BWD product stages BM x 32 row partials (32 KB at BM = 128) past its ring.  On the loader-wave tiles
    // (cfg 15 / 16: one workgroup a CU anyway, at most one wave of tiles) that costs no occupancy; on the 2-stage 4-wave
    // tile the many-tile shapes take (cfg 5: two workgroups a CU at 57 KB) it halves the workgroups a CU holds: 32
    // crops (M = 7328) ran the folded c_fc dX at 86 us against 45 + 16 us for the product + LayerNorm launch pair, bench
    // 3923 vs 4082 crops/s (r06h, profiles/r06h_ln_bwd_fold_32crops.txt).  The fold is taken where it pays.
    const int cfg = select_cfg(dtype != EBC_F32, M, N, K);
    return cfg == 15 || cfg == 16;
}

int gemm_rowstat_parts(int dtype, int M, int N, int K)
{
    const TileCfg* c = find_cfg(select_cfg(dtype != EBC_F32, M, N, K));
    return N / c->bn * 2;                       // every MODE 0 tile configuration has 2 wave columns
}

int gemm_nt_ln(int dtype, int epi, int out_f32, const void* A, const void* B, void* C, const float* bias,
               const float* resid, void* aux, int M, int N, int K, hipStream_t st, void* ws, size_t ws_bytes,
               const GemmLn& ln)
{
    const int bk = dtype == EBC_F32 ? 32 : 64;
    if (dtype == EBC_F32 || M <= 0 || N <= 0 || K <= 0 || K % bk != 0 || N % 64 != 0 || !A || !B || !C) return EBC_E_ARG;
    GemmArgs g{A, B, C, bias, resid, aux, M, N, K};
    if (epi == EPI_RESID) {
        if (!resid || !out_f32 || !ln.xh || !ln.rpart) return EBC_E_ARG;
        g.xh = ln.xh;
        g.rpart = ln.rpart;
        if (ln.vrep) {
            if (ln.vrep_L <= 0 || ln.vrep_nv <= 0 || ln.vrep_nv >= ln.vrep_L || ln.vrep_bs < 0) return EBC_E_ARG;
            g.vrep = ln.vrep; g.vrep_bs = ln.vrep_bs; g.vrep_L = ln.vrep_L; g.vrep_nv = ln.vrep_nv;
        }
    } else if (epi == EPI_LN || epi == EPI_LN_GELU) {
        if (out_f32 || !ln.lnp || !ln.lnw || ln.lnparts <= 0 || ln.lnparts > LN_PMAX || ln.lnparts % 2 || !ln.mean != !ln.rstd) return EBC_E_ARG;
        g.lnp = ln.lnp;
        g.lnparts = ln.lnparts;
        g.lnw = ln.lnw;
        g.ln_mean = ln.mean;
        g.ln_rstd = ln.rstd;
    } else if (epi == EPI_GELU_BWD) {
        // the LayerNorm-backward partials of the next product (bpart [M][gemm_rowstat_parts][2])
        if (out_f32 || !aux || !ln.bpart || !ln.lnb_s || !ln.lnb_c) return EBC_E_ARG;
        g.bpart = ln.bpart;
        g.lnb_s = ln.lnb_s;
        g.lnb_c = ln.lnb_c;
    } else if (epi == EPI_LN_BWD) {
        if (!out_f32 || !resid || !ln.xh || !ln.lnx || !ln.lnp || ln.lnparts <= 0 || ln.lnparts > LN_PMAX_B ||
            ln.lnparts % 2 || !ln.mean || !ln.rstd || bias)
            return EBC_E_ARG;
        g.xh = ln.xh;
        g.lnx = ln.lnx;
        g.lnp = ln.lnp;
        g.lnparts = ln.lnparts;
        g.ln_mean = ln.mean;
        g.ln_rstd = ln.rstd;
    } else {
        return EBC_E_ARG;
    }
    switch (dtype) {
        case EBC_F16: return dispatch_epi<EF16>(g, epi, out_f32, ws, ws_bytes, st);
        case EBC_BF16: return dispatch_epi<EBF16>(g, epi, out_f32, ws, ws_bytes, st);
    }
    return EBC_E_ARG;
}
}  // namespace ebc

namespace {
// weight-gradient GEMM (1x1 conv dW over K = pixels): tile and split-K from wgrad_plan
size_t wgrad_ws(int M, int N, int K, bool sixteen) {
    return wplan_ws(wgrad_plan(sixteen, false, M, N, K), M, N);
}
template <class E>
int wgrad_launch(GemmArgs g, void* ws, size_t wsb, hipStream_t st) {
    constexpr bool SIXTEEN = E::BYTES == 2;
    const WPlan wp = wgrad_plan(SIXTEEN, false, g.M, g.N, g.K);
    const TileCfg* c = find_cfg(wp.cfg);
    const int s = wp.splits;
    if (s > 1 && (!ws || wsb < wplan_ws(wp, g.M, g.N) || (!wp.partials && ntiles(g.M, g.N, c->bm, c->bn) > (long)(GEMM_CNT_BYTES / 4))))
        return EBC_E_ARG;
    if (s > 1) {
        g.cnt = wp.partials ? nullptr : reinterpret_cast<int*>(ws);
        g.part = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + GEMM_CNT_BYTES);
    }
    g.splits = s;
    g.kslice = g.K / s;
    g.group_m = 0;
    int rc = EBC_E_UNSUPPORTED;
    if constexpr (SIXTEEN) {
        switch (wp.cfg) {
            case 7: rc = launch_gemm<E, float, EPI_STORE, 256, 256, 2, 4, 2>(g, st); break;
            case 3: rc = launch_gemm<E, float, EPI_STORE, 256, 192, 2, 4, 2>(g, st); break;
            case 1: rc = launch_gemm<E, float, EPI_STORE, 128, 128, 2>(g, st); break;
            default: rc = launch_gemm<E, float, EPI_STORE, 128, 64, 2>(g, st); break;
        }
    } else {
        rc = launch_gemm<E, float, EPI_STORE, 128, 64, 2>(g, st);
    }
    if (rc || !(s > 1 && wp.partials)) return rc;
    return splitk_reduce(g.part, reinterpret_cast<float*>(g.C), (long)g.M * g.N, s, st);
}

// out[c][r] = in[r][c]: 64x64 tiles through LDS, 8-element (16 B for 16-bit) vectors both ways
template <class T>
__global__ __launch_bounds__(256) void transpose_kernel(const T* __restrict__ in, T* __restrict__ out, int R, int C, long ldo)
{
    __shared__ T sm[64][64 + 2];
    const int t = threadIdx.x, r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
    typedef T t8 __attribute__((ext_vector_type(8)));
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int e = t + 256 * k, rl = e >> 3, cl = (e & 7) * 8;
        if (r0 + rl < R && c0 + cl < C) {
            const t8 v = *reinterpret_cast<const t8*>(in + (size_t)(r0 + rl) * C + c0 + cl);
#pragma unroll
            for (int i = 0; i < 8; ++i) sm[rl][cl + i] = v[i];
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int e = t + 256 * k, cl = e >> 3, rl = (e & 7) * 8;
        if (c0 + cl < C && r0 + rl + 8 <= R) {
            t8 v;
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = sm[rl + i][cl];
            *reinterpret_cast<t8*>(out + (size_t)(c0 + cl) * ldo + r0 + rl) = v;
        } else if (c0 + cl < C && r0 + rl < R) {          // ragged last rows (R not a multiple of 8)
            for (int i = 0; r0 + rl + i < R; ++i) out[(size_t)(c0 + cl) * ldo + r0 + rl + i] = sm[rl + i][cl];
        }
    }
}
}  // namespace

extern "C" size_t ebc_gemm_wgrad_workspace_bytes(int dtype, int M, int N, int K)
{
    if (M <= 0 || N <= 0 || K <= 0) return 0;
    return wgrad_ws(M, N, K, dtype != EBC_F32);
}

extern "C" int ebc_gemm_wgrad(int dtype, const void* A, const void* B, float* C, int M, int N, int K,
                              void* workspace, size_t workspace_bytes, ebc_stream_t stream)
{
    const int bk = dtype == EBC_F32 ? 32 : 64;
    if (!A || !B || !C || M <= 0 || N <= 0 || K <= 0 || K % bk || N % 64) return EBC_E_ARG;
    GemmArgs g{A, B, C, nullptr, nullptr, nullptr, M, N, K};
    const hipStream_t st = (hipStream_t)stream;
    switch (dtype) {
        case EBC_F32: return wgrad_launch<EF32>(g, workspace, workspace_bytes, st);
        case EBC_F16: return wgrad_launch<EF16>(g, workspace, workspace_bytes, st);
        case EBC_BF16: return wgrad_launch<EBF16>(g, workspace, workspace_bytes, st);
    }
    return EBC_E_ARG;
}

extern "C" int ebc_transpose(int dtype, const void* in, void* out, int R, int C, long ld_out, ebc_stream_t stream)
{
    if (!in || !out || R <= 0 || C <= 0 || C % 8 || ld_out < R || ld_out % 8) return EBC_E_ARG;
    const dim3 grid((unsigned)((C + 63) / 64), (unsigned)((R + 63) / 64));
    const hipStream_t st = (hipStream_t)stream;
    switch (dtype) {
        case EBC_F32: hipLaunchKernelGGL(transpose_kernel<float>, grid, dim3(256), 0, st, (const float*)in, (float*)out, R, C, ld_out); break;
        case EBC_F16: hipLaunchKernelGGL(transpose_kernel<_Float16>, grid, dim3(256), 0, st, (const _Float16*)in, (_Float16*)out, R, C, ld_out); break;
        case EBC_BF16: hipLaunchKernelGGL(transpose_kernel<__bf16>, grid, dim3(256), 0, st, (const __bf16*)in, (__bf16*)out, R, C, ld_out); break;
        default: return EBC_E_ARG;
    }
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

extern "C" int ebc_gemm(int dtype, int epilogue, int out_f32, const void* A, const void* B, void* C,
                        const float* bias, const float* resid, void* aux, int M, int N, int K,
                        ebc_stream_t stream)
{
    return ebc::gemm_nt(dtype, epilogue, out_f32, A, B, C, bias, resid, aux, M, N, K, (hipStream_t)stream, nullptr, 0);
}

extern "C" size_t ebc_gemm_workspace_bytes(int dtype, int M, int N, int K)
{
    return ebc::gemm_workspace_bytes(dtype, M, N, K);
}

extern "C" int ebc_gemm_ws(int dtype, int epilogue, int out_f32, const void* A, const void* B, void* C,
                           const float* bias, const float* resid, void* aux, int M, int N, int K,
                           void* workspace, size_t workspace_bytes, ebc_stream_t stream)
{
    // workspace contract (include/ebc_hip.h): zero-filled before its first use, then owned by the
    // caller's stream; the kernels leave its counter block zero again after every call
    return ebc::gemm_nt(dtype, epilogue, out_f32, A, B, C, bias, resid, aux, M, N, K, (hipStream_t)stream,
                        workspace, workspace_bytes);
}

extern "C" int ebc_gemm_tile_config(int dtype, int M, int N, int K, int* out)
{
    if (M <= 0 || N <= 0 || K <= 0 || (dtype != EBC_F32 && dtype != EBC_F16 && dtype != EBC_BF16)) return EBC_E_ARG;
    const bool sixteen = dtype != EBC_F32;
    const int cfg = select_cfg(sixteen, M, N, K);
    const TileCfg* c = find_cfg(cfg);
    if (out) {
        out[0] = c->bm;
        out[1] = c->bn;
        out[2] = 1;
    }
    return cfg;
}

extern "C" int ebc_conv_tile_config(int dtype, int mode, int M, int N, int K, int* out)
{
    if (M <= 0 || N <= 0 || K <= 0 || (mode != 1 && mode != 2)) return EBC_E_ARG;
    const bool sixteen = dtype != EBC_F32;
    const int bk = !sixteen ? 32 : 64;
    int cfg, splits;
    if (mode == 2) {
        const WPlan wp = wgrad_plan(sixteen, true, M, N, K);
        cfg = wp.cfg;
        splits = wp.splits;
        if (wp.partials) splits = -splits;           // never stream-K: reported as split-K
    } else {
        cfg = conv_cfg(sixteen, mode, M, N);
        splits = conv_splits(cfg, mode, M, N, K / bk);
    }
    const TileCfg* c = find_cfg(cfg);
    if (splits < 0) {
        splits = -splits;
    } else if (sixteen) {
        // dispatch_conv: stream-K whenever sk_plan takes the launch (a workspace of conv_gemm_workspace_bytes)
        const SkPlan sk = sk_plan(mode, cfg, M, N, K, bk, ntiles(M, N, c->bm, c->bn) * splits);
        if (sk.total) splits = -sk.grid;
    }
    if (out) { out[0] = c->bm; out[1] = c->bn; out[2] = splits; }
    return cfg;
}
#endif  // EBC_GEMM_LAB
