// Fused DACE / DMCount loss for gfx950: one 1024-thread workgroup per crop, every Sinkhorn
// iteration on device, no host synchronisation.
//
// Reference: DACELoss.forward        losses/dace_loss.py:49-70  (+ _bin_count :42-47)
//            _reshape_density        losses/utils.py:4-9
//            DMLoss.forward          losses/dm_loss.py:99-124
//            OTLoss.forward          losses/dm_loss.py:38-79
//            sinkhorn                losses/bregman_pytorch.py:11-144
//
// Design:
//  * The DMCount cost is separable: C[i, iy*g+jx] = yd_i[iy] + xd_i[jx]
//    (dm_loss.py:53-59), so K = exp(C/-reg) = Ey_i[iy] * Ex_i[jx] with Ey = exp(yd/-reg),
//    Ex = exp(xd/-reg).  A crop's kernel matrix shrinks from n*g^2 to 2*n*g floats; the bucketed
//    path keeps only each point's 12-cell aligned window of Ey and Ex (2*n*12 floats), so a crop
//    stays LDS-resident up to ~1200 points (g = 28); wide windows or more points stream from L2.
//  * K^T u = (u*Ey)^T Ex is a dense [G x n] x [n x G] product, run as 4x4 register blocks over
//    b128 LDS reads with the points split across thread groups (partials summed by the v pass).
//  * exp(C/-reg) underflows to exactly 0 beyond ~32 px (reg = 10), so each point's factors are
//    nonzero on a <= 9-row x 9-column window: K v runs over those windows only, 8 lanes per point.
//  * The reference's control flow is kept exactly: err every eval_freq iterations
//    (bregman_pytorch.py:117-126), stop when err <= stopThr or it > maxIter, NaN/Inf rollback
//    to the previous (u, v) and break (:111-115), the 1e-16 epsilons, denormals kept (the build
//    never flushes f32 denormals).  The err pass's K^T u is reused by the next iteration.
#include <algorithm>
#include <type_traits>

#include "ebc_common.h"
#include "kernels.h"

using namespace ebc;

namespace {

// threads per workgroup (16 waves, 4 per SIMD): r02 measured the 100-iteration floor at 512 and 1024 threads the same,
// 256 threads 1.5x slower; 1024 keeps one pass over the cells / blocks per phase at G = 28
#ifndef EBC_DACE_NT
#define EBC_DACE_NT 1024
#endif
constexpr int NT = EBC_DACE_NT;
constexpr int LDS_MAX = 160 * 1024;
constexpr float M_EPS = 1e-16f;          // bregman_pytorch.py:8
#ifndef EBC_DACE_W16_MIN
#define EBC_DACE_W16_MIN 257
#endif
constexpr int SORTED_W16_MIN_POINTS = EBC_DACE_W16_MIN;   // crops from this many points: 16 lanes per block (r02 probe)
constexpr float EPS = 1e-8f;             // dm_loss.py:7

// Lab-only phase timer (-DEBC_DACE_PROF, tools/dbg/dace_prof.py): thread 0 of each crop's workgroup records core-clock
// stamps (s_memtime) at the crop body's phase boundaries and per-iteration phase sums; read by ebc_dace_prof_read.
#ifdef EBC_DACE_PROF
__device__ unsigned long long g_dace_prof[64][64];
#define PROF_AT(k) do { if (threadIdx.x == 0 && blockIdx.x < 64) g_dace_prof[blockIdx.x][k] = __builtin_amdgcn_s_memtime(); } while (0)
#define PROF_T() (__builtin_amdgcn_s_memtime())
#else
#define PROF_AT(k) do {} while (0)
#endif

// G = the LDS grid (a multiple of 4 >= the crop's density grid g = size / reduction); cells with a row or
// column >= g are dead: zero density, zero kernel factors, v = 0, never written out.
template <int G> struct Cfg {
    static_assert(G % 4 == 0, "LDS grid");
    static constexpr int GG = G * G;
    // K^T u: 4x4 cell blocks, the points split over KSPLIT thread groups whose partial sums live
    // in LDS (KSPLIT x GG) and are summed by the consumer (no atomics: LDS float atomics run at
    // ~3 cycles per lane).
    static constexpr int NB = (G / 4) * (G / 4);
    static constexpr int KSPLIT = 512 / NB;            // (sized for 512 threads: the dense fallback's LDS partials)
    // home buckets of the sorted Sinkhorn: one per BSxBS cell block; a <= 9-cell window starting in
    // block B reaches block B + HALO
    static constexpr int BS = 4, NB1 = G / BS, NBK = NB1 * NB1, HALO = 8 / BS;
    // fixed LDS (floats): pd, td, b, v0, v1, misc[64], bucket counts/starts, partial[KSPLIT][GG]
    static constexpr int BKT = (2 * NBK + 4 + 3) & ~3;
    static constexpr int FIXED = 5 * GG + 64 + BKT + KSPLIT * GG;
    static constexpr size_t FIXED_BYTES = (size_t)FIXED * 4;
    static constexpr int PER_POINT = 2 * G + 6;          // Ey, Ex (16-B aligned rows), u0, u1, window, key, x, y
    // bucketed path: factor rows cut to the 12 cells from the window's 4-aligned start (clamped to
    // G - 12): a <= 9-cell window starting at offset <= 3 fits, and a 4x4 block of any bucket that
    // gathers the point lies at offset 0, 4 or 8.  It needs only GG of the partials, so its factors
    // start at part + GG.
    static constexpr int CW = G < 12 ? G : 12;
    static constexpr int PER_POINT_C = 2 * CW + 6;
    static constexpr size_t FIXED_BYTES_C = (size_t)(5 * GG + 64 + BKT + GG) * 4;
};

// first cell of a point's compact factor row (window start lo, length len; 0 for an empty window)
template <int G, int CW>
__device__ __forceinline__ int row_base(int lo, int len) {
    if constexpr (CW == G) return 0;
    else return len ? min(lo & ~3, G - CW) : 0;
}

constexpr int HMETA_MAX = 64;
struct Params {
    const float* pred_class; const float* pred_density; const float* target_density;
    int target_is_reduced;
    const float* points; const int* offsets; const int* order;
    const float* bins_lo; const float* bins_hi;
    int B, N, size, red, count_mode, norm_cood;
    int g;                 // density grid size / red (<= the kernel's LDS grid G)
    float w_count, w_ot, w_tv, reg, stop_thr;
    int max_iter, eval_freq;
    float* grad_class; float* grad_density; float* crop_stats; float* beta_out; int* status;
    float* ws_factors;     // global factor storage for crops that do not fit LDS
    int lds_cap;           // max points kept in LDS with full factor rows (dense path)
    int lds_cap_s;         // max points kept in LDS with full factor rows (bucketed path)
    int lds_cap_c;         // max points kept in LDS with compact factor rows (bucketed path)
    int total_points;      // sum of n over the crops (probe records only)
    // ebc_dace_loss_h: the crop offsets / order as kernel arguments (B <= HMETA_MAX): no host-to-device copy
    int hmeta;
    int hoff[HMETA_MAX + 1], hord[HMETA_MAX];
};

// ---------------------------------------------------------------------------------------
// Sinkhorn-Knopp on the separable DMCount kernel.  `Ey`, `Ex` ([n][G]), `u0/u1` ([n]) live in
// LDS or global memory (FP = float* into either); everything else in LDS.
// cood of grid cell k (dm_loss.py:31-34): pixel centre, or normalised to [-1, 1] when norm_cood
__device__ __forceinline__ float cood(int k, int size, int red, int norm) {
    const float c = (float)(k * red) + 0.5f * (float)red;    // arange(0, size, red) + red / 2
    return norm ? c / (float)size * 2.0f - 1.0f : c;
}
__device__ __forceinline__ float pcoord(float p, int size, int norm) {
    return norm ? p / (float)size * 2.0f - 1.0f : p;     // dm_loss.py:51
}

// Per point, K's separable factors are exactly zero outside a short window (exp(C/-reg)
// underflows beyond ~32 px for reg = 10, i.e. <= 9 grid rows/columns): both products run over
// [ylo, ylo+ylen) x [xlo, xlo+xlen) only.  Skipping exact zeros leaves every value unchanged up to
// summation order; the windows are read off the computed factors, so any reg works.
// Accumulation uses LDS float atomics (order-nondeterministic at the ~1e-7 relative level).
__device__ __forceinline__ int block_max(int v, int* scratch) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    __syncthreads();
    if (lane == 0) scratch[w] = v;
    __syncthreads();
    int r = 0;
    for (int i = 0; i < nw; ++i) r = max(r, scratch[i]);
    return r;
}

// sum over aligned groups of 8 lanes with DPP moves (no LDS round trip): quad xor-1, quad xor-2,
// then half-row mirror pairs quad 0 with quad 1 of each 8-lane group
__device__ __forceinline__ float sum8_dpp(float x) {
    x += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, true));
    x += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x4E, 0xF, 0xF, true));
    x += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x141, 0xF, 0xF, true));
    return x;
}

template <int G, typename FP, typename IP>
__device__ void sinkhorn_crop(int n, int g, int size, int red, int norm, float reg, int max_iter, float stop_thr, int eval_freq,
                              const float* __restrict__ pts, FP Ey, FP Ex, FP u0, FP u1, IP win,
                              const float* b, float* v0, float* v1, float* part, float* misc,
                              int* iters_out, int* rolled_out, float* err_last_out)
{
    constexpr int GG = G * G;
    const int t = threadIdx.x;
    const float a = 1.0f / (float)n;                         // target_prob = ones/n
    // factors: Ey[i][iy] = exp(yd/-reg), Ex[i][jx] = exp(xd/-reg)
    for (int e = t; e < n * G; e += NT) {
        const int i = e / G, k = e - i * G;
        const float c = cood(k, size, red, norm);             // dm_loss.py:31-34
        const float x = pcoord(pts[2 * i], size, norm), y = pcoord(pts[2 * i + 1], size, norm);
        const float yd = (-2.0f * (y * c) + y * y) + c * c;
        const float xd = (-2.0f * (x * c) + x * x) + c * c;
        Ey[e] = k < g ? expf(yd / -reg) : 0.f;               // dead rows / columns of the LDS grid
        Ex[e] = k < g ? expf(xd / -reg) : 0.f;
    }
    for (int i = t; i < n; i += NT) u0[i] = 1.0f / (float)n;
    for (int j = t; j < GG; j += NT) v0[j] = (j / G < g && j % G < g) ? 1.0f / (float)(g * g) : 0.f;   // ones(M)/M
    __syncthreads();
    // nonzero windows (exp of a convex quadratic: the nonzeros are contiguous)
    int wy_max = 0;
    for (int i = t; i < n; i += NT) {
        int ylo = G, yhi = -1, xlo = G, xhi = -1;
        for (int k = 0; k < G; ++k) {
            if (Ey[i * G + k] != 0.f) { ylo = min(ylo, k); yhi = k; }
            if (Ex[i * G + k] != 0.f) { xlo = min(xlo, k); xhi = k; }
        }
        const int ylen = yhi >= ylo ? yhi - ylo + 1 : 0, xlen = xhi >= xlo ? xhi - xlo + 1 : 0;
        win[i] = (ylen ? ylo : 0) | (ylen << 8) | ((xlen ? xlo : 0) << 16) | (xlen << 24);
        wy_max = max(wy_max, ylen);
    }
    const int WY = block_max(wy_max, reinterpret_cast<int*>(misc));

    FP u = u0; FP un = u1;
    float* v = v0; float* vn = v1;
    int have_ktu = 0, it = 1, rolled = 0;
    float err = 1.0f, err_last = -1.0f;
    int* flag = reinterpret_cast<int*>(misc) + 16;            // NaN/Inf flags per iteration parity (misc[0..7]: block_sum scratch)
    if (t < 2) flag[t] = 0;
    __syncthreads();

    // K^T u partials: thread -> (4x4 block, point group); part[kg][GG] += (u_i Ey_i[iy]) Ex_i[jx]
    using C = Cfg<G>;
    constexpr int GB = G / 4;
    const int kb = t % C::NB, kg = t / C::NB;
    const int by = (kb / GB) * 4, bx = (kb % GB) * 4;
    auto ktu_pass = [&](FP uu) {
        if (kg < C::KSPLIT) {
            float4 acc[4] = {};
#pragma unroll 4
            for (int i = kg; i < n; i += C::KSPLIT) {
                const float ui = uu[i];
                const float4 ey = *reinterpret_cast<const float4*>(&Ey[i * G + by]);
                const float4 ex = *reinterpret_cast<const float4*>(&Ex[i * G + bx]);
                const float wy[4] = {ui * ey.x, ui * ey.y, ui * ey.z, ui * ey.w};
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    acc[r].x = fmaf(wy[r], ex.x, acc[r].x);
                    acc[r].y = fmaf(wy[r], ex.y, acc[r].y);
                    acc[r].z = fmaf(wy[r], ex.z, acc[r].z);
                    acc[r].w = fmaf(wy[r], ex.w, acc[r].w);
                }
            }
            float* pp = part + kg * GG + by * G + bx;
#pragma unroll
            for (int r = 0; r < 4; ++r) *reinterpret_cast<float4*>(pp + r * G) = acc[r];
        }
        __syncthreads();
    };
    auto ktu_at = [&](int j) {
        float sacc = 0.f;
#pragma unroll
        for (int k = 0; k < C::KSPLIT; ++k) sacc += part[k * GG + j];
        return sacc;
    };
    // K v: 8 lanes per point, lane q takes window rows q, q+8, ...; the 8 row sums meet by shuffles
    constexpr int WC = 10;
    const int q = t & 7;
    while (err > stop_thr && it <= max_iter) {               // bregman_pytorch.py:102
        if (!have_ktu) ktu_pass(u);
        have_ktu = 0;
        int* fl = flag + (it & 1);
        // v = b / (K^T u + eps)
        int bad = 0;
        for (int j = t; j < GG; j += NT) {
            const float val = b[j] / (ktu_at(j) + M_EPS);
            vn[j] = val;
            bad |= !isfinite(val);
        }
        if (bad) *fl = 1;
        __syncthreads();
        if (t == 0) flag[(it + 1) & 1] = 0;                   // nobody reads it until after the next barrier
        // u = a / (K v + eps); two points per 8-lane group per round so their LDS latencies overlap
        for (int i0 = 0; i0 < n; i0 += NT / 4) {
            float kv[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int i = i0 + h * (NT / 8) + (t >> 3);
                const bool live = i < n;
                const int w = live ? win[i] : 0;
                const int ylo = w & 255, ylen = (w >> 8) & 255, xlo = (w >> 16) & 255, xlen = (w >> 24) & 255;
                float acc = 0.f;
                if (live) {
                    const FP ex = Ex + i * G + xlo;
                    for (int c0 = 0; c0 < xlen; c0 += WC) {
                        float xv[WC];
#pragma unroll
                        for (int c = 0; c < WC; ++c) xv[c] = c0 + c < xlen ? ex[min(c0 + c, xlen - 1)] : 0.f;
                        for (int r = q; r < ylen; r += 8) {
                            const float* vr = vn + (ylo + r) * G + xlo;
                            float sacc = 0.f;
#pragma unroll
                            for (int c = 0; c < WC; ++c) sacc = fmaf(xv[c], vr[min(c0 + c, xlen - 1)], sacc);
                            acc = fmaf(Ey[i * G + ylo + r], sacc, acc);
                        }
                    }
                }
                kv[h] = acc;
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) kv[h] = sum8_dpp(kv[h]);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int i = i0 + h * (NT / 8) + (t >> 3);
                if (i < n && q == 0) {
                    const float val = a / (kv[h] + M_EPS);
                    un[i] = val;
                    if (!isfinite(val)) *fl = 1;
                }
            }
        }
        __syncthreads();
        if (*fl) { rolled = 1; break; }                       // keep (u, v): rollback, :111-115
        { FP tu = u; u = un; un = tu; float* tv = v; v = vn; vn = tv; }
        if (it % eval_freq == 0) {                            // :117-126
            ktu_pass(u);
            have_ktu = 1;
            float e = 0.f;
            for (int j = t; j < GG; j += NT) {
                const float d = b[j] - ktu_at(j) * v[j];
                e = fmaf(d, d, e);
            }
            err = block_sum(e, misc);
            err_last = err;
        }
        ++it;
    }
    // leave the final v in v0 and u in u0
    if (v != v0) { for (int j = t; j < GG; j += NT) v0[j] = v[j]; }
    if (u != u0) { for (int i = t; i < n; i += NT) u0[i] = u[i]; }
    __syncthreads();
    *iters_out = rolled ? it : it - 1;
    *rolled_out = rolled;
    *err_last_out = err_last;
    misc[1] = __int_as_float(WY);                            // for the wd pass
}

// sum over aligned groups of 4 lanes (quad xor-1, xor-2), every lane gets the sum
__device__ __forceinline__ float sum4_dpp(float x) {
    x += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, true));
    x += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x4E, 0xF, 0xF, true));
    return x;
}

// Sinkhorn-Knopp, bucketed form (LDS-resident crops whose K windows are <= 9 cells, i.e. reg = 10 and
// cell pitch 8: exp underflows beyond 32 px).  Same iteration, same control flow and epsilons as
// sinkhorn_crop / bregman_pytorch.py:102-126; only the summation order of the two products changes:
//  * the points are stably sorted into (G/4)^2 home buckets (the 4x4 cell block of their window
//    start); a window of <= 9 cells spans <= 3 blocks per axis, so K^T u of block (BY, BX) gathers
//    only the points of home buckets (BY-2..BY) x (BX-2..BX): 3 contiguous ranges of the sorted order;
//  * 8 adjacent lanes own a 4x4 block: they split its candidates, meet by DPP and form
//    v = b / (K^T u + eps) for it (no LDS partials), so an iteration is two phases and two barriers:
//    [K^T u, v] then [K v, u];
//  * K v: 4 lanes per point, each lane <= 3 window rows read as three aligned 16-B chunks of v.
// Factor rows are CW wide: G (full rows) or Cfg::CW (the 12 cells from row_base: compact).
// Returns false (nothing iterated) when a window is wider than 9 cells; the caller then runs
// sinkhorn_crop.  On return the factors, u (u0), windows and point coordinates (spts) are sorted.
template <int G, int CW, int LPB>
__device__ bool sinkhorn_sorted(int n, int g, int size, int red, int norm, float reg, int max_iter, float stop_thr, int eval_freq,
                                const float* __restrict__ pts, float* Ey, float* Ex, float* u0, float* u1, int* win,
                                int* key, float* spts, int* bk, const float* b, float* v0, float* v1, float* part,
                                float* misc, int* iters_out, int* rolled_out, float* err_last_out)
{
    using C = Cfg<G>;
    constexpr int GG = G * G, NB1 = C::NB1, NBK = C::NBK, HALO = C::HALO;
    const int t = threadIdx.x;
    int* cnt = bk;                 // [NBK] bucket sizes
    int* start = bk + NBK;         // [NBK + 1] bucket starts in the sorted order
    int* tmpwin = reinterpret_cast<int*>(u1);
    for (int k = t; k < NBK; k += NT) cnt[k] = 0;
    __syncthreads();
    // The scatter pass (ranks, factor rows) runs LPP lanes a point, as many as one pass of the workgroup takes (up to 32):
    // each lane counts every LPP-th earlier point and fills every LPP-th factor cell, the rank meets by lane shuffles; the
    // values are the one-lane form's, cell for cell.  r05 (kernel trace, 16 crops): 172 -> 163 us at 20 points a crop, 221
    // -> 215 us on a bench-like batch (one lane a point ran the 28-cell expf / division chain serially).  The windows pass
    // with LPP lanes a point as well measured no further gain on the bench's batches, and made the kernel spill: it stays
    // one lane a point.
    const int LG = n <= 32 ? 5 : n <= 64 ? 4 : n <= 128 ? 3 : n <= 256 ? 2 : n <= 512 ? 1 : 0, LPP = 1 << LG;
    auto grp_sum = [&](int v) { for (int o = LPP >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64); return v; };
    // 1. windows (read off the computed factors, as sinkhorn_crop) and home buckets, original order
    int wide = 0;
    for (int i = t; i < n; i += NT) {
        const float x = pcoord(pts[2 * i], size, norm), y = pcoord(pts[2 * i + 1], size, norm);
        int ylo = G, yhi = -1, xlo = G, xhi = -1;
        for (int k = 0; k < g; ++k) {
            const float c = cood(k, size, red, norm);
            const float yd = (-2.0f * (y * c) + y * y) + c * c;
            const float xd = (-2.0f * (x * c) + x * x) + c * c;
            if (expf(yd / -reg) != 0.f) { ylo = min(ylo, k); yhi = k; }
            if (expf(xd / -reg) != 0.f) { xlo = min(xlo, k); xhi = k; }
        }
        const int ylen = yhi >= ylo ? yhi - ylo + 1 : 0, xlen = xhi >= xlo ? xhi - xlo + 1 : 0;
        wide |= (ylen > 9) | (xlen > 9);
        const int kk = (ylen && xlen) ? (ylo / C::BS) * NB1 + (xlo / C::BS) : 0;
        key[i] = kk;
        tmpwin[i] = (ylen ? ylo : 0) | (ylen << 8) | ((xlen ? xlo : 0) << 16) | (xlen << 24);
        atomicAdd(&cnt[kk], 1);
    }
    if (block_or(wide, reinterpret_cast<int*>(misc))) return false;
    PROF_AT(48);
    if (t == 0) {
        int s = 0;
        for (int k = 0; k < NBK; ++k) { start[k] = s; s += cnt[k]; }
        start[NBK] = s;
    }
    __syncthreads();
    PROF_AT(49);
    // 2. stable scatter: slot = bucket start + rank among the earlier points of the same bucket
    for (int e0 = 0; e0 < n * LPP; e0 += NT) {
        const int e = e0 + t, i = e >> LG, sub = e & (LPP - 1);
        if (i >= n) break;                                   // whole groups (n * LPP is a multiple of LPP)
        const int kk = key[i];
        int r = 0;
        for (int j = sub; j < i; j += LPP) r += key[j] == kk;
        const int slot = start[kk] + grp_sum(r);
        const float px = pts[2 * i], py = pts[2 * i + 1];
        const float x = pcoord(px, size, norm), y = pcoord(py, size, norm);
        const int w = tmpwin[i];
        const int yb = row_base<G, CW>(w & 255, (w >> 8) & 255), xb = row_base<G, CW>((w >> 16) & 255, (w >> 24) & 255);
        for (int k = sub; k < CW; k += LPP) {
            const float cy = cood(yb + k, size, red, norm), cx = cood(xb + k, size, red, norm);
            const float yd = (-2.0f * (y * cy) + y * y) + cy * cy;
            const float xd = (-2.0f * (x * cx) + x * x) + cx * cx;
            Ey[slot * CW + k] = yb + k < g ? expf(yd / -reg) : 0.f;
            Ex[slot * CW + k] = xb + k < g ? expf(xd / -reg) : 0.f;
        }
        if (sub == 0) {
            spts[2 * slot] = px;
            spts[2 * slot + 1] = py;
            win[slot] = w;
        }
    }
    __syncthreads();
    PROF_AT(50);
    for (int i = t; i < n; i += NT) u0[i] = 1.0f / (float)n;
    for (int j = t; j < GG; j += NT) v0[j] = (j / G < g && j % G < g) ? 1.0f / (float)(g * g) : 0.f;
    const float a = 1.0f / (float)n;

    // candidate ranges of block blk: home rows BY-HALO..BY, columns BX-HALO..BX (contiguous per row)
    // (compact rows: bd[d][k] = first sorted index of home column hx0 + 1 + k in row d, so a
    // candidate's home column -- hence its row base -- follows from its index without a load)
    struct Ranges { int s[HALO + 1], pre[HALO + 2], bd[HALO + 1][HALO]; };
    auto ranges = [&](int blk, Ranges& R) {
        const int BY = blk / NB1, BX = blk - (blk / NB1) * NB1, hx0 = max(BX - HALO, 0);
        R.pre[0] = 0;
#pragma unroll
        for (int d = 0; d <= HALO; ++d) {
            const int hy = BY - HALO + d;
            int s0 = 0, e0 = 0;
            if (hy >= 0) { s0 = start[hy * NB1 + hx0]; e0 = start[hy * NB1 + BX + 1]; }
            R.s[d] = s0;
            R.pre[d + 1] = R.pre[d] + (e0 - s0);
#pragma unroll
            for (int k = 0; k < HALO; ++k) R.bd[d][k] = hy >= 0 ? start[hy * NB1 + min(hx0 + 1 + k, BX + 1)] : 0;
        }
    };
    // row base of a home bucket coordinate (compact rows; the 4x4 block at 4*B reads offset 4*B - base)
    auto hbase = [&](int h) { return CW == G ? 0 : min(C::BS * h, G - CW); };
    // LPB adjacent lanes per 4x4 block: lane kg takes candidates kg, kg+LPB, ... four at a time (all LDS
    // reads before the FMAs); the 16 block sums meet by DPP and lane kg keeps CPL = 16 / LPB cells from cell
    // CPL * kg.  LPB = 16 (one cell a lane) halves the heaviest block's candidate loop, which the phase barrier
    // waits for, at the cost of one more butterfly stage: the caller takes it for crops with many points only
    static_assert(LPB == 8 || (LPB == 16 && NBK * 16 <= NT), "lanes per block");
    constexpr int CPL = 16 / LPB;
    const int kg = t & (LPB - 1);
    auto ktu_block = [&](int blk, const Ranges& R, const float* uu, float& k0, float& k1) {
        const int BY = blk / NB1, BX = blk - (blk / NB1) * NB1, by = BY * 4, bx = BX * 4;
        float4 acc[4] = {};
        const int nc = R.pre[HALO + 1];
        const int hx0 = max(BX - HALO, 0);
        for (int c0 = kg; c0 < nc; c0 += 4 * LPB) {
            float ui[4];
            float4 ey[4], ex[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int c = c0 + k * LPB;
                int i = 0, oy = by, ox = bx;
#pragma unroll
                for (int d = 0; d <= HALO; ++d)
                    if (c >= R.pre[d] && c < R.pre[d + 1]) {
                        i = R.s[d] + c - R.pre[d];
                        if constexpr (CW != G) {
                            int hx = hx0;
#pragma unroll
                            for (int q2 = 0; q2 < HALO; ++q2) hx += i >= R.bd[d][q2];
                            oy = by - hbase(BY - HALO + d);
                            ox = bx - hbase(hx);
                        }
                    }
                if constexpr (CW != G) { if (c >= nc) { oy = 0; ox = 0; } }
                ui[k] = c < nc ? uu[i] : 0.f;
                ey[k] = *reinterpret_cast<const float4*>(&Ey[i * CW + oy]);
                ex[k] = *reinterpret_cast<const float4*>(&Ex[i * CW + ox]);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float wy[4] = {ui[k] * ey[k].x, ui[k] * ey[k].y, ui[k] * ey[k].z, ui[k] * ey[k].w};
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    acc[r].x = fmaf(wy[r], ex[k].x, acc[r].x);
                    acc[r].y = fmaf(wy[r], ex[k].y, acc[r].y);
                    acc[r].z = fmaf(wy[r], ex[k].z, acc[r].z);
                    acc[r].w = fmaf(wy[r], ex[k].w, acc[r].w);
                }
            }
        }
        // transposing butterfly over the 8 lanes (half-row mirror, then quad xor-2, xor-1): each stage
        // keeps half of the cells and adds the partner's copy of them; lane kg ends with cells 2kg, 2kg+1
        float c16[16];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            c16[4 * r] = acc[r].x; c16[4 * r + 1] = acc[r].y; c16[4 * r + 2] = acc[r].z; c16[4 * r + 3] = acc[r].w;
        }
        auto dpp = [](float x, auto ctl) {
            return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x),
                                                                      decltype(ctl)::value, 0xF, 0xF, true));
        };
        const bool b2 = kg & 4, b1 = kg & 2, b0 = kg & 1;
        float c8[8], c4[4];
        if constexpr (LPB == 16) {
            // first fold the two 8-lane halves (row mirror: lane kg <-> 15 - kg), then the 8-lane butterfly on the
            // half of the block's cells this lane keeps; lane kg ends with cell kg
            const bool b3 = kg & 8;
            float h8[8], h4[4], h2[2];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const float send = b3 ? c16[k] : c16[k + 8];
                h8[k] = (b3 ? c16[k + 8] : c16[k]) + dpp(send, std::integral_constant<int, 0x140>{});
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float send = b2 ? h8[k] : h8[k + 4];
                h4[k] = (b2 ? h8[k + 4] : h8[k]) + dpp(send, std::integral_constant<int, 0x141>{});
            }
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const float send = b1 ? h4[k] : h4[k + 2];
                h2[k] = (b1 ? h4[k + 2] : h4[k]) + dpp(send, std::integral_constant<int, 0x4E>{});
            }
            const float send = b0 ? h2[0] : h2[1];
            k0 = (b0 ? h2[1] : h2[0]) + dpp(send, std::integral_constant<int, 0xB1>{});
            k1 = 0.f;
            return;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const float send = b2 ? c16[k] : c16[k + 8];
            c8[k] = (b2 ? c16[k + 8] : c16[k]) + dpp(send, std::integral_constant<int, 0x141>{});
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float send = b1 ? c8[k] : c8[k + 4];
            c4[k] = (b1 ? c8[k + 4] : c8[k]) + dpp(send, std::integral_constant<int, 0x4E>{});
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const float send = b0 ? c4[k] : c4[k + 2];
            const float keep = (b0 ? c4[k + 2] : c4[k]) + dpp(send, std::integral_constant<int, 0xB1>{});
            if (k == 0) k0 = keep; else k1 = keep;
        }
    };
    // cell index of lane kg's first cell (cells 2kg, 2kg+1: row 2kg/4, columns 2kg%4, +1)
    auto cell0 = [&](int blk) {
        const int BY = blk / NB1, BX = blk - (blk / NB1) * NB1;
        return (BY * 4 + (CPL * kg) / 4) * G + BX * 4 + (CPL * kg) % 4;
    };
    constexpr int BPP = NT / LPB;                             // blocks per pass
    constexpr bool ONE = NBK <= BPP;                          // one block per 8-lane group (G = 28)
    Ranges R0;
    if (t / LPB < NBK) ranges(t / LPB, R0);

    float* u = u0; float* un = u1;
    float* v = v0; float* vn = v1;
    int have_ktu = 0, it = 1, rolled = 0;
    float err = 1.0f, err_last = -1.0f;
    int* flag = reinterpret_cast<int*>(misc) + 16;
    if (t < 2) flag[t] = 0;
    __syncthreads();
    // K v: LPT lanes per point, each <= ceil(9 / LPT) window rows; the heavy-crop instantiation (LPB = 16) uses 2,
    // so up to NT / 2 points take one pass instead of two
    constexpr int LPT = LPB == 16 ? 2 : 4;
    const int q = t & (LPT - 1);
    // K v's loop-invariant operands in registers when every point fits one pass (n <= NT / LPT, the bench's crops):
    // the point's 12-cell Ex chunk, its Ey values and v offsets of the lane's window rows -- per iteration the lane
    // then reads only the v rows (r03 re-read the window word, the Ex chunk and Ey through LDS every iteration,
    // one more dependent LDS round trip).  Same products in the same order: the bits do not change.
    constexpr int KW = G < 12 ? G : 12, MR = (9 + LPT - 1) / LPT;   // window rows <= 9
    const bool kv_regs = n <= NT / LPT;
    float4 kv_e[KW / 4];
    float kv_ey[MR];
    int kv_off[MR], kv_rows = 0;
    if (kv_regs && t / LPT < n) {
        const int i = t / LPT;
        const int w = win[i];
        const int ylo = w & 255, ylen = (w >> 8) & 255, xlo = (w >> 16) & 255, xlen = (w >> 24) & 255;
        if (xlen) {
            const int x4 = min(xlo & ~3, G - KW);
            const float* exr = Ex + i * CW + x4 - row_base<G, CW>(xlo, xlen);
            const float* eyr = Ey + i * CW + ylo - row_base<G, CW>(ylo, ylen);
#pragma unroll
            for (int c = 0; c < KW / 4; ++c) kv_e[c] = *reinterpret_cast<const float4*>(exr + 4 * c);
#pragma unroll
            for (int k = 0; k < MR; ++k) {
                const int r = q + k * LPT;
                kv_ey[k] = r < ylen ? eyr[r] : 0.f;
                kv_off[k] = (ylo + (r < ylen ? r : 0)) * G + x4;
                kv_rows += r < ylen;
            }
        }
    }
    int to_eval = eval_freq;
#ifdef EBC_DACE_PROF
    unsigned long long pa = 0, pb = 0, pe = 0, tp0 = 0, tp1 = 0, wa = 0, wb = 0;
    PROF_AT(4);
#endif
    while (err > stop_thr && it <= max_iter) {               // bregman_pytorch.py:102
        int* fl = flag + (it & 1);
#ifdef EBC_DACE_PROF
        tp0 = PROF_T();
#endif
        // phase A: v = b / (K^T u + eps) (K^T u reused from the err pass)
        int bad = 0;
        for (int blk = t / LPB; blk < NBK; blk += BPP) {
            Ranges R;
            if (!ONE) ranges(blk, R); else R = R0;
            const int j = cell0(blk);
            float k0, k1;
            if (have_ktu) { k0 = part[j]; k1 = CPL == 2 ? part[j + 1] : 0.f; }
            else ktu_block(blk, R, u, k0, k1);
            const float v0n = b[j] / (k0 + M_EPS);
            vn[j] = v0n;
            bad |= (int)!isfinite(v0n);
            if constexpr (CPL == 2) {
                const float v1n = b[j + 1] / (k1 + M_EPS);
                vn[j + 1] = v1n;
                bad |= (int)!isfinite(v1n);
            }
        }
        have_ktu = 0;
        if (bad) *fl = 1;
#ifdef EBC_DACE_PROF
        wa += PROF_T() - tp0;
#endif
        __syncthreads();
#ifdef EBC_DACE_PROF
        tp1 = PROF_T(); pa += tp1 - tp0;
#endif
        if (t == 0) flag[(it + 1) & 1] = 0;
        // phase B: u = a / (K v + eps)
        if (kv_regs) {
            const int i = t / LPT;
            float acc = 0.f;
#pragma unroll
            for (int k = 0; k < MR; ++k) {
                if (k < kv_rows) {
                    const float* vr = vn + kv_off[k];
                    float sum = 0.f;
#pragma unroll
                    for (int c = 0; c < KW / 4; ++c) {
                        const float4 a4 = *reinterpret_cast<const float4*>(vr + 4 * c);
                        sum = fmaf(kv_e[c].x, a4.x, sum); sum = fmaf(kv_e[c].y, a4.y, sum);
                        sum = fmaf(kv_e[c].z, a4.z, sum); sum = fmaf(kv_e[c].w, a4.w, sum);
                    }
                    acc = fmaf(kv_ey[k], sum, acc);
                }
            }
            if constexpr (LPT == 4) acc = sum4_dpp(acc);
            else acc += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, acc), 0xB1, 0xF, 0xF, true));
            if (i < n && q == 0) {
                const float val = a / (acc + M_EPS);
                un[i] = val;
                if (!isfinite(val)) *fl = 1;
            }
        }
        for (int i0 = 0; i0 < (kv_regs ? 0 : n); i0 += NT / LPT) {
            const int i = i0 + t / LPT;
            float acc = 0.f;
            if (i < n) {
                const int w = win[i];
                const int ylo = w & 255, ylen = (w >> 8) & 255, xlo = (w >> 16) & 255, xlen = (w >> 24) & 255;
                if (xlen) {
                    // KW cells from the window's 4-aligned start (12: a <= 9-cell window at offset <= 3; the
                    // whole row on grids narrower than 12)
                    constexpr int KW = G < 12 ? G : 12;
                    const int x4 = min(xlo & ~3, G - KW);
                    const float* exr = Ex + i * CW + x4 - row_base<G, CW>(xlo, xlen);
                    const float* eyr = Ey + i * CW + ylo - row_base<G, CW>(ylo, ylen);
                    float4 e[KW / 4];
#pragma unroll
                    for (int c = 0; c < KW / 4; ++c) e[c] = *reinterpret_cast<const float4*>(exr + 4 * c);
                    for (int r = q; r < ylen; r += LPT) {
                        const float* vr = vn + (ylo + r) * G + x4;
                        float sum = 0.f;
#pragma unroll
                        for (int c = 0; c < KW / 4; ++c) {
                            const float4 a4 = *reinterpret_cast<const float4*>(vr + 4 * c);
                            sum = fmaf(e[c].x, a4.x, sum); sum = fmaf(e[c].y, a4.y, sum);
                            sum = fmaf(e[c].z, a4.z, sum); sum = fmaf(e[c].w, a4.w, sum);
                        }
                        acc = fmaf(eyr[r], sum, acc);
                    }
                }
            }
            if constexpr (LPT == 4) acc = sum4_dpp(acc);
            else acc += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, acc), 0xB1, 0xF, 0xF, true));
            if (i < n && q == 0) {
                const float val = a / (acc + M_EPS);
                un[i] = val;
                if (!isfinite(val)) *fl = 1;
            }
        }
#ifdef EBC_DACE_PROF
        wb += PROF_T() - tp1;
#endif
        __syncthreads();
        if (*fl) { rolled = 1; break; }                       // keep (u, v): rollback, :111-115
#ifdef EBC_DACE_PROF
        tp0 = PROF_T(); pb += tp0 - tp1;
#endif
        { float* tu = u; u = un; un = tu; float* tv = v; v = vn; vn = tv; }
        if (--to_eval == 0) {                                 // it % eval_freq == 0 (:117-126); K^T u kept
            to_eval = eval_freq;
            float e = 0.f;
            for (int blk = t / LPB; blk < NBK; blk += BPP) {
                Ranges R;
                if (!ONE) ranges(blk, R); else R = R0;
                const int j = cell0(blk);
                float k0, k1;
                ktu_block(blk, R, u, k0, k1);
                part[j] = k0;
                const float d0 = b[j] - k0 * v[j];
                e = fmaf(d0, d0, e);
                if constexpr (CPL == 2) {
                    part[j + 1] = k1;
                    const float d1 = b[j + 1] - k1 * v[j + 1];
                    e = fmaf(d1, d1, e);
                }
            }
            err = block_sum(e, misc);
            err_last = err;
            have_ktu = 1;
#ifdef EBC_DACE_PROF
            pe += PROF_T() - tp0;
#endif
        }
        ++it;
    }
#ifdef EBC_DACE_PROF
    PROF_AT(5);
    if (t == 0 && blockIdx.x < 64) {
        g_dace_prof[blockIdx.x][8] = pa; g_dace_prof[blockIdx.x][9] = pb; g_dace_prof[blockIdx.x][10] = pe;
        g_dace_prof[blockIdx.x][11] = (unsigned long long)it; g_dace_prof[blockIdx.x][12] = (unsigned long long)n;
        g_dace_prof[blockIdx.x][13] = (unsigned long long)LPB;
    }
    if ((t & 63) == 0 && blockIdx.x < 64) { g_dace_prof[blockIdx.x][16 + t / 64] = wa; g_dace_prof[blockIdx.x][32 + t / 64] = wb; }
#endif
    if (v != v0) { for (int j = t; j < GG; j += NT) v0[j] = v[j]; }
    if (u != u0) { for (int i = t; i < n; i += NT) u0[i] = u[i]; }
    __syncthreads();
    *iters_out = rolled ? it : it - 1;
    *rolled_out = rolled;
    *err_last_out = err_last;
    misc[1] = __int_as_float(9);                             // window rows bound for the wd pass
    return true;
}

// Wasserstein distance sum(C * P) over the windows (dm_loss.py:77; reported, unused by training)
template <int G, int CW, typename FP, typename IP>
__device__ float transport_cost(int n, int size, int red, int norm, const float* pts, FP Ey, FP Ex, FP u, IP win,
                                const float* v, int WY, float* misc)
{
    float w = 0.f;
    for (int e = threadIdx.x; e < n * WY; e += NT) {
        const int i = e / WY, r = e - i * WY;
        const int wi = win[i];
        if (r >= ((wi >> 8) & 255)) continue;
        const int iy = (wi & 255) + r, xlo = (wi >> 16) & 255, xlen = (wi >> 24) & 255;
        const int yb = row_base<G, CW>(wi & 255, (wi >> 8) & 255), xb = row_base<G, CW>(xlo, xlen);
        const float x = pcoord(pts[2 * i], size, norm), y = pcoord(pts[2 * i + 1], size, norm);
        const float c = cood(iy, size, red, norm);
        const float yd = (-2.0f * (y * c) + y * y) + c * c;
        float t1 = 0.f, t2 = 0.f;
        for (int k = 0; k < xlen; ++k) {
            const int jx = xlo + k;
            const float cx = cood(jx, size, red, norm);
            const float xd = (-2.0f * (x * cx) + x * x) + cx * cx;
            const float kv = Ex[i * CW + jx - xb] * v[iy * G + jx];
            t1 += kv;
            t2 = fmaf(kv, xd, t2);
        }
        w += u[i] * Ey[i * CW + iy - yb] * (yd * t1 + t2);
    }
    return block_sum(w, misc);
}

template <int G>
__device__ void crop_body(const Params& P, int b, float* lds)
{
    using C = Cfg<G>;
    const int t = threadIdx.x;
    const int GG = C::GG, S = P.size;
    const int g = P.g, gg = g * g;                            // live cells: LDS j = y*G + x with y, x < g
    auto live = [&](int j) { return j / G < g && j % G < g; };
    auto gidx = [&](int j) { return (j / G) * g + j % G; };   // LDS cell -> index in the [g][g] global maps
    float* pd = lds;            // pred density
    float* td = pd + GG;        // target block sums
    float* bb = td + GG;        // normed pred density (Sinkhorn b)
    float* v0 = bb + GG;
    float* v1 = v0 + GG;
    float* misc = v1 + GG;
    int* bkt = reinterpret_cast<int*>(misc + 64);             // sorted-Sinkhorn bucket counts / starts
    float* part = misc + 64 + C::BKT;                         // K^T u partials [KSPLIT][GG]
    float* fac = part + C::KSPLIT * GG;                       // LDS factors, full rows (if they fit)
    float* facc = part + GG;                                  // LDS factors, compact rows (bucketed path)

    const int p0 = P.hmeta ? P.hoff[b] : P.offsets[b], n = (P.hmeta ? P.hoff[b + 1] : P.offsets[b + 1]) - p0;
    PROF_AT(0);

    // 1. pred density, target block sums (losses/utils.py:4-9)
    for (int j = t; j < GG; j += NT) { pd[j] = live(j) ? P.pred_density[(size_t)b * gg + gidx(j)] : 0.f; td[j] = 0.f; }
    __syncthreads();
    if (P.target_is_reduced) {
        for (int j = t; j < GG; j += NT) td[j] = live(j) ? P.target_density[(size_t)b * gg + gidx(j)] : 0.f;
    } else {
        const float4* src = reinterpret_cast<const float4*>(P.target_density + (size_t)b * S * S);
        const int q4 = S / 4;
        for (int e = t; e < S * q4; e += NT) {
            const int row = e / q4, c4 = e - row * q4;
            const float4 x = src[e];
            const float s = (x.x + x.y) + (x.z + x.w);
            if (s != 0.f) atomicAdd(&td[(row / P.red) * G + (c4 * 4) / P.red], s);
        }
    }
    __syncthreads();
    PROF_AT(1);
    const float pc = block_sum([&] { float s = 0.f; for (int j = t; j < GG; j += NT) s += pd[j]; return s; }(), misc);
    const float tc = (float)n;

    // 2. cross-entropy over bins (dace_loss.py:42-55), grad = (softmax - onehot) / B
    const float invB = 1.0f / (float)P.B;
    float ce = 0.f;
    for (int j = t; j < gg; j += NT) {                        // j: global cell index
        const float dv = td[(j / g) * G + j % g];
        int cls = 0;
        for (int k = 0; k < P.N; ++k)
            if (dv >= P.bins_lo[k] && dv <= P.bins_hi[k]) cls = k;
        const float* lg = P.pred_class + (size_t)b * P.N * gg + j;
        float mx = -INFINITY;
        for (int k = 0; k < P.N; ++k) mx = fmaxf(mx, lg[(size_t)k * gg]);
        float se = 0.f;
        for (int k = 0; k < P.N; ++k) se += expf(lg[(size_t)k * gg] - mx);
        const float lse = mx + logf(se);
        ce += lse - lg[(size_t)cls * gg];
        float* gc = P.grad_class + (size_t)b * P.N * gg + j;
        for (int k = 0; k < P.N; ++k)
            gc[(size_t)k * gg] = (expf(lg[(size_t)k * gg] - lse) - (k == cls ? 1.f : 0.f)) * invB;
    }
    ce = block_sum(ce, misc);
    PROF_AT(2);

    float cnt_b = 0.f, tv_b = 0.f, ot_b = 0.f, wd_b = 0.f, err_last = -1.f;
    int iters = 0, rolled = 0;
    const bool dm = P.count_mode == EBC_COUNT_DMCOUNT;           // EBC_COUNT_OT_ONLY: the OT term alone
    if (P.count_mode == EBC_COUNT_MAE || P.count_mode == EBC_COUNT_MSE) {
        // count_loss "mae" / "mse": per-pixel, summed over HW, mean over B (dace_loss.py:57-62)
        float s = 0.f;
        for (int j = t; j < GG; j += NT) {
            if (!live(j)) continue;
            const float d = pd[j] - td[j];
            s += (P.count_mode == EBC_COUNT_MAE) ? fabsf(d) : d * d;
            const float gd = (P.count_mode == EBC_COUNT_MAE) ? sgnf(d) : 2.f * d;
            P.grad_density[(size_t)b * gg + gidx(j)] = P.w_count * gd * invB;
        }
        cnt_b = block_sum(s, misc);
    } else {
        // 3. DMLoss pieces (dm_loss.py:99-124)
        const float inv_pc = 1.0f / (pc + EPS), inv_tc = 1.0f / (tc + EPS);
        float tvs = 0.f, tvk = 0.f;
        for (int j = t; j < GG; j += NT) {
            const float np_ = pd[j] * inv_pc;    // normed pred (dm_loss.py:106)
            bb[j] = pd[j] / (pc + EPS);
            const float d = np_ - td[j] * inv_tc;
            tvs += fabsf(d);
            tvk += sgnf(d) * pd[j];
        }
        tvs = block_sum(tvs, misc);
        tvk = block_sum(tvk, misc);
        tv_b = tvs * tc;
        cnt_b = fabsf(pc - tc);
        const float gcount = dm ? sgnf(pc - tc) * invB : 0.f;
        const float wtv = dm ? P.w_tv : 0.f;
        // 4. Sinkhorn OT (dm_loss.py:49-77)
        PROF_AT(3);
        if (n > 0) {
            const float* pts = P.points + 2 * (size_t)p0;
            // Inlined copies so each sees one address space for the factors: LDS-resident crops get
            // ds_* accesses (a select between LDS and global would make them flat_*).
            auto post = [&](auto cw, auto Ey, auto Ex, auto u0, auto win, const float* cpts) {
                const int WY = __float_as_int(misc[1]);
                __syncthreads();
                // beta = reg * log(v + eps); gradient (dm_loss.py:65-74)
                float sb = 0.f;
                for (int j = t; j < GG; j += NT) {
                    const float be = P.reg * logf(v0[j] + M_EPS);
                    v1[j] = be;
                    sb += pd[j] * be;
                    if (P.beta_out && live(j)) P.beta_out[(size_t)b * gg + gidx(j)] = be;
                }
                sb = block_sum(sb, misc);
                const float den = pc * pc + EPS;
                const float g1 = pc / den, g2 = sb / den;
                float ol = 0.f;
                for (int j = t; j < GG; j += NT) {
                    const float og = g1 * v1[j] - g2;
                    ol += pd[j] * og;
                    v1[j] = og;
                }
                ot_b = block_sum(ol, misc);
                wd_b = transport_cost<G, decltype(cw)::value>(n, S, P.red, P.norm_cood, cpts, Ey, Ex, u0, win, v0, WY, misc);
            };
            // dense path (full rows; wide windows or too many points for the compact rows)
            auto dense = [&](float* base, auto /*in_lds: one instantiation per address space*/) {
                float* Ey = base; float* Ex = Ey + (size_t)n * G; float* u0 = Ex + (size_t)n * G; float* u1 = u0 + n;
                int* win = reinterpret_cast<int*>(u1 + n);
                sinkhorn_crop<G>(n, P.g, P.size, P.red, P.norm_cood, P.reg, P.max_iter, P.stop_thr, P.eval_freq, pts, Ey, Ex, u0,
                                 u1, win, bb, v0, v1, part, misc, &iters, &rolled, &err_last);
                post(std::integral_constant<int, G>{}, Ey, Ex, u0, win, pts);
            };
            // bucketed path in LDS: full factor rows while they fit (fewest VALU per candidate), else
            // the compact 12-cell rows (a per-candidate row base, computed from its home bucket)
            auto bucketed = [&](auto cw) {
                constexpr int CW = decltype(cw)::value;
                float* Ey = facc; float* Ex = Ey + n * CW; float* u0 = Ex + n * CW; float* u1 = u0 + n;
                int* win = reinterpret_cast<int*>(u1 + n);
                int* key = win + n;
                float* spts = reinterpret_cast<float*>(key + n);
                // 16 lanes per 4x4 block for crops with many points (r02, tools/loss_probe.py: 600 points 883 -> 743 us,
                // 1000 points 1278 -> 950 us per 16-crop launch; the bench's light crops ran slower on it)
                constexpr bool W16 = C::NBK * 16 <= NT;
                const bool ok = (W16 && n >= SORTED_W16_MIN_POINTS)
                    ? sinkhorn_sorted<G, CW, W16 ? 16 : 8>(n, P.g, P.size, P.red, P.norm_cood, P.reg, P.max_iter, P.stop_thr,
                                                           P.eval_freq, pts, Ey, Ex, u0, u1, win, key, spts, bkt, bb, v0, v1,
                                                           part, misc, &iters, &rolled, &err_last)
                    : sinkhorn_sorted<G, CW, 8>(n, P.g, P.size, P.red, P.norm_cood, P.reg, P.max_iter, P.stop_thr,
                                                P.eval_freq, pts, Ey, Ex, u0, u1, win, key, spts, bkt, bb, v0, v1, part, misc,
                                                &iters, &rolled, &err_last);
                if (!ok) return false;
                post(cw, Ey, Ex, u0, win, spts);
                PROF_AT(6);
                return true;
            };
            bool done = false;
            if (n <= P.lds_cap_s) done = bucketed(std::integral_constant<int, G>{});
            else if (n <= P.lds_cap_c) done = bucketed(std::integral_constant<int, C::CW>{});
            if (!done) {
                if (n <= P.lds_cap) dense(fac, std::true_type{});
                else dense(P.ws_factors + (size_t)C::PER_POINT * p0, std::false_type{});
            }
        } else {
            for (int j = t; j < GG; j += NT) {
                v1[j] = 0.f;
                if (P.beta_out && live(j)) P.beta_out[(size_t)b * gg + gidx(j)] = 0.f;   // no OT for an empty crop (dm_loss.py:49)
            }
            __syncthreads();
        }
        // 5. d loss / d pred_density = w_count * (w_ot * ot_grad + w_tv * tv_grad + count_grad)
        const float ktv = tc * invB;
        for (int j = t; j < GG; j += NT) {
            if (!live(j)) continue;
            const float d = pd[j] * inv_pc - td[j] * inv_tc;
            const float gtv = ktv * (sgnf(d) * inv_pc - tvk * inv_pc * inv_pc);
            P.grad_density[(size_t)b * gg + gidx(j)] = P.w_count * (P.w_ot * v1[j] + wtv * gtv + gcount);
        }
    }
    PROF_AT(7);
    if (t == 0) {
        float* st = P.crop_stats + (size_t)b * 8;
        st[0] = ce; st[1] = tv_b; st[2] = cnt_b; st[3] = ot_b; st[4] = wd_b;
        st[5] = (float)iters; st[6] = (float)rolled; st[7] = err_last;
        if (P.status) P.status[b] = rolled ? -iters : iters;
    }
}

template <int G>
__global__ __launch_bounds__(NT) void dace_loss_kernel(Params P)
{
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int b = P.hmeta ? P.hord[blockIdx.x] : P.order ? P.order[blockIdx.x] : (int)blockIdx.x;
    crop_body<G>(P, b, lds);
}

// losses[5] = loss, ot_loss, tv_loss, count_loss, ce_loss  (dace_loss.py:64-70, dm_loss.py:111-122)
__global__ void dace_finalize_kernel(const float* stats, int B, int count_mode, float w_count, float w_ot,
                                     float w_tv, float* losses)
{
    __shared__ float scratch[8];
    const int t = threadIdx.x;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    for (int b = t; b < B; b += blockDim.x) {
        s[0] += stats[b * 8 + 0]; s[1] += stats[b * 8 + 1]; s[2] += stats[b * 8 + 2]; s[3] += stats[b * 8 + 3];
    }
    float r[4];
    for (int k = 0; k < 4; ++k) r[k] = block_sum(s[k], scratch);
    if (t == 0) {
        const float invB = 1.0f / (float)B;
        const float ce = r[0] * invB;
        if (count_mode == EBC_COUNT_DMCOUNT) {
            const float tv = r[1] * invB, cnt = r[2] * invB, ot = r[3];
            const float dm = ot * w_ot + tv * w_tv + cnt;
            losses[0] = ce + w_count * dm; losses[1] = ot; losses[2] = tv; losses[3] = cnt; losses[4] = ce;
        } else if (count_mode == EBC_COUNT_OT_ONLY) {
            const float ot = r[3];
            losses[0] = w_count * w_ot * ot; losses[1] = ot; losses[2] = 0.f; losses[3] = 0.f; losses[4] = ce;
        } else {
            const float cnt = r[2] * invB;
            losses[0] = ce + w_count * cnt; losses[1] = 0.f; losses[2] = 0.f; losses[3] = cnt; losses[4] = ce;
        }
    }
}

template <int G> int launch(const Params& P0, hipStream_t st)
{
    using C = Cfg<G>;
    Params P = P0;
    P.lds_cap = (int)((LDS_MAX - C::FIXED_BYTES) / (sizeof(float) * C::PER_POINT));
    P.lds_cap_s = (int)((LDS_MAX - C::FIXED_BYTES_C) / (sizeof(float) * C::PER_POINT));
    P.lds_cap_c = (int)((LDS_MAX - C::FIXED_BYTES_C) / (sizeof(float) * C::PER_POINT_C));
    if (!ensure_lds<dace_loss_kernel<G>>(LDS_MAX, st)) return EBC_E_LAUNCH;
    const int pi = probe_on() ? probe_start(EBC_PROBE_DACE, P.count_mode, 0, 0, 0, P.B, P.total_points, G, st) : -1;
    hipLaunchKernelGGL(dace_loss_kernel<G>, dim3(P.B), dim3(NT), LDS_MAX, st, P);
    probe_stop(pi, st);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

}  // namespace

// the LDS grid a density grid g runs on (dead cells pad it to an instantiated size), 0 = unsupported
static int lds_grid(int g)
{
    static const int grids[] = {8, 16, 24, 28, 32, 40, 48, 56, 64};
    for (int G : grids) if (g <= G) return G;
    return 0;
}

extern "C" size_t ebc_dace_workspace_bytes(int B, int total_points, int size, int reduction)
{
    const int G = reduction > 0 ? lds_grid(size / reduction) : 0;
    return sizeof(float) * ((size_t)(2 * (G ? G : 64) + 6) * (size_t)(total_points > 0 ? total_points : 1)) + 256;
}

namespace {
int dace_loss_impl(const float* pred_class, const float* pred_density, const float* target_density,
                   int target_is_reduced, const float* points, const int* offsets, const int* order, bool host_meta,
                   const float* bins_lo, const float* bins_hi, int B, int N, int size, int reduction,
                   int count_mode, int norm_cood, float weight_count_loss, float weight_ot, float weight_tv,
                   float reg, int max_iter, float stop_thr, int eval_freq,
                   float* grad_class, float* grad_density, float* losses, float* crop_stats,
                   float* beta_out, int* status, void* workspace, size_t workspace_bytes,
                   ebc_stream_t stream)
{
    if (B <= 0 || N <= 0 || reduction <= 0 || size % reduction != 0 || eval_freq <= 0 || reg <= 0.f)
        return EBC_E_ARG;
    if (count_mode < EBC_COUNT_DMCOUNT || count_mode > EBC_COUNT_OT_ONLY) return EBC_E_ARG;
    if (!target_is_reduced && reduction % 4 != 0) return EBC_E_UNSUPPORTED;   // float4 row pieces per cell
    if (!pred_class || !pred_density || !target_density || !offsets || !bins_lo || !bins_hi ||
        !grad_class || !grad_density || !losses || !crop_stats)
        return EBC_E_ARG;
    if (!target_is_reduced && (size % 4) != 0) return EBC_E_ARG;
    const int g = size / reduction;
    hipStream_t st = (hipStream_t)stream;
    Params P{};
    P.pred_class = pred_class; P.pred_density = pred_density; P.target_density = target_density;
    P.target_is_reduced = target_is_reduced; P.points = points;
    if (host_meta) {
        if (B > HMETA_MAX) return EBC_E_UNSUPPORTED;
        P.hmeta = 1;
        for (int i = 0; i <= B; ++i) P.hoff[i] = offsets[i];
        for (int i = 0; i < B; ++i) {
            if (order && (order[i] < 0 || order[i] >= B)) return EBC_E_ARG;
            P.hord[i] = order ? order[i] : i;
        }
    } else {
        P.offsets = offsets; P.order = order;
    }
    P.bins_lo = bins_lo; P.bins_hi = bins_hi; P.B = B; P.N = N; P.size = size; P.red = reduction;
    P.count_mode = count_mode; P.norm_cood = norm_cood; P.w_count = weight_count_loss; P.w_ot = weight_ot; P.w_tv = weight_tv;
    P.reg = reg; P.stop_thr = stop_thr; P.max_iter = max_iter; P.eval_freq = eval_freq;
    P.grad_class = grad_class; P.grad_density = grad_density; P.crop_stats = crop_stats;
    P.beta_out = beta_out; P.status = status; P.ws_factors = (float*)workspace;
    const int G = lds_grid(g);
    if (g <= 0 || !G) return EBC_E_UNSUPPORTED;                 // density grids up to 64 x 64 (LDS-resident state)
    P.g = g;
    P.total_points = (int)((workspace_bytes - 256) / (sizeof(float) * (2 * (size_t)G + 6)));
    int rc;
    switch (G) {
        case 8: rc = launch<8>(P, st); break;
        case 16: rc = launch<16>(P, st); break;
        case 24: rc = launch<24>(P, st); break;
        case 28: rc = launch<28>(P, st); break;
        case 32: rc = launch<32>(P, st); break;
        case 40: rc = launch<40>(P, st); break;
        case 48: rc = launch<48>(P, st); break;
        case 56: rc = launch<56>(P, st); break;
        default: rc = launch<64>(P, st); break;
    }
    if (rc) return rc;
    hipLaunchKernelGGL(dace_finalize_kernel, dim3(1), dim3(256), 0, st, crop_stats, B, count_mode,
                       weight_count_loss, weight_ot, weight_tv, losses);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}
}  // namespace

extern "C" int ebc_dace_loss(const float* pred_class, const float* pred_density, const float* target_density,
                             int target_is_reduced, const float* points, const int* offsets, const int* order,
                             const float* bins_lo, const float* bins_hi, int B, int N, int size, int reduction,
                             int count_mode, int norm_cood, float weight_count_loss, float weight_ot, float weight_tv,
                             float reg, int max_iter, float stop_thr, int eval_freq,
                             float* grad_class, float* grad_density, float* losses, float* crop_stats,
                             float* beta_out, int* status, void* workspace, size_t workspace_bytes,
                             ebc_stream_t stream)
{
    return dace_loss_impl(pred_class, pred_density, target_density, target_is_reduced, points, offsets, order, false,
                          bins_lo, bins_hi, B, N, size, reduction, count_mode, norm_cood, weight_count_loss, weight_ot,
                          weight_tv, reg, max_iter, stop_thr, eval_freq, grad_class, grad_density, losses, crop_stats,
                          beta_out, status, workspace, workspace_bytes, stream);
}
extern "C" int ebc_dace_loss_h(const float* pred_class, const float* pred_density, const float* target_density,
                               int target_is_reduced, const float* points, const int* offsets_host,
                               const int* order_host, const float* bins_lo, const float* bins_hi, int B, int N, int size,
                               int reduction, int count_mode, int norm_cood, float weight_count_loss, float weight_ot,
                               float weight_tv, float reg, int max_iter, float stop_thr, int eval_freq,
                               float* grad_class, float* grad_density, float* losses, float* crop_stats,
                               float* beta_out, int* status, void* workspace, size_t workspace_bytes,
                               ebc_stream_t stream)
{
    return dace_loss_impl(pred_class, pred_density, target_density, target_is_reduced, points, offsets_host,
                          order_host, true, bins_lo, bins_hi, B, N, size, reduction, count_mode, norm_cood,
                          weight_count_loss, weight_ot, weight_tv, reg, max_iter, stop_thr, eval_freq, grad_class,
                          grad_density, losses, crop_stats, beta_out, status, workspace, workspace_bytes, stream);
}

// The loss's backward (_DaceFn): both kernel-made gradients times the upstream scalar (GradScaler's scale) in one
// launch, out of place (a retained graph may run the backward again)
__global__ __launch_bounds__(256) void scale2_kernel(const float* __restrict__ s, const float* __restrict__ a, float* ao,
                                                     long na, const float* __restrict__ b, float* bo, long nb)
{
    const float f = *s;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < na + nb; i += (long)gridDim.x * 256) {
        if (i < na) ao[i] = a[i] * f;
        else bo[i - na] = b[i - na] * f;
    }
}
extern "C" int ebc_scale2(const float* s, const float* a, float* a_out, long na, const float* b, float* b_out, long nb,
                          ebc_stream_t stream)
{
    if (!s || na < 0 || nb < 0 || (na && (!a || !a_out)) || (nb && (!b || !b_out))) return EBC_E_ARG;
    if (na + nb == 0) return EBC_OK;
    const long blocks = std::min<long>((na + nb + 255) / 256, 1024);
    hipLaunchKernelGGL(scale2_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, s, a, a_out, na, b, b_out, nb);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

extern "C" int ebc_version(void) { return 1; }

#ifdef EBC_DACE_PROF
extern "C" int ebc_dace_prof_read(unsigned long long* host, int nbytes)
{
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dace_prof), std::min<size_t>(nbytes, sizeof(g_dace_prof)), 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
