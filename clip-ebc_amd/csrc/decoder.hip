// Decoder BasicBlock of CLIP-EBC (ViT-B/16 backbone) on gfx950: bilinear x2 upsample, two 3x3
// convolutions as implicit GEMMs on the MFMA GEMM (gemm.hip MODE 1 / 2), training-mode BatchNorm
// (batch statistics from the GEMM epilogue), ReLU, the residual add, and the whole backward.
//
// Reference: reduction adapt F.interpolate(x2, bilinear)   models/clip/model.py:195-196
//            BasicBlock conv-bn-relu-conv-bn-add-relu     models/utils.py:254-303
//            (BatchNorm2d train statistics / running stats, SyncBatchNorm under DDP: trainer.py:147)
//
// Layouts (T = compute dtype: f32 parity mode, f16 / bf16 under autocast):
//   feat   [B][h][w][C] f32            encoder output (ln_post patch tokens, NHWC)
//   xpad   [B][Hp][Wp][C] T            zero-padded NHWC conv input (Hp = H+2, Wp >= W+2, see geo)
//   z      [B*H*W][N] T                conv output before BatchNorm
//   y      [B*H*W][C] T                block output (the projection GEMM's A operand)
//   xT3    [3][C][Qs] T                kx-shifted transposed copies for the weight gradient:
//                                      xT3[kx][c][G + q] = xpad[q + kx - 1][c] (0 outside)
//   dzT    [N][Qs] T                   transposed padded dz (0 outside the interior)
//   dw     [N][C][3][3] f32            weight gradient, nn.Conv2d layout
// Every kernel is HBM-bound elementwise / transpose work (4-wide vector accesses).
#include <algorithm>

#include "ebc_common.h"
#include "mfma.h"
#include "kernels.h"

using namespace ebc;

namespace {

template <class T> __device__ __forceinline__ void st4(T* p, float4 v);
template <> __device__ __forceinline__ void st4<float>(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
template <> __device__ __forceinline__ void st4<_Float16>(_Float16* p, float4 v) {
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    *reinterpret_cast<h4*>(p) = h4{(_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
}
template <> __device__ __forceinline__ void st4<__bf16>(__bf16* p, float4 v) {
    typedef __bf16 b4 __attribute__((ext_vector_type(4)));
    *reinterpret_cast<b4*>(p) = b4{(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
}
template <class T> __device__ __forceinline__ float4 ld4(const T* p);
template <> __device__ __forceinline__ float4 ld4<float>(const float* p) { return *reinterpret_cast<const float4*>(p); }
template <> __device__ __forceinline__ float4 ld4<_Float16>(const _Float16* p) {
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    const h4 v = *reinterpret_cast<const h4*>(p);
    return make_float4((float)v[0], (float)v[1], (float)v[2], (float)v[3]);
}
template <> __device__ __forceinline__ float4 ld4<__bf16>(const __bf16* p) {
    typedef __bf16 b4 __attribute__((ext_vector_type(4)));
    const b4 v = *reinterpret_cast<const b4*>(p);
    return make_float4((float)v[0], (float)v[1], (float)v[2], (float)v[3]);
}
__device__ __forceinline__ float4 f4(float a) { return make_float4(a, a, a, a); }
__device__ __forceinline__ float4 fma4(float4 a, float4 b, float4 c) {
    return make_float4(fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y), fmaf(a.z, b.z, c.z), fmaf(a.w, b.w, c.w));
}
__device__ __forceinline__ float4 relu4(float4 a) {
    return make_float4(fmaxf(a.x, 0.f), fmaxf(a.y, 0.f), fmaxf(a.z, 0.f), fmaxf(a.w, 0.f));
}

// Decoder geometry shared by every entry point (the transposed images' guards and row stride let the
// weight-gradient GEMM run its K loop over whole 64-pixel slabs with 16-B aligned rows).
struct Geo {
    int B, H, W, C, Hp, Wp, G, kpi, bk;
    long Q, Qs;
};
Geo make_geo(int dtype, int B, int H, int W, int C) {
    Geo g;
    g.B = B; g.H = H; g.W = W; g.C = C;
    g.Hp = H + 2;
    g.Wp = std::max(((W + 2 + 7) / 8) * 8, 32);      // >= bk/2: a slab overshoots into pad rows only
    g.bk = dtype == EBC_F32 ? 32 : 64;
    g.G = ((g.Wp + 1 + 63) / 64) * 64;
    g.Q = (long)B * g.Hp * g.Wp;
    g.kpi = (H * g.Wp + g.bk - 1) / g.bk;
    g.Qs = ((g.G + g.Q + g.bk + g.Wp + 63) / 64) * 64;
    return g;
}
struct DGeo {               // device copy
    int B, H, W, C, Hp, Wp, G;
    long Q, Qs;
};
DGeo dgeo(const Geo& g) { return DGeo{g.B, g.H, g.W, g.C, g.Hp, g.Wp, g.G, g.Q, g.Qs}; }

// padded position q -> interior pixel index p = (b*H + y)*W + x, or -1
__device__ __forceinline__ long interior(const DGeo& g, long q) {
    if (q < 0 || q >= g.Q) return -1;
    const int hw = g.Hp * g.Wp;
    const int b = (int)(q / hw), r = (int)(q - (long)b * hw), yp = r / g.Wp, xp = r - yp * g.Wp;
    if (yp < 1 || yp > g.H || xp < 1 || xp > g.W) return -1;
    return ((long)b * g.H + yp - 1) * g.W + xp - 1;
}

// F.interpolate(mode="bilinear", align_corners=False, scale_factor=up) source taps
// (aten area_pixel_compute_source_index + upsample_bilinear2d's h1/h1p/h1lambda)
struct Taps { int i0, i1; float l0, l1; };
__device__ __forceinline__ Taps taps(int o, int n, float scale) {
    float src = scale * ((float)o + 0.5f) - 0.5f;
    src = src < 0.f ? 0.f : src;
    const int i0 = (int)src;
    const float l1 = src - (float)i0;
    return Taps{i0, i0 + (i0 < n - 1 ? 1 : 0), 1.0f - l1, l1};
}
__device__ __forceinline__ float4 bilinear4(const float* feat, int b, int y, int x, int h, int w, int C, int c,
                                            float scale) {
    const Taps ty = taps(y, h, scale), tx = taps(x, w, scale);
    const float* f0 = feat + ((size_t)(b * h + ty.i0) * w) * C + c;
    const float* f1 = feat + ((size_t)(b * h + ty.i1) * w) * C + c;
    const float4 a = ld4(f0 + (size_t)tx.i0 * C), bb = ld4(f0 + (size_t)tx.i1 * C);
    const float4 cc = ld4(f1 + (size_t)tx.i0 * C), d = ld4(f1 + (size_t)tx.i1 * C);
    float4 r;
    r.x = ty.l0 * (tx.l0 * a.x + tx.l1 * bb.x) + ty.l1 * (tx.l0 * cc.x + tx.l1 * d.x);
    r.y = ty.l0 * (tx.l0 * a.y + tx.l1 * bb.y) + ty.l1 * (tx.l0 * cc.y + tx.l1 * d.y);
    r.z = ty.l0 * (tx.l0 * a.z + tx.l1 * bb.z) + ty.l1 * (tx.l0 * cc.z + tx.l1 * d.z);
    r.w = ty.l0 * (tx.l0 * a.w + tx.l1 * bb.w) + ty.l1 * (tx.l0 * cc.w + tx.l1 * d.w);
    return r;
}

// ------------------------------------------------------------------ forward
template <class T>
__global__ __launch_bounds__(256) void upsample_pad_kernel(const float* __restrict__ feat, T* __restrict__ xpad,
                                                           DGeo g, int h, int w, float scale)
{
    const int C4 = g.C / 4;
    const long e = (long)blockIdx.x * 256 + threadIdx.x;
    if (e >= g.Q * C4) return;
    const long q = e / C4;
    const int c = (int)(e - q * C4) * 4;
    const long p = interior(g, q);
    float4 v = f4(0.f);
    if (p >= 0) {
        const int hw = g.H * g.W, b = (int)(p / hw), r = (int)(p - (long)b * hw), y = r / g.W, x = r - y * g.W;
        v = bilinear4(feat, b, y, x, h, w, g.C, c, scale);
    }
    st4(xpad + q * g.C + c, v);
}

template <class T>
__global__ __launch_bounds__(256) void bn_relu_pad_kernel(const T* __restrict__ z, const float* __restrict__ scale,
                                                          const float* __restrict__ shift, T* __restrict__ hpad, DGeo g)
{
    const int C4 = g.C / 4;
    const long e = (long)blockIdx.x * 256 + threadIdx.x;
    if (e >= g.Q * C4) return;
    const long q = e / C4;
    const int c = (int)(e - q * C4) * 4;
    const long p = interior(g, q);
    float4 v = f4(0.f);
    if (p >= 0) v = relu4(fma4(ld4(z + p * g.C + c), ld4(scale + c), ld4(shift + c)));
    st4(hpad + q * g.C + c, v);
}

template <class T>
__global__ __launch_bounds__(256) void bn_add_relu_kernel(const T* __restrict__ z, const float* __restrict__ scale,
                                                          const float* __restrict__ shift, const float* __restrict__ feat,
                                                          T* __restrict__ y, long P, int H, int W, int C, int h, int w,
                                                          float fscale)
{
    const int C4 = C / 4;
    const long e = (long)blockIdx.x * 256 + threadIdx.x;
    if (e >= P * C4) return;
    const long p = e / C4;
    const int c = (int)(e - p * C4) * 4;
    const int hw = H * W, b = (int)(p / hw), r = (int)(p - (long)b * hw), yy = r / W, xx = r - yy * W;
    float4 v = fma4(ld4(z + p * C + c), ld4(scale + c), ld4(shift + c));
    const float4 res = bilinear4(feat, b, yy, xx, h, w, C, c, fscale);       // downsample = Identity: + x
    v.x += res.x; v.y += res.y; v.z += res.z; v.w += res.w;
    st4(y + p * C + c, relu4(v));
}

// per-tile column partials [nb][2C] -> f64 column sums [2C]: 64 columns x 16 row groups per block
// (many independent loads in flight; the partial count is ~50-200)
__global__ __launch_bounds__(1024) void reduce_partials_kernel(const float* __restrict__ part, int nb, int C2,
                                                               double* __restrict__ out)
{
    __shared__ double red[16][64];
    const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + cl;
    double s = 0.0;
    if (c < C2) {
#pragma unroll 4
        for (int i = rg; i < nb; i += 16) s += (double)part[(size_t)i * C2 + c];
    }
    red[rg][cl] = s;
    __syncthreads();
    if (rg == 0 && c < C2) {
        double r = 0.0;
#pragma unroll
        for (int k = 0; k < 16; ++k) r += red[k][cl];
        out[c] = r;
    }
}

// BatchNorm2d (training: batch mean / biased variance, running stats with momentum and the unbiased
// variance; eval: running stats), folded into a per-channel scale/shift
__global__ __launch_bounds__(256) void bn_fwd_finalize_kernel(const double* __restrict__ sums, double count, float eps,
                                                              float momentum, const float* __restrict__ gamma,
                                                              const float* __restrict__ beta, float* mean, float* rstd,
                                                              float* scale, float* shift, float* rmean, float* rvar, int C)
{
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= C) return;
    double m, var;
    if (sums) {
        m = sums[c] / count;
        var = sums[C + c] / count - m * m;
        var = var > 0.0 ? var : 0.0;
        if (rmean) rmean[c] = (float)((1.0 - momentum) * (double)rmean[c] + momentum * m);
        if (rvar) rvar[c] = (float)((1.0 - momentum) * (double)rvar[c] + momentum * var * count / (count - 1.0));
    } else {
        m = rmean[c];
        var = rvar[c];
    }
    const float rs = (float)(1.0 / sqrt(var + (double)eps));
    const float sc = gamma[c] * rs;
    mean[c] = (float)m;
    rstd[c] = rs;
    scale[c] = sc;
    shift[c] = beta[c] - (float)m * sc;
}

// ------------------------------------------------------------------ backward
// g = gy * relu'(.)  with the ReLU mask from the stored output (mask_y) or recomputed from z
template <class T>
__device__ __forceinline__ float4 masked_grad(const T* gy, const T* my, const T* z, const float* scale,
                                              const float* shift, long off, int c) {
    const float4 gv = ld4(gy + off);
    float4 m;
    if (my) {
        m = ld4(my + off);
    } else {
        m = fma4(ld4(z + off), ld4(scale + c), ld4(shift + c));
    }
    return make_float4(m.x > 0.f ? gv.x : 0.f, m.y > 0.f ? gv.y : 0.f, m.z > 0.f ? gv.z : 0.f, m.w > 0.f ? gv.w : 0.f);
}

// column partials of sum(g) and sum(g * xhat), xhat = (z - mean) * rstd; block = (C/4) x RL threads
template <class T>
__global__ __launch_bounds__(512) void bn_bwd_partial_kernel(const T* __restrict__ gy, const T* __restrict__ my,
                                                             const T* __restrict__ z, const float* __restrict__ mean,
                                                             const float* __restrict__ rstd,
                                                             const float* __restrict__ scale,
                                                             const float* __restrict__ shift, float* __restrict__ part,
                                                             long P, int C, int rows_per_block)
{
    extern __shared__ float red[];                // [RL][2][C]
    const int C4 = C / 4, RL = blockDim.x / C4;
    const int cg = threadIdx.x % C4, rl = threadIdx.x / C4, c = cg * 4;
    const long r0 = (long)blockIdx.x * rows_per_block;
    const long r1 = std::min<long>(P, r0 + rows_per_block);
    const float4 mu = ld4(mean + c), rs = ld4(rstd + c);
    float4 s1 = f4(0.f), s2 = f4(0.f);
    if (rl < RL) {
        for (long r = r0 + rl; r < r1; r += RL) {
            const long off = r * C + c;
            const float4 gv = masked_grad(gy, my, z, scale, shift, off, c);
            const float4 zv = ld4(z + off);
            s1.x += gv.x; s1.y += gv.y; s1.z += gv.z; s1.w += gv.w;
            s2.x = fmaf(gv.x, (zv.x - mu.x) * rs.x, s2.x);
            s2.y = fmaf(gv.y, (zv.y - mu.y) * rs.y, s2.y);
            s2.z = fmaf(gv.z, (zv.z - mu.z) * rs.z, s2.z);
            s2.w = fmaf(gv.w, (zv.w - mu.w) * rs.w, s2.w);
        }
        *reinterpret_cast<float4*>(red + (size_t)rl * 2 * C + c) = s1;
        *reinterpret_cast<float4*>(red + (size_t)rl * 2 * C + C + c) = s2;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 2 * C; e += blockDim.x) {
        float s = 0.f;
        for (int k = 0; k < RL; ++k) s += red[(size_t)k * 2 * C + e];
        part[(size_t)blockIdx.x * 2 * C + e] = s;
    }
}

// dgamma = sum(g*xhat), dbeta = sum(g); coef = [gamma*rstd, sum(g)/count, sum(g*xhat)/count]
__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(const double* __restrict__ sums, double count,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ rstd, float* dgamma,
                                                              float* dbeta, float* coef, int C)
{
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= C) return;
    const double sg = sums[c], sgx = sums[C + c];
    if (dgamma) dgamma[c] = (float)sgx;
    if (dbeta) dbeta[c] = (float)sg;
    coef[c] = gamma[c] * rstd[c];
    coef[C + c] = (float)(sg / count);
    coef[2 * C + c] = (float)(sgx / count);
}

// Tiles of 64 padded positions x 64 channels, staged through LDS so that both the NHWC-padded image
// (rows of channels) and the transposed image (rows of positions) are written with contiguous rows.
constexpr int TQ = 64, TC = 64;

// dz = gamma*rstd * (g - mean(g) - xhat * mean(g*xhat)) -> dzpad [Q][C] and dzT [C][Qs]
template <class T>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const T* __restrict__ gy, const T* __restrict__ my,
                                                           const T* __restrict__ z, const float* __restrict__ mean,
                                                           const float* __restrict__ rstd,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ shift,
                                                           const float* __restrict__ coef, T* __restrict__ dzpad,
                                                           T* __restrict__ dzT, DGeo g)
{
    __shared__ float sm[TQ][TC + 1];
    const int t = threadIdx.x;
    const long j0 = (long)blockIdx.x * TQ;
    const int c0 = blockIdx.y * TC;
    {
        const int ql = t >> 2, cl = (t & 3) * 16;
        const long q = j0 + ql - g.G;
        const long p = interior(g, q);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int c = c0 + cl + 4 * k;
            float4 v = f4(0.f);
            if (p >= 0) {
                const long off = p * g.C + c;
                const float4 gv = masked_grad(gy, my, z, scale, shift, off, c);
                const float4 zv = ld4(z + off), mu = ld4(mean + c), rs = ld4(rstd + c);
                const float4 a = ld4(coef + c), mg = ld4(coef + g.C + c), mgx = ld4(coef + 2 * g.C + c);
                v.x = a.x * (gv.x - mg.x - (zv.x - mu.x) * rs.x * mgx.x);
                v.y = a.y * (gv.y - mg.y - (zv.y - mu.y) * rs.y * mgx.y);
                v.z = a.z * (gv.z - mg.z - (zv.z - mu.z) * rs.z * mgx.z);
                v.w = a.w * (gv.w - mg.w - (zv.w - mu.w) * rs.w * mgx.w);
            }
            if (q >= 0 && q < g.Q) st4(dzpad + q * g.C + c, v);
            sm[ql][cl + 4 * k] = v.x; sm[ql][cl + 4 * k + 1] = v.y;
            sm[ql][cl + 4 * k + 2] = v.z; sm[ql][cl + 4 * k + 3] = v.w;
        }
    }
    __syncthreads();
    {
        const int cr = t >> 2, jl = (t & 3) * 16;
        T* dst = dzT + (size_t)(c0 + cr) * g.Qs + j0 + jl;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            st4(dst + 4 * k, make_float4(sm[jl + 4 * k][cr], sm[jl + 4 * k + 1][cr], sm[jl + 4 * k + 2][cr],
                                         sm[jl + 4 * k + 3][cr]));
    }
}

// xT3[kx][c][G + q] = xpad[q + kx - 1][c]  (xpad is zero outside the interior; 0 beyond [0, Q))
template <class T>
__global__ __launch_bounds__(256) void transpose3_kernel(const T* __restrict__ xpad, T* __restrict__ xT3, DGeo g)
{
    __shared__ float sm[TQ + 2][TC + 1];
    const int t = threadIdx.x;
    const long j0 = (long)blockIdx.x * TQ;
    const int c0 = blockIdx.y * TC;
    constexpr int NE = (TQ + 2) * (TC / 4), PER = (NE + 255) / 256;
    float4 v[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {                // all loads in flight before the LDS writes
        const int e = t + 256 * k, ql = e / (TC / 4), cl = (e % (TC / 4)) * 4;
        const long q = j0 - g.G + ql - 1;
        v[k] = (e < NE && q >= 0 && q < g.Q) ? ld4(xpad + q * g.C + c0 + cl) : f4(0.f);
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int e = t + 256 * k, ql = e / (TC / 4), cl = (e % (TC / 4)) * 4;
        if (e < NE) { sm[ql][cl] = v[k].x; sm[ql][cl + 1] = v[k].y; sm[ql][cl + 2] = v[k].z; sm[ql][cl + 3] = v[k].w; }
    }
    __syncthreads();
    const int cr = t >> 2, jl = (t & 3) * 16;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
        T* dst = xT3 + ((size_t)kx * g.C + c0 + cr) * g.Qs + j0 + jl;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int s = jl + 4 * k + kx;
            st4(dst + 4 * k, make_float4(sm[s][cr], sm[s + 1][cr], sm[s + 2][cr], sm[s + 3][cr]));
        }
    }
}

// dfeat = bilinear^T (g), g = conv1's input gradient + the residual branch's (already summed by the
// dgrad GEMM epilogue): input cell i collects output rows/columns UP*i - UP/2 .. +2*UP-1 (zero weight
// where a tap misses i); all loads issued without data-dependent branches
template <class T, int UP>
__global__ __launch_bounds__(256) void upsample_bwd_kernel(const T* __restrict__ g, float* __restrict__ dfeat, int B,
                                                           int h, int w, int H, int W, int C)
{
    constexpr int NCAND = 2 * UP;
    constexpr float scale = 1.0f / (float)UP;
    const int C4 = C / 4;
    const long e = (long)blockIdx.x * 256 + threadIdx.x;
    if (e >= (long)B * h * w * C4) return;
    const long cell = e / C4;
    const int c = (int)(e - cell * C4) * 4;
    const int b = (int)(cell / (h * w)), r = (int)(cell - (long)b * h * w), i = r / w, j = r - i * w;
    float wy[NCAND], wx[NCAND];
    int oy[NCAND], ox[NCAND];
#pragma unroll
    for (int k = 0; k < NCAND; ++k) {
        const int y = UP * i - UP / 2 + k, x = UP * j - UP / 2 + k;
        oy[k] = min(max(y, 0), H - 1);
        ox[k] = min(max(x, 0), W - 1);
        const Taps ty = taps(oy[k], h, scale), tx = taps(ox[k], w, scale);
        wy[k] = (y >= 0 && y < H) ? (ty.i0 == i ? ty.l0 : 0.f) + (ty.i1 == i ? ty.l1 : 0.f) : 0.f;
        wx[k] = (x >= 0 && x < W) ? (tx.i0 == j ? tx.l0 : 0.f) + (tx.i1 == j ? tx.l1 : 0.f) : 0.f;
    }
    float4 acc = f4(0.f);
#pragma unroll
    for (int a = 0; a < NCAND; ++a)
#pragma unroll
        for (int k = 0; k < NCAND; ++k)
            acc = fma4(f4(wy[a] * wx[k]), ld4(g + (((long)b * H + oy[a]) * W + ox[k]) * C + c), acc);
    *reinterpret_cast<float4*>(dfeat + cell * C + c) = acc;
}

// conv weight [N][C][3][3] f32 (nn.Conv2d) -> forward operand wk [N][3][3][C] and flipped data-gradient
// operand wf [C][3][3][N] (wf[c][t][o] = w[o][c][8 - t]) in the compute dtype; 32x32 (o, c) tiles in LDS
template <class T>
__global__ __launch_bounds__(256) void prep_weights_kernel(const float* __restrict__ w, T* __restrict__ wk,
                                                           T* __restrict__ wf, int N, int C)
{
    __shared__ float sm[32][32 * 9 + 1];           // [o][c*9 + t]
    const int o0 = blockIdx.x * 32, c0 = blockIdx.y * 32, t = threadIdx.x;
    constexpr int PER = 32 * 32 * 9 / 256;         // 36 loads per thread, all issued before the LDS writes
    float v[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int e = t + 256 * k, ol = e / (32 * 9), r = e - ol * 32 * 9;
        v[k] = (o0 + ol < N && c0 + r / 9 < C) ? w[((size_t)(o0 + ol) * C + c0) * 9 + r] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int e = t + 256 * k, ol = e / (32 * 9), r = e - ol * 32 * 9;
        sm[ol][r] = v[k];
    }
    __syncthreads();
    for (int e = t; e < 32 * 9 * 32; e += 256) {   // wk rows (o, tap): 32 contiguous c
        const int cl = e & 31, r = e >> 5, ol = r / 9, tap = r - ol * 9;
        if (o0 + ol < N && c0 + cl < C) wk[((size_t)(o0 + ol) * 9 + tap) * C + c0 + cl] = (T)sm[ol][cl * 9 + tap];
    }
    for (int e = t; e < 32 * 9 * 32; e += 256) {   // wf rows (c, tap): 32 contiguous o
        const int ol = e & 31, r = e >> 5, cl = r / 9, tap = r - cl * 9;
        if (o0 + ol < N && c0 + cl < C) wf[((size_t)(c0 + cl) * 9 + tap) * N + o0 + ol] = (T)sm[ol][cl * 9 + 8 - tap];
    }
}

inline unsigned nblk(long n) { return (unsigned)((n + 255) / 256); }

template <class T>
int bn_bwd_reduce_t(const void* gy, const void* my, const void* z, const float* mean, const float* rstd,
                    const float* scale, const float* shift, double* sums, void* ws, size_t wsb, long P, int C,
                    hipStream_t st)
{
    const int C4 = C / 4;
    const int RL = std::max(1, 512 / C4);
    const int threads = C4 * RL;
    const int rpb = 64;
    const long nb = (P + rpb - 1) / rpb;
    const size_t need = CONV_WS_STATS_OFFSET + (size_t)nb * 2 * C * 4;
    if (!ws || wsb < need || threads > 1024) return EBC_E_ARG;
    float* part = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + CONV_WS_STATS_OFFSET);
    hipLaunchKernelGGL(bn_bwd_partial_kernel<T>, dim3((unsigned)nb), dim3(threads), (size_t)RL * 2 * C * 4, st,
                       (const T*)gy, (const T*)my, (const T*)z, mean, rstd, scale, shift, part, P, C, rpb);
    hipLaunchKernelGGL(reduce_partials_kernel, dim3((2 * C + 63) / 64), dim3(1024), 0, st, (const float*)part, (int)nb,
                       2 * C, sums);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

}  // namespace

// ---------------------------------------------------------------------------------------- C-ABI
#define EBC_DTYPE_SWITCH(dtype, ...)                                   \
    switch (dtype) {                                                   \
        case EBC_F32: { using T = float; __VA_ARGS__; } break;         \
        case EBC_F16: { using T = _Float16; __VA_ARGS__; } break;      \
        case EBC_BF16: { using T = __bf16; __VA_ARGS__; } break;       \
        default: return EBC_E_ARG;                                     \
    }

extern "C" int ebc_dec_geometry(int dtype, int B, int H, int W, int C, long* out)
{
    if (B <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 64 || !out) return EBC_E_ARG;
    const Geo g = make_geo(dtype, B, H, W, C);
    out[0] = g.Hp; out[1] = g.Wp; out[2] = g.G; out[3] = g.kpi; out[4] = g.Q; out[5] = g.Qs;
    return EBC_OK;
}

extern "C" size_t ebc_dec_workspace_bytes(int dtype, int B, int H, int W, int C, int N)
{
    const Geo g = make_geo(dtype, B, H, W, C);
    const int M = B * H * W;
    size_t need = ebc::conv_gemm_workspace_bytes(dtype, 1, M, N, 9 * C);
    need = std::max(need, ebc::conv_gemm_workspace_bytes(dtype, 1, M, C, 9 * N));
    need = std::max(need, ebc::conv_gemm_workspace_bytes(dtype, 2, N, 9 * C, B * g.kpi * g.bk));
    const long nb = ((long)M + 63) / 64;
    need = std::max(need, CONV_WS_STATS_OFFSET + (size_t)nb * 2 * std::max(C, N) * 4);
    return need;
}

extern "C" int ebc_dec_upsample_pad(int dtype, const float* feat, void* xpad, int B, int h, int w, int C, int up,
                                    ebc_stream_t stream)
{
    if (!feat || !xpad || up < 1 || C % 64) return EBC_E_ARG;
    const Geo g = make_geo(dtype, B, h * up, w * up, C);
    const DGeo d = dgeo(g);
    EBC_DTYPE_SWITCH(dtype, hipLaunchKernelGGL(upsample_pad_kernel<T>, dim3(nblk(g.Q * (C / 4))), dim3(256), 0,
                                               (hipStream_t)stream, feat, (T*)xpad, d, h, w, 1.0f / (float)up));
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

extern "C" int ebc_conv3x3_fwd(int dtype, const void* xpad, const void* weight, void* out, double* colsum,
                               const void* add_gy, const void* add_y, void* ws, size_t wsb, int B, int H, int W, int C,
                               int N, ebc_stream_t stream)
{
    if (!xpad || !weight || !out || C % 64 || N % 64 || (colsum && add_gy) || (!add_gy != !add_y)) return EBC_E_ARG;
    const Geo g = make_geo(dtype, B, H, W, C);
    ebc::ConvGeom cg{H, W, C, g.Hp, g.Wp, 0, 0, 0};
    const int M = B * H * W;
    int tiles = 0;
    const hipStream_t st = (hipStream_t)stream;
    const int epi = colsum ? 4 : (add_gy ? 5 : 0);
    EBC_TRY(ebc::conv_gemm(dtype, 1, epi, xpad, weight, out, cg, M, N, 9 * C, ws, wsb, &tiles, st, add_gy, add_y));
    if (colsum) {
        const float* part = reinterpret_cast<const float*>(reinterpret_cast<const char*>(ws) + CONV_WS_STATS_OFFSET);
        hipLaunchKernelGGL(reduce_partials_kernel, dim3((2 * N + 63) / 64), dim3(1024), 0, st, part, tiles, 2 * N, colsum);
        EBC_CHECK_LAUNCH();
    }
    return EBC_OK;
}

extern "C" int ebc_conv3x3_wgrad(int dtype, const void* dzT, const void* xT3, float* dw, void* ws, size_t wsb, int B,
                                 int H, int W, int C, int N, ebc_stream_t stream)
{
    if (!dzT || !xT3 || !dw || C % 64 || N % 64) return EBC_E_ARG;
    const Geo g = make_geo(dtype, B, H, W, C);
    ebc::ConvGeom cg{H, W, C, g.Hp, g.Wp, g.kpi, g.Qs, g.G};
    return ebc::conv_gemm(dtype, 2, 0, dzT, xT3, dw, cg, N, 9 * C, B * g.kpi * g.bk, ws, wsb, nullptr,
                          (hipStream_t)stream);
}

extern "C" int ebc_bn_finalize(const double* colsum, double count, float eps, float momentum, const float* gamma,
                               const float* beta, float* mean, float* rstd, float* scale, float* shift,
                               float* running_mean, float* running_var, int C, ebc_stream_t stream)
{
    if (!gamma || !beta || !mean || !rstd || !scale || !shift) return EBC_E_ARG;
    if (!colsum && (!running_mean || !running_var)) return EBC_E_ARG;
    if (colsum && count <= 1.0) return EBC_E_ARG;
    hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3(nblk(C)), dim3(256), 0, (hipStream_t)stream, colsum, count, eps,
                       momentum, gamma, beta, mean, rstd, scale, shift, running_mean, running_var, C);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

extern "C" int ebc_bn_relu_pad(int dtype, const void* z, const float* scale, const float* shift, void* hpad, int B,
                               int H, int W, int C, ebc_stream_t stream)
{
    if (!z || !scale || !shift || !hpad || C % 64) return EBC_E_ARG;
    const Geo g = make_geo(dtype, B, H, W, C);
    const DGeo d = dgeo(g);
    EBC_DTYPE_SWITCH(dtype, hipLaunchKernelGGL(bn_relu_pad_kernel<T>, dim3(nblk(g.Q * (C / 4))), dim3(256), 0,
                                               (hipStream_t)stream, (const T*)z, scale, shift, (T*)hpad, d));
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

extern "C" int ebc_bn_add_relu(int dtype, const void* z, const float* scale, const float* shift, const float* feat,
                               int up, void* y, int B, int H, int W, int C, ebc_stream_t stream)
{
    if (!z || !scale || !shift || !feat || !y || up < 1 || H % up || W % up || C % 4) return EBC_E_ARG;
    const long P = (long)B * H * W;
    EBC_DTYPE_SWITCH(dtype, hipLaunchKernelGGL(bn_add_relu_kernel<T>, dim3(nblk(P * (C / 4))), dim3(256), 0,
                                               (hipStream_t)stream, (const T*)z, scale, shift, feat, (T*)y, P, H, W, C,
                                               H / up, W / up, 1.0f / (float)up));
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

extern "C" int ebc_bn_bwd_reduce(int dtype, const void* gy, const void* mask_y, const void* z, const float* mean,
                                 const float* rstd, const float* scale, const float* shift, double* sums, void* ws,
                                 size_t wsb, long P, int C, ebc_stream_t stream)
{
    if (!gy || !z || !mean || !rstd || !sums || C % 4 || (!mask_y && (!scale || !shift))) return EBC_E_ARG;
    const hipStream_t st = (hipStream_t)stream;
    switch (dtype) {
        case EBC_F32: return bn_bwd_reduce_t<float>(gy, mask_y, z, mean, rstd, scale, shift, sums, ws, wsb, P, C, st);
        case EBC_F16: return bn_bwd_reduce_t<_Float16>(gy, mask_y, z, mean, rstd, scale, shift, sums, ws, wsb, P, C, st);
        case EBC_BF16: return bn_bwd_reduce_t<__bf16>(gy, mask_y, z, mean, rstd, scale, shift, sums, ws, wsb, P, C, st);
    }
    return EBC_E_ARG;
}

extern "C" int ebc_bn_bwd_finalize(const double* sums, double count, const float* gamma, const float* rstd,
                                   float* dgamma, float* dbeta, float* coef, int C, ebc_stream_t stream)
{
    if (!sums || !gamma || !rstd || !coef || count <= 0.0) return EBC_E_ARG;
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(nblk(C)), dim3(256), 0, (hipStream_t)stream, sums, count, gamma,
                       rstd, dgamma, dbeta, coef, C);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

extern "C" int ebc_bn_bwd_apply(int dtype, const void* gy, const void* mask_y, const void* z, const float* mean,
                                const float* rstd, const float* scale, const float* shift, const float* coef,
                                void* dzpad, void* dzT, int B, int H, int W, int C, ebc_stream_t stream)
{
    if (!gy || !z || !mean || !rstd || !coef || !dzpad || !dzT || C % TC || (!mask_y && (!scale || !shift)))
        return EBC_E_ARG;
    const Geo g = make_geo(dtype, B, H, W, C);
    const DGeo d = dgeo(g);
    const dim3 grid((unsigned)(g.Qs / TQ), (unsigned)(C / TC));
    EBC_DTYPE_SWITCH(dtype, hipLaunchKernelGGL(bn_bwd_apply_kernel<T>, grid, dim3(256), 0, (hipStream_t)stream,
                                               (const T*)gy, (const T*)mask_y, (const T*)z, mean, rstd, scale, shift,
                                               coef, (T*)dzpad, (T*)dzT, d));
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

extern "C" int ebc_dec_transpose3(int dtype, const void* xpad, void* xT3, int B, int H, int W, int C,
                                  ebc_stream_t stream)
{
    if (!xpad || !xT3 || C % TC) return EBC_E_ARG;
    const Geo g = make_geo(dtype, B, H, W, C);
    const DGeo d = dgeo(g);
    const dim3 grid((unsigned)(g.Qs / TQ), (unsigned)(C / TC));
    EBC_DTYPE_SWITCH(dtype, hipLaunchKernelGGL(transpose3_kernel<T>, grid, dim3(256), 0, (hipStream_t)stream,
                                               (const T*)xpad, (T*)xT3, d));
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

extern "C" int ebc_dec_upsample_bwd(int dtype, const void* g, float* dfeat, int B, int h, int w, int C, int up,
                                    ebc_stream_t stream)
{
    if (!g || !dfeat || C % 4) return EBC_E_ARG;
    if (up != 1 && up != 2) return EBC_E_UNSUPPORTED;
    const long cells = (long)B * h * w;
    const unsigned grid = nblk(cells * (C / 4));
    const hipStream_t st = (hipStream_t)stream;
    if (up == 2) {
        EBC_DTYPE_SWITCH(dtype, hipLaunchKernelGGL((upsample_bwd_kernel<T, 2>), dim3(grid), dim3(256), 0, st,
                                                   (const T*)g, dfeat, B, h, w, 2 * h, 2 * w, C));
    } else {
        EBC_DTYPE_SWITCH(dtype, hipLaunchKernelGGL((upsample_bwd_kernel<T, 1>), dim3(grid), dim3(256), 0, st,
                                                   (const T*)g, dfeat, B, h, w, h, w, C));
    }
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

extern "C" int ebc_dec_prep_weights(int dtype, const float* w, void* wk, void* wf, int N, int C, ebc_stream_t stream)
{
    if (!w || !wk || !wf || N <= 0 || C <= 0) return EBC_E_ARG;
    const dim3 grid((unsigned)((N + 31) / 32), (unsigned)((C + 31) / 32));
    EBC_DTYPE_SWITCH(dtype, hipLaunchKernelGGL(prep_weights_kernel<T>, grid, dim3(256), 0, (hipStream_t)stream, w,
                                               (T*)wk, (T*)wf, N, C));
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}
