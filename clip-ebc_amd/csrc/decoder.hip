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
//   xT3    [3][C][Qs] T                kx-shifted transposed row-padded copies for the weight gradient:
//                                      xT3[kx][c][b*Pimg + yp*W + x] = x[b][yp - 1][x + kx - 1] (0 outside),
//                                      Pimg = (H + 2) * W rounded up to 8 and >= HWp (a zero row above and below
//                                      every image, zeros to the next image)
//   dzT    [N][Qs] T                   transposed dz over the weight gradient's K: column b*HWp + r = interior
//                                      pixel r of image b (HWp = H*W rounded up to 8; 0 beyond H*W)
//   dw     [N][C][3][3] f32            weight gradient, nn.Conv2d layout
// Every kernel is HBM-bound elementwise / transpose work (4-wide vector accesses).
//
// The ResNet-50 decoder Bottleneck (models/utils.py:306-363, expansion 1: conv1x1-bn-relu-conv3x3-bn-relu-
// conv1x1-bn-add-relu) reuses the 3x3 machinery for its middle conv; its two 1x1 convs are plain MFMA GEMMs
// on the unpadded [B*H*W][C] rows, with the flat-layout helpers below (upsample, BN statistics, BN+ReLU,
// BN input gradient with the identity branch's masked gradient).
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
// 8 consecutive elements (16 B for 16-bit types, 32 B for f32) <-> float[8]
template <class T> __device__ __forceinline__ void ld8(const T* p, float* v) {
    typedef T t8 __attribute__((ext_vector_type(8)));
    const t8 x = *reinterpret_cast<const t8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)x[i];
}
template <class T> __device__ __forceinline__ void st8(T* p, const float* v) {
    typedef T t8 __attribute__((ext_vector_type(8)));
    t8 x;
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = (T)v[i];
    *reinterpret_cast<t8*>(p) = x;
}
__device__ __forceinline__ float4 f4(float a) { return make_float4(a, a, a, a); }
// 8 consecutive per-channel f32 parameters (two 16-B loads; c a multiple of 8)
__device__ __forceinline__ void ldp8(const float* p, float* v) {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ float4 fma4(float4 a, float4 b, float4 c) {
    return make_float4(fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y), fmaf(a.z, b.z, c.z), fmaf(a.w, b.w, c.w));
}
__device__ __forceinline__ float4 relu4(float4 a) {
    return make_float4(fmaxf(a.x, 0.f), fmaxf(a.y, 0.f), fmaxf(a.z, 0.f), fmaxf(a.w, 0.f));
}

// Decoder geometry shared by every entry point.  MODE 1 (convs, data gradient): zero-padded NHWC images
// [B][Hp][Wp][C], Wp a multiple of 8 (16-B aligned tap shifts).  MODE 2 (weight gradient): its K runs over the
// interior pixels only -- B*H*W of them, each image's rounded up to HWp = a multiple of 8 (and >= 64) so a 16-B K
// chunk never spans two images -- (r03's K loop ran over the padded rows of pitch Wp: 12.5 % of its MFMA work multiplied zeros
// at 28x28); the kx shift of a tap is baked into three transposed copies of the input, the ky shift is a row offset
// into their row-padded images (Pimg >= (H + 2) * W positions each).  Kq = the GEMM's K (B*HWp rounded up to 64),
// Qs = the row stride of dz^T and of the x^T copies (room for the K tail's reads past the last image).
struct Geo {
    int B, H, W, C, Hp, Wp, HWp;
    long Q, Kq, Pimg, Qs;
};
Geo make_geo(int /*dtype*/, int B, int H, int W, int C) {
    Geo g;
    g.B = B; g.H = H; g.W = W; g.C = C;
    g.Hp = H + 2;
    g.Wp = std::max(((W + 2 + 7) / 8) * 8, 32);
    g.Q = (long)B * g.Hp * g.Wp;
    g.HWp = std::max(((H * W + 7) / 8) * 8, 64);        // >= 64: a 64-wide K tile crosses at most one image edge
    g.Kq = (((long)B * g.HWp + 63) / 64) * 64;
    g.Pimg = ((std::max((long)(H + 2) * W, (long)g.HWp) + 7) / 8) * 8;    // image bases 16-B aligned, >= HWp
    const long tail = (long)(B + 2 + 64 / g.HWp) * g.Pimg + g.HWp + 2L * W + 64;
    g.Qs = ((std::max(g.Kq, tail) + 63) / 64) * 64;
    return g;
}
struct DGeo {               // device copy
    int B, H, W, C, Hp, Wp, HWp;
    long Q, Kq, Pimg, Qs;
};
DGeo dgeo(const Geo& g) { return DGeo{g.B, g.H, g.W, g.C, g.Hp, g.Wp, g.HWp, g.Q, g.Kq, g.Pimg, g.Qs}; }

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
// The row kernels below: one image row per blockIdx.y (b * rows + r: the position / pixel row is wave-uniform),
// blockIdx.x * 256 + threadIdx.x = (position in the row, a V-channel chunk), 32-bit index math, V = 8 channels a lane
// (16-B stores of the 16-bit outputs) where C allows.  (r06: the flat form -- one 64-bit division of the element
// index and two more in interior() per 4 channels -- was VALU-bound: upsample_pad 19.3, bn_relu_pad 13.6,
// bn_add_relu 18.2 us in-step at 16 crops.)  Same arithmetic per element.
// XCD order for the 2-D row grids (mfma.h xcd_remap on the dispatch-linear id, x fastest): each XCD takes a contiguous
// run of image rows, so the bilinear taps that neighbouring rows share are fetched into one XCD's L2 (r06 PMC: the
// dispatch order spread them over the XCDs -- upsample_pad fetched 4x, bn_add_relu 7x, upsample_bwd 3x its bytes)
__device__ __forceinline__ void xcd_block2d(int& bx, int& by) {
    const int nx = (int)gridDim.x, id = xcd_remap((int)(blockIdx.y * gridDim.x + blockIdx.x), nx * (int)gridDim.y);
    by = id / nx;
    bx = id - by * nx;
}
template <class T, int V> __device__ __forceinline__ void stv(T* p, const float* v) {
    if constexpr (V == 8) st8(p, v);
    else st4(p, make_float4(v[0], v[1], v[2], v[3]));
}
template <class T, int V>
__global__ __launch_bounds__(256) void upsample_pad_kernel(const float* __restrict__ feat, T* __restrict__ xpad,
                                                           DGeo g, int h, int w, float scale)
{
    int bx, row;
    xcd_block2d(bx, row);
    const int b = row / g.Hp, yp = row - b * g.Hp;                         // padded row yp of image b
    const int CV = g.C / V, i = bx * 256 + threadIdx.x;
    if (i >= g.Wp * CV) return;
    const int xp = i / CV, c = (i - xp * CV) * V;
    float v[V];
#pragma unroll
    for (int k = 0; k < V; ++k) v[k] = 0.f;
    if (yp >= 1 && yp <= g.H && xp >= 1 && xp <= g.W) {
#pragma unroll
        for (int k = 0; k < V; k += 4) {
            const float4 r = bilinear4(feat, b, yp - 1, xp - 1, h, w, g.C, c + k, scale);
            v[k] = r.x; v[k + 1] = r.y; v[k + 2] = r.z; v[k + 3] = r.w;
        }
    }
    stv<T, V>(xpad + ((size_t)row * g.Wp + xp) * g.C + c, v);
}

template <class T, int V>
__global__ __launch_bounds__(256) void bn_relu_pad_kernel(const T* __restrict__ z, const float* __restrict__ scale,
                                                          const float* __restrict__ shift, T* __restrict__ hpad, DGeo g)
{
    const int row = blockIdx.y, b = row / g.Hp, yp = row - b * g.Hp;
    const int CV = g.C / V, i = blockIdx.x * 256 + threadIdx.x;
    if (i >= g.Wp * CV) return;
    const int xp = i / CV, c = (i - xp * CV) * V;
    float v[V];
#pragma unroll
    for (int k = 0; k < V; ++k) v[k] = 0.f;
    if (yp >= 1 && yp <= g.H && xp >= 1 && xp <= g.W) {
        const T* zp = z + ((size_t)(b * g.H + yp - 1) * g.W + xp - 1) * g.C + c;
#pragma unroll
        for (int k = 0; k < V; k += 4) {
            const float4 r = relu4(fma4(ld4(zp + k), ld4(scale + c + k), ld4(shift + c + k)));
            v[k] = r.x; v[k + 1] = r.y; v[k + 2] = r.z; v[k + 3] = r.w;
        }
    }
    stv<T, V>(hpad + ((size_t)row * g.Wp + xp) * g.C + c, v);
}

template <class T, int V>
__global__ __launch_bounds__(256) void bn_add_relu_kernel(const T* __restrict__ z, const float* __restrict__ scale,
                                                          const float* __restrict__ shift, const float* __restrict__ feat,
                                                          T* __restrict__ y, int H, int W, int C, int h, int w, float fscale)
{
    int bx, row;
    xcd_block2d(bx, row);
    const int b = row / H, yy = row - b * H;                                // pixel row yy of image b
    const int CV = C / V, i = bx * 256 + threadIdx.x;
    if (i >= W * CV) return;
    const int xx = i / CV, c = (i - xx * CV) * V;
    const size_t o = ((size_t)row * W + xx) * C + c;
    float v[V];
#pragma unroll
    for (int k = 0; k < V; k += 4) {
        float4 a = fma4(ld4(z + o + k), ld4(scale + c + k), ld4(shift + c + k));
        const float4 res = bilinear4(feat, b, yy, xx, h, w, C, c + k, fscale);       // downsample = Identity: + x
        a.x += res.x; a.y += res.y; a.z += res.z; a.w += res.w;
        a = relu4(a);
        v[k] = a.x; v[k + 1] = a.y; v[k + 2] = a.z; v[k + 3] = a.w;
    }
    stv<T, V>(y + o, v);
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
// count_dev != NULL: the element count is a device value (SyncBatchNorm: the ranks' counts all-reduced
// together with the sums, so ranks may hold different batch sizes)
__global__ __launch_bounds__(256) void bn_fwd_finalize_kernel(const double* __restrict__ sums, double count,
                                                              const double* __restrict__ count_dev, float eps,
                                                              float momentum, const float* __restrict__ gamma,
                                                              const float* __restrict__ beta, float* mean, float* rstd,
                                                              float* scale, float* shift, float* rmean, float* rvar, int C,
                                                              long long* nbt)
{
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= C) return;
    if (nbt && c == 0) *nbt += 1;                 // BatchNorm2d.num_batches_tracked (no torch launch for it)
    double m, var;
    if (count_dev) count = *count_dev;
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

// The two halves of a BatchNorm statistics pass fused for the ranks that exchange nothing in between (plain
// BatchNorm, or SyncBatchNorm in a world of one): per-tile column partials [nb][2C] -> f64 sums in reduce_partials'
// exact order (row groups strided by 16, then the 16 groups in order) -> the finalize of bn_fwd_finalize_kernel /
// bn_bwd_finalize_kernel, one launch instead of two.  64 channels (both halves of the partial row) per block.
__device__ __forceinline__ void reduce_pair(const float* __restrict__ part, int nb, int C, double (*red)[16][64],
                                            double& S, double& Q)
{
    const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + cl;
    double s = 0.0, q = 0.0;
    if (c < C) {
#pragma unroll 4
        for (int i = rg; i < nb; i += 16) {
            s += (double)part[(size_t)i * 2 * C + c];
            q += (double)part[(size_t)i * 2 * C + C + c];
        }
    }
    red[0][rg][cl] = s;
    red[1][rg][cl] = q;
    __syncthreads();
    S = 0.0; Q = 0.0;
    if (rg == 0 && c < C) {
#pragma unroll
        for (int k = 0; k < 16; ++k) { S += red[0][k][cl]; Q += red[1][k][cl]; }
    }
}

__global__ __launch_bounds__(1024) void reduce_fwd_finalize_kernel(const float* __restrict__ part, int nb, int C,
                                                                   double count, float eps, float momentum,
                                                                   const float* __restrict__ gamma,
                                                                   const float* __restrict__ beta, float* mean,
                                                                   float* rstd, float* scale, float* shift,
                                                                   float* rmean, float* rvar, double* colsum_out,
                                                                   long long* nbt)
{
    __shared__ double red[2][16][64];
    double S, Q;
    reduce_pair(part, nb, C, red, S, Q);
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    if (threadIdx.x >= 64 || c >= C) return;
    if (nbt && c == 0) *nbt += 1;                 // BatchNorm2d.num_batches_tracked
    if (colsum_out) { colsum_out[c] = S; colsum_out[C + c] = Q; }
    const double m = S / count;
    double var = Q / count - m * m;
    var = var > 0.0 ? var : 0.0;
    if (rmean) rmean[c] = (float)((1.0 - momentum) * (double)rmean[c] + momentum * m);
    if (rvar) rvar[c] = (float)((1.0 - momentum) * (double)rvar[c] + momentum * var * count / (count - 1.0));
    const float rs = (float)(1.0 / sqrt(var + (double)eps));
    const float sc = gamma[c] * rs;
    mean[c] = (float)m;
    rstd[c] = rs;
    scale[c] = sc;
    shift[c] = beta[c] - (float)m * sc;
}

__global__ __launch_bounds__(1024) void reduce_bwd_finalize_kernel(const float* __restrict__ part, int nb, int C,
                                                                   double count, const float* __restrict__ gamma,
                                                                   const float* __restrict__ rstd, float* dgamma,
                                                                   float* dbeta, float* coef)
{
    __shared__ double red[2][16][64];
    double sg, sgx;
    reduce_pair(part, nb, C, red, sg, sgx);
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    if (threadIdx.x >= 64 || c >= C) return;
    if (dgamma) dgamma[c] = (float)sgx;
    if (dbeta) dbeta[c] = (float)sg;
    coef[c] = gamma[c] * rstd[c];
    coef[C + c] = (float)(sg / count);
    coef[2 * C + c] = (float)(sgx / count);
}

// x[p][c] = bilinear x`up` upsample of feat, unpadded rows (the Bottleneck's conv1x1 input)
template <class T>
__global__ __launch_bounds__(256) void upsample_kernel(const float* __restrict__ feat, T* __restrict__ x, long P, int H,
                                                       int W, int C, int h, int w, float scale)
{
    const int C4 = C / 4;
    const long e = (long)blockIdx.x * 256 + threadIdx.x;
    if (e >= P * C4) return;
    const long p = e / C4;
    const int c = (int)(e - p * C4) * 4;
    const int hw = H * W, b = (int)(p / hw), r = (int)(p - (long)b * hw), yy = r / W, xx = r - yy * W;
    st4(x + p * C + c, bilinear4(feat, b, yy, xx, h, w, C, c, scale));
}

// out = relu(z*scale + shift), unpadded rows, 8 channels per thread
template <class T>
__global__ __launch_bounds__(256) void bn_relu_kernel(const T* __restrict__ z, const float* __restrict__ scale,
                                                      const float* __restrict__ shift, T* __restrict__ out, long P, int C)
{
    const int C8 = C / 8;
    const long e = (long)blockIdx.x * 256 + threadIdx.x;
    if (e >= P * C8) return;
    const long p = e / C8;
    const int c = (int)(e - p * C8) * 8;
    float v[8];
    ld8(z + p * C + c, v);
    const float4 s0 = ld4(scale + c), s1 = ld4(scale + c + 4), h0 = ld4(shift + c), h1 = ld4(shift + c + 4);
    const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = fmaxf(fmaf(v[i], sc[i], sh[i]), 0.f);
    st8(out + p * C + c, v);
}

// ---- ModifiedResNet encoder blocks (image_encoder.py:10-115, blocks.py:56-101), NHWC rows [B*H*W][C]
// out[b][y][x] = mean of the 2x2 window of relu(z*scale + shift) (the Bottleneck's conv2 -> bn2 -> relu2 ->
// AvgPool2d(2) when stride 2); 8 channels per thread
template <class T>
__global__ __launch_bounds__(256) void bn_relu_avgpool_kernel(const T* __restrict__ z, const float* __restrict__ scale,
                                                              const float* __restrict__ shift, T* __restrict__ out, int B,
                                                              int H, int W, int C)
{
    const int C8 = C / 8, Ho = H / 2, Wo = W / 2;
    const long e = (long)blockIdx.x * 256 + threadIdx.x;
    if (e >= (long)B * Ho * Wo * C8) return;
    const long po = e / C8;
    const int c = (int)(e - po * C8) * 8;
    const int b = (int)(po / (Ho * Wo)), r = (int)(po - (long)b * Ho * Wo), yo = r / Wo, xo = r - yo * Wo;
    const float4 s0 = ld4(scale + c), s1 = ld4(scale + c + 4), h0 = ld4(shift + c), h1 = ld4(shift + c + 4);
    const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
    float v[4][8];
#pragma unroll
    for (int k = 0; k < 4; ++k) ld8(z + (((size_t)b * H + 2 * yo + (k >> 1)) * W + 2 * xo + (k & 1)) * C + c, v[k]);
    float o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        // AvgPool2d: sum of the window in row-major order, then / 4 (aten avg_pool2d, count_include_pad)
        const float a = fmaxf(fmaf(v[0][i], sc[i], sh[i]), 0.f), bb = fmaxf(fmaf(v[1][i], sc[i], sh[i]), 0.f);
        const float cc = fmaxf(fmaf(v[2][i], sc[i], sh[i]), 0.f), d = fmaxf(fmaf(v[3][i], sc[i], sh[i]), 0.f);
        o[i] = (((a + bb) + cc) + d) / 4.0f;
    }
    st8(out + po * C + c, o);
}

// out = AvgPool2d(2)(x) on NHWC rows (the downsample branch's "-1" pool); TI -> TO, 8 channels per thread
template <class TI, class TO>
__global__ __launch_bounds__(256) void avgpool2_kernel(const TI* __restrict__ x, TO* __restrict__ out, int B, int H, int W,
                                                       int C)
{
    const int C8 = C / 8, Ho = H / 2, Wo = W / 2;
    const long e = (long)blockIdx.x * 256 + threadIdx.x;
    if (e >= (long)B * Ho * Wo * C8) return;
    const long po = e / C8;
    const int c = (int)(e - po * C8) * 8;
    const int b = (int)(po / (Ho * Wo)), r = (int)(po - (long)b * Ho * Wo), yo = r / Wo, xo = r - yo * Wo;
    float v[4][8];
#pragma unroll
    for (int k = 0; k < 4; ++k) ld8(x + (((size_t)b * H + 2 * yo + (k >> 1)) * W + 2 * xo + (k & 1)) * C + c, v[k]);
    float o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (((v[0][i] + v[1][i]) + v[2][i]) + v[3][i]) / 4.0f;
    st8(out + po * C + c, o);
}

// AvgPool2d(2) backward: gx[b][y][x] = g[b][y/2][x/2] / 4 (TI -> TO), 8 channels per thread
template <class TI, class TO>
__global__ __launch_bounds__(256) void avgpool2_bwd_kernel(const TI* __restrict__ g, TO* __restrict__ gx, int B, int H, int W,
                                                           int C)
{
    const int C8 = C / 8, Ho = H / 2, Wo = W / 2;
    const long e = (long)blockIdx.x * 256 + threadIdx.x;
    if (e >= (long)B * H * W * C8) return;
    const long p = e / C8;
    const int c = (int)(e - p * C8) * 8;
    const int b = (int)(p / (H * W)), r = (int)(p - (long)b * H * W), y = r / W, x = r - y * W;
    float v[8];
    ld8(g + (((size_t)b * Ho + y / 2) * Wo + x / 2) * C + c, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] *= 0.25f;
    st8(gx + p * C + c, v);
}

// y = relu(z*scale + shift + identity), identity = idt*iscale + ishift (the downsample branch's BatchNorm) or
// idt itself (iscale == NULL): bn3 -> += identity -> relu3 of the Bottleneck; 8 channels per thread
template <class T>
__global__ __launch_bounds__(256) void bn_add_relu_flat_kernel(const T* __restrict__ z, const float* __restrict__ scale,
                                                               const float* __restrict__ shift, const T* __restrict__ idt,
                                                               const float* __restrict__ iscale,
                                                               const float* __restrict__ ishift, T* __restrict__ y, long P,
                                                               int C)
{
    const int C8 = C / 8;
    const long e = (long)blockIdx.x * 256 + threadIdx.x;
    if (e >= P * C8) return;
    const long p = e / C8;
    const int c = (int)(e - p * C8) * 8;
    const size_t off = (size_t)p * C + c;
    float zv[8], iv[8], sc[8], sh[8], isc[8], ish[8];
    ld8(z + off, zv);
    ld8(idt + off, iv);
    ldp8(scale + c, sc); ldp8(shift + c, sh);
    if (iscale) { ldp8(iscale + c, isc); ldp8(ishift + c, ish); }
    float o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const float idn = iscale ? fmaf(iv[i], isc[i], ish[i]) : iv[i];
        o[i] = fmaxf(fmaf(zv[i], sc[i], sh[i]) + idn, 0.f);
    }
    st8(y + off, o);
}

// column partials of sum(z) and sum(z*z) (BatchNorm batch statistics of a 1x1 conv output); the
// bn_bwd_partial_kernel scheme: (C/8) x RL threads, UNR rows per load batch, row order kept
template <class T, int UNR>
__global__ __launch_bounds__(512) void bn_stats_partial_kernel(const T* __restrict__ z, float* __restrict__ part, long P,
                                                               int C, int rows_per_block)
{
    extern __shared__ float red[];                // [RL][2][C]
    const int C8 = C / 8, RL = blockDim.x / C8;
    const int rl = threadIdx.x / C8, c = (threadIdx.x - rl * C8) * 8;
    const long r0 = (long)blockIdx.x * rows_per_block;
    const long r1 = std::min<long>(P, r0 + rows_per_block);
    float s1[8], s2[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) { s1[i] = 0.f; s2[i] = 0.f; }
    for (long r = r0 + rl; r < r1; r += UNR * RL) {
        float zv[UNR][8];
#pragma unroll
        for (int k = 0; k < UNR; ++k) ld8(z + std::min<long>(r + k * RL, r1 - 1) * C + c, zv[k]);
#pragma unroll
        for (int k = 0; k < UNR; ++k) {
            if (r + k * RL >= r1) continue;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                s1[i] += zv[k][i];
                s2[i] = fmaf(zv[k][i], zv[k][i], s2[i]);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        red[(size_t)rl * 2 * C + c + i] = s1[i];
        red[(size_t)rl * 2 * C + C + c + i] = s2[i];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 2 * C; e += blockDim.x) {
        float s = 0.f;
        for (int k = 0; k < RL; ++k) s += red[(size_t)k * 2 * C + e];
        part[(size_t)blockIdx.x * 2 * C + e] = s;
    }
}

// ------------------------------------------------------------------ backward
// g = gy * relu'(.)  with the ReLU mask from the stored output (mask_y) or recomputed from z (HAS_MY false)

// column partials of sum(g) and sum(g * xhat), xhat = (z - mean) * rstd; block = (C/8) x RL threads, 8
// channels (one 16-B vector) per thread.  Each thread walks its rows UNR at a time with every load issued
// first (row-clamped, unconditional); the sums keep the row order.
template <class T, bool HAS_MY, int UNR>
__global__ __launch_bounds__(512) void bn_bwd_partial_kernel(const T* __restrict__ gy, const T* __restrict__ my,
                                                             const T* __restrict__ z, const float* __restrict__ mean,
                                                             const float* __restrict__ rstd,
                                                             const float* __restrict__ scale,
                                                             const float* __restrict__ shift, float* __restrict__ part,
                                                             long P, int C, int rows_per_block)
{
    extern __shared__ float red[];                // [RL][2][C]
    const int C8 = C / 8, RL = blockDim.x / C8;
    const int rl = threadIdx.x / C8, c = (threadIdx.x - rl * C8) * 8;
    const long r0 = (long)blockIdx.x * rows_per_block;
    const long r1 = std::min<long>(P, r0 + rows_per_block);
    float mu[8], rs[8], sc[8], sh[8], s1[8], s2[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        mu[i] = mean[c + i]; rs[i] = rstd[c + i];
        sc[i] = HAS_MY ? 0.f : scale[c + i]; sh[i] = HAS_MY ? 0.f : shift[c + i];
        s1[i] = 0.f; s2[i] = 0.f;
    }
    for (long r = r0 + rl; r < r1; r += UNR * RL) {
        float gv[UNR][8], zv[UNR][8], mv[HAS_MY ? UNR : 1][8];
#pragma unroll
        for (int k = 0; k < UNR; ++k) {
            const long off = std::min<long>(r + k * RL, r1 - 1) * C + c;
            ld8(gy + off, gv[k]);
            ld8(z + off, zv[k]);
            if (HAS_MY) ld8(my + off, mv[k]);
        }
#pragma unroll
        for (int k = 0; k < UNR; ++k) {
            if (r + k * RL >= r1) continue;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const float m = HAS_MY ? mv[k][i] : fmaf(zv[k][i], sc[i], sh[i]);
                const float g = m > 0.f ? gv[k][i] : 0.f;
                s1[i] += g;
                s2[i] = fmaf(g, (zv[k][i] - mu[i]) * rs[i], s2[i]);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        red[(size_t)rl * 2 * C + c + i] = s1[i];
        red[(size_t)rl * 2 * C + C + c + i] = s2[i];
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
                                                              const double* __restrict__ count_dev,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ rstd, float* dgamma,
                                                              float* dbeta, float* coef, int C)
{
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= C) return;
    const double sg = sums[c], sgx = sums[C + c];
    if (count_dev) count = *count_dev;
    if (dgamma) dgamma[c] = (float)sgx;
    if (dbeta) dbeta[c] = (float)sg;
    coef[c] = gamma[c] * rstd[c];
    coef[C + c] = (float)(sg / count);
    coef[2 * C + c] = (float)(sgx / count);
}

// dz = gamma*rstd * (g - mean(g) - xhat * mean(g*xhat)), g = gy * relu'(.), unpadded rows (a 1x1 conv's
// output gradient); gmask != NULL also gets g itself in f32 (the identity branch's gradient of the block)
template <class T, bool HAS_MY>
__global__ __launch_bounds__(256) void bn_bwd_apply_flat_kernel(const T* __restrict__ gy, const T* __restrict__ my,
                                                                const T* __restrict__ z, const float* __restrict__ mean,
                                                                const float* __restrict__ rstd,
                                                                const float* __restrict__ scale,
                                                                const float* __restrict__ shift,
                                                                const float* __restrict__ coef, T* __restrict__ dz,
                                                                float* __restrict__ gmask, long P, int C)
{
    const int C8 = C / 8;
    const long e = (long)blockIdx.x * 256 + threadIdx.x;
    if (e >= P * C8) return;
    const long p = e / C8;
    const int c = (int)(e - p * C8) * 8;
    const size_t off = (size_t)p * C + c;
    float gv[8], zv[8], mv[8];
    ld8(gy + off, gv);
    ld8(z + off, zv);
    if (HAS_MY) ld8(my + off, mv);
    float k0[8], k1[8], k2[8], mu[8], rs[8], sc[8], sh[8];
    ldp8(coef + c, k0); ldp8(coef + C + c, k1); ldp8(coef + 2 * C + c, k2); ldp8(mean + c, mu); ldp8(rstd + c, rs);
    if (!HAS_MY) { ldp8(scale + c, sc); ldp8(shift + c, sh); }
    float v[8], gm[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const float m = HAS_MY ? mv[i] : fmaf(zv[i], sc[i], sh[i]);
        gm[i] = m > 0.f ? gv[i] : 0.f;
        v[i] = k0[i] * (gm[i] - k1[i] - (zv[i] - mu[i]) * rs[i] * k2[i]);
    }
    st8(dz + off, v);
    if (gmask) {
        *reinterpret_cast<float4*>(gmask + off) = make_float4(gm[0], gm[1], gm[2], gm[3]);
        *reinterpret_cast<float4*>(gmask + off + 4) = make_float4(gm[4], gm[5], gm[6], gm[7]);
    }
}

// Tiles of 64 padded positions x 64 channels, staged through LDS so that both the NHWC-padded image
// (rows of channels) and the transposed image (rows of positions) are written with contiguous rows.
constexpr int TQ = 64, TC = 64;

// dz = gamma*rstd * (g - mean(g) - xhat * mean(g*xhat)) -> dzpad [Q][C] (interior pixels) and dzT [C][Kq] (the
// weight gradient's K columns, 0 past each image's H*W).  A 64-column x 64-channel tile per block: the per-channel
// factors staged in LDS once, every thread's 16 channels of gy / mask / z loaded up front (row-clamped: no load
// behind a branch), 16-B stores both ways.  Blocks past Kq / 64 write dzpad's zero border (the data-gradient
// conv reads it as its zero padding).
template <class T, bool HAS_MY>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const T* __restrict__ gy, const T* __restrict__ my,
                                                           const T* __restrict__ z, const float* __restrict__ mean,
                                                           const float* __restrict__ rstd,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ shift,
                                                           const float* __restrict__ coef, T* __restrict__ dzpad,
                                                           T* __restrict__ dzT, DGeo g)
{
    __shared__ float sm[TQ][TC + 1];
    __shared__ float cf[7][TC];                   // gamma*rstd, mean(g), mean(g*xhat), mean, rstd, scale, shift
    const int t = threadIdx.x;
    const int c0 = blockIdx.y * TC;
    const int ql = t >> 2, cl = (t & 3) * 16;
    const long nkb = g.Kq / TQ;
    if (blockIdx.x >= nkb) {                      // dzpad's border: zeros
        const long q = (blockIdx.x - nkb) * TQ + ql;
        if (q < g.Q && interior(g, q) < 0) {
            const float z16[16] = {};
            st8(dzpad + q * g.C + c0 + cl, z16);
            st8(dzpad + q * g.C + c0 + cl + 8, z16 + 8);
        }
        return;
    }
    const long j0 = (long)blockIdx.x * TQ;
    const long j = j0 + ql;                       // K column: image b, interior pixel r
    const int hw = g.H * g.W;
    const long bimg = j / g.HWp;
    const int r = (int)(j - bimg * g.HWp);
    const long p = (bimg < g.B && r < hw) ? bimg * hw + r : -1;
    const long q = p >= 0 ? (bimg * g.Hp + r / g.W + 1) * g.Wp + r % g.W + 1 : -1;
    const long off = (p >= 0 ? p : 0) * g.C + c0 + cl;
    float gv[16], zv[16], mv[HAS_MY ? 16 : 1];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        ld8(gy + off + 8 * h, gv + 8 * h);
        ld8(z + off + 8 * h, zv + 8 * h);
        if (HAS_MY) ld8(my + off + 8 * h, mv + 8 * h);
    }
    if (t < TC) {
        const int c = c0 + t;
        cf[0][t] = coef[c]; cf[1][t] = coef[g.C + c]; cf[2][t] = coef[2 * g.C + c];
        cf[3][t] = mean[c]; cf[4][t] = rstd[c];
        if (!HAS_MY) { cf[5][t] = scale[c]; cf[6][t] = shift[c]; }
    }
    __syncthreads();
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int cc = cl + i;
        const float m = HAS_MY ? mv[i] : fmaf(zv[i], cf[5][cc], cf[6][cc]);
        const float gg = m > 0.f ? gv[i] : 0.f;
        v[i] = p >= 0 ? cf[0][cc] * (gg - cf[1][cc] - (zv[i] - cf[3][cc]) * cf[4][cc] * cf[2][cc]) : 0.f;
        sm[ql][cc] = v[i];
    }
    if (q >= 0) {
        st8(dzpad + q * g.C + c0 + cl, v);
        st8(dzpad + q * g.C + c0 + cl + 8, v + 8);
    }
    __syncthreads();
    {
        const int cr = t >> 2, jl = (t & 3) * 16;
        T* dst = dzT + (size_t)(c0 + cr) * g.Qs + j0 + jl;
        float w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = sm[jl + i][cr];
        st8(dst, w);
        st8(dst + 8, w + 8);
    }
}

// xT3[kx][c][pos] = xpad[(b * Hp + yp) * Wp + x + kx][c] for pos = b * Pimg + yp * W + x (b < B), else 0: every
// position of a row (the zero guard rows, the tail past the last image included).  A 64-position x 64-channel tile
// per block.  The three taps are one row of centre values shifted: tap 1 is column x + 1 of xpad's row, taps 0 / 2
// the centre of position pos -1 / +1 within the same image row, and at x = 0 / W - 1 xpad's border column 0 / W + 1
// (staged beside the centres: the pad cells are copied as they are).  So the block loads the 66 centre rows of its
// positions (one halo position each side) once and transposes them through LDS once for all three taps (r06: the r05
// form loaded each position's three taps, 3x the rows, and transposed three times).
template <class T>
__global__ __launch_bounds__(256) void transpose3_kernel(const T* __restrict__ xpad, T* __restrict__ xT3, DGeo g)
{
    __shared__ float sm[TQ + 2][TC + 1];           // centre of position j0 - 1 + slot
    __shared__ float se[2][TQ][TC + 1];            // border column 0 / W + 1 of position j0 + slot's row (x = 0 / W - 1)
    const int t = threadIdx.x;
    const int j0 = blockIdx.x * TQ;                 // (Qs < 2^31: checked by the launcher)
    const int c0 = blockIdx.y * TC;
    const int HpW = g.Hp * g.W, Pimg = (int)g.Pimg;
    float v[2][16], e[2][16];
    int pls[2], edg[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {                   // (TQ + 2) x 4 chunks of 16 channels over 256 threads
        const int k = t + 256 * r, pl = k >> 2, cl = (k & 3) * 16;
        pls[r] = k < (TQ + 2) * 4 ? pl : -1;
        edg[r] = -1;
        const int pos = j0 - 1 + pl;
        bool ok = pls[r] >= 0 && pos >= 0;
        long q = 0;
        int x = 0;
        if (ok) {
            const int pb = pos / Pimg, prem = pos - pb * Pimg;
            ok = pb < g.B && prem < HpW;
            const int pyp = prem / g.W;
            x = prem - pyp * g.W;
            q = ((long)pb * g.Hp + pyp) * g.Wp + x + 1;
        }
        if (ok) {
            ld8(xpad + q * g.C + c0 + cl, v[r]);
            ld8(xpad + q * g.C + c0 + cl + 8, v[r] + 8);
            const bool inb = pl >= 1 && pl <= TQ;           // one of the block's own positions
            if (inb && (x == 0 || x == g.W - 1)) {
                const long qe = x == 0 ? q - 1 : q + 1;
                ld8(xpad + qe * g.C + c0 + cl, e[r]);
                ld8(xpad + qe * g.C + c0 + cl + 8, e[r] + 8);
                edg[r] = x == 0 ? 0 : 1;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) v[r][i] = 0.f;
        }
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        if (pls[r] < 0) continue;
        const int cl = ((t + 256 * r) & 3) * 16;
#pragma unroll
        for (int i = 0; i < 16; ++i) sm[pls[r]][cl + i] = v[r][i];
        if (edg[r] >= 0) {
#pragma unroll
            for (int i = 0; i < 16; ++i) se[edg[r]][pls[r] - 1][cl + i] = e[r][i];
        }
    }
    __syncthreads();
    // output: 8 lanes a channel row, each 8 consecutive positions (16-B stores, a whole 128-B line per 8 lanes); this
    // thread's 8 positions' x and validity walked from the first (no division in the loop)
    const int jl = (t & 7) * 8;
    const int p0 = j0 + jl;
    int b = p0 / Pimg, rem = p0 - b * Pimg, x = rem % g.W;
    bool lft[8], rgt[8], val[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        val[i] = b < g.B && rem < HpW;
        lft[i] = x > 0;
        rgt[i] = x < g.W - 1;
        if (++rem == Pimg) { rem = 0; x = 0; ++b; }
        else if (++x == g.W) x = 0;
    }
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
        const int cr = pass * 32 + (t >> 3);
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            float w[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const float s = kx == 1 ? sm[jl + i + 1][cr] : kx == 0 ? (lft[i] ? sm[jl + i][cr] : se[0][jl + i][cr])
                                                                      : (rgt[i] ? sm[jl + i + 2][cr] : se[1][jl + i][cr]);
                w[i] = val[i] ? s : 0.f;
            }
            st8(xT3 + ((size_t)kx * g.C + c0 + cr) * g.Qs + j0 + jl, w);
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
    // one input row (b, i) per blockIdx.y, 32-bit index math (r06: was a 64-bit division per 4 channels)
    int bx, row;
    xcd_block2d(bx, row);
    const int b = row / h, i = row - b * h;
    const int C4 = C / 4, e = bx * 256 + threadIdx.x;
    if (e >= w * C4) return;
    const int j = e / C4, c = (e - j * C4) * 4;
    const long cell = (long)row * w + j;
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
    // 16-B stores of 8 consecutive elements (N, C multiples of 32: checked by the launcher)
    for (int e = t; e < 32 * 9 * 4; e += 256) {    // wk rows (o, tap): 32 contiguous c
        const int cv = (e & 3) * 8, r = e >> 2, ol = r / 9, tap = r - ol * 9;
        float x[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = sm[ol][(cv + i) * 9 + tap];
        st8(wk + ((size_t)(o0 + ol) * 9 + tap) * C + c0 + cv, x);
    }
    for (int e = t; e < 32 * 9 * 4; e += 256) {    // wf rows (c, tap): 32 contiguous o
        const int ov = (e & 3) * 8, r = e >> 2, cl = r / 9, tap = r - cl * 9;
        float x[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = sm[ov + i][cl * 9 + 8 - tap];
        st8(wf + ((size_t)(c0 + cl) * 9 + tap) * N + o0 + ov, x);
    }
}

// 1x1 conv weight [N][K] f32 -> wk [N][K] and its transpose wt [K][N] in the compute dtype (the GEMM's forward
// and data-gradient operands), 32x32 tiles through LDS
template <class T>
__global__ __launch_bounds__(256) void prep_weights_1x1_kernel(const float* __restrict__ w, T* __restrict__ wk,
                                                               T* __restrict__ wt, int N, int K)
{
    __shared__ float sm[32][33];
    const int n0 = blockIdx.x * 32, k0 = blockIdx.y * 32, t = threadIdx.x;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int nl = r * 8 + t / 32, kl = t % 32;
        const float v = w[(size_t)(n0 + nl) * K + k0 + kl];
        sm[nl][kl] = v;
        wk[(size_t)(n0 + nl) * K + k0 + kl] = (T)v;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int kl = r * 8 + t / 32, nl = t % 32;
        wt[(size_t)(k0 + kl) * N + n0 + nl] = (T)sm[nl][kl];
    }
}

inline unsigned nblk(long n) { return (unsigned)((n + 255) / 256); }
// bn_bwd_partial rows per block: 8 rows per thread-row-lane (two 4-row load batches)
inline int bn_partial_rows(int C) { return 8 * std::max(1, 512 / std::max(1, C / 8)); }

// optional fused finalize (reduce_fwd_finalize_kernel / reduce_bwd_finalize_kernel) instead of reduce_partials
struct FwdFin { float eps, momentum; const float *gamma, *beta; float *mean, *rstd, *scale, *shift, *rmean, *rvar; long long* nbt; };
struct BwdFin { const float* gamma; float *dgamma, *dbeta, *coef; };

template <class T>
int bn_bwd_reduce_t(const void* gy, const void* my, const void* z, const float* mean, const float* rstd,
                    const float* scale, const float* shift, double* sums, void* ws, size_t wsb, long P, int C,
                    hipStream_t st, const BwdFin* fin = nullptr)
{
    if (C % 8 || C / 8 > 512) return EBC_E_UNSUPPORTED;
    const int C8 = C / 8;
    const int RL = std::max(1, 512 / C8);
    const int threads = C8 * RL;
    const int rpb = bn_partial_rows(C);
    const long nb = (P + rpb - 1) / rpb;
    const size_t need = CONV_WS_STATS_OFFSET + (size_t)nb * 2 * C * 4;
    if (!ws || wsb < need) return EBC_E_ARG;
    float* part = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + CONV_WS_STATS_OFFSET);
    const size_t lds = (size_t)RL * 2 * C * 4;
    if (my)
        hipLaunchKernelGGL((bn_bwd_partial_kernel<T, true, 4>), dim3((unsigned)nb), dim3(threads), lds, st,
                           (const T*)gy, (const T*)my, (const T*)z, mean, rstd, scale, shift, part, P, C, rpb);
    else
        hipLaunchKernelGGL((bn_bwd_partial_kernel<T, false, 4>), dim3((unsigned)nb), dim3(threads), lds, st,
                           (const T*)gy, (const T*)my, (const T*)z, mean, rstd, scale, shift, part, P, C, rpb);
    if (fin)
        hipLaunchKernelGGL(reduce_bwd_finalize_kernel, dim3((C + 63) / 64), dim3(1024), 0, st, (const float*)part, (int)nb,
                           C, (double)P, fin->gamma, rstd, fin->dgamma, fin->dbeta, fin->coef);
    else
        hipLaunchKernelGGL(reduce_partials_kernel, dim3((2 * C + 63) / 64), dim3(1024), 0, st, (const float*)part, (int)nb,
                           2 * C, sums);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

template <class T>
int bn_stats_t(const void* z, double* colsum, void* ws, size_t wsb, long P, int C, hipStream_t st,
               const FwdFin* fin = nullptr)
{
    if (C % 8 || C / 8 > 512) return EBC_E_UNSUPPORTED;
    const int C8 = C / 8;
    const int RL = std::max(1, 512 / C8);
    const int rpb = bn_partial_rows(C);
    const long nb = (P + rpb - 1) / rpb;
    const size_t need = CONV_WS_STATS_OFFSET + (size_t)nb * 2 * C * 4;
    if (!ws || wsb < need) return EBC_E_ARG;
    float* part = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + CONV_WS_STATS_OFFSET);
    hipLaunchKernelGGL((bn_stats_partial_kernel<T, 4>), dim3((unsigned)nb), dim3(C8 * RL), (size_t)RL * 2 * C * 4, st,
                       (const T*)z, part, P, C, rpb);
    if (fin)
        hipLaunchKernelGGL(reduce_fwd_finalize_kernel, dim3((C + 63) / 64), dim3(1024), 0, st, (const float*)part, (int)nb,
                           C, (double)P, fin->eps, fin->momentum, fin->gamma, fin->beta, fin->mean, fin->rstd, fin->scale,
                           fin->shift, fin->rmean, fin->rvar, colsum, fin->nbt);
    else
        hipLaunchKernelGGL(reduce_partials_kernel, dim3((2 * C + 63) / 64), dim3(1024), 0, st, (const float*)part, (int)nb,
                           2 * C, colsum);
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
    out[0] = g.Hp; out[1] = g.Wp; out[2] = g.HWp; out[3] = g.Kq; out[4] = g.Q; out[5] = g.Qs;
    return EBC_OK;
}

extern "C" size_t ebc_dec_workspace_bytes(int dtype, int B, int H, int W, int C, int N)
{
    const Geo g = make_geo(dtype, B, H, W, C);
    const int M = B * H * W;
    size_t need = ebc::conv_gemm_workspace_bytes(dtype, 1, M, N, 9 * C);
    need = std::max(need, ebc::conv_gemm_workspace_bytes(dtype, 1, M, C, 9 * N));
    need = std::max(need, ebc::conv_gemm_workspace_bytes(dtype, 2, N, 9 * C, (int)g.Kq));
    const int rpb = std::min(bn_partial_rows(C), bn_partial_rows(N));
    const long nb = std::max(((long)M + 63) / 64, ((long)M + rpb - 1) / rpb);
    need = std::max(need, CONV_WS_STATS_OFFSET + (size_t)nb * 2 * std::max(C, N) * 4);
    return need;
}

extern "C" int ebc_dec_upsample_pad(int dtype, const float* feat, void* xpad, int B, int h, int w, int C, int up,
                                    ebc_stream_t stream)
{
    if (!feat || !xpad || up < 1 || C % 64 || B <= 0 || (long)B * (h * up + 2) >= 65536) return EBC_E_ARG;
    const Geo g = make_geo(dtype, B, h * up, w * up, C);
    const DGeo d = dgeo(g);
    const dim3 grid((unsigned)((g.Wp * (C / 8) + 255) / 256), (unsigned)(B * g.Hp));
    EBC_DTYPE_SWITCH(dtype, hipLaunchKernelGGL((upsample_pad_kernel<T, 8>), grid, dim3(256), 0,
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
    ebc::ConvGeom cg{H, W, C, g.Hp, g.Wp, 0, 0, 0, B};
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

extern "C" int ebc_conv3x3_fwd_bn(int dtype, const void* xpad, const void* weight, void* out, void* ws, size_t wsb,
                                  int B, int H, int W, int C, int N, float eps, float momentum, const float* gamma,
                                  const float* beta, float* mean, float* rstd, float* scale, float* shift,
                                  float* running_mean, float* running_var, long long* num_batches_tracked,
                                  double* colsum_out, ebc_stream_t stream)
{
    if (!xpad || !weight || !out || C % 64 || N % 64 || !gamma || !beta || !mean || !rstd || !scale || !shift)
        return EBC_E_ARG;
    if ((running_mean == nullptr) != (running_var == nullptr) || B * H * W <= 1) return EBC_E_ARG;
    const Geo g = make_geo(dtype, B, H, W, C);
    ebc::ConvGeom cg{H, W, C, g.Hp, g.Wp, 0, 0, 0, B};
    const int M = B * H * W;
    int tiles = 0;
    const hipStream_t st = (hipStream_t)stream;
    EBC_TRY(ebc::conv_gemm(dtype, 1, 4, xpad, weight, out, cg, M, N, 9 * C, ws, wsb, &tiles, st, nullptr, nullptr));
    // the conv epilogue's per-tile column sums -> f64 in reduce_partials' order -> batch statistics, running stats,
    // scale / shift: one launch (reduce_fwd_finalize_kernel) where ebc_conv3x3_fwd + ebc_bn_finalize take two
    const float* part = reinterpret_cast<const float*>(reinterpret_cast<const char*>(ws) + CONV_WS_STATS_OFFSET);
    hipLaunchKernelGGL(reduce_fwd_finalize_kernel, dim3((N + 63) / 64), dim3(1024), 0, st, part, tiles, N, (double)M,
                       eps, momentum, gamma, beta, mean, rstd, scale, shift, running_mean, running_var, colsum_out,
                       num_batches_tracked);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

extern "C" int ebc_conv3x3_wgrad(int dtype, const void* dzT, const void* xT3, float* dw, void* ws, size_t wsb, int B,
                                 int H, int W, int C, int N, ebc_stream_t stream)
{
    if (!dzT || !xT3 || !dw || C % 64 || N % 64) return EBC_E_ARG;
    const Geo g = make_geo(dtype, B, H, W, C);
    ebc::ConvGeom cg{H, W, C, g.Hp, g.Wp, g.HWp, g.Qs, g.Pimg, B};
    return ebc::conv_gemm(dtype, 2, 0, dzT, xT3, dw, cg, N, 9 * C, (int)g.Kq, ws, wsb, nullptr, (hipStream_t)stream);
}

extern "C" int ebc_bn_finalize(const double* colsum, double count, float eps, float momentum, const float* gamma,
                               const float* beta, float* mean, float* rstd, float* scale, float* shift,
                               float* running_mean, float* running_var, long long* num_batches_tracked, int C,
                               ebc_stream_t stream)
{
    if (!gamma || !beta || !mean || !rstd || !scale || !shift) return EBC_E_ARG;
    if (!colsum && (!running_mean || !running_var)) return EBC_E_ARG;
    if (colsum && count >= 0.0 && count <= 1.0) return EBC_E_ARG;
    const double* cdev = colsum && count < 0.0 ? colsum + 2 * C : nullptr;     // device count at colsum[2C]
    hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3(nblk(C)), dim3(256), 0, (hipStream_t)stream, colsum, count, cdev, eps,
                       momentum, gamma, beta, mean, rstd, scale, shift, running_mean, running_var, C, num_batches_tracked);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

extern "C" int ebc_bn_relu_pad(int dtype, const void* z, const float* scale, const float* shift, void* hpad, int B,
                               int H, int W, int C, ebc_stream_t stream)
{
    if (!z || !scale || !shift || !hpad || C % 64 || B <= 0 || (long)B * (H + 2) >= 65536) return EBC_E_ARG;
    const Geo g = make_geo(dtype, B, H, W, C);
    const DGeo d = dgeo(g);
    const dim3 grid((unsigned)((g.Wp * (C / 8) + 255) / 256), (unsigned)(B * g.Hp));
    EBC_DTYPE_SWITCH(dtype, hipLaunchKernelGGL((bn_relu_pad_kernel<T, 8>), grid, dim3(256), 0,
                                               (hipStream_t)stream, (const T*)z, scale, shift, (T*)hpad, d));
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

extern "C" int ebc_bn_add_relu(int dtype, const void* z, const float* scale, const float* shift, const float* feat,
                               int up, void* y, int B, int H, int W, int C, ebc_stream_t stream)
{
    if (!z || !scale || !shift || !feat || !y || up < 1 || H % up || W % up || C % 4) return EBC_E_ARG;
    if (B <= 0 || H <= 0 || W <= 0 || (long)W * C >= (1L << 31) || (long)B * H >= 65536) return EBC_E_ARG;
    const hipStream_t st = (hipStream_t)stream;
    if (C % 8 == 0) {
        const dim3 grid((unsigned)((W * (C / 8) + 255) / 256), (unsigned)(B * H));
        EBC_DTYPE_SWITCH(dtype, hipLaunchKernelGGL((bn_add_relu_kernel<T, 8>), grid, dim3(256), 0, st, (const T*)z, scale,
                                                   shift, feat, (T*)y, H, W, C, H / up, W / up, 1.0f / (float)up));
    } else {
        const dim3 grid((unsigned)((W * (C / 4) + 255) / 256), (unsigned)(B * H));
        EBC_DTYPE_SWITCH(dtype, hipLaunchKernelGGL((bn_add_relu_kernel<T, 4>), grid, dim3(256), 0, st, (const T*)z, scale,
                                                   shift, feat, (T*)y, H, W, C, H / up, W / up, 1.0f / (float)up));
    }
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
    if (!sums || !gamma || !rstd || !coef || count == 0.0) return EBC_E_ARG;
    const double* cdev = count < 0.0 ? sums + 2 * C : nullptr;                 // device count at sums[2C]
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(nblk(C)), dim3(256), 0, (hipStream_t)stream, sums, count, cdev, gamma,
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
    const dim3 grid((unsigned)(g.Kq / TQ + (g.Q + TQ - 1) / TQ), (unsigned)(C / TC));
    if (mask_y) {
        EBC_DTYPE_SWITCH(dtype, hipLaunchKernelGGL((bn_bwd_apply_kernel<T, true>), grid, dim3(256), 0, (hipStream_t)stream,
                                                   (const T*)gy, (const T*)mask_y, (const T*)z, mean, rstd, scale,
                                                   shift, coef, (T*)dzpad, (T*)dzT, d));
    } else {
        EBC_DTYPE_SWITCH(dtype, hipLaunchKernelGGL((bn_bwd_apply_kernel<T, false>), grid, dim3(256), 0, (hipStream_t)stream,
                                                   (const T*)gy, (const T*)mask_y, (const T*)z, mean, rstd, scale,
                                                   shift, coef, (T*)dzpad, (T*)dzT, d));
    }
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

extern "C" int ebc_dec_transpose3(int dtype, const void* xpad, void* xT3, int B, int H, int W, int C,
                                  ebc_stream_t stream)
{
    if (!xpad || !xT3 || C % TC) return EBC_E_ARG;
    const Geo g = make_geo(dtype, B, H, W, C);
    const DGeo d = dgeo(g);
    // (r05: a register-transpose form without LDS -- a lane's 4 positions x 8 channels, 8-B stores -- ran 26.1 vs 23.4 us
    // in-step, not kept)
    if (g.Qs >= (1L << 31) - TQ || W < 2) return EBC_E_ARG;
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
    if (B <= 0 || h <= 0 || w <= 0 || (long)w * C >= (1L << 31) || (long)B * h >= 65536) return EBC_E_ARG;
    const dim3 grid((unsigned)((w * (C / 4) + 255) / 256), (unsigned)(B * h));
    const hipStream_t st = (hipStream_t)stream;
    if (up == 2) {
        EBC_DTYPE_SWITCH(dtype, hipLaunchKernelGGL((upsample_bwd_kernel<T, 2>), grid, dim3(256), 0, st,
                                                   (const T*)g, dfeat, B, h, w, 2 * h, 2 * w, C));
    } else {
        EBC_DTYPE_SWITCH(dtype, hipLaunchKernelGGL((upsample_bwd_kernel<T, 1>), grid, dim3(256), 0, st,
                                                   (const T*)g, dfeat, B, h, w, h, w, C));
    }
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

extern "C" int ebc_dec_prep_weights(int dtype, const float* w, void* wk, void* wf, int N, int C, ebc_stream_t stream)
{
    if (!w || !wk || !wf || N <= 0 || C <= 0 || N % 32 || C % 32) return EBC_E_ARG;
    const dim3 grid((unsigned)(N / 32), (unsigned)(C / 32));
    EBC_DTYPE_SWITCH(dtype, hipLaunchKernelGGL(prep_weights_kernel<T>, grid, dim3(256), 0, (hipStream_t)stream, w,
                                               (T*)wk, (T*)wf, N, C));
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

// ------------------------------------------------------------------ flat-layout helpers (Bottleneck decoder)
extern "C" int ebc_dec_upsample(int dtype, const float* feat, void* x, int B, int h, int w, int C, int up,
                                ebc_stream_t stream)
{
    if (!feat || !x || up < 1 || B <= 0 || h <= 0 || w <= 0 || C % 4) return EBC_E_ARG;
    const int H = h * up, W = w * up;
    const long P = (long)B * H * W;
    EBC_DTYPE_SWITCH(dtype, hipLaunchKernelGGL(upsample_kernel<T>, dim3(nblk(P * (C / 4))), dim3(256), 0,
                                               (hipStream_t)stream, feat, (T*)x, P, H, W, C, h, w, 1.0f / (float)up));
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

extern "C" int ebc_bn_stats(int dtype, const void* z, double* colsum, void* ws, size_t wsb, long P, int C,
                            ebc_stream_t stream)
{
    if (!z || !colsum || P <= 0 || C % 8) return EBC_E_ARG;
    const hipStream_t st = (hipStream_t)stream;
    switch (dtype) {
        case EBC_F32: return bn_stats_t<float>(z, colsum, ws, wsb, P, C, st);
        case EBC_F16: return bn_stats_t<_Float16>(z, colsum, ws, wsb, P, C, st);
        case EBC_BF16: return bn_stats_t<__bf16>(z, colsum, ws, wsb, P, C, st);
    }
    return EBC_E_ARG;
}

extern "C" int ebc_bn_stats_finalize(int dtype, const void* z, void* ws, size_t wsb, long P, int C, float eps,
                                     float momentum, const float* gamma, const float* beta, float* mean, float* rstd,
                                     float* scale, float* shift, float* running_mean, float* running_var,
                                     double* colsum_out, long long* num_batches_tracked, ebc_stream_t stream)
{
    if (!z || P <= 1 || C % 8 || !gamma || !beta || !mean || !rstd || !scale || !shift) return EBC_E_ARG;
    if ((running_mean == nullptr) != (running_var == nullptr)) return EBC_E_ARG;
    const FwdFin fin{eps, momentum, gamma, beta, mean, rstd, scale, shift, running_mean, running_var, num_batches_tracked};
    const hipStream_t st = (hipStream_t)stream;
    switch (dtype) {
        case EBC_F32: return bn_stats_t<float>(z, colsum_out, ws, wsb, P, C, st, &fin);
        case EBC_F16: return bn_stats_t<_Float16>(z, colsum_out, ws, wsb, P, C, st, &fin);
        case EBC_BF16: return bn_stats_t<__bf16>(z, colsum_out, ws, wsb, P, C, st, &fin);
    }
    return EBC_E_ARG;
}

extern "C" int ebc_bn_bwd_reduce_finalize(int dtype, const void* gy, const void* mask_y, const void* z, const float* mean,
                                          const float* rstd, const float* scale, const float* shift, const float* gamma,
                                          float* dgamma, float* dbeta, float* coef, void* ws, size_t wsb, long P, int C,
                                          ebc_stream_t stream)
{
    if (!gy || !z || !mean || !rstd || !gamma || !coef || P <= 0 || C % 4 || (!mask_y && (!scale || !shift)))
        return EBC_E_ARG;
    const BwdFin fin{gamma, dgamma, dbeta, coef};
    const hipStream_t st = (hipStream_t)stream;
    switch (dtype) {
        case EBC_F32: return bn_bwd_reduce_t<float>(gy, mask_y, z, mean, rstd, scale, shift, nullptr, ws, wsb, P, C, st, &fin);
        case EBC_F16: return bn_bwd_reduce_t<_Float16>(gy, mask_y, z, mean, rstd, scale, shift, nullptr, ws, wsb, P, C, st, &fin);
        case EBC_BF16: return bn_bwd_reduce_t<__bf16>(gy, mask_y, z, mean, rstd, scale, shift, nullptr, ws, wsb, P, C, st, &fin);
    }
    return EBC_E_ARG;
}

extern "C" int ebc_bn_relu(int dtype, const void* z, const float* scale, const float* shift, void* out, long P, int C,
                           ebc_stream_t stream)
{
    if (!z || !scale || !shift || !out || P <= 0 || C % 8) return EBC_E_ARG;
    EBC_DTYPE_SWITCH(dtype, hipLaunchKernelGGL(bn_relu_kernel<T>, dim3(nblk(P * (C / 8))), dim3(256), 0,
                                               (hipStream_t)stream, (const T*)z, scale, shift, (T*)out, P, C));
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

extern "C" int ebc_bn_bwd_apply_flat(int dtype, const void* gy, const void* mask_y, const void* z, const float* mean,
                                     const float* rstd, const float* scale, const float* shift, const float* coef,
                                     void* dz, float* gmask, long P, int C, ebc_stream_t stream)
{
    if (!gy || !z || !mean || !rstd || !coef || !dz || P <= 0 || C % 8 || (!mask_y && (!scale || !shift)))
        return EBC_E_ARG;
    const unsigned grid = nblk(P * (C / 8));
    const hipStream_t st = (hipStream_t)stream;
    if (mask_y) {
        EBC_DTYPE_SWITCH(dtype, hipLaunchKernelGGL((bn_bwd_apply_flat_kernel<T, true>), dim3(grid), dim3(256), 0, st,
                                                   (const T*)gy, (const T*)mask_y, (const T*)z, mean, rstd, scale, shift,
                                                   coef, (T*)dz, gmask, P, C));
    } else {
        EBC_DTYPE_SWITCH(dtype, hipLaunchKernelGGL((bn_bwd_apply_flat_kernel<T, false>), dim3(grid), dim3(256), 0, st,
                                                   (const T*)gy, (const T*)mask_y, (const T*)z, mean, rstd, scale, shift,
                                                   coef, (T*)dz, gmask, P, C));
    }
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

// ------------------------------------------------------------------ ModifiedResNet block helpers
extern "C" int ebc_bn_relu_avgpool(int dtype, const void* z, const float* scale, const float* shift, void* out, int B, int H,
                                   int W, int C, ebc_stream_t stream)
{
    if (!z || !scale || !shift || !out || B <= 0 || H % 2 || W % 2 || H <= 0 || W <= 0 || C % 8) return EBC_E_ARG;
    const long n = (long)B * (H / 2) * (W / 2) * (C / 8);
    EBC_DTYPE_SWITCH(dtype, hipLaunchKernelGGL(bn_relu_avgpool_kernel<T>, dim3(nblk(n)), dim3(256), 0, (hipStream_t)stream,
                                               (const T*)z, scale, shift, (T*)out, B, H, W, C));
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

// dtype_in / dtype_out: the element types of x and out (EBC_F32 or the compute dtype)
extern "C" int ebc_avgpool2(int dtype_in, int dtype_out, const void* x, void* out, int B, int H, int W, int C,
                            ebc_stream_t stream)
{
    if (!x || !out || B <= 0 || H % 2 || W % 2 || H <= 0 || W <= 0 || C % 8 || dtype_in != dtype_out) return EBC_E_ARG;
    const long n = (long)B * (H / 2) * (W / 2) * (C / 8);
    EBC_DTYPE_SWITCH(dtype_in, hipLaunchKernelGGL((avgpool2_kernel<T, T>), dim3(nblk(n)), dim3(256), 0, (hipStream_t)stream,
                                                  (const T*)x, (T*)out, B, H, W, C));
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

extern "C" int ebc_avgpool2_bwd(int dtype_in, int dtype_out, const void* g, void* gx, int B, int H, int W, int C,
                                ebc_stream_t stream)
{
    if (!g || !gx || B <= 0 || H % 2 || W % 2 || H <= 0 || W <= 0 || C % 8) return EBC_E_ARG;
    const long n = (long)B * H * W * (C / 8);
    const hipStream_t st = (hipStream_t)stream;
    if (dtype_in == dtype_out) {
        EBC_DTYPE_SWITCH(dtype_in, hipLaunchKernelGGL((avgpool2_bwd_kernel<T, T>), dim3(nblk(n)), dim3(256), 0, st,
                                                      (const T*)g, (T*)gx, B, H, W, C));
    } else if (dtype_in == EBC_F32) {
        EBC_DTYPE_SWITCH(dtype_out, hipLaunchKernelGGL((avgpool2_bwd_kernel<float, T>), dim3(nblk(n)), dim3(256), 0, st,
                                                       (const float*)g, (T*)gx, B, H, W, C));
    } else {
        return EBC_E_ARG;
    }
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

extern "C" int ebc_bn_add_relu_flat(int dtype, const void* z, const float* scale, const float* shift, const void* idt,
                                    const float* iscale, const float* ishift, void* y, long P, int C, ebc_stream_t stream)
{
    if (!z || !scale || !shift || !idt || !y || P <= 0 || C % 8 || (!iscale != !ishift)) return EBC_E_ARG;
    EBC_DTYPE_SWITCH(dtype, hipLaunchKernelGGL(bn_add_relu_flat_kernel<T>, dim3(nblk(P * (C / 8))), dim3(256), 0,
                                               (hipStream_t)stream, (const T*)z, scale, shift, (const T*)idt, iscale,
                                               ishift, (T*)y, P, C));
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

extern "C" int ebc_prep_weights_1x1(int dtype, const float* w, void* wk, void* wt, int N, int K, ebc_stream_t stream)
{
    if (!w || !wk || !wt || N <= 0 || K <= 0 || N % 32 || K % 32) return EBC_E_ARG;
    const dim3 grid((unsigned)(N / 32), (unsigned)(K / 32));
    EBC_DTYPE_SWITCH(dtype, hipLaunchKernelGGL(prep_weights_1x1_kernel<T>, grid, dim3(256), 0, (hipStream_t)stream, w,
                                               (T*)wk, (T*)wt, N, K));
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}
