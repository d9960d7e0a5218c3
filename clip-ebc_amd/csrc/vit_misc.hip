// Memory-bound pieces of the CLIP-EBC ViT path on gfx950: LayerNorm fwd/bwd, patch im2col,
// token embedding (+CLS, +pos, ln_pre, VPT rows), VPT insert / gradient, the blockwise
// image-text similarity head fwd/bwd, and the attention-backward row statistic.
//
// Reference: LayerNorm (fp32 math)        models/clip/_clip/blocks.py:8-14
//            token prologue               models/clip/model.py:147-158, image_encoder.py:141-148
//            VPT assemble / disassemble   models/clip/model.py:131-140, 161-183
//            ln_post + drop CLS           models/clip/model.py:185-188
//            similarity head              models/clip/model.py:198-217
// Every kernel is one wave per row (D = 256*NV), 16-B vector accesses, fp32 statistics.
#include <climits>
#include "ebc_common.h"
#include "kernels.h"
#include "mfma.h"
#include "touch.h"

using namespace ebc;

namespace {

constexpr float LN_EPS = 1e-5f;

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
template <class T> __device__ __forceinline__ float4 ld4(const T* p) {
    return make_float4((float)p[0], (float)p[1], (float)p[2], (float)p[3]);
}
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

struct RowMap {            // out row r -> source row (r / rpg) * gstride + goff + r % rpg
    int rpg, gstride, goff;
    __device__ __forceinline__ size_t operator()(int r) const {
        return (size_t)(r / rpg) * gstride + goff + (r % rpg);
    }
};

// Normalise NV float4 per lane of one row held in registers.
template <int NV>
__device__ __forceinline__ void ln_row(float4 (&v)[NV], const float4 (&gb)[2 * NV], float& mean, float& rstd) {
    constexpr float inv = 1.0f / (256.0f * NV);
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    mean = wave_sum(s) * inv;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const float a = v[i].x - mean, b = v[i].y - mean, c = v[i].z - mean, d = v[i].w - mean;
        q += (a * a + b * b) + (c * c + d * d);
    }
    rstd = 1.0f / sqrtf(wave_sum(q) * inv + LN_EPS);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const float4 g = gb[2 * i], b = gb[2 * i + 1];
        v[i] = make_float4((v[i].x - mean) * rstd * g.x + b.x, (v[i].y - mean) * rstd * g.y + b.y,
                           (v[i].z - mean) * rstd * g.z + b.z, (v[i].w - mean) * rstd * g.w + b.w);
    }
}

// Row blocks in XCD order (xcd_remap): each XCD takes a contiguous run of rows, the same rows the GEMM tiles that
// produce and consume them run on that XCD (gemm.hip maps its tiles the same way), so the row operands a kernel
// reads were last written on its own XCD
__device__ __forceinline__ int row_block() { return xcd_remap(blockIdx.x, (int)gridDim.x); }

// deep-VPT insert fused into ln_1 (model.py:131-140, 161-168): rows 1..NV of every crop are read from
// the prompt (vpt + b * bstride + (l-1) * D) instead of X, and written into X for the residual path
struct VptIns {
    const float* vpt;       // null: plain LayerNorm
    long bstride;
    int L, NV;
    float* X;
};

template <class T, int NV>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ x, RowMap map, const float* gamma,
                                                     const float* beta, T* out, float* outf, float* mean_out,
                                                     float* rstd_out, int M, VptIns vi)
{
    constexpr int D = 256 * NV;
    const int r = row_block() * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (r >= M) return;
    const float* xr = x + map(r) * D;
    bool ins = false;
    if (vi.vpt) {
        const int b = r / vi.L, l = r - b * vi.L;
        if (l >= 1 && l <= vi.NV) { xr = vi.vpt + b * vi.bstride + (size_t)(l - 1) * D; ins = true; }
    }
    float4 v[NV], gb[2 * NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = *reinterpret_cast<const float4*>(xr + 4 * lane + 256 * i);
    // gamma / beta issued with the row (not after the two reductions): one dependent L2 round trip fewer
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        gb[2 * i] = *reinterpret_cast<const float4*>(gamma + 4 * lane + 256 * i);
        gb[2 * i + 1] = *reinterpret_cast<const float4*>(beta + 4 * lane + 256 * i);
    }
    if (ins) {
#pragma unroll
        for (int i = 0; i < NV; ++i) *reinterpret_cast<float4*>(vi.X + (size_t)r * D + 4 * lane + 256 * i) = v[i];
    }
    float mean, rstd;
    ln_row<NV>(v, gb, mean, rstd);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const size_t o = (size_t)r * D + 4 * lane + 256 * i;
        if (out) st4<T>(out + o, v[i]);
        if (outf) st4<float>(outf + o, v[i]);
    }
    if (lane == 0 && mean_out) { mean_out[r] = mean; rstd_out[r] = rstd; }
}

// dx_out = dx_in + LN'(dy):  rstd * (g - mean(g) - xhat * mean(g * xhat)),  g = dy * gamma
// deep-VPT gradient fused into ln_1's backward (model.py:131-140): rows 1..NV of every crop are the
// gradient of that layer's prompt tokens; they go to rows[(b*NV + l-1)*D] and the token-stream
// gradient of those rows (dx_out, dx_out_t) becomes zero (the prompt replaced them at this layer's input)
struct VptOut {
    float* rows;            // null: plain LayerNorm backward
    int L, NV;
};

// RD: rows-dense output (layer 0's prompt rows): x, dx_in, mean and rstd at the mapped row, dy and dx_out dense
// touch (ZF, ln_post's backward, the ViT backward's first launch): the first block's dX weights read onto the die
// (touch.h) -- the later blocks' are touched by the attention backward above them, the first block's had none (r06
// kernel trace: its c_fc dX product 38.3 us against 29 us for the others)
template <class T, class DY, int NV, bool ZF = false, bool RD = false>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const DY* __restrict__ dy, const float* __restrict__ x, RowMap map,
                                                     const float* mean_in, const float* rstd_in, const float* gamma,
                                                     const float* dx_in, float* dx_out, T* dx_out_t, int M, VptOut vo,
                                                     TouchList touch)
{
    constexpr int D = 256 * NV;
    constexpr float inv = 1.0f / (float)D;
    int r = row_block() * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    // the touch loads first: in flight beside the row's loads (issued after them, hipcc's waits for the row data at
    // the kernel-argument branches below drained them too), waited at the wave's end
    TouchSink ts;
    if constexpr (ZF) { if (touch.n) touch_issue1<4>(touch, ts); }
    if constexpr (ZF) {
        // grid over every destination row (M = groups * gstride): rows outside the mapped groups get a zero
        // gradient (ln_post: the CLS / prompt rows), the others run as mapped row r = their index in the groups
        if (r >= M) {
            if (touch.n) touch_wait(ts);
            return;
        }
        const int grp = r / map.gstride, l = r - grp * map.gstride;
        if (l < map.goff || l >= map.goff + map.rpg) {
#pragma unroll
            for (int i = 0; i < NV; ++i) {
                const int c = 4 * lane + 256 * i;
                *reinterpret_cast<float4*>(dx_out + (size_t)r * D + c) = make_float4(0.f, 0.f, 0.f, 0.f);
                if (dx_out_t) st4<T>(dx_out_t + (size_t)r * D + c, make_float4(0.f, 0.f, 0.f, 0.f));
            }
            if (touch.n) touch_wait(ts);
            return;
        }
        r = grp * map.rpg + l - map.goff;
    } else {
        if (r >= M) return;
    }
    const size_t mrow = map(r), xr = mrow * D;
    const float mean = mean_in[RD ? mrow : r], rstd = rstd_in[RD ? mrow : r];
    const size_t orow = RD ? (size_t)r * D : xr;
    float4 g[NV], xh[NV], din[NV];
    float s1 = 0.f, s2 = 0.f;
    // the incoming gradient is loaded with the row operands (not after the reductions)
#pragma unroll
    for (int i = 0; i < NV; ++i)
        din[i] = dx_in ? *reinterpret_cast<const float4*>(dx_in + xr + 4 * lane + 256 * i) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int c = 4 * lane + 256 * i;
        const float4 d = ld4<DY>(dy + (size_t)r * D + c);
        const float4 gm = *reinterpret_cast<const float4*>(gamma + c);
        const float4 xv = *reinterpret_cast<const float4*>(x + xr + c);
        g[i] = make_float4(d.x * gm.x, d.y * gm.y, d.z * gm.z, d.w * gm.w);
        xh[i] = make_float4((xv.x - mean) * rstd, (xv.y - mean) * rstd, (xv.z - mean) * rstd, (xv.w - mean) * rstd);
        s1 += (g[i].x + g[i].y) + (g[i].z + g[i].w);
        s2 += (g[i].x * xh[i].x + g[i].y * xh[i].y) + (g[i].z * xh[i].z + g[i].w * xh[i].w);
    }
    s1 = wave_sum(s1) * inv;
    s2 = wave_sum(s2) * inv;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int c = 4 * lane + 256 * i;
        float4 o = make_float4(rstd * (g[i].x - s1 - xh[i].x * s2), rstd * (g[i].y - s1 - xh[i].y * s2),
                               rstd * (g[i].z - s1 - xh[i].z * s2), rstd * (g[i].w - s1 - xh[i].w * s2));
        if (dx_in) { o.x += din[i].x; o.y += din[i].y; o.z += din[i].z; o.w += din[i].w; }
        if (vo.rows) {
            const int b = r / vo.L, l = r - b * vo.L;
            if (l >= 1 && l <= vo.NV) {
                *reinterpret_cast<float4*>(vo.rows + ((size_t)b * vo.NV + l - 1) * D + c) = o;
                o = make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
        *reinterpret_cast<float4*>(dx_out + orow + c) = o;
        if (!RD && dx_out_t) st4<T>(dx_out_t + xr + c, o);
    }
    if constexpr (ZF) { if (touch.n) touch_wait(ts); }
}

// dvpt_l[r][c] = sum_b rows_l[b][r][c] for every layer l with a destination (crop order), one launch
struct VptSum {
    float* dst[64];
};
__global__ void vpt_sum_kernel(const float* __restrict__ rows, VptSum vs, int layers, int B, int n4)
{
    const int e = blockIdx.x * blockDim.x + threadIdx.x;        // float4 index within one layer's [NV][D]
    const int l = blockIdx.y;
    if (e >= n4 || !vs.dst[l]) return;
    const float4* src = reinterpret_cast<const float4*>(rows) + (size_t)l * B * n4 + e;
    // sixteen crops' loads in flight before their adds (r06: one dependent HBM round trip per crop took 10 us a step;
    // batches of eight left the 16-crop step's last seven crops one load at a time): indices past B re-read the last
    // crop and are not added, and the adds keep crop order, so the sums keep their bits
    constexpr int NB = 16;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int b0 = 0; b0 < B; b0 += NB) {
        float4 v[NB];
#pragma unroll
        for (int i = 0; i < NB; ++i) v[i] = src[(size_t)min(b0 + i, B - 1) * n4];
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const int b = b0 + i;
            if (b == 0) acc = v[i];
            else if (b < B) { acc.x += v[i].x; acc.y += v[i].y; acc.z += v[i].z; acc.w += v[i].w; }
        }
    }
    reinterpret_cast<float4*>(vs.dst[l])[e] = acc;
}

// x [B,3,H,W] f32 -> patches [B*gh*gw, 3*P*P] (k = c*P*P + kh*P + kw, conv1 weight order).  One workgroup a patch
// row, one float4 of it a thread, 32-bit index math (r06: the grid-stride form's 64-bit divisions made it VALU-bound,
// 9.1 us a step for 14 MB)
template <class T>
__global__ __launch_bounds__(1024) void im2col_kernel(const float* __restrict__ x, T* __restrict__ out, int H, int W, int P)
{
    const int gh = H / P, gw = W / P, PP = P * P, KD = 3 * PP;
    const int row = blockIdx.x, k = 4 * threadIdx.x;
    if (k >= KD) return;
    const int px = row % gw, t = row / gw, py = t % gh, b = t / gh;
    const int c = k / PP, r = k - c * PP, kh = r / P, kw = r - kh * P;
    const float4 v = *reinterpret_cast<const float4*>(x + ((size_t)(b * 3 + c) * H + (py * P + kh)) * W + px * P + kw);
    st4<T>(out + (size_t)row * KD + k, v);
}

// X[b, s] for the first block (models/clip/model.py:147-168):
//   s = 0: ln_pre(cls + pos[0]);  1 <= s <= NVPT: vpt_0;  s > NVPT: ln_pre(patch[b, s-1-NVPT] + pos[s-NVPT])
template <int NV>
__global__ __launch_bounds__(256) void embed_kernel(const float* __restrict__ patch, const float* cls, const float* pos,
                                                    const float* gamma, const float* beta, const float* vpt,
                                                    long vpt_bstride, float* X, int B, int L, int G, int NVPT)
{
    constexpr int D = 256 * NV;
    const int r = row_block() * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (r >= B * L) return;
    const int b = r / L, s = r % L;
    float* xo = X + (size_t)r * D;
    if (s >= 1 && s <= NVPT) {
        const float* vp = vpt + b * vpt_bstride + (size_t)(s - 1) * D;
#pragma unroll
        for (int i = 0; i < NV; ++i)
            *reinterpret_cast<float4*>(xo + 4 * lane + 256 * i) = *reinterpret_cast<const float4*>(vp + 4 * lane + 256 * i);
        return;
    }
    const int p = s == 0 ? -1 : s - 1 - NVPT;
    float4 v[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int c = 4 * lane + 256 * i;
        const float4 e = p < 0 ? *reinterpret_cast<const float4*>(cls + c)
                               : *reinterpret_cast<const float4*>(patch + ((size_t)b * G + p) * D + c);
        const float4 q = *reinterpret_cast<const float4*>(pos + (size_t)(p + 1) * D + c);
        v[i] = make_float4(e.x + q.x, e.y + q.y, e.z + q.z, e.w + q.w);
    }
    float4 gb[2 * NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        gb[2 * i] = *reinterpret_cast<const float4*>(gamma + 4 * lane + 256 * i);
        gb[2 * i + 1] = *reinterpret_cast<const float4*>(beta + 4 * lane + 256 * i);
    }
    float mean, rstd;
    ln_row<NV>(v, gb, mean, rstd);
#pragma unroll
    for (int i = 0; i < NV; ++i) *reinterpret_cast<float4*>(xo + 4 * lane + 256 * i) = v[i];
}

__global__ void insert_vpt_kernel(float* X, const float* vpt, long vpt_bstride, int B, int L, int NVPT, int D)
{
    const size_t total = (size_t)B * NVPT * D / 4;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
        const int c4 = (int)(e % (D / 4));
        const int r = (int)((e / (D / 4)) % NVPT), b = (int)(e / ((size_t)(D / 4) * NVPT));
        reinterpret_cast<float4*>(X + ((size_t)b * L + 1 + r) * D)[c4] =
            reinterpret_cast<const float4*>(vpt + b * vpt_bstride + (size_t)r * D)[c4];
    }
}

// dvpt[r, c] (+)= sum_b dX[b, 1+r, c]  (or per batch when per_batch), then zero those rows of dX / dXt.
// Block = 64 column groups of 4 x 4 crop lanes for one 256-column chunk of prompt row r: crop lane bl sums
// crops bl, bl+4, ... (all its loads in flight at once), the 4 lane sums meet in LDS in lane order.
template <class T>
__global__ __launch_bounds__(256) void vpt_grad_kernel(float* __restrict__ dX, T* __restrict__ dXt,
                                                       float* __restrict__ dvpt, int B, int L, int NVPT, int D,
                                                       int per_batch, int accumulate)
{
    __shared__ float4 red[4][64];
    const int cg = threadIdx.x & 63, bl = threadIdx.x >> 6;
    const int chunks = D / 256, r = blockIdx.x / chunks, c = (blockIdx.x - r * chunks) * 256 + 4 * cg;
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 s = z;
    constexpr int MAXB = 16;                      // crops per lane held in registers per pass
    for (int b0 = bl; b0 < B; b0 += 4 * MAXB) {
        float4 x[MAXB];
#pragma unroll
        for (int k = 0; k < MAXB; ++k) {
            const int b = b0 + 4 * k;
            x[k] = b < B ? *reinterpret_cast<const float4*>(dX + ((size_t)b * L + 1 + r) * D + c) : z;
        }
#pragma unroll
        for (int k = 0; k < MAXB; ++k) {
            const int b = b0 + 4 * k;
            if (b >= B) continue;
            const size_t o = ((size_t)b * L + 1 + r) * D + c;
            if (per_batch) {
                float4* dst = reinterpret_cast<float4*>(dvpt + ((size_t)b * NVPT + r) * D + c);
                float4 y = x[k];
                if (accumulate) { const float4 d = *dst; y.x += d.x; y.y += d.y; y.z += d.z; y.w += d.w; }
                *dst = y;
            } else {
                s.x += x[k].x; s.y += x[k].y; s.z += x[k].z; s.w += x[k].w;
            }
            *reinterpret_cast<float4*>(dX + o) = z;
            if (dXt) st4<T>(dXt + o, z);
        }
    }
    if (per_batch) return;
    red[bl][cg] = s;
    __syncthreads();
    if (bl == 0) {
        float4 t = red[0][cg];
#pragma unroll
        for (int k = 1; k < 4; ++k) { const float4 u = red[k][cg]; t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w; }
        float4* dst = reinterpret_cast<float4*>(dvpt + (size_t)r * D + c);
        if (accumulate) { const float4 d = *dst; t.x += d.x; t.y += d.y; t.z += d.z; t.w += d.w; }
        *dst = t;
    }
}

// ----------------------------------------------------------------------------- similarity head
// One wave per pixel, CH channels (CH / 64 per lane, in float4 pieces 256 apart), NB <= 16 bins; the text
// features are normalised in LDS.  CH = 512 (ViT-B/16) or 1024 (ResNet-50, models/clip/model.py:85-95).
// pixels per 4-wave block (r02, tools/kbench.py head): the forward is fastest with one pixel per wave (4: 15.7 us vs
// 18.5 at 16, 16 crops); the backward with 8 per wave (32: 38.2 vs 42.2 us; fewer blocks also mean fewer d bias
// partial rows for head_bias_finalize_kernel to sum)
constexpr int HEAD_FWD_PPB = 4, HEAD_BWD_PPB = 32;

template <class TZ, int CH>
__device__ __forceinline__ void load_pix(const TZ* z, float (&v)[CH / 64]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int q = 0; q < CH / 256; ++q) {
        const float4 a = ld4<TZ>(z + 256 * q + 4 * lane);
        v[4 * q] = a.x; v[4 * q + 1] = a.y; v[4 * q + 2] = a.z; v[4 * q + 3] = a.w;
    }
}

template <int CH>
__device__ void load_text(const float* text, int NB, float* tn) {
    // tn[k][c] = text[k][c] / max(||text[k]||, 1e-12)   (F.normalize, model.py:204): each text row read once, as
    // float4 pieces held in registers across the norm (the per-element loop re-read it, 2 x CH/64 dependent loads)
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    for (int k = w; k < NB; k += blockDim.x / 64) {
        float4 x[CH / 256];
        float s = 0.f;
#pragma unroll
        for (int q = 0; q < CH / 256; ++q) {
            x[q] = *reinterpret_cast<const float4*>(text + k * CH + 256 * q + 4 * lane);
            s += (x[q].x * x[q].x + x[q].y * x[q].y) + (x[q].z * x[q].z + x[q].w * x[q].w);
        }
        s = wave_sum(s);
        const float inv = 1.0f / fmaxf(sqrtf(s), 1e-12f);
#pragma unroll
        for (int q = 0; q < CH / 256; ++q)
            *reinterpret_cast<float4*>(tn + k * CH + 256 * q + 4 * lane) =
                make_float4(x[q].x * inv, x[q].y * inv, x[q].z * inv, x[q].w * inv);
    }
    __syncthreads();
}

// <scaled pixel, normalised text row> partial of this lane (its CH / 64 channels)
template <int CH>
__device__ __forceinline__ float text_dot(const float* t, const float* zs) {
    const int lane = threadIdx.x & 63;
    float d = 0.f;
#pragma unroll
    for (int q = 0; q < CH / 256; ++q) {
        const float4 a = *reinterpret_cast<const float4*>(t + 256 * q + 4 * lane);
        d += zs[4 * q] * a.x + zs[4 * q + 1] * a.y + zs[4 * q + 2] * a.z + zs[4 * q + 3] * a.w;
    }
    return d;
}

template <class TZ, int CH>
__global__ __launch_bounds__(256) void head_fwd_kernel(const TZ* __restrict__ Z, const float* text, const float* logit_scale,
                                                       const float* anchors, float* logits, float* expo, int P, int HW, int NB)
{
    constexpr int NV = CH / 64;
    extern __shared__ __attribute__((aligned(16))) float tn[];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    constexpr int PPW = HEAD_FWD_PPB / 4;            // pixels per wave: every row load issued up front,
    float vv[PPW][NV];                                // before the text normalisation (latencies overlap)
#pragma unroll
    for (int j = 0; j < PPW; ++j) load_pix<TZ, CH>(Z + (size_t)min(blockIdx.x * HEAD_FWD_PPB + w + 4 * j, P - 1) * CH, vv[j]);
    const float s = expf(*logit_scale);
    load_text<CH>(text, NB, tn);
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
        const int p = blockIdx.x * HEAD_FWD_PPB + w + 4 * j;
        if (p >= P) break;
        float* v = vv[j];
        float ss = 0.f;
#pragma unroll
        for (int j = 0; j < NV; ++j) ss += v[j] * v[j];
        const float inv = 1.0f / fmaxf(sqrtf(wave_sum(ss)), 1e-12f);
        float zs[NV];
#pragma unroll
        for (int j = 0; j < NV; ++j) zs[j] = s * (v[j] * inv);
        float lg[16];
        float mx = -INFINITY;
        for (int k = 0; k < NB; ++k) {
            lg[k] = wave_sum(text_dot<CH>(tn + k * CH, zs));
            mx = fmaxf(mx, lg[k]);
        }
        float se = 0.f;
        for (int k = 0; k < NB; ++k) se += expf(lg[k] - mx);
        float e = 0.f;
        for (int k = 0; k < NB; ++k) e += (expf(lg[k] - mx) / se) * anchors[k];
        if (lane == 0) {
            const int b = p / HW, hw = p % HW;
            for (int k = 0; k < NB; ++k) logits[((size_t)b * NB + k) * HW + hw] = lg[k];
            expo[(size_t)b * HW + hw] = e;
        }
    }
}

// dZ = d/dZ of (logits, exp) given upstream dlogits [B,NB,HW], dexp [B,1,HW] (x *gscale if given);
// also this block's d bias (column sums of its dZ rows) and d logit_scale partial: part[block][0..CH) and
// part[block][CH] (plain stores; head_bias_finalize_kernel sums the blocks in order -- bit-reproducible, where float
// atomics from every block into the same CH addresses were neither reproducible nor free of contention).
template <class TZ, class TD, int CH>
__global__ __launch_bounds__(256) void head_bwd_kernel(const TZ* __restrict__ Z, const float* text, const float* logit_scale,
                                                       const float* anchors, const float* dlogits, const float* dexp,
                                                       const float* gscale, TD* dZ, float* part, int P, int HW, int NB)
{
    constexpr int NV = CH / 64;
    extern __shared__ __attribute__((aligned(16))) float tn[];
    float* dbias_l = tn + NB * CH;       // [4 waves][CH]
    float* dsc_l = dbias_l + 4 * CH;     // [4]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    constexpr int PPW = HEAD_BWD_PPB / 4;            // pixels per wave: every row load issued up front,
    float vv[PPW][NV];                                // before the text normalisation (latencies overlap)
#pragma unroll
    for (int j = 0; j < PPW; ++j) load_pix<TZ, CH>(Z + (size_t)min(blockIdx.x * HEAD_BWD_PPB + w + 4 * j, P - 1) * CH, vv[j]);
    const float ls = *logit_scale, s = expf(ls);
    const float gs = gscale ? *gscale : 1.0f;
    load_text<CH>(text, NB, tn);
    float db[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) db[j] = 0.f;
    float dsc = 0.f;
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
        const int p = blockIdx.x * HEAD_BWD_PPB + w + 4 * j;
        if (p >= P) break;
        float* v = vv[j];
        float ss = 0.f;
#pragma unroll
        for (int j = 0; j < NV; ++j) ss += v[j] * v[j];
        const float nrm = sqrtf(wave_sum(ss));
        const float den = fmaxf(nrm, 1e-12f), inv = 1.0f / den;
        float zn[NV], zs[NV];
#pragma unroll
        for (int j = 0; j < NV; ++j) { zn[j] = v[j] * inv; zs[j] = s * zn[j]; }
        float lg[16], pr[16];
        float mx = -INFINITY;
        for (int k = 0; k < NB; ++k) {
            lg[k] = wave_sum(text_dot<CH>(tn + k * CH, zs));
            mx = fmaxf(mx, lg[k]);
        }
        float se = 0.f;
        for (int k = 0; k < NB; ++k) { pr[k] = expf(lg[k] - mx); se += pr[k]; }
        float e = 0.f;
        for (int k = 0; k < NB; ++k) { pr[k] /= se; e += pr[k] * anchors[k]; }
        const int b = p / HW, hw = p % HW;
        const float de = dexp[(size_t)b * HW + hw] * gs;
        float dzn[NV];
#pragma unroll
        for (int j = 0; j < NV; ++j) dzn[j] = 0.f;
        for (int k = 0; k < NB; ++k) {
            // d logit_k = dlogits_k + dexp * p_k (anchor_k - e)   (softmax + expectation backward)
            const float dl = dlogits[((size_t)b * NB + k) * HW + hw] * gs + de * pr[k] * (anchors[k] - e);
            dsc += dl * lg[k];                             // logits = exp(ls) * cos  ->  d ls = dl * logits
            const float* t = tn + k * CH;
            const float c = dl * s;
#pragma unroll
            for (int q = 0; q < NV / 4; ++q) {
                const float4 a = *reinterpret_cast<const float4*>(t + 256 * q + 4 * lane);
                dzn[4 * q] += c * a.x; dzn[4 * q + 1] += c * a.y; dzn[4 * q + 2] += c * a.z; dzn[4 * q + 3] += c * a.w;
            }
        }
        // F.normalize backward: dz = (dzn - zn * <zn, dzn>) / ||z||   (or dzn / eps when clamped)
        float dot = 0.f;
#pragma unroll
        for (int j = 0; j < NV; ++j) dot += zn[j] * dzn[j];
        dot = (nrm > 1e-12f) ? wave_sum(dot) : 0.f;
        float dz[NV];
#pragma unroll
        for (int j = 0; j < NV; ++j) { dz[j] = (dzn[j] - zn[j] * dot) * inv; db[j] += dz[j]; }
#pragma unroll
        for (int q = 0; q < NV / 4; ++q)
            st4<TD>(dZ + (size_t)p * CH + 256 * q + 4 * lane, make_float4(dz[4 * q], dz[4 * q + 1], dz[4 * q + 2], dz[4 * q + 3]));
    }
    // lane 0's dsc is the wave's per-pixel sum (wave_sum results are lane-uniform)
#pragma unroll
    for (int q = 0; q < NV / 4; ++q)
#pragma unroll
        for (int j = 0; j < 4; ++j) dbias_l[w * CH + 256 * q + 4 * lane + j] = db[4 * q + j];
    if (lane == 0) dsc_l[w] = dsc;
    __syncthreads();
    if (!part) return;
    float* pr = part + (size_t)blockIdx.x * (CH + 1);
    for (int c = threadIdx.x; c < CH; c += blockDim.x)
        pr[c] = (dbias_l[c] + dbias_l[CH + c]) + (dbias_l[2 * CH + c] + dbias_l[3 * CH + c]);
    if (threadIdx.x == 0) pr[CH] = (dsc_l[0] + dsc_l[1]) + (dsc_l[2] + dsc_l[3]);
}

// dbias[c] = sum over blocks of part[b][c] (c < CH), dscale = sum of part[b][CH], blocks in order
// 64 columns per workgroup, 8 waves: wave w sums blocks w, w + 8, ... in eight interleaved chains (all eight loads
// of a round in flight: one serial chain of nblk dependent L2 round trips per lane took 31 us per step at 392 blocks),
// then the 8 wave sums are combined in wave order -- a fixed order, so the result is bit-reproducible
template <int CH>
__global__ __launch_bounds__(512) void head_bias_finalize_kernel(const float* __restrict__ part, int nblk, float* dbias,
                                                                 float* dscale)
{
    __shared__ float ws[8][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + lane;
    const bool live = c <= CH;
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int b = w;
    for (; b + 56 < nblk; b += 64) {
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += live ? part[(size_t)(b + 8 * j) * (CH + 1) + c] : 0.f;
    }
    for (int j = 0; b < nblk; b += 8, ++j) s[j & 7] += live ? part[(size_t)b * (CH + 1) + c] : 0.f;
    ws[w][lane] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
    __syncthreads();
    if (w == 0 && live) {
        float t = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) t += ws[k][lane];
        if (c < CH) { if (dbias) dbias[c] = t; }
        else if (dscale) *dscale = t;
    }
}

// delta[b, h, q] = sum_d dO[b*L+q, h*64+d] * O[b*L+q, h*64+d]   (FA-style backward row statistic)
template <class T>
__global__ void attn_delta_kernel(const T* dO, const T* O, float* delta, int B, int L, int H)
{
    const int total = B * L * H;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
        const int h = e % H, row = e / H;
        const int b = row / L, q = row % L;
        const T* a = dO + (size_t)row * H * 64 + h * 64;
        const T* o = O + (size_t)row * H * 64 + h * 64;
        float s = 0.f;
#pragma unroll
        for (int d = 0; d < 64; d += 4) {
            const float4 x = ld4<T>(a + d), y = ld4<T>(o + d);
            s += (x.x * y.x + x.y * y.y) + (x.z * y.z + x.w * y.w);
        }
        delta[((size_t)b * H + h) * L + q] = s;
    }
}

template <class T>
__global__ void cast_kernel(const float* in, T* out, size_t n4)
{
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n4; e += (size_t)gridDim.x * blockDim.x)
        st4<T>(out + 4 * e, reinterpret_cast<const float4*>(in)[e]);
}

inline int grid_for(size_t n, int block = 256) {
    const size_t g = (n + block - 1) / block;
    return (int)(g < 8192 ? (g ? g : 1) : 8192);
}

}  // namespace

// ------------------------------------------------------------------------------- launchers
namespace ebc {

static int ln_fwd_launch(int dtype, const float* x, RowMap map, const float* gamma, const float* beta, void* out,
                         float* outf, float* mean, float* rstd, int M, VptIns vi, hipStream_t st)
{
    const dim3 grid((M + 3) / 4);
    const int pi = probe_on() ? probe_start(EBC_PROBE_LN_FWD, 0, 0, 0, 0, M, 768, 0, st) : -1;
    struct Stop { int i; hipStream_t s; ~Stop() { probe_stop(i, s); } } stop{pi, st};
    switch (dtype) {
        case EBC_F32: hipLaunchKernelGGL((ln_fwd_kernel<float, 3>), grid, dim3(256), 0, st, x, map, gamma, beta, (float*)out, outf, mean, rstd, M, vi); break;
        case EBC_F16: hipLaunchKernelGGL((ln_fwd_kernel<_Float16, 3>), grid, dim3(256), 0, st, x, map, gamma, beta, (_Float16*)out, outf, mean, rstd, M, vi); break;
        case EBC_BF16: hipLaunchKernelGGL((ln_fwd_kernel<__bf16, 3>), grid, dim3(256), 0, st, x, map, gamma, beta, (__bf16*)out, outf, mean, rstd, M, vi); break;
        default: return EBC_E_ARG;
    }
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

int layernorm_fwd(int dtype, const float* x, int rpg, int gstride, int goff, const float* gamma, const float* beta,
                  void* out, float* outf, float* mean, float* rstd, int M, int D, hipStream_t st)
{
    if (D != 768 || M <= 0) return EBC_E_UNSUPPORTED;
    const RowMap map{rpg > 0 ? rpg : M, gstride, goff};
    return ln_fwd_launch(dtype, x, map, gamma, beta, out, outf, mean, rstd, M, VptIns{nullptr, 0, 1, 0, nullptr}, st);
}

int layernorm_fwd_vpt(int dtype, float* X, const float* vpt, long vpt_bstride, int L, int NVPT, const float* gamma,
                      const float* beta, void* out, float* mean, float* rstd, int M, int D, hipStream_t st)
{
    if (D != 768 || M <= 0 || L <= NVPT || M % L) return EBC_E_UNSUPPORTED;
    const RowMap map{M, 0, 0};
    return ln_fwd_launch(dtype, X, map, gamma, beta, out, nullptr, mean, rstd, M,
                         VptIns{vpt, vpt_bstride, L, NVPT, X}, st);
}

template <class T>
static int ln_bwd_t(int dy_f32, const void* dy, const float* x, RowMap map, const float* mean, const float* rstd,
                    const float* gamma, const float* dx_in, float* dx_out, void* dx_out_t, int M, VptOut vo, hipStream_t st)
{
    const dim3 grid((M + 3) / 4);
    const int pi = probe_on() ? probe_start(EBC_PROBE_LN_BWD, 0, 0, 0, 0, M, 768, 0, st) : -1;
    struct Stop { int i; hipStream_t s; ~Stop() { probe_stop(i, s); } } stop{pi, st};
    if (dy_f32)
        hipLaunchKernelGGL((ln_bwd_kernel<T, float, 3>), grid, dim3(256), 0, st, (const float*)dy, x, map, mean, rstd, gamma, dx_in, dx_out, (T*)dx_out_t, M, vo, TouchList{});
    else
        hipLaunchKernelGGL((ln_bwd_kernel<T, T, 3>), grid, dim3(256), 0, st, (const T*)dy, x, map, mean, rstd, gamma, dx_in, dx_out, (T*)dx_out_t, M, vo, TouchList{});
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

// ln_post's backward (dy f32 over the patch rows, no incoming dx): also writes the zero gradient of every row
// outside the groups, so dx_out / dx_out_t need no memset: one launch over all M / rpg * gstride rows
int layernorm_bwd_fill(int dtype, const float* dy, const float* x, int rpg, int gstride, int goff, const float* mean,
                       const float* rstd, const float* gamma, float* dx_out, void* dx_out_t, int M, int D, hipStream_t st,
                       const TouchList* touch)
{
    if (D != 768 || M <= 0 || rpg <= 0 || M % rpg || goff + rpg > gstride) return EBC_E_UNSUPPORTED;
    const RowMap map{rpg, gstride, goff};
    const VptOut vo{nullptr, 1, 0};
    TouchList t = touch && touch_enabled() ? *touch : TouchList{};
    size_t lines = 0;                                   // at most one line a lane (touch_issue1)
    for (int i = 0; i < t.n; ++i) lines += t.bytes[i] >> 7;
    const int Mf = M / rpg * gstride;
    const dim3 grid((Mf + 3) / 4);
    if (lines > (size_t)grid.x * 256) t = TouchList{};
    const int pi = probe_on() ? probe_start(EBC_PROBE_LN_BWD, 0, 0, 0, 0, Mf, 768, 0, st) : -1;
    switch (dtype) {
        case EBC_F32: hipLaunchKernelGGL((ln_bwd_kernel<float, float, 3, true>), grid, dim3(256), 0, st, dy, x, map, mean, rstd,
                                         gamma, nullptr, dx_out, (float*)dx_out_t, Mf, vo, t); break;
        case EBC_F16: hipLaunchKernelGGL((ln_bwd_kernel<_Float16, float, 3, true>), grid, dim3(256), 0, st, dy, x, map, mean,
                                         rstd, gamma, nullptr, dx_out, (_Float16*)dx_out_t, Mf, vo, t); break;
        case EBC_BF16: hipLaunchKernelGGL((ln_bwd_kernel<__bf16, float, 3, true>), grid, dim3(256), 0, st, dy, x, map, mean,
                                          rstd, gamma, nullptr, dx_out, (__bf16*)dx_out_t, Mf, vo, t); break;
        default: probe_stop(pi, st); return EBC_E_ARG;
    }
    probe_stop(pi, st);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

int layernorm_bwd(int dtype, int dy_f32, const void* dy, const float* x, int rpg, int gstride, int goff,
                  const float* mean, const float* rstd, const float* gamma, const float* dx_in, float* dx_out,
                  void* dx_out_t, int M, int D, hipStream_t st)
{
    if (D != 768 || M <= 0) return EBC_E_UNSUPPORTED;
    const RowMap map{rpg > 0 ? rpg : M, gstride, goff};
    const VptOut vo{nullptr, 1, 0};
    switch (dtype) {
        case EBC_F32: return ln_bwd_t<float>(1, dy, x, map, mean, rstd, gamma, dx_in, dx_out, dx_out_t, M, vo, st);
        case EBC_F16: return ln_bwd_t<_Float16>(dy_f32, dy, x, map, mean, rstd, gamma, dx_in, dx_out, dx_out_t, M, vo, st);
        case EBC_BF16: return ln_bwd_t<__bf16>(dy_f32, dy, x, map, mean, rstd, gamma, dx_in, dx_out, dx_out_t, M, vo, st);
    }
    return EBC_E_ARG;
}

int im2col(int dtype, const float* x, void* out, int B, int H, int W, int P, hipStream_t st)
{
    if (H % P || W % P || (P * P * 3) % 4 || P % 4) return EBC_E_ARG;
    const long rows = (long)B * (H / P) * (W / P);
    const int k4 = 3 * P * P / 4, blk = (k4 + 63) / 64 * 64;
    if (rows <= 0 || rows > INT_MAX || blk > 1024 || (size_t)B * 3 * H * W > (size_t)INT_MAX * 4) return EBC_E_ARG;
    const dim3 grid((unsigned)rows);
    switch (dtype) {
        case EBC_F32: hipLaunchKernelGGL(im2col_kernel<float>, grid, dim3(blk), 0, st, x, (float*)out, H, W, P); break;
        case EBC_F16: hipLaunchKernelGGL(im2col_kernel<_Float16>, grid, dim3(blk), 0, st, x, (_Float16*)out, H, W, P); break;
        case EBC_BF16: hipLaunchKernelGGL(im2col_kernel<__bf16>, grid, dim3(blk), 0, st, x, (__bf16*)out, H, W, P); break;
        default: return EBC_E_ARG;
    }
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

int embed_tokens(const float* patch, const float* cls, const float* pos, const float* gamma, const float* beta,
                 const float* vpt, long vpt_bstride, float* X, int B, int L, int G, int NVPT, int D, hipStream_t st)
{
    if (D != 768 || L != 1 + NVPT + G) return EBC_E_ARG;
    hipLaunchKernelGGL(embed_kernel<3>, dim3((B * L + 3) / 4), dim3(256), 0, st, patch, cls, pos, gamma, beta, vpt,
                       vpt_bstride, X, B, L, G, NVPT);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

int layernorm_bwd_vpt(int dtype, const void* dy, const float* x, const float* mean, const float* rstd,
                      const float* gamma, const float* dx_in, float* dx_out, void* dx_out_t, int M, int D, float* vpt_rows,
                      int L, int NVPT, hipStream_t st)
{
    if (D != 768 || M <= 0 || M % L || NVPT < 1 || NVPT >= L || !vpt_rows) return EBC_E_UNSUPPORTED;
    const RowMap map{M, 0, 0};
    const VptOut vo{vpt_rows, L, NVPT};
    switch (dtype) {
        case EBC_F32: return ln_bwd_t<float>(1, dy, x, map, mean, rstd, gamma, dx_in, dx_out, dx_out_t, M, vo, st);
        case EBC_F16: return ln_bwd_t<_Float16>(0, dy, x, map, mean, rstd, gamma, dx_in, dx_out, dx_out_t, M, vo, st);
        case EBC_BF16: return ln_bwd_t<__bf16>(0, dy, x, map, mean, rstd, gamma, dx_in, dx_out, dx_out_t, M, vo, st);
    }
    return EBC_E_ARG;
}

int layernorm_bwd_rows(int dtype, const void* dy, const float* x, int rpg, int gstride, int goff, const float* mean,
                       const float* rstd, const float* gamma, const float* dx_in, float* dx_out, int M, int D,
                       hipStream_t st)
{
    if (D != 768 || M <= 0 || rpg <= 0 || M % rpg || goff < 0 || goff + rpg > gstride) return EBC_E_UNSUPPORTED;
    const RowMap map{rpg, gstride, goff};
    const VptOut vo{nullptr, 1, 0};
    const dim3 grid((M + 3) / 4);
    const int pi = probe_on() ? probe_start(EBC_PROBE_LN_BWD, 0, 0, 0, 0, M, 768, 0, st) : -1;
    struct Stop { int i; hipStream_t s; ~Stop() { probe_stop(i, s); } } stop{pi, st};
    switch (dtype) {
        case EBC_F32: hipLaunchKernelGGL((ln_bwd_kernel<float, float, 3, false, true>), grid, dim3(256), 0, st, (const float*)dy,
                                         x, map, mean, rstd, gamma, dx_in, dx_out, (float*)nullptr, M, vo, TouchList{}); break;
        case EBC_F16: hipLaunchKernelGGL((ln_bwd_kernel<_Float16, _Float16, 3, false, true>), grid, dim3(256), 0, st,
                                         (const _Float16*)dy, x, map, mean, rstd, gamma, dx_in, dx_out, (_Float16*)nullptr, M, vo, TouchList{}); break;
        case EBC_BF16: hipLaunchKernelGGL((ln_bwd_kernel<__bf16, __bf16, 3, false, true>), grid, dim3(256), 0, st,
                                          (const __bf16*)dy, x, map, mean, rstd, gamma, dx_in, dx_out, (__bf16*)nullptr, M, vo, TouchList{}); break;
        default: return EBC_E_ARG;
    }
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

int vpt_sum(const float* rows, float* const* dst, int layers, int B, int NVPT, int D, hipStream_t st)
{
    if (layers <= 0 || layers > 64 || B <= 0 || D % 4) return EBC_E_ARG;
    VptSum vs{};
    bool any = false;
    for (int l = 0; l < layers; ++l) { vs.dst[l] = dst[l]; any |= dst[l] != nullptr; }
    if (!any) return EBC_OK;
    const int n4 = NVPT * D / 4;
    hipLaunchKernelGGL(vpt_sum_kernel, dim3((n4 + 255) / 256, layers), dim3(256), 0, st, rows, vs, layers, B, n4);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

int insert_vpt(float* X, const float* vpt, long vpt_bstride, int B, int L, int NVPT, int D, hipStream_t st)
{
    const size_t n = (size_t)B * NVPT * D / 4;
    hipLaunchKernelGGL(insert_vpt_kernel, dim3(grid_for(n)), dim3(256), 0, st, X, vpt, vpt_bstride, B, L, NVPT, D);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

int vpt_grad(int dtype, float* dX, void* dXt, float* dvpt, int B, int L, int NVPT, int D, int per_batch, int accumulate, hipStream_t st)
{
    if (D % 256 || NVPT <= 0 || B <= 0) return NVPT == 0 ? EBC_OK : EBC_E_UNSUPPORTED;
    const dim3 grid((unsigned)(NVPT * (D / 256)));
    switch (dtype) {
        case EBC_F32: hipLaunchKernelGGL(vpt_grad_kernel<float>, grid, dim3(256), 0, st, dX, (float*)dXt, dvpt, B, L, NVPT, D, per_batch, accumulate); break;
        case EBC_F16: hipLaunchKernelGGL(vpt_grad_kernel<_Float16>, grid, dim3(256), 0, st, dX, (_Float16*)dXt, dvpt, B, L, NVPT, D, per_batch, accumulate); break;
        case EBC_BF16: hipLaunchKernelGGL(vpt_grad_kernel<__bf16>, grid, dim3(256), 0, st, dX, (__bf16*)dXt, dvpt, B, L, NVPT, D, per_batch, accumulate); break;
        default: return EBC_E_ARG;
    }
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

template <int CH>
static int head_fwd_t(int dtype_z, const void* Z, const float* text, const float* logit_scale, const float* anchors,
                      float* logits, float* expo, int P, int HW, int NB, hipStream_t st)
{
    const dim3 grid((P + HEAD_FWD_PPB - 1) / HEAD_FWD_PPB);
    const size_t lds = (size_t)NB * CH * 4;
    switch (dtype_z) {
        case EBC_F32: hipLaunchKernelGGL((head_fwd_kernel<float, CH>), grid, dim3(256), lds, st, (const float*)Z, text, logit_scale, anchors, logits, expo, P, HW, NB); break;
        case EBC_F16: hipLaunchKernelGGL((head_fwd_kernel<_Float16, CH>), grid, dim3(256), lds, st, (const _Float16*)Z, text, logit_scale, anchors, logits, expo, P, HW, NB); break;
        case EBC_BF16: hipLaunchKernelGGL((head_fwd_kernel<__bf16, CH>), grid, dim3(256), lds, st, (const __bf16*)Z, text, logit_scale, anchors, logits, expo, P, HW, NB); break;
        default: return EBC_E_ARG;
    }
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

int head_fwd(int dtype_z, const void* Z, const float* text, const float* logit_scale, const float* anchors,
             float* logits, float* expo, int P, int HW, int NB, int embed, hipStream_t st)
{
    if (NB <= 0 || NB > 16) return EBC_E_UNSUPPORTED;
    if (embed == 512) return head_fwd_t<512>(dtype_z, Z, text, logit_scale, anchors, logits, expo, P, HW, NB, st);
    if (embed == 1024) return head_fwd_t<1024>(dtype_z, Z, text, logit_scale, anchors, logits, expo, P, HW, NB, st);
    return EBC_E_UNSUPPORTED;
}

template <int CH>
static int head_bwd_t(int dtype_z, int dtype_dz, const void* Z, const float* text, const float* logit_scale,
                      const float* anchors, const float* dlogits, const float* dexp, const float* gscale, void* dZ,
                      float* dbias, float* dscale, int P, int HW, int NB, void* ws, size_t wsb, hipStream_t st)
{
    const int nblk = (P + HEAD_BWD_PPB - 1) / HEAD_BWD_PPB;
    const bool sums = dbias || dscale;
    float* part = sums ? reinterpret_cast<float*>(ws) : nullptr;
    if (sums && (!ws || wsb < head_bwd_ws_bytes(P, CH))) return EBC_E_ARG;
    const dim3 grid(nblk);
    const size_t lds = ((size_t)NB * CH + 4 * CH + 4) * 4;
    constexpr int LDS_MAX = (16 * CH + 4 * CH + 4) * 4;      // NB <= 16 (embed 1024: 81 KiB)
#define HB(TZ, TD) if (!ensure_lds<head_bwd_kernel<TZ, TD, CH>>(LDS_MAX, st)) return EBC_E_LAUNCH; \
    hipLaunchKernelGGL((head_bwd_kernel<TZ, TD, CH>), grid, dim3(256), lds, st, (const TZ*)Z, text, logit_scale, anchors, dlogits, dexp, gscale, (TD*)dZ, part, P, HW, NB)
    // the dZ element type is the caller's buffer type (dtype_dz), independent of Z's
#define HBZ(TZ)                                                   \
    switch (dtype_dz) {                                           \
        case EBC_F32: HB(TZ, float); break;                       \
        case EBC_F16: HB(TZ, _Float16); break;                    \
        case EBC_BF16: HB(TZ, __bf16); break;                     \
        default: return EBC_E_ARG;                                \
    }
    switch (dtype_z) {
        case EBC_F32: HBZ(float); break;
        case EBC_F16: HBZ(_Float16); break;
        case EBC_BF16: HBZ(__bf16); break;
        default: return EBC_E_ARG;
    }
#undef HBZ
#undef HB
    EBC_CHECK_LAUNCH();
    if (sums) {
        hipLaunchKernelGGL(head_bias_finalize_kernel<CH>, dim3(CH / 64 + 1), dim3(512), 0, st, part, nblk, dbias, dscale);
        EBC_CHECK_LAUNCH();
    }
    return EBC_OK;
}

size_t head_bwd_ws_bytes(int P, int embed)
{
    return P > 0 ? (size_t)((P + HEAD_BWD_PPB - 1) / HEAD_BWD_PPB) * (embed + 1) * sizeof(float) : 0;
}

int head_bwd(int dtype_z, int dtype_dz, const void* Z, const float* text, const float* logit_scale, const float* anchors,
             const float* dlogits, const float* dexp, const float* gscale, void* dZ, float* dbias, float* dscale,
             int P, int HW, int NB, int embed, void* ws, size_t wsb, hipStream_t st)
{
    if (NB <= 0 || NB > 16 || P <= 0) return EBC_E_UNSUPPORTED;
    if (embed == 512)
        return head_bwd_t<512>(dtype_z, dtype_dz, Z, text, logit_scale, anchors, dlogits, dexp, gscale, dZ, dbias, dscale, P, HW, NB,
                               ws, wsb, st);
    if (embed == 1024)
        return head_bwd_t<1024>(dtype_z, dtype_dz, Z, text, logit_scale, anchors, dlogits, dexp, gscale, dZ, dbias, dscale, P, HW,
                                NB, ws, wsb, st);
    return EBC_E_UNSUPPORTED;
}

int attn_delta(int dtype, const void* dO, const void* O, float* delta, int B, int L, int H, hipStream_t st)
{
    const int n = B * L * H;
    switch (dtype) {
        case EBC_F32: hipLaunchKernelGGL(attn_delta_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, (const float*)dO, (const float*)O, delta, B, L, H); break;
        case EBC_F16: hipLaunchKernelGGL(attn_delta_kernel<_Float16>, dim3(grid_for(n)), dim3(256), 0, st, (const _Float16*)dO, (const _Float16*)O, delta, B, L, H); break;
        case EBC_BF16: hipLaunchKernelGGL(attn_delta_kernel<__bf16>, dim3(grid_for(n)), dim3(256), 0, st, (const __bf16*)dO, (const __bf16*)O, delta, B, L, H); break;
        default: return EBC_E_ARG;
    }
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

int cast_f32(int dtype, const float* in, void* out, size_t n, hipStream_t st)
{
    if (n % 4) return EBC_E_ARG;
    switch (dtype) {
        case EBC_F16: hipLaunchKernelGGL(cast_kernel<_Float16>, dim3(grid_for(n / 4)), dim3(256), 0, st, in, (_Float16*)out, n / 4); break;
        case EBC_BF16: hipLaunchKernelGGL(cast_kernel<__bf16>, dim3(grid_for(n / 4)), dim3(256), 0, st, in, (__bf16*)out, n / 4); break;
        case EBC_F32: hipLaunchKernelGGL(cast_kernel<float>, dim3(grid_for(n / 4)), dim3(256), 0, st, in, (float*)out, n / 4); break;
        default: return EBC_E_ARG;
    }
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

}  // namespace ebc
