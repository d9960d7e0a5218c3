// Training-crop augmentation on device: crop + antialiased bicubic resize + flip + colour jitter +
// Gaussian blur + salt-and-pepper noise + ImageNet normalisation, and the dot-map targets.
//
// Reference (the reference runs all of this on CPU in DataLoader workers):
//   RandomResizedCrop / _crop / _resize   datasets/transforms.py:9-43,133-171
//       TF.resize(bicubic, antialias=True) = torch F.interpolate(mode="bicubic", antialias=True)
//   RandomHorizontalFlip                  datasets/transforms.py:174-187
//   ColorJitter (brightness/contrast/saturation/hue)      datasets/transforms.py:190-201
//   GaussianBlur(kernel_size, sigma=(0.1, 5.0))           datasets/transforms.py:217-223
//   PepperSaltNoise                       datasets/transforms.py:242-255
//   Normalize(ImageNet mean/std)          datasets/crowd.py:64,162
//   generate_density_map (sigma = None)   datasets/utils.py:11-28
//
// Launches per batch of crops (all crops of all images in each launch, RB-row blocks):
//   resize_h: rows of each crop window -> [3][crop_h][out_w] scratch (horizontal AA-bicubic taps)
//   resize_v: scratch -> [3][out_h][out_w] output (vertical taps), horizontal flip on the store
//   gray_partial, pointwise, blur_v, blur_h: the per-crop op lists (see pointwise_kernel)
// Byte work (HBM/L2-bound): every thread owns output columns, so all loads/stores are row-contiguous.
#include "ebc_common.h"

namespace {

constexpr int RB = 4;          // rows per workgroup in the resize passes

// torch's antialias bicubic filter (a = -0.5), UpSampleKernel.cpp aa path
__device__ __forceinline__ float aa_cubic(float x) {
    constexpr float a = -0.5f;
    x = fabsf(x);
    if (x < 1.f) return ((a + 2.f) * x - (a + 3.f)) * x * x + 1.f;
    if (x < 2.f) return (((x - 5.f) * x + 8.f) * x - 4.f) * a;
    return 0.f;
}

// taps of output index i for an in_size -> out_size AA resize: first input index, count, 1/sum
struct Taps { int lo, n; float center, inv, norm; };
__device__ __forceinline__ Taps aa_taps(int i, int in_size, int out_size) {
    const float scale = (float)in_size / (float)out_size;
    const float support = scale >= 1.f ? 2.f * scale : 2.f;
    Taps t;
    t.inv = scale >= 1.f ? 1.f / scale : 1.f;
    t.center = scale * ((float)i + 0.5f);
    t.lo = max((int)(t.center - support + 0.5f), 0);
    const int hi = min((int)(t.center + support + 0.5f), in_size);
    t.n = hi - t.lo;
    float s = 0.f;
    for (int j = 0; j < t.n; ++j) s += aa_cubic(((float)(j + t.lo) - t.center + 0.5f) * t.inv);
    t.norm = s != 0.f ? 1.f / s : 0.f;
    return t;
}
__device__ __forceinline__ float tap_w(const Taps& t, int j) {
    return aa_cubic(((float)(j + t.lo) - t.center + 0.5f) * t.inv) * t.norm;
}

__global__ __launch_bounds__(256) void resize_h_kernel(const float* __restrict__ src, const EbcCropDesc* __restrict__ desc,
                                                       float* __restrict__ ws)
{
    const EbcCropDesc d = desc[blockIdx.y / 3];
    const int c = blockIdx.y % 3, r0 = blockIdx.x * RB;
    if (r0 >= d.crop_h) return;
    const float* plane = src + d.src_off + (size_t)c * d.src_h * d.src_w;
    float* tmp = ws + d.tmp_off + (size_t)c * d.crop_h * d.out_w;
    for (int ox = threadIdx.x; ox < d.out_w; ox += blockDim.x) {
        const Taps t = aa_taps(ox, d.crop_w, d.out_w);
        for (int r = r0; r < min(r0 + RB, d.crop_h); ++r) {
            const float* row = plane + (size_t)(d.top + r) * d.src_w + d.left + t.lo;
            float acc = 0.f;
            for (int j = 0; j < t.n; ++j) acc = fmaf(tap_w(t, j), row[j], acc);
            tmp[(size_t)r * d.out_w + ox] = acc;
        }
    }
}

__global__ __launch_bounds__(256) void resize_v_kernel(const EbcCropDesc* __restrict__ desc, const float* __restrict__ ws,
                                                       float* __restrict__ out)
{
    const EbcCropDesc d = desc[blockIdx.y / 3];
    const int c = blockIdx.y % 3, y0 = blockIdx.x * RB;
    if (y0 >= d.out_h) return;
    const float* tmp = ws + d.tmp_off + (size_t)c * d.crop_h * d.out_w;
    float* o = out + d.out_off + (size_t)c * d.out_h * d.out_w;
    for (int y = y0; y < min(y0 + RB, d.out_h); ++y) {
        const Taps t = aa_taps(y, d.crop_h, d.out_h);
        for (int ox = threadIdx.x; ox < d.out_w; ox += blockDim.x) {
            float acc = 0.f;
            for (int j = 0; j < t.n; ++j) acc = fmaf(tap_w(t, j), tmp[(size_t)(t.lo + j) * d.out_w + ox], acc);
            o[(size_t)y * d.out_w + (d.flip ? d.out_w - 1 - ox : ox)] = acc;
        }
    }
}

__device__ __forceinline__ float clamp01(float x) { return fminf(fmaxf(x, 0.f), 1.f); }
// TF.rgb_to_grayscale for float images: 0.2989 r + 0.587 g + 0.114 b
__device__ __forceinline__ float gray(float r, float g, float b) { return 0.2989f * r + 0.587f * g + 0.114f * b; }

// counter-based uniform [0, 1): murmur3 finaliser of (seed, element index), 24 random bits
__device__ __forceinline__ float hash_uniform(uint32_t seed, uint32_t idx) {
    uint32_t h = seed ^ (idx * 0x9E3779B9u);
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
    return (float)(h >> 8) * (1.0f / 16777216.0f);
}

__device__ __forceinline__ int reflect(int i, int n) { return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i); }

// The per-crop op list, spread over many workgroups per crop (a single CU per crop is bound by the
// bytes one CU keeps in flight): rows are cut into RB-row blocks, every pass is its own launch.
//   gray_partial : crops with a contrast op -- per-block grey sums of the image as it stands before
//                  that op (the earlier jitter ops applied on the fly), into the crop's scratch
//   pointwise    : all jitter ops (contrast's mean = the fixed-order sum of those partials); crops
//                  without blur also get noise + normalisation here
//   blur_v/blur_h: GaussianBlur (vertical taps into scratch, horizontal taps + noise + normalisation)
struct Pix { float r, g, b; };

// torchvision F.adjust_hue on one float pixel, in its float32 operations (_rgb2hsv, h = (h + f) % 1, _hsv2rgb; the
// reference's masks select exactly one term, so the masked sums are that term); no contraction into FMAs, so each
// operation rounds as the reference's separate tensor ops do
__device__ __forceinline__ Pix adjust_hue(Pix px, float hf) {
#pragma clang fp contract(off)
    const float r = px.r, g = px.g, b = px.b;
    const float maxc = fmaxf(fmaxf(r, g), b), minc = fminf(fminf(r, g), b);
    const bool eqc = maxc == minc;
    const float cr = maxc - minc;
    const float s = cr / (eqc ? 1.0f : maxc);
    const float crd = eqc ? 1.0f : cr;
    const float rc = (maxc - r) / crd, gc = (maxc - g) / crd, bc = (maxc - b) / crd;
    float h;
    if (maxc == r) h = bc - gc;
    else if (maxc == g) h = (2.0f + rc) - bc;
    else h = (4.0f + gc) - rc;
    h = fmodf(h / 6.0f + 1.0f, 1.0f);
    // (h + hue) % 1.0: torch.remainder (fmod, then + 1 for a negative remainder)
    float hh = fmodf(h + hf, 1.0f);
    if (hh != 0.0f && hh < 0.0f) hh += 1.0f;
    const float v = maxc;
    const float fi = floorf(hh * 6.0f);
    const float f = hh * 6.0f - fi;
    int i = (int)fi % 6;
    if (i < 0) i += 6;
    const float p = fminf(fmaxf(v * (1.0f - s), 0.0f), 1.0f);
    const float q = fminf(fmaxf(v * (1.0f - s * f), 0.0f), 1.0f);
    const float t = fminf(fmaxf(v * (1.0f - s * (1.0f - f)), 0.0f), 1.0f);
    switch (i) {
        case 0: return {v, t, p};
        case 1: return {q, v, p};
        case 2: return {p, v, t};
        case 3: return {p, q, v};
        case 4: return {t, p, v};
        default: return {v, p, q};
    }
}

__device__ __forceinline__ Pix jitter_apply(Pix p, int ops, int from, int to, const EbcCropDesc& d, float cmean) {
    for (int slot = from; slot < to; ++slot) {
        const int op = (ops >> (3 * slot)) & 7;
        if (op == 1) {
            p.r = clamp01(d.brightness * p.r); p.g = clamp01(d.brightness * p.g); p.b = clamp01(d.brightness * p.b);
        } else if (op == 2) {
            const float f = d.contrast, mb = (1.f - f) * cmean;
            p.r = clamp01(f * p.r + mb); p.g = clamp01(f * p.g + mb); p.b = clamp01(f * p.b + mb);
        } else if (op == 3) {
            const float f = d.saturation, gm = (1.f - f) * gray(p.r, p.g, p.b);
            p.r = clamp01(f * p.r + gm); p.g = clamp01(f * p.g + gm); p.b = clamp01(f * p.b + gm);
        } else if (op == 4) {
            p = adjust_hue(p, d.hue);
        }
    }
    return p;
}

__device__ __forceinline__ float finish_px(float v, int c, int e, const EbcCropDesc& d, const float* __restrict__ noise,
                                          const EbcAugConst& k) {
    if (d.noise) {
        const float u = d.noise_off >= 0 && noise ? noise[d.noise_off + e] : hash_uniform(d.seed, (uint32_t)e);
        if (u < d.saltiness) v = 1.f;
        if (u > 1.f - d.spiciness) v = 0.f;
    }
    if (d.normalize) v = (v - k.mean[c]) / k.std[c];
    return v;
}

__device__ __forceinline__ int n_ops(int ops) { int n = 0; while (n < 4 && ((ops >> (3 * n)) & 7)) ++n; return n; }
__device__ __forceinline__ int contrast_slot(int ops) {
    int c = -1;
    for (int s = 0; s < 4; ++s) if (((ops >> (3 * s)) & 7) == 2) c = s;
    return c;
}

constexpr int PT = 256;        // pointwise / blur threads

__device__ float block_sum_pt(float v, float* red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(PT) void gray_partial_kernel(const EbcCropDesc* __restrict__ desc, const float* __restrict__ out,
                                                         float* __restrict__ ws)
{
    __shared__ float red[PT / 64];
    const EbcCropDesc d = desc[blockIdx.y];
    const int cs = contrast_slot(d.jitter_ops), y0 = blockIdx.x * RB;
    if (cs < 0 || y0 >= d.out_h) return;
    const int HW = d.out_h * d.out_w;
    const float* R = out + d.out_off;
    float s = 0.f;
    for (int y = y0; y < min(y0 + RB, d.out_h); ++y)
        for (int x = threadIdx.x; x < d.out_w; x += PT) {
            const int e = y * d.out_w + x;
            const Pix p = jitter_apply({R[e], R[HW + e], R[2 * HW + e]}, d.jitter_ops, 0, cs, d, 0.f);
            s += gray(p.r, p.g, p.b);
        }
    s = block_sum_pt(s, red);
    if (threadIdx.x == 0) ws[d.tmp_off + blockIdx.x] = s;
}

__global__ __launch_bounds__(PT) void pointwise_kernel(const EbcCropDesc* __restrict__ desc, float* __restrict__ out,
                                                      const float* __restrict__ ws, const float* __restrict__ noise,
                                                      EbcAugConst k)
{
    const EbcCropDesc d = desc[blockIdx.y];
    const int y0 = blockIdx.x * RB, nops = n_ops(d.jitter_ops);
    if (y0 >= d.out_h || (nops == 0 && d.blur) || (nops == 0 && !d.noise && !d.normalize)) return;
    float cmean = 0.f;
    if (contrast_slot(d.jitter_ops) >= 0) {
        const int nb = (d.out_h + RB - 1) / RB;
        for (int i = 0; i < nb; ++i) cmean += ws[d.tmp_off + i];       // fixed order: reproducible
        cmean /= (float)(d.out_h * d.out_w);
    }
    const int HW = d.out_h * d.out_w;
    float* R = out + d.out_off;
    for (int y = y0; y < min(y0 + RB, d.out_h); ++y)
        for (int x = threadIdx.x; x < d.out_w; x += PT) {
            const int e = y * d.out_w + x;
            Pix p = jitter_apply({R[e], R[HW + e], R[2 * HW + e]}, d.jitter_ops, 0, nops, d, cmean);
            if (!d.blur) {
                p.r = finish_px(p.r, 0, e, d, noise, k);
                p.g = finish_px(p.g, 1, HW + e, d, noise, k);
                p.b = finish_px(p.b, 2, 2 * HW + e, d, noise, k);
            }
            R[e] = p.r; R[HW + e] = p.g; R[2 * HW + e] = p.b;
        }
}

// normalised pdf over linspace(-(ks-1)/2, (ks-1)/2, ks) (torchvision _get_gaussian_kernel1d)
__device__ void blur_taps(float* kk, int ks, float sigma) {
    if (threadIdx.x == 0) {
        float s = 0.f;
        for (int i = 0; i < ks; ++i) {
            const float x = (float)i - 0.5f * (float)(ks - 1);
            kk[i] = expf(-0.5f * (x / sigma) * (x / sigma));
            s += kk[i];
        }
        for (int i = 0; i < ks; ++i) kk[i] /= s;
    }
    __syncthreads();
}

__global__ __launch_bounds__(PT) void blur_v_kernel(const EbcCropDesc* __restrict__ desc, const float* __restrict__ out,
                                                   float* __restrict__ ws, EbcAugConst k)
{
    __shared__ float ky[EBC_AUG_MAX_BLUR];
    const EbcCropDesc d = desc[blockIdx.y / 3];
    const int c = blockIdx.y % 3, y0 = blockIdx.x * RB, H = d.out_h, W = d.out_w, hk = k.blur_k / 2;
    if (!d.blur || y0 >= H) return;
    blur_taps(ky, k.blur_k, k.sigma_y);
    const float* P = out + d.out_off + (size_t)c * H * W;
    float* S = ws + d.tmp_off + (size_t)c * H * W;
    for (int y = y0; y < min(y0 + RB, H); ++y)
        for (int x = threadIdx.x; x < W; x += PT) {
            float acc = 0.f;
            for (int i = 0; i < k.blur_k; ++i) acc = fmaf(ky[i], P[reflect(y + i - hk, H) * W + x], acc);
            S[y * W + x] = acc;
        }
}

__global__ __launch_bounds__(PT) void blur_h_kernel(const EbcCropDesc* __restrict__ desc, float* __restrict__ out,
                                                   const float* __restrict__ ws, const float* __restrict__ noise,
                                                   EbcAugConst k)
{
    __shared__ float kx[EBC_AUG_MAX_BLUR];
    const EbcCropDesc d = desc[blockIdx.y / 3];
    const int c = blockIdx.y % 3, y0 = blockIdx.x * RB, H = d.out_h, W = d.out_w, hk = k.blur_k / 2;
    if (!d.blur || y0 >= H) return;
    blur_taps(kx, k.blur_k, k.sigma_x);
    const float* S = ws + d.tmp_off + (size_t)c * H * W;
    float* O = out + d.out_off + (size_t)c * H * W;
    for (int y = y0; y < min(y0 + RB, H); ++y)
        for (int x = threadIdx.x; x < W; x += PT) {
            float acc = 0.f;
            for (int i = 0; i < k.blur_k; ++i) acc = fmaf(kx[i], S[y * W + reflect(x + i - hk, W)], acc);
            O[y * W + x] = finish_px(acc, c, c * H * W + y * W + x, d, noise, k);
        }
}

// dot map: out[b][0][clamp(int y)][clamp(int x)] = 1 (zeroed by the launcher)
__global__ void point_map_kernel(const float* __restrict__ pts, const int* __restrict__ offsets, int B, int H, int W,
                                 float* __restrict__ out)
{
    const int b = blockIdx.y;
    const int p0 = offsets[b], n = offsets[b + 1] - p0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int x = min(max((int)pts[2 * (p0 + i)], 0), W - 1);
        const int y = min(max((int)pts[2 * (p0 + i) + 1], 0), H - 1);
        out[((size_t)b * H + y) * W + x] = 1.0f;
    }
}

}  // namespace

extern "C" int ebc_augment_crops(const float* src, const EbcCropDesc* desc, int n, int max_crop_h, int max_out_h,
                                 float* out, float* workspace, const float* noise, EbcAugConst k, ebc_stream_t stream)
{
    if (n < 0 || !desc || !out || !workspace || max_crop_h < 0 || max_out_h < 0) return EBC_E_ARG;
    if (k.blur_k < 1 || k.blur_k > EBC_AUG_MAX_BLUR || (k.blur_k & 1) == 0) return EBC_E_ARG;
    if (n == 0) return EBC_OK;
    hipStream_t st = (hipStream_t)stream;
    if (src && max_crop_h > 0) {
        hipLaunchKernelGGL(resize_h_kernel, dim3((max_crop_h + RB - 1) / RB, 3 * n), dim3(256), 0, st, src, desc, workspace);
        EBC_CHECK_LAUNCH();
        hipLaunchKernelGGL(resize_v_kernel, dim3((max_out_h + RB - 1) / RB, 3 * n), dim3(256), 0, st, desc, workspace, out);
        EBC_CHECK_LAUNCH();
    }
    const int nb = (max_out_h + RB - 1) / RB;
    hipLaunchKernelGGL(gray_partial_kernel, dim3(nb, n), dim3(PT), 0, st, desc, out, workspace);
    EBC_CHECK_LAUNCH();
    hipLaunchKernelGGL(pointwise_kernel, dim3(nb, n), dim3(PT), 0, st, desc, out, workspace, noise, k);
    EBC_CHECK_LAUNCH();
    hipLaunchKernelGGL(blur_v_kernel, dim3(nb, 3 * n), dim3(PT), 0, st, desc, out, workspace, k);
    EBC_CHECK_LAUNCH();
    hipLaunchKernelGGL(blur_h_kernel, dim3(nb, 3 * n), dim3(PT), 0, st, desc, out, workspace, noise, k);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

extern "C" int ebc_point_map(const float* points, const int* offsets, int B, int H, int W, int max_points, float* out,
                             ebc_stream_t stream)
{
    if (B < 0 || H <= 0 || W <= 0 || !out || (B > 0 && !offsets)) return EBC_E_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(out, 0, sizeof(float) * (size_t)B * H * W, st) != hipSuccess) return EBC_E_LAUNCH;
    if (B == 0 || max_points <= 0) return EBC_OK;
    hipLaunchKernelGGL(point_map_kernel, dim3((max_points + 255) / 256, B), dim3(256), 0, st, points, offsets, B, H, W, out);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}
