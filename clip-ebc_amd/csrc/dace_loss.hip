// Fused DACE / DMCount loss for gfx950: one 512-thread workgroup per crop, every Sinkhorn
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
//    Ex = exp(xd/-reg).  A crop's kernel matrix shrinks from n*g^2 to 2*n*g floats, which fits
//    the 160 KiB LDS for n <= ~470 (g = 28) and streams from L2 above that.
//  * K^T u (a [g x n][n x g] product) is register-tiled 4x4 per thread and split over point
//    slices; K v is computed per point as sum_iy Ey[iy] * (sum_jx Ex[jx] v[iy][jx]) with the
//    v rows of a row-group held in registers (wave-uniform broadcast LDS reads).
//  * The reference's control flow is kept exactly: err every eval_freq iterations
//    (bregman_pytorch.py:117-126), stop when err <= stopThr or it > maxIter, NaN/Inf rollback
//    to the previous (u, v) and break (:111-115), the 1e-16 epsilons, denormals kept (the build
//    never flushes f32 denormals).  The err pass's K^T u is reused by the next iteration.
#include "ebc_common.h"

using namespace ebc;

namespace {

constexpr int NT = 512;                  // threads per workgroup (8 waves, 2 per SIMD)
constexpr int NWAVE = NT / 64;
constexpr int LDS_MAX = 160 * 1024;
constexpr float M_EPS = 1e-16f;          // bregman_pytorch.py:8
constexpr float EPS = 1e-8f;             // dm_loss.py:7

template <int G> struct Cfg {
    static constexpr int GG = G * G;
    static constexpr int NTILE = (G / 4) * (G / 4);      // 4x4 output tiles of K^T u
    static constexpr int SL = NT / NTILE;                // point slices
    static constexpr int R = (G <= 28) ? 4 : 2;          // rows per group in the K v pass
    static constexpr int NG = G / R;                     // row groups
    // fixed LDS (floats): pd, td, b, v0, v1, ktu, red[SL*GG], kvred[NWAVE*64], misc[64]
    static constexpr int FIXED = 6 * GG + SL * GG + NWAVE * 64 + 64;
    static constexpr size_t FIXED_BYTES = (size_t)FIXED * 4;
    static constexpr int PER_POINT = 2 * G + 2;          // Ey, Ex, u0, u1
    static_assert(NTILE * SL <= NT && SL >= 1, "tiling");
    static_assert(G % 4 == 0 && G % R == 0, "grid");
};

struct Params {
    const float* pred_class; const float* pred_density; const float* target_density;
    int target_is_reduced;
    const float* points; const int* offsets; const int* order;
    const float* bins_lo; const float* bins_hi;
    int B, N, size, red, count_mode, norm_cood;
    float w_count, w_ot, w_tv, reg, stop_thr;
    int max_iter, eval_freq;
    float* grad_class; float* grad_density; float* crop_stats; float* beta_out; int* status;
    float* ws_factors;     // global factor storage for crops that do not fit LDS
    int lds_cap;           // max points kept in LDS
};

// ---------------------------------------------------------------------------------------
// Sinkhorn-Knopp on the separable DMCount kernel.  `Ey`, `Ex` ([n][G]), `u0/u1` ([n]) live in
// LDS or global memory (FP = float* into either); everything else in LDS.
// cood of grid cell k (dm_loss.py:31-34): pixel centre, or normalised to [-1, 1] when norm_cood
__device__ __forceinline__ float cood(int k, int size, int norm) {
    const float c = (float)(k * 8) + 4.0f;
    return norm ? c / (float)size * 2.0f - 1.0f : c;
}
__device__ __forceinline__ float pcoord(float p, int size, int norm) {
    return norm ? p / (float)size * 2.0f - 1.0f : p;     // dm_loss.py:51
}

template <int G, typename FP>
__device__ void sinkhorn_crop(int n, int size, int norm, float reg, int max_iter, float stop_thr, int eval_freq,
                              const float* __restrict__ pts, FP Ey, FP Ex, FP u0, FP u1,
                              const float* b, float* v0, float* v1, float* ktu, float* red,
                              float* kvred, float* misc, int* iters_out, int* rolled_out, float* err_last_out)
{
    using C = Cfg<G>;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const float a = 1.0f / (float)n;                         // target_prob = ones/n
    // factors: Ey[i][iy] = exp(yd/-reg), Ex[i][jx] = exp(xd/-reg)
    for (int e = t; e < n * G; e += NT) {
        const int i = e / G, k = e - i * G;
        const float c = cood(k, size, norm);                  // dm_loss.py:31-34 (reduction 8)
        const float x = pcoord(pts[2 * i], size, norm), y = pcoord(pts[2 * i + 1], size, norm);
        const float yd = (-2.0f * (y * c) + y * y) + c * c;
        const float xd = (-2.0f * (x * c) + x * x) + c * c;
        Ey[e] = expf(yd / -reg);
        Ex[e] = expf(xd / -reg);
    }
    for (int i = t; i < n; i += NT) u0[i] = 1.0f / (float)n;
    for (int j = t; j < C::GG; j += NT) v0[j] = 1.0f / (float)C::GG;
    __syncthreads();

    FP u = u0; FP un = u1;
    float* v = v0; float* vn = v1;
    int have_ktu = 0, it = 1, rolled = 0;
    float err = 1.0f, err_last = -1.0f;

    // K^T u into ktu[GG] (or reuse)
    auto ktu_pass = [&](FP uu) {
        const int tile = t % C::NTILE, s = t / C::NTILE;
        if (s < C::SL) {
            const int ty = tile / (G / 4), tx = tile % (G / 4);
            float acc[4][4];
#pragma unroll
            for (int p = 0; p < 4; ++p)
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[p][q] = 0.f;
            for (int i = s; i < n; i += C::SL) {
                const float w = uu[i];
                const float4 ey = *reinterpret_cast<const float4*>(&Ey[i * G + 4 * ty]);
                const float4 ex = *reinterpret_cast<const float4*>(&Ex[i * G + 4 * tx]);
                const float wy[4] = {w * ey.x, w * ey.y, w * ey.z, w * ey.w};
                const float xx[4] = {ex.x, ex.y, ex.z, ex.w};
#pragma unroll
                for (int p = 0; p < 4; ++p)
#pragma unroll
                    for (int q = 0; q < 4; ++q) acc[p][q] = fmaf(wy[p], xx[q], acc[p][q]);
            }
#pragma unroll
            for (int p = 0; p < 4; ++p)
                *reinterpret_cast<float4*>(&red[s * C::GG + (4 * ty + p) * G + 4 * tx]) =
                    make_float4(acc[p][0], acc[p][1], acc[p][2], acc[p][3]);
        }
        __syncthreads();
        for (int j = t; j < C::GG; j += NT) {
            float sacc = 0.f;
#pragma unroll
            for (int s2 = 0; s2 < C::SL; ++s2) sacc += red[s2 * C::GG + j];
            ktu[j] = sacc;
        }
        __syncthreads();
    };

    while (err > stop_thr && it <= max_iter) {               // bregman_pytorch.py:102
        if (!have_ktu) ktu_pass(u);
        have_ktu = 0;
        // v = b / (K^T u + eps)
        int bad = 0;
        for (int j = t; j < C::GG; j += NT) {
            const float val = b[j] / (ktu[j] + M_EPS);
            vn[j] = val;
            bad |= !isfinite(val);
        }
        __syncthreads();
        // u = a / (K v + eps): per point, sum_iy Ey[iy] * (sum_jx Ex[jx] * v[iy][jx])
        for (int c0 = 0; c0 < n; c0 += 64) {
            const int i = c0 + lane;
            float kv = 0.f;
            if (i < n) {
                float ex[G];
#pragma unroll
                for (int q = 0; q < G; q += 4) {
                    const float4 e4 = *reinterpret_cast<const float4*>(&Ex[i * G + q]);
                    ex[q] = e4.x; ex[q + 1] = e4.y; ex[q + 2] = e4.z; ex[q + 3] = e4.w;
                }
                for (int grp = wv; grp < C::NG; grp += NWAVE) {
#pragma unroll
                    for (int r = 0; r < C::R; ++r) {
                        const int iy = grp * C::R + r;
                        const float* vr = &vn[iy * G];
                        float tr = 0.f;
#pragma unroll
                        for (int q = 0; q < G; q += 4) {
                            const float4 v4 = *reinterpret_cast<const float4*>(&vr[q]);
                            tr = fmaf(ex[q], v4.x, tr);
                            tr = fmaf(ex[q + 1], v4.y, tr);
                            tr = fmaf(ex[q + 2], v4.z, tr);
                            tr = fmaf(ex[q + 3], v4.w, tr);
                        }
                        kv = fmaf(Ey[i * G + iy], tr, kv);
                    }
                }
            }
            kvred[wv * 64 + lane] = kv;
            __syncthreads();
            if (t < 64 && c0 + t < n) {
                float s = 0.f;
#pragma unroll
                for (int w2 = 0; w2 < NWAVE; ++w2) s += kvred[w2 * 64 + t];
                const float val = a / (s + M_EPS);
                un[c0 + t] = val;
                bad |= !isfinite(val);
            }
            __syncthreads();
        }
        bad = block_or(bad, reinterpret_cast<int*>(misc));
        if (bad) { rolled = 1; break; }                       // keep (u, v): rollback, :111-115
        { FP tu = u; u = un; un = tu; float* tv = v; v = vn; vn = tv; }
        if (it % eval_freq == 0) {                            // :117-126
            ktu_pass(u);
            have_ktu = 1;
            float e = 0.f;
            for (int j = t; j < C::GG; j += NT) {
                const float d = b[j] - ktu[j] * v[j];
                e = fmaf(d, d, e);
            }
            err = block_sum(e, misc);
            err_last = err;
        }
        ++it;
    }
    // leave the final v in v0 and u in u0
    if (v != v0) { for (int j = t; j < C::GG; j += NT) v0[j] = v[j]; }
    if (u != u0) { for (int i = t; i < n; i += NT) u0[i] = u[i]; }
    __syncthreads();
    *iters_out = rolled ? it : it - 1;
    *rolled_out = rolled;
    *err_last_out = err_last;
}

template <int G>
__device__ void crop_body(const Params& P, int b, float* lds)
{
    using C = Cfg<G>;
    const int t = threadIdx.x;
    const int GG = C::GG, S = P.size;
    float* pd = lds;            // pred density
    float* td = pd + GG;        // target block sums
    float* bb = td + GG;        // normed pred density (Sinkhorn b)
    float* v0 = bb + GG;
    float* v1 = v0 + GG;
    float* ktu = v1 + GG;
    float* red = ktu + GG;
    float* kvred = red + C::SL * GG;
    float* misc = kvred + NWAVE * 64;
    float* fac = misc + 64;     // LDS factors (if they fit)

    const int p0 = P.offsets[b], n = P.offsets[b + 1] - p0;

    // 1. pred density, target block sums (losses/utils.py:4-9)
    for (int j = t; j < GG; j += NT) { pd[j] = P.pred_density[(size_t)b * GG + j]; td[j] = 0.f; }
    __syncthreads();
    if (P.target_is_reduced) {
        for (int j = t; j < GG; j += NT) td[j] = P.target_density[(size_t)b * GG + j];
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
    const float pc = block_sum([&] { float s = 0.f; for (int j = t; j < GG; j += NT) s += pd[j]; return s; }(), misc);
    const float tc = (float)n;

    // 2. cross-entropy over bins (dace_loss.py:42-55), grad = (softmax - onehot) / B
    const float invB = 1.0f / (float)P.B;
    float ce = 0.f;
    for (int j = t; j < GG; j += NT) {
        const float dv = td[j];
        int cls = 0;
        for (int k = 0; k < P.N; ++k)
            if (dv >= P.bins_lo[k] && dv <= P.bins_hi[k]) cls = k;
        const float* lg = P.pred_class + (size_t)b * P.N * GG + j;
        float mx = -INFINITY;
        for (int k = 0; k < P.N; ++k) mx = fmaxf(mx, lg[(size_t)k * GG]);
        float se = 0.f;
        for (int k = 0; k < P.N; ++k) se += expf(lg[(size_t)k * GG] - mx);
        const float lse = mx + logf(se);
        ce += lse - lg[(size_t)cls * GG];
        float* gc = P.grad_class + (size_t)b * P.N * GG + j;
        for (int k = 0; k < P.N; ++k)
            gc[(size_t)k * GG] = (expf(lg[(size_t)k * GG] - lse) - (k == cls ? 1.f : 0.f)) * invB;
    }
    ce = block_sum(ce, misc);

    float cnt_b = 0.f, tv_b = 0.f, ot_b = 0.f, wd_b = 0.f, err_last = -1.f;
    int iters = 0, rolled = 0;
    if (P.count_mode != EBC_COUNT_DMCOUNT) {
        // count_loss "mae" / "mse": per-pixel, summed over HW, mean over B (dace_loss.py:57-62)
        float s = 0.f;
        for (int j = t; j < GG; j += NT) {
            const float d = pd[j] - td[j];
            s += (P.count_mode == EBC_COUNT_MAE) ? fabsf(d) : d * d;
            const float g = (P.count_mode == EBC_COUNT_MAE) ? sgnf(d) : 2.f * d;
            P.grad_density[(size_t)b * GG + j] = P.w_count * g * invB;
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
        const float gcount = sgnf(pc - tc) * invB;
        // 4. Sinkhorn OT (dm_loss.py:49-77)
        if (n > 0) {
            const float* pts = P.points + 2 * (size_t)p0;
            if (n <= P.lds_cap) {
                float* Ey = fac; float* Ex = Ey + n * G; float* u0 = Ex + n * G; float* u1 = u0 + n;
                sinkhorn_crop<G>(n, P.size, P.norm_cood, P.reg, P.max_iter, P.stop_thr, P.eval_freq, pts, Ey, Ex, u0, u1,
                                 bb, v0, v1, ktu, red, kvred, misc, &iters, &rolled, &err_last);
            } else {
                float* base = P.ws_factors + (size_t)C::PER_POINT * p0;
                float* Ey = base; float* Ex = Ey + (size_t)n * G; float* u0 = Ex + (size_t)n * G; float* u1 = u0 + n;
                sinkhorn_crop<G>(n, P.size, P.norm_cood, P.reg, P.max_iter, P.stop_thr, P.eval_freq, pts, Ey, Ex, u0, u1,
                                 bb, v0, v1, ktu, red, kvred, misc, &iters, &rolled, &err_last);
            }
            // beta = reg * log(v + eps); gradient (dm_loss.py:65-74)
            float sb = 0.f;
            for (int j = t; j < GG; j += NT) {
                const float be = P.reg * logf(v0[j] + M_EPS);
                v1[j] = be;
                sb += pd[j] * be;
                if (P.beta_out) P.beta_out[(size_t)b * GG + j] = be;
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
            // Wasserstein distance sum(C * P) (dm_loss.py:77; reported, unused by training)
            const bool in_lds = n <= P.lds_cap;
            const float* Ey = in_lds ? fac : P.ws_factors + (size_t)C::PER_POINT * p0;
            const float* Ex = Ey + (size_t)n * G;
            const float* uu = Ex + (size_t)n * G;
            float w = 0.f;
            for (int i = t; i < n; i += NT) {
                const float x = pcoord(pts[2 * i], S, P.norm_cood), y = pcoord(pts[2 * i + 1], S, P.norm_cood);
                float acc = 0.f;
                for (int iy = 0; iy < G; ++iy) {
                    const float c = cood(iy, S, P.norm_cood);
                    const float yd = (-2.0f * (y * c) + y * y) + c * c;
                    float t1 = 0.f, t2 = 0.f;
                    for (int jx = 0; jx < G; ++jx) {
                        const float cx = cood(jx, S, P.norm_cood);
                        const float xd = (-2.0f * (x * cx) + x * x) + cx * cx;
                        const float kv = Ex[(size_t)i * G + jx] * v0[iy * G + jx];
                        t1 = fmaf(kv, 1.0f, t1);
                        t2 = fmaf(kv, xd, t2);
                    }
                    acc += Ey[(size_t)i * G + iy] * (yd * t1 + t2);
                }
                w += uu[i] * acc;
            }
            wd_b = block_sum(w, misc);
        } else {
            for (int j = t; j < GG; j += NT) v1[j] = 0.f;
            __syncthreads();
        }
        // 5. d loss / d pred_density = w_count * (w_ot * ot_grad + w_tv * tv_grad + count_grad)
        const float ktv = tc * invB;
        for (int j = t; j < GG; j += NT) {
            const float d = pd[j] * inv_pc - td[j] * inv_tc;
            const float gtv = ktv * (sgnf(d) * inv_pc - tvk * inv_pc * inv_pc);
            P.grad_density[(size_t)b * GG + j] = P.w_count * (P.w_ot * v1[j] + P.w_tv * gtv + gcount);
        }
    }
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
    const int b = P.order ? P.order[blockIdx.x] : (int)blockIdx.x;
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
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute((const void*)dace_loss_kernel<G>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX) != hipSuccess)
            return EBC_E_LAUNCH;
        attr = true;
    }
    hipLaunchKernelGGL(dace_loss_kernel<G>, dim3(P.B), dim3(NT), LDS_MAX, st, P);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

}  // namespace

extern "C" size_t ebc_dace_workspace_bytes(int B, int total_points, int size, int reduction)
{
    const int g = size / reduction;
    return sizeof(float) * ((size_t)(2 * g + 2) * (size_t)(total_points > 0 ? total_points : 1)) + 256;
}

extern "C" int ebc_dace_loss(const float* pred_class, const float* pred_density, const float* target_density,
                             int target_is_reduced, const float* points, const int* offsets, const int* order,
                             const float* bins_lo, const float* bins_hi, int B, int N, int size, int reduction,
                             int count_mode, int norm_cood, float weight_count_loss, float weight_ot, float weight_tv,
                             float reg, int max_iter, float stop_thr, int eval_freq,
                             float* grad_class, float* grad_density, float* losses, float* crop_stats,
                             float* beta_out, int* status, void* workspace, size_t workspace_bytes,
                             ebc_stream_t stream)
{
    if (B <= 0 || N <= 0 || reduction != 8 || size % reduction != 0 || eval_freq <= 0 || reg <= 0.f)
        return EBC_E_ARG;
    if (!pred_class || !pred_density || !target_density || !offsets || !bins_lo || !bins_hi ||
        !grad_class || !grad_density || !losses || !crop_stats)
        return EBC_E_ARG;
    if (!target_is_reduced && (size % 4) != 0) return EBC_E_ARG;
    const int g = size / reduction;
    hipStream_t st = (hipStream_t)stream;
    Params P{};
    P.pred_class = pred_class; P.pred_density = pred_density; P.target_density = target_density;
    P.target_is_reduced = target_is_reduced; P.points = points; P.offsets = offsets; P.order = order;
    P.bins_lo = bins_lo; P.bins_hi = bins_hi; P.B = B; P.N = N; P.size = size; P.red = reduction;
    P.count_mode = count_mode; P.norm_cood = norm_cood; P.w_count = weight_count_loss; P.w_ot = weight_ot; P.w_tv = weight_tv;
    P.reg = reg; P.stop_thr = stop_thr; P.max_iter = max_iter; P.eval_freq = eval_freq;
    P.grad_class = grad_class; P.grad_density = grad_density; P.crop_stats = crop_stats;
    P.beta_out = beta_out; P.status = status; P.ws_factors = (float*)workspace;
    int rc;
    if (g == 28) rc = launch<28>(P, st);
    else if (g == 56) rc = launch<56>(P, st);
    else return EBC_E_UNSUPPORTED;
    if (rc) return rc;
    hipLaunchKernelGGL(dace_finalize_kernel, dim3(1), dim3(256), 0, st, crop_stats, B, count_mode,
                       weight_count_loss, weight_ot, weight_tv, losses);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

extern "C" int ebc_version(void) { return 1; }
