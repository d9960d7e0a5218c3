// General dense Sinkhorn-Knopp (one problem, one 1024-thread workgroup, every iteration on device).
//
// Reference: sinkhorn(a, b, C, reg, maxIter, stopThr, verbose, log, eval_freq, print_freq)
//            losses/bregman_pytorch.py:11-144
//
// The DMCount hot path never comes here: its cost matrix is separable and ebc_dace_loss solves it
// in factored form (dace_loss.hip).  This entry point is the drop-in for a caller of `sinkhorn()`
// itself, with an arbitrary cost matrix C [na, nb]:
//   K = exp(C / -reg) materialised once (LDS when it fits, else the workspace: 2 K passes per
//   iteration stream it from L2), u / v double-buffered in LDS;
//   per iteration KTu = u^T K (one column per thread), v = b / (KTu + 1e-16), Kv = K v (one row per
//   wave, DPP reduction), u = a / (Kv + 1e-16); any NaN/Inf in the new (u, v) restores the previous
//   pair and stops (:111-115); with `log`, err = ||b - (u^T K) * v||^2 every eval_freq iterations
//   (:117-126; that K^T u is reused by the next iteration's v, the same u gives the same product);
//   stop when err <= stopThr or it > maxIter.  Without `log` the reference never updates err, so all
//   maxIter iterations run; this kernel keeps that.
// Outputs: u, v, alpha = reg log(u + 1e-16), beta = reg log(v + 1e-16), P = u_i K_ij v_j, the err list,
// and info = {iterations (negative: rolled back at that iteration), number of err entries}.
// f32 throughout, no fast-math: the 1e-16 epsilons act on denormal-range sums.
#include "ebc_common.h"

using namespace ebc;

namespace {

constexpr int NT = 1024, NW = NT / 64;
constexpr float M_EPS = 1e-16f;           // bregman_pytorch.py:8
constexpr int LDS_MAX = 160 * 1024;

struct SkArgs {
    const float* a; const float* b; const float* C;
    int na, nb;
    float reg, stop_thr;
    int max_iter, eval_freq, log;
    float* P; float* u_out; float* v_out; float* alpha; float* beta; float* err; int* info;
    float* kws;        // K in global memory (when it does not fit LDS)
};

__device__ __forceinline__ int block_any(int v, int* scratch) {
    v = wave_or(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) scratch[threadIdx.x >> 6] = v;
    __syncthreads();
    int r = 0;
    for (int i = 0; i < NW; ++i) r |= scratch[i];
    return r;
}

template <bool KLDS>
__global__ __launch_bounds__(NT) void sinkhorn_dense_kernel(SkArgs p)
{
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int na = p.na, nb = p.nb;
    float* u0 = sm;
    float* u1 = u0 + na;
    float* v0 = u1 + na;
    float* v1 = v0 + nb;
    float* ktu = v1 + nb;                    // K^T u kept from the err pass
    float* misc = ktu + nb;                  // [64]
    float* K = KLDS ? misc + 64 : p.kws;
    // K = exp(C / -reg): torch.div(C, -reg) then torch.exp (:89-91)
    for (long e = t; e < (long)na * nb; e += NT) K[e] = expf(p.C[e] / -p.reg);
    for (int i = t; i < na; i += NT) u0[i] = 1.0f / (float)na;      // ones / na (:86-87)
    for (int j = t; j < nb; j += NT) v0[j] = 1.0f / (float)nb;
    __syncthreads();
    float* u = u0; float* un = u1;
    float* v = v0; float* vn = v1;
    int it = 1, rolled = 0, have_ktu = 0, nerr = 0;
    float err = 1.0f;
    int* flag = reinterpret_cast<int*>(misc) + 32;
    auto ktu_col = [&](const float* uu, int j) {
        float s = 0.f;
        for (int i = 0; i < na; ++i) s = fmaf(uu[i], K[(long)i * nb + j], s);
        return s;
    };
    while (err > p.stop_thr && it <= p.max_iter) {           // :102
        int bad = 0;
        // v = b / (u^T K + eps)
        for (int j = t; j < nb; j += NT) {
            const float s = have_ktu ? ktu[j] : ktu_col(u, j);
            const float val = p.b[j] / (s + M_EPS);
            vn[j] = val;
            bad |= !isfinite(val);
        }
        have_ktu = 0;
        __syncthreads();
        // u = a / (K v + eps): one row per wave
        for (int i = w; i < na; i += NW) {
            const float* kr = K + (long)i * nb;
            float s = 0.f;
            for (int j = lane; j < nb; j += 64) s = fmaf(kr[j], vn[j], s);
            s = wave_sum(s);
            const float val = p.a[i] / (s + M_EPS);
            if (lane == 0) un[i] = val;
            bad |= !isfinite(val);
        }
        if (block_any(bad, flag)) { rolled = 1; break; }     // restore (upre, vpre) and stop (:111-115)
        { float* tu = u; u = un; un = tu; float* tv = v; v = vn; vn = tv; }
        if (p.log && it % p.eval_freq == 0) {                 // :117-126
            float e = 0.f;
            for (int j = t; j < nb; j += NT) {
                const float s = ktu_col(u, j);
                ktu[j] = s;
                const float d = p.b[j] - s * v[j];
                e = fmaf(d, d, e);
            }
            err = block_sum(e, misc);
            if (t == 0 && p.err) p.err[nerr] = err;
            ++nerr;
            have_ktu = 1;
        }
        ++it;
    }
    __syncthreads();
    for (int i = t; i < na; i += NT) {
        if (p.u_out) p.u_out[i] = u[i];
        if (p.alpha) p.alpha[i] = p.reg * logf(u[i] + M_EPS);   // :133-137
    }
    for (int j = t; j < nb; j += NT) {
        if (p.v_out) p.v_out[j] = v[j];
        if (p.beta) p.beta[j] = p.reg * logf(v[j] + M_EPS);
    }
    if (p.P) {                                                 // P = u K v (:140)
        for (long e = t; e < (long)na * nb; e += NT) {
            const int i = (int)(e / nb), j = (int)(e - (long)i * nb);
            p.P[e] = u[i] * K[e] * v[j];
        }
    }
    if (t == 0) {
        const int iters = rolled ? it : it - 1;
        p.info[0] = rolled ? -iters : iters;
        p.info[1] = nerr;
    }
}

size_t uv_bytes(int na, int nb) { return sizeof(float) * ((size_t)2 * na + 2 * (size_t)nb + nb + 64); }
bool k_in_lds(int na, int nb) { return uv_bytes(na, nb) + sizeof(float) * (size_t)na * nb <= (size_t)LDS_MAX; }

}  // namespace

extern "C" size_t ebc_sinkhorn_workspace_bytes(int na, int nb)
{
    if (na <= 0 || nb <= 0) return 0;
    return k_in_lds(na, nb) ? 0 : sizeof(float) * (size_t)na * nb;
}

extern "C" int ebc_sinkhorn(const float* a, const float* b, const float* C, int na, int nb, float reg, int max_iter,
                            float stop_thr, int eval_freq, int log, float* P, float* u, float* v, float* alpha,
                            float* beta, float* err, int* info, void* workspace, size_t workspace_bytes,
                            ebc_stream_t stream)
{
    if (!a || !b || !C || !info || na <= 0 || nb <= 0 || !(reg > 0.f) || eval_freq <= 0) return EBC_E_ARG;
    if (uv_bytes(na, nb) > (size_t)LDS_MAX) return EBC_E_UNSUPPORTED;            // u, v must stay in LDS
    const bool klds = k_in_lds(na, nb);
    if (!klds && (!workspace || workspace_bytes < sizeof(float) * (size_t)na * nb)) return EBC_E_ARG;
    SkArgs p{a, b, C, na, nb, reg, stop_thr, max_iter, eval_freq, log, P, u, v, alpha, beta, err, info,
             (float*)workspace};
    const hipStream_t st = (hipStream_t)stream;
    if (klds) {
        if (!ensure_lds<sinkhorn_dense_kernel<true>>(LDS_MAX, st)) return EBC_E_LAUNCH;
        const size_t lds = uv_bytes(na, nb) + sizeof(float) * (size_t)na * nb;
        hipLaunchKernelGGL(sinkhorn_dense_kernel<true>, dim3(1), dim3(NT), lds, st, p);
    } else {
        if (!ensure_lds<sinkhorn_dense_kernel<false>>(LDS_MAX, st)) return EBC_E_LAUNCH;
        hipLaunchKernelGGL(sinkhorn_dense_kernel<false>, dim3(1), dim3(NT), uv_bytes(na, nb), st, p);
    }
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}
