// Adam with the GradScaler's dynamic loss scaling folded in: the reference's optimizer step
// (utils/train_utils.py:80-85 Adam(lr, weight_decay) + trainer.py:123 GradScaler, driven as train.py:53-57
// scale(loss).backward(); step(optimizer); update()).
//
// Two launches per step over every trainable tensor (any count: groups of MAXT tensors per launch):
//   amp_check_kernel   found_inf |= any non-finite gradient     (GradScaler._unscale_grads_ / check_inf)
//   adam_kernel        if !found_inf: unscale, L2 weight decay, moments, bias-corrected update, unscaled grad
//                      written back (torch's fused Adam with grad_scale / found_inf); workgroup 0 of the last group
//                      also writes the NEXT scaler state (GradScaler.update: backoff / growth tracker / growth)
// The state is ping-ponged: the optimizer's step count float step[2] and the scaler's float sc[2][3] = {scale,
// growth_tracker, found_inf}; a step reads entry [parity] and writes entry [1 - parity], so nothing reads a word
// another workgroup of the same launch writes and there is no separate update launch.
//
// Arithmetic follows torch's fused Adam (ADAM_MODE::ORIGINAL) operation for operation, including its double-
// precision hyper-parameter products (beta * m + (1 - beta) * g with beta a double) and the bias corrections
// computed in double from the step count: against torch's fused Adam the scale sequence and unscaled gradients are the
// same bits and parameters / moments agree to f32 rounding (fp-contraction choices may differ; tests/test_gpu_optim.py).
#include <cmath>

#include "ebc_common.h"

namespace {

constexpr int MAXT = 32;          // tensors per launch (kernel-argument pack)
constexpr int CHUNK = 4096;       // elements per workgroup: 256 threads x 4 float4

struct AdamPack {
    float* p[MAXT];
    float* g[MAXT];
    float* m[MAXT];
    float* v[MAXT];
    long numel[MAXT];
    int blk0[MAXT + 1];           // first workgroup of tensor t; blk0[n] = the launch's workgroups
    int n;
    unsigned vec;                 // bit t: the four operands of tensor t are 16-B aligned
};

__device__ __forceinline__ int pack_tensor(const AdamPack& k, int b) {
    int t = 0;
    while (t + 1 < k.n && k.blk0[t + 1] <= b) ++t;
    return t;
}

__global__ __launch_bounds__(256) void amp_check_kernel(AdamPack k, float* found)
{
    const int t = pack_tensor(k, blockIdx.x);
    const long base = (long)(blockIdx.x - k.blk0[t]) * CHUNK;
    const long n = k.numel[t] - base < CHUNK ? k.numel[t] - base : CHUNK;
    const float* g = k.g[t] + base;
    bool bad = false;
    if (((k.vec >> t) & 1) && n == CHUNK) {
        // a whole chunk: the thread's four 16-B pieces in flight together (r05: the strided loop issued one at a time,
        // 17.5 us a step for 45 MB)
        float4 x[CHUNK / 1024];
#pragma unroll
        for (int q = 0; q < CHUNK / 1024; ++q) x[q] = *reinterpret_cast<const float4*>(g + 4 * (threadIdx.x + 256 * q));
#pragma unroll
        for (int q = 0; q < CHUNK / 1024; ++q)
            bad |= !(isfinite(x[q].x) && isfinite(x[q].y) && isfinite(x[q].z) && isfinite(x[q].w));
    } else if ((k.vec >> t) & 1) {
        const long n4 = n & ~3L;
        for (long i = 4 * threadIdx.x; i < n4; i += 4 * 256) {
            const float4 x = *reinterpret_cast<const float4*>(g + i);
            bad |= !(isfinite(x.x) && isfinite(x.y) && isfinite(x.z) && isfinite(x.w));
        }
        for (long i = n4 + threadIdx.x; i < n; i += 256) bad |= !isfinite(g[i]);
    } else {
        for (long i = threadIdx.x; i < n; i += 256) bad |= !isfinite(g[i]);
    }
    // one store per wave that saw a non-finite value (every writer stores the same value; no workgroup barrier)
    if (__any(bad) && (threadIdx.x & 63) == 0) *found = 1.0f;
}

struct AdamHyper {
    double lr, beta1, beta2, eps, wd, growth, backoff;
    int interval, amp, write_grad, last_group;
};

// torch fused Adam's adam_math for one element (opmath float, hyper-parameters double)
__device__ __forceinline__ void adam_elem(float& param, float& grad, float& exp_avg, float& exp_avg_sq, const AdamHyper& h,
                                          float scale, float step_size, float bc2_sqrt)
{
    float gr = grad;
    if (h.amp) {
        gr = (float)((double)gr / (double)scale);
        grad = gr;
    }
    if (h.wd != 0.0) gr = (float)((double)gr + (double)param * h.wd);
    exp_avg = (float)(h.beta1 * (double)exp_avg + (1.0 - h.beta1) * (double)gr);
    exp_avg_sq = (float)(h.beta2 * (double)exp_avg_sq + (1.0 - h.beta2) * (double)gr * (double)gr);
    const float denom = (float)((double)(sqrtf(exp_avg_sq) / bc2_sqrt) + h.eps);
    param -= step_size * exp_avg / denom;
}

__global__ __launch_bounds__(256) void adam_kernel(AdamPack k, const float* __restrict__ stp, float* __restrict__ stp_next,
                                                   const float* __restrict__ sc, float* __restrict__ sc_next, AdamHyper h)
{
    const float step = *stp;
    const float scale = h.amp ? sc[0] : 1.0f, tracker = h.amp ? sc[1] : 0.0f;
    const bool found = h.amp && sc[2] != 0.0f;
    if (h.last_group && blockIdx.x == 0 && threadIdx.x == 0) {
        // next state (torch._amp_update_scale_; the step count advances only on an applied step)
        if (h.amp) {
            float ns = scale, nt = tracker;
            if (found) {
                ns = (float)((double)scale * h.backoff);
                nt = 0.0f;
            } else {
                const float succ = tracker + 1.0f;
                if (succ == (float)h.interval) {
                    const float g = (float)((double)scale * h.growth);
                    if (isfinite(g)) ns = g;
                    nt = 0.0f;
                } else {
                    nt = succ;
                }
            }
            sc_next[0] = ns;
            sc_next[1] = nt;
            sc_next[2] = 0.0f;
        }
        *stp_next = found ? step : step + 1.0f;
    }
    if (found) return;
    // bias corrections of the step this update counts (torch adds 1 to the step before the kernel)
    const double sd = (double)(step + 1.0f);
    const float bc1 = (float)(1.0 - pow(h.beta1, sd));
    const float bc2_sqrt = (float)sqrt(1.0 - pow(h.beta2, sd));
    const float step_size = (float)(h.lr / (double)bc1);

    const int t = pack_tensor(k, blockIdx.x);
    const long base = (long)(blockIdx.x - k.blk0[t]) * CHUNK;
    const long n = k.numel[t] - base < CHUNK ? k.numel[t] - base : CHUNK;
    float* P = k.p[t] + base;
    float* G = k.g[t] + base;
    float* M = k.m[t] + base;
    float* V = k.v[t] + base;
    long i0 = 0;
    if ((k.vec >> t) & 1) {
        const long n4 = n & ~3L;
        for (long i = 4 * threadIdx.x; i < n4; i += 4 * 256) {
            float4 p = *reinterpret_cast<const float4*>(P + i), g = *reinterpret_cast<const float4*>(G + i);
            float4 m = *reinterpret_cast<const float4*>(M + i), v = *reinterpret_cast<const float4*>(V + i);
            adam_elem(p.x, g.x, m.x, v.x, h, scale, step_size, bc2_sqrt);
            adam_elem(p.y, g.y, m.y, v.y, h, scale, step_size, bc2_sqrt);
            adam_elem(p.z, g.z, m.z, v.z, h, scale, step_size, bc2_sqrt);
            adam_elem(p.w, g.w, m.w, v.w, h, scale, step_size, bc2_sqrt);
            *reinterpret_cast<float4*>(P + i) = p;
            *reinterpret_cast<float4*>(M + i) = m;
            *reinterpret_cast<float4*>(V + i) = v;
            if (h.amp && h.write_grad) *reinterpret_cast<float4*>(G + i) = g;
        }
        i0 = n4;
    }
    for (long i = i0 + threadIdx.x; i < n; i += 256) {
        float p = P[i], g = G[i], m = M[i], v = V[i];
        adam_elem(p, g, m, v, h, scale, step_size, bc2_sqrt);
        P[i] = p;
        M[i] = m;
        V[i] = v;
        if (h.amp && h.write_grad) G[i] = g;
    }
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// groups of MAXT tensors -> kernel-argument packs
int make_pack(const EbcAdamTensor* ts, int n0, int n1, AdamPack& k)
{
    k.n = n1 - n0;
    k.vec = 0;
    long blocks = 0;
    for (int i = 0; i < k.n; ++i) {
        const EbcAdamTensor& e = ts[n0 + i];
        if (!e.param || !e.grad || !e.exp_avg || !e.exp_avg_sq || e.numel <= 0) return EBC_E_ARG;
        k.p[i] = e.param; k.g[i] = e.grad; k.m[i] = e.exp_avg; k.v[i] = e.exp_avg_sq; k.numel[i] = e.numel;
        if (aligned16(e.param) && aligned16(e.grad) && aligned16(e.exp_avg) && aligned16(e.exp_avg_sq)) k.vec |= 1u << i;
        k.blk0[i] = (int)blocks;
        blocks += (e.numel + CHUNK - 1) / CHUNK;
        if (blocks > (1L << 30)) return EBC_E_UNSUPPORTED;
    }
    k.blk0[k.n] = (int)blocks;
    return EBC_OK;
}

}  // namespace

namespace {
int amp_check_all(const EbcAdamTensor* tensors, int n, float* found, hipStream_t st)
{
    AdamPack k;
    for (int g0 = 0; g0 < n; g0 += MAXT) {
        const int rc = make_pack(tensors, g0, g0 + MAXT < n ? g0 + MAXT : n, k);
        if (rc) return rc;
        hipLaunchKernelGGL(amp_check_kernel, dim3(k.blk0[k.n]), dim3(256), 0, st, k, found);
        EBC_CHECK_LAUNCH();
    }
    return EBC_OK;
}
int adam_update_all(const EbcAdamTensor* tensors, int n, float* step, int step_parity, float* scaler, int scaler_parity,
                    double lr, double beta1, double beta2, double eps, double weight_decay, double growth_factor,
                    double backoff_factor, int growth_interval, int write_unscaled_grad, hipStream_t st)
{
    const bool amp = scaler != nullptr;
    float* cur = amp ? scaler + 3 * scaler_parity : nullptr;
    float* nxt = amp ? scaler + 3 * (1 - scaler_parity) : nullptr;
    AdamHyper h{lr, beta1, beta2, eps, weight_decay, growth_factor, backoff_factor, growth_interval, amp ? 1 : 0,
                write_unscaled_grad ? 1 : 0, 0};
    AdamPack k;
    for (int g0 = 0; g0 < n; g0 += MAXT) {
        const int g1 = g0 + MAXT < n ? g0 + MAXT : n;
        const int rc = make_pack(tensors, g0, g1, k);
        if (rc) return rc;
        h.last_group = g1 == n;
        hipLaunchKernelGGL(adam_kernel, dim3(k.blk0[k.n]), dim3(256), 0, st, k, (const float*)(step + step_parity),
                           step + (1 - step_parity), (const float*)cur, nxt, h);
        EBC_CHECK_LAUNCH();
    }
    return EBC_OK;
}
}  // namespace

extern "C" int ebc_adam_step(const EbcAdamTensor* tensors, int n, float* step, int step_parity, float* scaler,
                             int scaler_parity, double lr, double beta1, double beta2, double eps, double weight_decay,
                             double growth_factor, double backoff_factor, int growth_interval, int write_unscaled_grad,
                             ebc_stream_t stream)
{
    if (!tensors || n <= 0 || !step || (step_parity & ~1) || (scaler_parity & ~1) || growth_interval <= 0) return EBC_E_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (scaler) {
        const int rc = amp_check_all(tensors, n, scaler + 3 * scaler_parity + 2, st);
        if (rc) return rc;
    }
    return adam_update_all(tensors, n, step, step_parity, scaler, scaler_parity, lr, beta1, beta2, eps, weight_decay,
                           growth_factor, backoff_factor, growth_interval, write_unscaled_grad, st);
}

extern "C" int ebc_amp_check(const EbcAdamTensor* tensors, int n, float* scaler, int scaler_parity, ebc_stream_t stream)
{
    if (!tensors || n <= 0 || !scaler || (scaler_parity & ~1)) return EBC_E_ARG;
    return amp_check_all(tensors, n, scaler + 3 * scaler_parity + 2, (hipStream_t)stream);
}

extern "C" int ebc_adam_update(const EbcAdamTensor* tensors, int n, float* step, int step_parity, float* scaler,
                               int scaler_parity, double lr, double beta1, double beta2, double eps, double weight_decay,
                               double growth_factor, double backoff_factor, int growth_interval, int write_unscaled_grad,
                               ebc_stream_t stream)
{
    if (!tensors || n <= 0 || !step || (step_parity & ~1) || (scaler_parity & ~1) || growth_interval <= 0) return EBC_E_ARG;
    return adam_update_all(tensors, n, step, step_parity, scaler, scaler_parity, lr, beta1, beta2, eps, weight_decay,
                           growth_factor, backoff_factor, growth_interval, write_unscaled_grad, (hipStream_t)stream);
}
