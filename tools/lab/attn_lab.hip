// Attention lab (experiment harness, not product code): attention.hip's forward / fused backward kernels at the
// 16-crop ViT-B/16 + VPT(32) shape (B 16, L 229, 12 heads) by waves per workgroup (queries per workgroup = 16 x
// waves), interleaved rounds in one process; every variant's output compared bitwise with the 16-wave forward.
//   build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/lab/attn_lab.hip -o tools/lab/bin/attn_lab
#include "../../clip-ebc_amd/csrc/attention.hip"

#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

namespace ebc {
bool probe_on() { return false; }
int probe_start(int, int, int, int, int, int, int, int, hipStream_t) { return -1; }
void probe_stop(int, hipStream_t) {}
}  // namespace ebc

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void fill_f16(_Float16* p, size_t n, unsigned seed, float scale)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
        p[i] = (_Float16)(((h & 0xffff) / 32768.0f - 1.0f) * scale);
    }
}

int main(int argc, char** argv)
{
    const int rounds = argc > 1 ? atoi(argv[1]) : 3, reps = argc > 2 ? atoi(argv[2]) : 50;
    const int B = 16, L = 229, H = 12, D = H * 64;
    _Float16 *qkv, *out, *out2, *dout, *dqkv;
    float *lse, *lse2;
    CK(hipMalloc(&qkv, (size_t)B * L * 3 * D * 2));
    CK(hipMalloc(&out, (size_t)B * L * D * 2));
    CK(hipMalloc(&out2, (size_t)B * L * D * 2));
    CK(hipMalloc(&dout, (size_t)B * L * D * 2));
    CK(hipMalloc(&dqkv, (size_t)B * L * 3 * D * 2));
    CK(hipMalloc(&lse, (size_t)B * H * L * 4));
    CK(hipMalloc(&lse2, (size_t)B * H * L * 4));
    hipLaunchKernelGGL(fill_f16, dim3(512), dim3(256), 0, 0, qkv, (size_t)B * L * 3 * D, 1u, 1.0f);
    hipLaunchKernelGGL(fill_f16, dim3(512), dim3(256), 0, 0, dout, (size_t)B * L * D, 2u, 0.1f);
    CK(hipDeviceSynchronize());
    struct V { std::string name; std::function<int(void*, float*)> fn; };
    std::vector<V> fwd = {
        {"fwd NW16", [&](void* o, float* l) { return attn_fwd_nw<EF16, 16, L_VPT32>(qkv, o, l, B, L, H, 0); }},
        {"fwd NW8", [&](void* o, float* l) { return attn_fwd_nw<EF16, 8, L_VPT32>(qkv, o, l, B, L, H, 0); }},
        {"fwd NW4", [&](void* o, float* l) { return attn_fwd_nw<EF16, 4, L_VPT32>(qkv, o, l, B, L, H, 0); }},
        {"fwd NW8 QT2", [&](void* o, float* l) { return attn_fwd_nw<EF16, 8, L_VPT32, 2>(qkv, o, l, B, L, H, 0); }},
        {"fwd NW4 QT2", [&](void* o, float* l) { return attn_fwd_nw<EF16, 4, L_VPT32, 2>(qkv, o, l, B, L, H, 0); }},
        {"fwd NW2 QT2", [&](void* o, float* l) { return attn_fwd_nw<EF16, 2, L_VPT32, 2>(qkv, o, l, B, L, H, 0); }},
        {"fwd NW4 QT4", [&](void* o, float* l) { return attn_fwd_nw<EF16, 4, L_VPT32, 4>(qkv, o, l, B, L, H, 0); }},
    };
    std::vector<V> bwd = {
        {"bwd fused NW8", [&](void*, float*) { return attn_bwd_fused_nw<EF16, 8, L_VPT32>(qkv, dout, out, lse, dqkv, B, L, H, 0); }},
        {"bwd fused NW4", [&](void*, float*) { return attn_bwd_fused_nw<EF16, 4, L_VPT32>(qkv, dout, out, lse, dqkv, B, L, H, 0); }},
        {"bwd fused NW16", [&](void*, float*) { return attn_bwd_fused_nw<EF16, 16, L_VPT32>(qkv, dout, out, lse, dqkv, B, L, H, 0); }},
    };
    std::vector<unsigned short> ref((size_t)B * L * D), got((size_t)B * L * D);
    for (size_t v = 0; v < fwd.size(); ++v) {
        if (fwd[v].fn(v ? out2 : out, v ? lse2 : lse)) { printf("launch error %s\n", fwd[v].name.c_str()); return 1; }
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(v ? got.data() : ref.data(), v ? out2 : out, ref.size() * 2, hipMemcpyDeviceToHost));
        if (v) {
            size_t bad = 0;
            for (size_t i = 0; i < ref.size(); ++i) bad += ref[i] != got[i];
            printf("%s vs NW16: %zu of %zu elements differ\n", fwd[v].name.c_str(), bad, ref.size());
        }
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; ++r) {
        for (auto* set : {&fwd, &bwd})
            for (auto& v : *set) {
                v.fn(out2, lse2);
                CK(hipEventRecord(e0));
                for (int i = 0; i < reps; ++i) v.fn(out2, lse2);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                printf("r%d %-16s %7.2f us\n", r, v.name.c_str(), ms / reps * 1e3);
            }
    }
    // ---- operand residency: qkv (and dout for the backward) rewritten by a producer kernel right before each launch
    // (as the QKV GEMM writes it in the step), vs after a 512 MB scrub (HBM), vs back to back (above)
    {
        char* scrub2;
        CK(hipMalloc(&scrub2, (size_t)512 << 20));
        for (int r = 0; r < rounds; ++r)
            for (int mode = 0; mode < 2; ++mode)
                for (int which = 0; which < 2; ++which) {
                    float tot = 0;
                    const int n = reps / 5 + 2;
                    for (int i = 0; i < n; ++i) {
                        if (mode == 0) {
                            hipLaunchKernelGGL(fill_f16, dim3(2048), dim3(256), 0, 0, qkv, (size_t)B * L * 3 * D, 1u, 1.0f);
                            hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, dout, (size_t)B * L * D, 2u, 0.1f);
                        } else {
                            CK(hipMemsetAsync(scrub2, i & 0xff, (size_t)512 << 20, 0));
                        }
                        CK(hipEventRecord(e0));
                        const int rc = which == 0 ? attn_fwd_nw<EF16, 16, L_VPT32>(qkv, out2, lse2, B, L, H, 0)
                                                  : attn_bwd_fused_nw<EF16, 8, L_VPT32>(qkv, dout, out, lse, dqkv, B, L, H, 0);
                        if (rc) { printf("launch error\n"); return 1; }
                        CK(hipEventRecord(e1));
                        CK(hipEventSynchronize(e1));
                        float ms = 0;
                        CK(hipEventElapsedTime(&ms, e0, e1));
                        if (i >= 2) tot += ms;
                    }
                    printf("r%d %-14s %s %7.2f us\n", r, mode == 0 ? "after producer" : "after scrub", which == 0 ? "fwd NW16     " : "bwd fused NW8",
                           tot / (n - 2) * 1e3);
                }
    }
    // ---- weight-touch cost: the forward with its in-kernel touch of T MB of cold buffers (a 512 MB scrub write runs
    // before every launch, so the touched lines come from HBM as the next layer's weights do in the step)
    {
        const size_t WB = (size_t)14200000 & ~(size_t)127, SB = (size_t)512 << 20;
        char* wbuf;
        char* scrub;
        CK(hipMalloc(&wbuf, WB));
        CK(hipMalloc(&scrub, SB));
        CK(hipMemset(wbuf, 1, WB));
        const size_t sizes[] = {0, WB / 3 & ~(size_t)127, 2 * (WB / 3) & ~(size_t)127, WB};
        for (int r = 0; r < rounds; ++r)
            for (size_t sz : sizes)
                for (int qt = 1; qt <= 2; ++qt) {
                    float tot = 0;
                    for (int i = 0; i < reps / 5 + 2; ++i) {
                        CK(hipMemsetAsync(scrub, i & 0xff, SB, 0));
                        TouchList t{};
                        if (sz) t.add(wbuf, sz);
                        CK(hipEventRecord(e0));
                        const int rc = qt == 1 ? attn_fwd_nw<EF16, 16, L_VPT32>(qkv, out2, lse2, B, L, H, 0, &t)
                                               : attn_fwd_nw<EF16, 8, L_VPT32, 2>(qkv, out2, lse2, B, L, H, 0, &t);
                        if (rc) { printf("launch error\n"); return 1; }
                        CK(hipEventRecord(e1));
                        CK(hipEventSynchronize(e1));
                        float ms = 0;
                        CK(hipEventElapsedTime(&ms, e0, e1));
                        if (i >= 2) tot += ms;
                    }
                    printf("r%d touch %5.1f MB cold  fwd %s %7.2f us\n", r, sz / 1e6, qt == 1 ? "NW16    " : "NW8 QT2 ",
                           tot / (reps / 5) * 1e3);
                }
    }
    return 0;
}
