// Attention lab (experiment harness, not product code): attention.hip's forward kernel by waves per workgroup
// (queries per workgroup = 16 x waves x QT) and the one-workgroup backward at the ViT-B/16 + VPT(32) shape (L 229,
// 12 heads), B crops (argv[3], 16 or 32), interleaved rounds in one process; every forward variant's output compared
// bitwise with the 16-wave one.
//   build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/lab/attn_lab.hip -o tools/lab/bin/attn_lab
//   run:   tools/lab/bin/attn_lab ROUNDS REPS B
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
    const int B = argc > 3 ? atoi(argv[3]) : 16, L = 229, H = 12, D = H * 64;
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
        {"fwd NW8 QT2", [&](void* o, float* l) { return attn_fwd_nw<EF16, 8, L_VPT32, 2>(qkv, o, l, B, L, H, 0); }},
        {"fwd NW4 QT2", [&](void* o, float* l) { return attn_fwd_nw<EF16, 4, L_VPT32, 2>(qkv, o, l, B, L, H, 0); }},
    };
    std::vector<V> bwd = {
        {"bwd one", [&](void*, float*) { return attn_bwd_one<EF16, L_VPT32>(qkv, dout, out, lse, dqkv, B, L, H, 0, 0, nullptr); }},
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
                printf("r%d B%d %-16s %7.2f us\n", r, B, v.name.c_str(), ms / reps * 1e3);
            }
    }
    return 0;
}
