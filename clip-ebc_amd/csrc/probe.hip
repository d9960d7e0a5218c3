// In-step kernel timing for the benchmark (host side only; no device code beyond a named no-op).
//
// ebc_probe_begin arms recording: every launch of the instrumented kernels (GEMM / implicit-GEMM conv,
// the DACE/Sinkhorn loss, attention, LayerNorm) is bracketed by two HIP events recorded on the stream
// it is launched on, so the durations are the kernels' own, measured inside a real training step.
// ebc_probe_end synchronises on the last event and returns one record per launch.  The events come
// from a pool created once (hipEventCreate is not free), so an armed step adds only the event records.
// ebc_marker launches a named empty kernel: profile readers (tools/kstats.py --window) keep only the
// kernels between two markers, i.e. exactly the timed steps.
#include <vector>

#include "ebc_common.h"
#include "kernels.h"

namespace ebc {
namespace {
struct Rec { EbcProbeRecord r; hipEvent_t e0, e1; };
std::vector<Rec> g_recs;
std::vector<hipEvent_t> g_pool;
bool g_on = false;
}  // namespace

bool probe_on() { return g_on; }

int probe_start(int kind, int epi, int bm, int bn, int mode, int m, int n, int k, hipStream_t st)
{
    if (!g_on || 2 * (g_recs.size() + 1) > g_pool.size()) return -1;
    Rec rec{};
    rec.r = EbcProbeRecord{kind, epi, bm, bn, mode, m, n, k, 0.f};
    rec.e0 = g_pool[2 * g_recs.size()];
    rec.e1 = g_pool[2 * g_recs.size() + 1];
    if (hipEventRecord(rec.e0, st) != hipSuccess) return -1;
    g_recs.push_back(rec);
    return (int)g_recs.size() - 1;
}

void probe_stop(int idx, hipStream_t st)
{
    if (idx >= 0 && idx < (int)g_recs.size()) (void)hipEventRecord(g_recs[idx].e1, st);
}
}  // namespace ebc

namespace {
__global__ void ebc_marker_kernel(int) {}
}

extern "C" int ebc_probe_begin(int capacity)
{
    using namespace ebc;
    if (capacity <= 0) return EBC_E_ARG;
    while ((int)g_pool.size() < 2 * capacity) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return EBC_E_LAUNCH;
        g_pool.push_back(e);
    }
    g_recs.clear();
    g_on = true;
    return EBC_OK;
}

extern "C" int ebc_probe_end(EbcProbeRecord* out, int capacity)
{
    using namespace ebc;
    g_on = false;
    int n = 0;
    for (Rec& rec : g_recs) {
        if (hipEventSynchronize(rec.e1) != hipSuccess) return EBC_E_LAUNCH;
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, rec.e0, rec.e1) != hipSuccess) return EBC_E_LAUNCH;
        rec.r.ms = ms;
        if (out && n < capacity) out[n] = rec.r;
        ++n;
    }
    g_recs.clear();
    return n;
}

extern "C" int ebc_marker(int id, ebc_stream_t stream)
{
    hipLaunchKernelGGL(ebc_marker_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, id);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}
