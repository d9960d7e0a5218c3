// Device side of the weight touch (kernels.h TouchList), shared by the attention kernels and ln_post's backward.
#pragma once
#include <hip/hip_runtime.h>
#include "kernels.h"

namespace ebc {
// Weight touch (kernels.h TouchList): once its operands are staged (no later global load in the wave to wait behind
// them), every wave of the launch reads one dword of each of its share of the listed buffers' 128-B lines (64 lines
// per instruction), so the weights of the GEMMs that follow are on-die when they start.  Measured on the c_proj
// product (tools/lab/gemm_lab.hip "mlp-seq"): 37.5 us with its weight in HBM, 28.4 us read onto the die beforehand;
// a separate touch kernel on a side stream instead cost more in the kernels it ran beside (r03 same-box A/B).
// The lines of all listed buffers are dealt out as one sequence over every lane of the grid, so no lane loads a
// second line before every lane has one (the bench's sets are 8-14 MB: at most one line per lane).  The loads are
// ordinary loads the compiler counts: a lane's first two lines land in registers that only touch_wait (an empty asm
// at the wave's end that names them) consumes, so the compiler's own s_waitcnt insertion waits for them there and
// nothing stalls mid-kernel; further lines (a set larger than twice the grid's lanes) load in a loop that waits for
// each.  (r03's form -- inline-asm loads into a "+v" register -- let the register allocator reuse that register
// while a load was still in flight: the compiler takes an asm output as written at the statement.)
struct TouchSink { unsigned a = 0, b = 0; };
template <int NW>
__device__ __forceinline__ void touch_issue(const TouchList& t, TouchSink& s)
{
    const size_t me = ((size_t)blockIdx.x * NW + (threadIdx.x >> 6)) * 64 + (threadIdx.x & 63);
    const size_t tot = (size_t)gridDim.x * NW * 64;
    // the buffer walk is wave-uniform (the list's pointers stay scalar kernel-argument loads)
    const unsigned* p0 = nullptr;
    const unsigned* p1 = nullptr;
    size_t cum = 0;
    for (int b = 0; b < t.n; ++b) {
        const size_t n = t.bytes[b] >> 7;
        const char* base = reinterpret_cast<const char*>(t.ptr[b]);
        if (me >= cum && me < cum + n) p0 = reinterpret_cast<const unsigned*>(base + ((me - cum) << 7));
        if (me + tot >= cum && me + tot < cum + n) p1 = reinterpret_cast<const unsigned*>(base + ((me + tot - cum) << 7));
        cum += n;
    }
    if (p0) s.a = *p0;
    if (p1) s.b = *p1;
    if (me + 2 * tot < cum) {                    // more lines than twice the grid's lanes: the rest, waited one by one
        size_t c = 0;
        for (int b = 0; b < t.n; ++b) {
            const size_t n = t.bytes[b] >> 7;
            const char* base = reinterpret_cast<const char*>(t.ptr[b]);
            for (size_t gi = me + 2 * tot; gi < c + n; gi += tot)
                if (gi >= c) s.b ^= *reinterpret_cast<const unsigned*>(base + ((gi - c) << 7));
            c += n;
        }
    }
    asm volatile("" ::: "memory");               // the loads stay here (no memory access moves across)
}
__device__ __forceinline__ void touch_wait(const TouchSink& s) { asm volatile("" :: "v"(s.a), "v"(s.b)); }
// At most one line a lane (the caller checks lines <= the grid's lanes): one unconditional load a lane (lanes past the
// lines re-read the first one), so no branch joins the wave's load sequence -- at a join hipcc's vmcnt bookkeeping
// takes the shortest path's count, and the row loads' wait in ln_post's backward drained the touch with them.
template <int NW>
__device__ __forceinline__ void touch_issue1(const TouchList& t, TouchSink& s)
{
    const size_t me = ((size_t)blockIdx.x * NW + (threadIdx.x >> 6)) * 64 + (threadIdx.x & 63);
    const unsigned* p0 = reinterpret_cast<const unsigned*>(t.ptr[0]);
    size_t cum = 0;
    for (int b = 0; b < t.n; ++b) {
        const size_t n = t.bytes[b] >> 7;
        if (me >= cum && me < cum + n) p0 = reinterpret_cast<const unsigned*>(reinterpret_cast<const char*>(t.ptr[b]) + ((me - cum) << 7));
        cum += n;
    }
    s.a = *p0;
    asm volatile("" ::: "memory");
}
}  // namespace ebc
