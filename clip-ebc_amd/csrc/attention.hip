// Multi-head self-attention for the CLIP ViT-B/16 + VPT encoder on gfx950: forward, and the
// FA2-style backward split into a dQ kernel and a dK/dV kernel (no atomics).
//
// Reference: nn.MultiheadAttention(d_model=768, n_head=12) called as attn(x, x, x,
// need_weights=False) in ResidualAttentionBlock.attention (models/clip/_clip/blocks.py:35-37),
// i.e. softmax(Q K^T / sqrt(64)) V per head with the packed in-projection layout
// qkv[row] = [q(768) | k(768) | v(768)], head h at columns h*64 .. h*64+63.
//
// The sequence is short (1 CLS + 32 VPT + 196 patches = 229 tokens), so a workgroup keeps the
// whole K and V (or Q and dO) of one (crop, head) in LDS, padded to LP = 256 rows; scores for 16
// query rows x 256 keys live in registers, so no online softmax.  16-bit rows are 128 B with their
// eight 16-B chunks XOR-swizzled per row pair (chunk c of row r at c ^ SWZ[(r >> 1) & 7]): the
// ds_read_b128 row fragments (lane groups {0-3,12-15,20-27}, ...) and the ds_read_b64_tr_b16 column
// fragments (32-lane groups) both cover the 64 banks once per group (the former 144-B pitch left
// 43-47 % of the LDS cycles as bank conflicts, PMC r02); f32 (parity mode) keeps a padded pitch.
// Operand orientation ("swapped" S^T = K Q^T) puts each query on one lane, so the probability
// accumulators are directly the A operand of P.V with no LDS round trip (mfma.h).
//   grid: B * H * ceil(L/(16 NW)) workgroups of NW waves; wave w owns 16 queries (fwd, dQ) or 16 keys (dKV).
#include <algorithm>
#include <cstdlib>
#include <string>

#include "ebc_common.h"
#include "kernels.h"
#include "mfma.h"
#include "touch.h"

using namespace ebc;

// lab-only phase stamps (tools/lab/attn_tl_lab.hip): 0 entry, 1 operands staged (after the barrier), 2 a wave's end
#ifndef EBC_ATTN_STAMP
#define EBC_ATTN_STAMP(phase) ((void)0)
#endif

namespace {

constexpr int HD = 64;          // head dim
constexpr int LP = 256;         // padded sequence (>= L)
constexpr int NKT = LP / 16;    // 16-row tiles
// NW waves per workgroup (16 queries / keys each): 16 for the ViT-B/16 sequence (one workgroup per
// (crop, head), K/V or Q/dO staged once), 8 for short sequences
constexpr float LOG2E = 1.4426950408889634f;
// (crop, head) work in XCD order (xcd_remap): each XCD takes a contiguous run of crops, i.e. the token rows the
// QKV / dO GEMM tiles of that XCD wrote and the next GEMM's tiles on it read; in the backward the dQ and dK/dV
// workgroups of one (crop, head) are adjacent, so the second reader of K/V (Q/dO) finds them in the same L2
__device__ __forceinline__ int attn_block() { return xcd_remap(blockIdx.x, (int)gridDim.x); }

template <class E> struct AttnCfg {
    using T = typename E::T;
    static constexpr int EB = E::BYTES;
    static constexpr bool SW = EB == 2;                      // 16-bit: swizzled 128-B rows
    static constexpr int LDR = SW ? HD : HD + 16 / EB;       // row pitch in elements (128 B / 272 B)
    static constexpr int CPR = HD * EB / 16;                 // 16-B chunks per row
    static constexpr size_t TILE_BYTES = (size_t)LP * LDR * EB;
};

// chunk swizzle of row r (16-bit tiles): a permutation f of 0..7 indexed by the row pair, chosen so that
// {f(0),f(1),f(6),f(7)} and {f(2..5)} ^ 1 are disjoint (row fragments) and f(0..3), f(4..7) each take one
// value from every pair {2k, 2k+1} (transposed column fragments)
__device__ __forceinline__ int attn_swz(int r) { return (0x71534260u >> (4 * ((r >> 1) & 7))) & 7; }

// element offset of (row, col) in an LDS tile; col a multiple of 4 (16-bit) so a fragment piece stays in its chunk
template <class E>
__device__ __forceinline__ int attn_off(int row, int col) {
    using C = AttnCfg<E>;
    if constexpr (C::SW) return row * C::LDR + ((((col >> 3) ^ attn_swz(row)) << 3) | (col & 7));
    else return row * C::LDR + col;
}

// One tile of rows into LDS (dst[s][0..63] = src[s*ld + 0..63] for s < L, zero up to LP) in two halves, so that several tiles' (and the fragments') global loads are all in flight before
// the first LDS store waits on one of them: fetch -> (other loads) -> store
template <class E, int NWV> struct RowFetch {
    static constexpr int PER = LP * AttnCfg<E>::CPR / (64 * NWV);
    uint4 v[PER];
};
template <class E, int NWV>
__device__ __forceinline__ void rows_fetch(RowFetch<E, NWV>& f, const typename E::T* src, int ld, int L)
{
    using C = AttnCfg<E>;
#pragma unroll
    for (int k = 0; k < RowFetch<E, NWV>::PER; ++k) {
        const int e = threadIdx.x + k * 64 * NWV;
        const int s = e / C::CPR, c = e % C::CPR;
        f.v[k] = s < L ? *reinterpret_cast<const uint4*>(src + (size_t)s * ld + c * (16 / C::EB)) : make_uint4(0, 0, 0, 0);
    }
}
template <class E, int NWV>
__device__ __forceinline__ void rows_store(typename E::T* dst, const RowFetch<E, NWV>& f)
{
    using C = AttnCfg<E>;
#pragma unroll
    for (int k = 0; k < RowFetch<E, NWV>::PER; ++k) {
        const int e = threadIdx.x + k * 64 * NWV;
        const int s = e / C::CPR, c = e % C::CPR;
        *reinterpret_cast<uint4*>(dst + attn_off<E>(s, c * (16 / C::EB))) = f.v[k];
    }
}

// B-operand column fragment of rows r0 .. r0+31, columns n0 .. n0+15 (mfma.h load_colfrag on the
// swizzled 16-bit tiles: each lane's 8-B ds_read_b64_tr_b16 piece stays inside one 16-B chunk)
template <class E>
__device__ __forceinline__ typename E::Frag attn_colfrag(const typename E::T* lds, int r0, int n0) {
    using C = AttnCfg<E>;
    if constexpr (!C::SW) {
        return load_colfrag<E>(lds, C::LDR, r0, n0);
    } else {
        const int l = threadIdx.x & 63, g = l >> 4, w = l & 15, q = w >> 2, p = w & 3;
        const int r = r0 + 4 * g + q;
        const typename E::T* a0 = lds + attn_off<E>(r, n0 + 4 * p);
        const typename E::T* a1 = lds + attn_off<E>(r + 16, n0 + 4 * p);
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a0));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a1));
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        return __builtin_bit_cast(typename E::Frag, v);
    }
}

// 8 contiguous elements of a global row (zeros when !valid)
template <class E>
__device__ __forceinline__ typename E::Frag gload8(const typename E::T* p, bool valid) {
    if (valid) return load8<E>(p);
    typename E::Frag z;
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = E::from(0.f);
    return z;
}

// 4 consecutive output elements (8 B for 16-bit): the P.V / dS.K products are issued with the column fragment as the
// A operand, so each lane ends with 4 consecutive head-dim columns of ONE row (its query / key fr) and stores them in
// one instruction (16 two-byte stores per lane before)
template <class E>
__device__ __forceinline__ void store4(typename E::T* p, float a, float b, float c, float d) {
    typedef typename E::T t4 __attribute__((ext_vector_type(4)));
    *reinterpret_cast<t4*>(p) = t4{E::from(a), E::from(b), E::from(c), E::from(d)};
}

// Two 16-column blocks' outputs of one row as 16-B stores (cdna_hip_programming.md T21): lane group fg holds columns
// 4 fg .. 4 fg + 3 of blocks da and db (x sa, x sb); v_permlane16_swap (odd 16-lane rows of the first operand <-> even
// rows of the second) leaves each lane 8 contiguous columns -- block (fg odd ? db : da), columns 8 (fg >> 1) .. -- one
// dwordx4 store where two dwordx2 stores were (r06).  `row` is the output row's first element; the swaps run on every
// lane (call it outside divergent code), the store only where `live`.
template <class E>
__device__ __forceinline__ void store8_pair(typename E::T* row, bool live, const f32x4& a, const f32x4& b, float sa, float sb,
                                            int da, int db) {
    typedef typename E::T t4 __attribute__((ext_vector_type(4)));
    const int fg = (threadIdx.x & 63) >> 4;
    const uint2 pa = __builtin_bit_cast(uint2, t4{E::from(a[0] * sa), E::from(a[1] * sa), E::from(a[2] * sa), E::from(a[3] * sa)});
    const uint2 pb = __builtin_bit_cast(uint2, t4{E::from(b[0] * sb), E::from(b[1] * sb), E::from(b[2] * sb), E::from(b[3] * sb)});
    const auto r0 = __builtin_amdgcn_permlane16_swap(pa.x, pb.x, false, false);
    const auto r1 = __builtin_amdgcn_permlane16_swap(pa.y, pb.y, false, false);
    if (live) *reinterpret_cast<uint4*>(row + 16 * ((fg & 1) ? db : da) + 8 * (fg >> 1)) = make_uint4(r0[0], r1[0], r0[1], r1[1]);
}

template <class E>
__device__ __forceinline__ typename E::Frag lds_rowfrag(const typename E::T* base, int row, int col) {
    return load8<E>(base + attn_off<E>(row, col));
}

// Weight touch: touch.h (touch_issue / touch_wait)

// Softmax row arithmetic in the swapped layout (a query's 256 keys on the lanes fr, fr + 16, fr + 32, fr + 48, four
// per lane per 16-key tile).  r03's PMC put the forward at 9.2 VALU instructions per MFMA; per score it issued a
// canonicalising v_max before every fmaxf (IEEE maxNum), one v_fma and one v_add, and per row reduction two
// ds_bpermute round trips with their lane-index arithmetic.  Here: v_maximum3_f32 (IEEE maximum: no canonicalise, 2
// scores an instruction), packed f32 FMA / add (v_pk_fma_f32, v_pk_add_f32: 2 scores an instruction) and the row
// reductions across the four 16-lane rows by v_permlane16_swap / v_permlane32_swap (each lane receives its own and its
// partner's value, in either order, so max / + of the pair is the same on both lanes).
typedef float f32x2 __attribute__((ext_vector_type(2)));
// softmax pair arithmetic as two single-lane instructions (EBC_ATTN_SCALAR 1; the Makefile builds this file with
// -fno-slp-vectorize so they stay single) or packed f32 (v_pk_fma_f32 / v_pk_add_f32 / v_pk_mul_f32, 0).  Beside the
// MFMAs a packed f32 instruction costs more issue than the two it replaces (MI355X_MICROARCH.md per-instruction
// constants); r06, tools/lab/attn_tl_lab.hip, 16 crops: forward 11.8 -> 11.5 us, backward 25.3 -> 24.7 us
#ifndef EBC_ATTN_SCALAR
#define EBC_ATTN_SCALAR 1
#endif
// backward: the MFMA chain of dP starts from -delta (cdna_hip_programming.md "row constants as the initial accumulator"),
// so dS = p dP' needs no subtraction (r06: backward 24.7 -> 24.0 us, compute phase 14.9 -> 14.3 us)
#ifndef EBC_ATTN_DINIT
#define EBC_ATTN_DINIT 1
#endif
__device__ __forceinline__ f32x2 fma2(f32x2 a, f32x2 b, f32x2 c) {
    if constexpr (EBC_ATTN_SCALAR) return f32x2{__builtin_fmaf(a.x, b.x, c.x), __builtin_fmaf(a.y, b.y, c.y)};
    else return __builtin_elementwise_fma(a, b, c);
}
__device__ __forceinline__ f32x2 add2(f32x2 a, f32x2 b) {
    if constexpr (EBC_ATTN_SCALAR) return f32x2{a.x + b.x, a.y + b.y};
    else return a + b;
}
__device__ __forceinline__ f32x2 mul2(f32x2 a, f32x2 b) {
    if constexpr (EBC_ATTN_SCALAR) return f32x2{a.x * b.x, a.y * b.y};
    else return a * b;
}
__device__ __forceinline__ float max3f(float a, float b, float c) {
    return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c);
}
__device__ __forceinline__ float rows_max(float x) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = __builtin_elementwise_maximum(__uint_as_float(a[0]), __uint_as_float(a[1]));
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __builtin_elementwise_maximum(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float rows_sum(float x) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// ------------------------------------------------------------------------------ forward
// QT query tiles of 16 per wave: every K row fragment and V column fragment read from LDS feeds QT MFMAs (the LDS
// reads per query halve at QT = 2; with one tile per wave the forward was bound by re-reading K and V per 16 queries)
template <class E, int NWV, int LFIX, int QT = 1>
__global__ __launch_bounds__(64 * NWV) void attn_fwd_kernel(const typename E::T* __restrict__ qkv, typename E::T* __restrict__ out,
                                                       float* __restrict__ lse, int B, int L_, int H, float scale,
                                                       TouchList touch)
{
    const int L = LFIX > 0 ? LFIX : L_;                        // compile-time sequence: tile loops and masks fold
    using T = typename E::T;
    using C = AttnCfg<E>;
    EBC_ATTN_STAMP(0);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* Ks = reinterpret_cast<T*>(smem);
    T* Vs = reinterpret_cast<T*>(smem + C::TILE_BYTES);
    constexpr int QB = 16 * NWV * QT;
    const int nqb = (L + QB - 1) / QB;
    const int bid = attn_block();
    const int bh = bid / nqb, qb = bid % nqb;
    const int b = bh / H, h = bh % H;
    const int D3 = 3 * H * HD, D = H * HD;
    const T* base = qkv + (size_t)b * L * D3 + h * HD;
    // K, V and this wave's Q fragments: every global load issued before the first LDS store
    RowFetch<E, NWV> fk, fv;
    rows_fetch<E, NWV>(fk, base + D, D3, L);
    rows_fetch<E, NWV>(fv, base + 2 * D, D3, L);

    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, fg = lane >> 4;
    const int q0 = qb * QB + w * 16 * QT;                      // this wave's first query; tile t starts at q0 + 16 t
    typename E::Frag qf[QT][2];
#pragma unroll
    for (int t = 0; t < QT; ++t) {
        const int qme = q0 + 16 * t + fr;                      // this lane's query in tile t (column of S^T)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) qf[t][ks] = gload8<E>(base + (size_t)qme * D3 + 32 * ks + 8 * fg, qme < L);
    }
    rows_store<E, NWV>(Ks, fk);
    rows_store<E, NWV>(Vs, fv);
    __syncthreads();
    EBC_ATTN_STAMP(1);

    TouchSink tsink;
    if (touch.n) touch_issue<NWV>(touch, tsink);               // every wave takes its share of the touch lines
    if (q0 >= L) {                                             // no live query in this wave (no barrier follows)
        if (touch.n) touch_wait(tsink);
        EBC_ATTN_STAMP(2);
        return;
    }
    // key tiles past L are skipped; only the ragged last tile is masked; the softmax scale is folded
    // into the exp2 argument: p = 2^(s*c - max*c), c = scale*log2(e)
    const int nkt = (L + 15) >> 4;
    const bool ragged = (L & 15) != 0;
    const float c2 = scale * LOG2E;
    f32x4 s[QT][NKT];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
        for (int t = 0; t < QT; ++t) s[t][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (kt < nkt) {
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const typename E::Frag kf = lds_rowfrag<E>(Ks, 16 * kt + fr, 32 * ks + 8 * fg);
#pragma unroll
                for (int t = 0; t < QT; ++t) s[t][kt] = mma(kf, qf[t][ks], s[t][kt]);
            }
        }
    }
    // s[t][kt][i] = S[q = q0 + 16 t + fr][key = 16 kt + 4 fg + i]
    float mx[QT], sum[QT];
#pragma unroll
    for (int t = 0; t < QT; ++t) {
        float m0 = -INFINITY, m1 = -INFINITY;
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt) {
            if (kt < nkt) {
                if (ragged && kt == nkt - 1) {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if (16 * kt + 4 * fg + i >= L) s[t][kt][i] = -INFINITY;
                }
                m0 = max3f(m0, s[t][kt][0], s[t][kt][1]);
                m1 = max3f(m1, s[t][kt][2], s[t][kt][3]);
            }
        }
        mx[t] = rows_max(__builtin_elementwise_maximum(m0, m1));
        const float mc = mx[t] * c2;
        const f32x2 c2v = {c2, c2}, mcv = {-mc, -mc};
        f32x2 acc = {0.f, 0.f};
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt) {
            if (kt < nkt) {
#pragma unroll
                for (int i = 0; i < 4; i += 2) {
                    f32x2 e = fma2(f32x2{s[t][kt][i], s[t][kt][i + 1]}, c2v, mcv);
                    e.x = __builtin_amdgcn_exp2f(e.x);
                    e.y = __builtin_amdgcn_exp2f(e.y);
                    s[t][kt][i] = e.x;
                    s[t][kt][i + 1] = e.y;
                    acc = add2(acc, e);
                }
            }
        }
        sum[t] = rows_sum(acc.x + acc.y);
    }

    f32x4 o[QT][HD / 16];
#pragma unroll
    for (int t = 0; t < QT; ++t)
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) o[t][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int st = 0; st < NKT / 2; ++st) {
        if (2 * st >= nkt) continue;
        typename E::Frag pf[QT];
#pragma unroll
        for (int t = 0; t < QT; ++t) {
            const float pv[8] = {s[t][2 * st][0], s[t][2 * st][1], s[t][2 * st][2], s[t][2 * st][3],
                                 s[t][2 * st + 1][0], s[t][2 * st + 1][1], s[t][2 * st + 1][2], s[t][2 * st + 1][3]};
            pf[t] = pack8<E>(pv);
        }
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) {
            const typename E::Frag vf = attn_colfrag<E>(Vs, 32 * st, 16 * dt);
#pragma unroll
            for (int t = 0; t < QT; ++t) o[t][dt] = mma(vf, pf[t], o[t][dt]);      // O^T tile
        }
    }
    // o[t][dt][i] = O[q = q0 + 16 t + fr][d = 16 dt + 4 fg + i]; this lane holds query fr's row sum itself
#pragma unroll
    for (int t = 0; t < QT; ++t) {
        const float inv = 1.0f / sum[t];
        const int q = q0 + 16 * t + fr;
        if constexpr (E::BYTES == 2) {
            T* orow = out + ((size_t)b * L + q) * D + h * HD;
            store8_pair<E>(orow, q < L, o[t][0], o[t][1], inv, inv, 0, 1);
            store8_pair<E>(orow, q < L, o[t][2], o[t][3], inv, inv, 2, 3);
        } else if (q < L) {
            T* orow = out + ((size_t)b * L + q) * D + h * HD + 4 * fg;
#pragma unroll
            for (int dt = 0; dt < HD / 16; ++dt)
                store4<E>(orow + 16 * dt, o[t][dt][0] * inv, o[t][dt][1] * inv, o[t][dt][2] * inv, o[t][dt][3] * inv);
        }
        const int qme = q0 + 16 * t + fr;
        if (fg == 0 && qme < L && lse) lse[((size_t)b * H + h) * L + qme] = mx[t] * scale + logf(sum[t]);   // natural-log units
    }
    if (touch.n) touch_wait(tsink);
    EBC_ATTN_STAMP(2);
}

// ------------------------------------------------------------------------------ backward dQ
template <class E, int NWV, int LFIX>
__device__ __forceinline__ void attn_bwd_dq_body(int bid, const typename E::T* __restrict__ qkv, const typename E::T* __restrict__ dout,
                                                 const typename E::T* __restrict__ out, const float* __restrict__ lse,
                                                 float* __restrict__ delta, typename E::T* __restrict__ dqkv, int B,
                                                 int L_, int H, float scale)
{
    const int L = LFIX > 0 ? LFIX : L_;
    using T = typename E::T;
    using C = AttnCfg<E>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* Ks = reinterpret_cast<T*>(smem);
    T* Vs = reinterpret_cast<T*>(smem + C::TILE_BYTES);
    constexpr int QB = 16 * NWV;
    const int nqb = (L + QB - 1) / QB;
    const int bh = bid / nqb, qb = bid % nqb;
    const int b = bh / H, h = bh % H;
    const int D3 = 3 * H * HD, D = H * HD;
    const T* base = qkv + (size_t)b * L * D3 + h * HD;
    // K, V, and this wave's Q / dO / O fragments and lse: every global load before the first LDS store
    RowFetch<E, NWV> fk, fv;
    rows_fetch<E, NWV>(fk, base + D, D3, L);
    rows_fetch<E, NWV>(fv, base + 2 * D, D3, L);

    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, fg = lane >> 4;
    const int q0 = qb * QB + w * 16;
    const int qme = q0 + fr;
    const bool qv = qme < L;
    typename E::Frag qf[2], df[2], of[2];
    const T* drow = dout + ((size_t)b * L + qme) * D + h * HD;
    const T* orow = out + ((size_t)b * L + qme) * D + h * HD;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
        qf[ks] = gload8<E>(base + (size_t)qme * D3 + 32 * ks + 8 * fg, qv);
        df[ks] = gload8<E>(drow + 32 * ks + 8 * fg, qv);
        of[ks] = gload8<E>(orow + 32 * ks + 8 * fg, qv);
    }
    const float lq = qv ? lse[((size_t)b * H + h) * L + qme] : INFINITY;
    rows_store<E, NWV>(Ks, fk);
    rows_store<E, NWV>(Vs, fv);
    // delta = rowsum(dO * O) (FA2 D_i), computed here and published for the dK/dV kernel
    float dq;
    {
        float dd = 0.f;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
            for (int j = 0; j < 8; ++j) dd = fmaf((float)df[ks][j], (float)of[ks][j], dd);
        }
        dd += __shfl_xor(dd, 16, 64);
        dd += __shfl_xor(dd, 32, 64);
        dq = qv ? dd : 0.f;
        if (fg == 0 && qv && delta) delta[((size_t)b * H + h) * L + qme] = dd;
    }
    __syncthreads();

    if (q0 >= L) return;                                       // no live query in this wave (no barrier follows)
    const int nkt = (L + 15) >> 4;
    const bool ragged = (L & 15) != 0;
    const float c2 = scale * LOG2E, lq2 = lq * LOG2E;          // p = 2^(s*c - lse*log2 e)
    f32x4 dq_acc[HD / 16];
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) dq_acc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int st = 0; st < NKT / 2; ++st) {
        if (2 * st >= nkt) continue;
        float ds[8];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            const int kt = 2 * st + hf;
            if (kt >= nkt) {
#pragma unroll
                for (int i = 0; i < 4; ++i) ds[4 * hf + i] = 0.f;
                continue;
            }
            f32x4 sv = f32x4{0.f, 0.f, 0.f, 0.f}, pv = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                sv = mma(lds_rowfrag<E>(Ks, 16 * kt + fr, 32 * ks + 8 * fg), qf[ks], sv);
                pv = mma(lds_rowfrag<E>(Vs, 16 * kt + fr, 32 * ks + 8 * fg), df[ks], pv);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float p = __builtin_amdgcn_exp2f(fmaf(sv[i], c2, -lq2));
                if (ragged && kt == nkt - 1 && 16 * kt + 4 * fg + i >= L) p = 0.f;
                ds[4 * hf + i] = p * (pv[i] - dq);
            }
        }
        const typename E::Frag dsf = pack8<E>(ds);
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) dq_acc[dt] = mma(dsf, attn_colfrag<E>(Ks, 32 * st, 16 * dt), dq_acc[dt]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int q = q0 + 4 * fg + i;
        if (q < L) {
            T* row = dqkv + ((size_t)b * L + q) * D3 + h * HD;
#pragma unroll
            for (int dt = 0; dt < HD / 16; ++dt) row[16 * dt + fr] = E::from(dq_acc[dt][i] * scale);
        }
    }
}

template <class E, int NWV, int LFIX>
__global__ __launch_bounds__(64 * NWV) void attn_bwd_dq_kernel(const typename E::T* __restrict__ qkv, const typename E::T* __restrict__ dout,
                                                          const typename E::T* __restrict__ out, const float* __restrict__ lse,
                                                          float* __restrict__ delta, typename E::T* __restrict__ dqkv, int B,
                                                          int L_, int H, float scale)
{
    attn_bwd_dq_body<E, NWV, LFIX>(attn_block(), qkv, dout, out, lse, delta, dqkv, B, L_, H, scale);
}

// ------------------------------------------------------------------------------ backward dK, dV
// delta = rowsum(dO * O) of query q, summed in the dQ kernel's order (per 16-lane group fg: a 16-term fma
// chain over columns 32 ks + 8 fg + j, then (p0 + p1) + (p2 + p3)), so both kernels see the same bits
template <class E>
__device__ __forceinline__ float attn_delta_row(const typename E::T* drow, const typename E::T* orow) {
    float p[4];
#pragma unroll
    for (int fg = 0; fg < 4; ++fg) {
        float dd = 0.f;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const typename E::Frag df = load8<E>(drow + 32 * ks + 8 * fg), of = load8<E>(orow + 32 * ks + 8 * fg);
#pragma unroll
            for (int j = 0; j < 8; ++j) dd = fmaf((float)df[j], (float)of[j], dd);
        }
        p[fg] = dd;
    }
    return (p[0] + p[1]) + (p[2] + p[3]);
}

// delta of one query for the one-workgroup backward: 4 lanes a query (16 columns each, v_dot2 products accumulated in
// f32), the quad's partial sums added by DPP.  Its bits differ from attn_delta_row's; only this kernel uses it, for
// both the dQ and the dK / dV products, so they agree with each other.  (r03: one lane a query, 64 conversions and 32
// FMAs per row on 4 of the 16 waves, ahead of the workgroup's first barrier.)
template <class E>
__device__ __forceinline__ float attn_delta_quad(const typename E::T* drow, const typename E::T* orow) {
    const typename E::Frag d0 = load8<E>(drow), d1 = load8<E>(drow + 8), o0 = load8<E>(orow), o1 = load8<E>(orow + 8);
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
        if constexpr (std::is_same<E, EF16>::value) {
            typedef _Float16 h2 __attribute__((ext_vector_type(2)));
            acc = __builtin_amdgcn_fdot2(h2{d0[j], d0[j + 1]}, h2{o0[j], o0[j + 1]}, acc, false);
            acc = __builtin_amdgcn_fdot2(h2{d1[j], d1[j + 1]}, h2{o1[j], o1[j + 1]}, acc, false);
        } else {
            typedef __bf16 b2 __attribute__((ext_vector_type(2)));
            acc = __builtin_amdgcn_fdot2_f32_bf16(b2{d0[j], d0[j + 1]}, b2{o0[j], o0[j + 1]}, acc, false);
            acc = __builtin_amdgcn_fdot2_f32_bf16(b2{d1[j], d1[j + 1]}, b2{o1[j], o1[j + 1]}, acc, false);
        }
    }
    acc += __builtin_amdgcn_update_dpp(0.f, acc, 0xB1, 0xF, 0xF, false);      // quad_perm [1, 0, 3, 2]
    acc += __builtin_amdgcn_update_dpp(0.f, acc, 0x4E, 0xF, 0xF, false);      // quad_perm [2, 3, 0, 1]
    return acc;
}

template <class E, int NWV, int LFIX>
__device__ __forceinline__ void attn_bwd_dkv_body(int bid, const typename E::T* __restrict__ qkv, const typename E::T* __restrict__ dout,
                                                  const typename E::T* __restrict__ out, const float* __restrict__ lse,
                                                  const float* __restrict__ delta, typename E::T* __restrict__ dqkv, int B,
                                                  int L_, int H, float scale)
{
    const int L = LFIX > 0 ? LFIX : L_;
    using T = typename E::T;
    using C = AttnCfg<E>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* Qs = reinterpret_cast<T*>(smem);
    T* Ds = reinterpret_cast<T*>(smem + C::TILE_BYTES);
    float* ls = reinterpret_cast<float*>(smem + 2 * C::TILE_BYTES);
    float* dl = ls + LP;
    constexpr int QB = 16 * NWV;
    const int nkb = (L + QB - 1) / QB;
    const int bh = bid / nkb, kb = bid % nkb;
    const int b = bh / H, h = bh % H;
    const int D3 = 3 * H * HD, D = H * HD;
    const T* base = qkv + (size_t)b * L * D3 + h * HD;
    // Q, dO and this wave's K / V fragments: every global load before the first LDS store
    RowFetch<E, NWV> fq, fd;
    rows_fetch<E, NWV>(fq, base, D3, L);
    rows_fetch<E, NWV>(fd, dout + (size_t)b * L * D + h * HD, D, L);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, fg = lane >> 4;
    const int k0 = kb * QB + w * 16;
    const int kme = k0 + fr;
    const bool kv = kme < L;
    typename E::Frag kf[2], vf[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
        kf[ks] = gload8<E>(base + (size_t)kme * D3 + D + 32 * ks + 8 * fg, kv);
        vf[ks] = gload8<E>(base + (size_t)kme * D3 + 2 * D + 32 * ks + 8 * fg, kv);
    }
    rows_store<E, NWV>(Qs, fq);
    rows_store<E, NWV>(Ds, fd);
    for (int q = threadIdx.x; q < LP; q += blockDim.x) {              // lse pre-scaled by log2(e)
        ls[q] = q < L ? lse[((size_t)b * H + h) * L + q] * LOG2E : INFINITY;
        if (delta) dl[q] = q < L ? delta[((size_t)b * H + h) * L + q] : 0.f;
        else dl[q] = q < L ? attn_delta_row<E>(dout + ((size_t)b * L + q) * D + h * HD, out + ((size_t)b * L + q) * D + h * HD) : 0.f;
    }

    __syncthreads();

    if (k0 >= L) return;                                       // no live key in this wave (no barrier follows)
    const int nqt = (L + 15) >> 4;                             // query tiles past L: lse = +inf, p = 0
    const float c2 = scale * LOG2E;
    f32x4 dk[HD / 16], dv[HD / 16];
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) { dk[dt] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[dt] = f32x4{0.f, 0.f, 0.f, 0.f}; }
#pragma unroll 2
    for (int st = 0; st < NKT / 2; ++st) {
        if (2 * st >= nqt) break;
        float pp[8], ds[8];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            const int qt = 2 * st + hf;
            f32x4 sv = f32x4{0.f, 0.f, 0.f, 0.f}, pv = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                sv = mma(lds_rowfrag<E>(Qs, 16 * qt + fr, 32 * ks + 8 * fg), kf[ks], sv);   // S^T[q][key]
                pv = mma(lds_rowfrag<E>(Ds, 16 * qt + fr, 32 * ks + 8 * fg), vf[ks], pv);   // dP^T[q][key]
            }
            const float4 l4 = *reinterpret_cast<const float4*>(ls + 16 * qt + 4 * fg);
            const float4 d4 = *reinterpret_cast<const float4*>(dl + 16 * qt + 4 * fg);
            const float lq[4] = {l4.x, l4.y, l4.z, l4.w}, dq[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float p = __builtin_amdgcn_exp2f(fmaf(sv[i], c2, -lq[i]));   // lse = +inf (padding) -> 0
                pp[4 * hf + i] = p;
                ds[4 * hf + i] = p * (pv[i] - dq[i]);
            }
        }
        const typename E::Frag pf = pack8<E>(pp), dsf = pack8<E>(ds);
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) {
            dv[dt] = mma(pf, attn_colfrag<E>(Ds, 32 * st, 16 * dt), dv[dt]);
            dk[dt] = mma(dsf, attn_colfrag<E>(Qs, 32 * st, 16 * dt), dk[dt]);
        }
            }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int key = k0 + 4 * fg + i;
        if (key < L) {
            T* row = dqkv + ((size_t)b * L + key) * D3 + h * HD;
#pragma unroll
            for (int dt = 0; dt < HD / 16; ++dt) {
                row[D + 16 * dt + fr] = E::from(dk[dt][i] * scale);
                row[2 * D + 16 * dt + fr] = E::from(dv[dt][i]);
            }
        }
    }
}

template <class E, int NWV, int LFIX>
__global__ __launch_bounds__(64 * NWV) void attn_bwd_dkv_kernel(const typename E::T* __restrict__ qkv, const typename E::T* __restrict__ dout,
                                                           const float* __restrict__ lse, const float* __restrict__ delta,
                                                           typename E::T* __restrict__ dqkv, int B, int L_, int H, float scale)
{
    attn_bwd_dkv_body<E, NWV, LFIX>(attn_block(), qkv, dout, nullptr, lse, delta, dqkv, B, L_, H, scale);
}

// One 16-wave workgroup per (crop, head) for the whole backward: K, V, Q and dO staged once into LDS (4 x 32 KiB),
// lse and the row statistic delta (attn_delta_row, the dK/dV body's bits) for every query beside them; then each wave
// forms dQ of its 16 queries and dK / dV of its 16 keys from LDS alone.  Per (crop, head) the operands are fetched
// once (5 rows of 128 B per token with O), where the two-role grid fetched K/V per dQ block, Q/dO per dK/dV block
// and dO + O again per dK/dV block for delta: 2.2x the bytes (PMC r03a: 85 MB per launch) over 1.5 waves of
// 8-wave workgroups.  The arithmetic is the two-role kernels', operation for operation.
// rows > 0: only dQ of queries < rows and dK / dV of keys < rows (layer 0's prompt rows).
// Lane-constant LDS addressing of the swizzled 16-bit tiles: a row fragment (rows 16 t + fr, columns 32 ks + 8 fg) and a
// column fragment (rows 32 st + 4 g + q (+16), columns 16 dt + 4 p) land at a per-lane byte offset (ks or dt) plus a
// compile-time one (t, st), because the chunk swizzle depends on (row >> 1) & 7 only, which those row steps keep: every
// fragment read is one VGPR address + an immediate (the generic attn_off form cost ~470 address VALU per wave).
struct AttnLaneOffsets {
    int row[2];                // ks = 0, 1
    int col[HD / 16];          // dt = 0 .. 3
    __device__ __forceinline__ AttnLaneOffsets() {
        const int l = threadIdx.x & 63, fr = l & 15, fg = l >> 4;
        const int sr = attn_swz(fr);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) row[ks] = (fr * HD + (((4 * ks + fg) ^ sr) << 3)) * 2;
        const int g = l >> 4, w = l & 15, q = w >> 2, p = w & 3, rr = 4 * g + q, sc = attn_swz(rr);
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) col[dt] = (rr * HD + ((((2 * dt + (p >> 1)) ^ sc) << 3) | (4 * (p & 1)))) * 2;
    }
};
template <class E>
__device__ __forceinline__ typename E::Frag rowfrag_at(const char* tile, int off, int t) {
    return __builtin_bit_cast(typename E::Frag, *reinterpret_cast<const uint4*>(tile + off + t * 16 * HD * 2));
}
template <class E>
__device__ __forceinline__ typename E::Frag colfrag_at(const char* tile, int off, int st) {
    const char* a = tile + off + st * 32 * HD * 2;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a + 16 * HD * 2));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(typename E::Frag, v);
}

template <class E, int LFIX>
__global__ __launch_bounds__(1024) void attn_bwd_one_kernel(const typename E::T* __restrict__ qkv, const typename E::T* __restrict__ dout,
                                                           const typename E::T* __restrict__ out, const float* __restrict__ lse,
                                                           typename E::T* __restrict__ dqkv, int B, int L_, int H, float scale,
                                                           int rows, TouchList touch)
{
    constexpr int NWV = 16;
    const int L = LFIX > 0 ? LFIX : L_;
    using T = typename E::T;
    using C = AttnCfg<E>;
    EBC_ATTN_STAMP(0);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* Ks = reinterpret_cast<T*>(smem);
    T* Vs = reinterpret_cast<T*>(smem + C::TILE_BYTES);
    T* Qs = reinterpret_cast<T*>(smem + 2 * C::TILE_BYTES);
    T* Ds = reinterpret_cast<T*>(smem + 3 * C::TILE_BYTES);
    float* ls = reinterpret_cast<float*>(smem + 4 * C::TILE_BYTES);
    float* dl = ls + LP;
    const int bh = attn_block(), b = bh / H, h = bh % H;
    const int D3 = 3 * H * HD, D = H * HD;
    const T* base = qkv + (size_t)b * L * D3 + h * HD;
    const T* dob = dout + (size_t)b * L * D + h * HD;
    RowFetch<E, NWV> fk, fv, fq, fd;
    rows_fetch<E, NWV>(fk, base + D, D3, L);
    rows_fetch<E, NWV>(fv, base + 2 * D, D3, L);
    rows_fetch<E, NWV>(fq, base, D3, L);
    rows_fetch<E, NWV>(fd, dob, D, L);
    const int qd = threadIdx.x >> 2, qj = threadIdx.x & 3;    // lse / delta of query qd, a quarter of its row
    float lsv = INFINITY, dlv = 0.f;                            // padding queries: p = 0, delta 0
    if (qd < L) {                                               // (a lane quad is all in or all out)
        if (qj == 0) lsv = lse[((size_t)b * H + h) * L + qd] * LOG2E;       // lse pre-scaled by log2(e)
        dlv = attn_delta_quad<E>(dob + (size_t)qd * D + 16 * qj, out + ((size_t)b * L + qd) * D + h * HD + 16 * qj);
    }
    rows_store<E, NWV>(Ks, fk);
    rows_store<E, NWV>(Vs, fv);
    rows_store<E, NWV>(Qs, fq);
    rows_store<E, NWV>(Ds, fd);
    static_assert(64 * NWV >= 4 * LP, "a lane quad per padded query");
    if (qj == 0) { ls[qd] = lsv; dl[qd] = dlv; }
    __syncthreads();
    EBC_ATTN_STAMP(1);

    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, fg = lane >> 4;
    const int lim = rows > 0 && rows < L ? rows : L;
    // every wave takes its share of the weight touch (the lines are dealt over all of the grid's lanes), then a wave
    // with no live query / key waits for its touch loads and leaves (no barrier follows)
    TouchSink tsink;
    if (touch.n) touch_issue<NWV>(touch, tsink);
    if (16 * w >= lim) {
        if (touch.n) touch_wait(tsink);
        EBC_ATTN_STAMP(2);
        return;
    }
    const int nkt = (L + 15) >> 4;
    const bool ragged = (L & 15) != 0;
    const float c2 = scale * LOG2E;
    static_assert(E::BYTES == 2, "swizzled 16-bit tiles");
    const AttnLaneOffsets lo;
    // per-lane fragment base pointers of each tile (the row / column steps are immediates on these)
    const char* Kr[2] = {reinterpret_cast<const char*>(Ks) + lo.row[0], reinterpret_cast<const char*>(Ks) + lo.row[1]};
    const char* Vr[2] = {reinterpret_cast<const char*>(Vs) + lo.row[0], reinterpret_cast<const char*>(Vs) + lo.row[1]};
    const char* Qr[2] = {reinterpret_cast<const char*>(Qs) + lo.row[0], reinterpret_cast<const char*>(Qs) + lo.row[1]};
    const char* Dr[2] = {reinterpret_cast<const char*>(Ds) + lo.row[0], reinterpret_cast<const char*>(Ds) + lo.row[1]};
    const char* Kc[HD / 16];
    const char* Qc[HD / 16];
    const char* Dc[HD / 16];
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) {
        Kc[dt] = reinterpret_cast<const char*>(Ks) + lo.col[dt];
        Qc[dt] = reinterpret_cast<const char*>(Qs) + lo.col[dt];
        Dc[dt] = reinterpret_cast<const char*>(Ds) + lo.col[dt];
    }
    {
        // dQ of queries q0 .. q0 + 15 (the dQ body: S, dP per key tile, dS packed as the A operand of dS K)
        const int q0 = 16 * w, qme = q0 + fr;
        typename E::Frag qf[2], df[2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            qf[ks] = rowfrag_at<E>(Qr[ks], 0, w);
            df[ks] = rowfrag_at<E>(Dr[ks], 0, w);
        }
        const float lq2 = ls[qme], dq = dl[qme];
        f32x4 dq_acc[HD / 16];
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) dq_acc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
        // software-pipelined over key-tile pairs: the S / dP products of pair st + 1 are issued before the softmax
        // arithmetic of pair st, so each wave has independent MFMAs in flight under its VALU chain
        f32x4 sv[2][2], pv[2][2];                              // [pair parity][tile of the pair]
        auto sdp = [&](int kt, f32x4& s_, f32x4& p_) {
            s_ = f32x4{0.f, 0.f, 0.f, 0.f};
            p_ = EBC_ATTN_DINIT ? f32x4{-dq, -dq, -dq, -dq} : f32x4{0.f, 0.f, 0.f, 0.f};   // dP - delta from the MFMA chain
            if (kt < nkt) {
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
                    s_ = mma(rowfrag_at<E>(Kr[ks], 0, kt), qf[ks], s_);
                    p_ = mma(rowfrag_at<E>(Vr[ks], 0, kt), df[ks], p_);
                }
            }
        };
        sdp(0, sv[0][0], pv[0][0]);
        sdp(1, sv[0][1], pv[0][1]);
#pragma unroll
        for (int st = 0; st < NKT / 2; ++st) {
            if (2 * st >= nkt) break;
            const int cur = st & 1;
            if (2 * st + 2 < nkt) {
                sdp(2 * st + 2, sv[cur ^ 1][0], pv[cur ^ 1][0]);
                sdp(2 * st + 3, sv[cur ^ 1][1], pv[cur ^ 1][1]);
            }
            // packed f32 (softmax arithmetic note above the forward): p = 2^(s c - lse c), dS = p (dP - delta)
            float ds[8];
            const f32x2 c2v = {c2, c2}, nlv = {-lq2, -lq2}, ndv = {-dq, -dq};
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
                const int kt = 2 * st + hf;
#pragma unroll
                for (int i = 0; i < 4; i += 2) {
                    f32x2 p = fma2(f32x2{sv[cur][hf][i], sv[cur][hf][i + 1]}, c2v, nlv);
                    p.x = __builtin_amdgcn_exp2f(p.x);
                    p.y = __builtin_amdgcn_exp2f(p.y);
                    if (kt >= nkt || (ragged && kt == nkt - 1 && 16 * kt + 4 * fg + i >= L)) p.x = 0.f;
                    if (kt >= nkt || (ragged && kt == nkt - 1 && 16 * kt + 4 * fg + i + 1 >= L)) p.y = 0.f;
                    const f32x2 d = EBC_ATTN_DINIT ? mul2(p, f32x2{pv[cur][hf][i], pv[cur][hf][i + 1]})
                                                   : mul2(p, add2(f32x2{pv[cur][hf][i], pv[cur][hf][i + 1]}, ndv));
                    ds[4 * hf + i] = d.x;
                    ds[4 * hf + i + 1] = d.y;
                }
            }
            const typename E::Frag dsf = pack8<E>(ds);
#pragma unroll
            for (int dt = 0; dt < HD / 16; ++dt) dq_acc[dt] = mma(colfrag_at<E>(Kc[dt], 0, st), dsf, dq_acc[dt]);   // dQ^T
        }
        // dq_acc[dt][i] = dQ[q0 + fr][16 dt + 4 fg + i]
        {
            T* row = dqkv + ((size_t)b * L + qme) * D3 + h * HD;
            store8_pair<E>(row, qme < L, dq_acc[0], dq_acc[1], scale, scale, 0, 1);
            store8_pair<E>(row, qme < L, dq_acc[2], dq_acc[3], scale, scale, 2, 3);
        }
    }
    {
        // dK, dV of keys k0 .. k0 + 15 (the dK/dV body: S^T, dP^T per query tile, P and dS as A operands)
        const int k0 = 16 * w;
        typename E::Frag kf[2], vf[2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            kf[ks] = rowfrag_at<E>(Kr[ks], 0, w);
            vf[ks] = rowfrag_at<E>(Vr[ks], 0, w);
        }
        const int nqt = nkt;                                   // query tiles past L: lse = +inf, p = 0
        f32x4 dk[HD / 16], dv[HD / 16];
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) { dk[dt] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[dt] = f32x4{0.f, 0.f, 0.f, 0.f}; }
        f32x4 sv[2][2], pv[2][2];                              // pipelined as the dQ phase, over query-tile pairs
        auto sdp = [&](int qt, f32x4& s_, f32x4& p_) {
            s_ = f32x4{0.f, 0.f, 0.f, 0.f};
            if constexpr (EBC_ATTN_DINIT) {                    // dP^T - delta of the tile's queries from the MFMA chain
                const float4 d4 = *reinterpret_cast<const float4*>(dl + 16 * qt + 4 * fg);
                p_ = f32x4{-d4.x, -d4.y, -d4.z, -d4.w};
            } else {
                p_ = f32x4{0.f, 0.f, 0.f, 0.f};
            }
            if (qt < nqt) {
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
                    s_ = mma(rowfrag_at<E>(Qr[ks], 0, qt), kf[ks], s_);   // S^T[q][key]
                    p_ = mma(rowfrag_at<E>(Dr[ks], 0, qt), vf[ks], p_);   // dP^T[q][key]
                }
            }
        };
        sdp(0, sv[0][0], pv[0][0]);
        sdp(1, sv[0][1], pv[0][1]);
#pragma unroll
        for (int st = 0; st < NKT / 2; ++st) {
            if (2 * st >= nqt) break;
            const int cur = st & 1;
            if (2 * st + 2 < nqt) {
                sdp(2 * st + 2, sv[cur ^ 1][0], pv[cur ^ 1][0]);
                sdp(2 * st + 3, sv[cur ^ 1][1], pv[cur ^ 1][1]);
            }
            float pp[8], ds[8];
            const f32x2 c2v = {c2, c2};
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
                const int qt = 2 * st + hf;
                const float4 l4 = *reinterpret_cast<const float4*>(ls + 16 * qt + 4 * fg);
                const float4 d4 = *reinterpret_cast<const float4*>(dl + 16 * qt + 4 * fg);
                const f32x2 lq[2] = {{l4.x, l4.y}, {l4.z, l4.w}}, dq[2] = {{d4.x, d4.y}, {d4.z, d4.w}};
#pragma unroll
                for (int i = 0; i < 4; i += 2) {
                    // lse = +inf (padding) -> p = 0
                    f32x2 p = fma2(f32x2{sv[cur][hf][i], sv[cur][hf][i + 1]}, c2v, -lq[i / 2]);
                    p.x = __builtin_amdgcn_exp2f(p.x);
                    p.y = __builtin_amdgcn_exp2f(p.y);
                    const f32x2 d = EBC_ATTN_DINIT ? mul2(p, f32x2{pv[cur][hf][i], pv[cur][hf][i + 1]})
                                                   : mul2(p, add2(f32x2{pv[cur][hf][i], pv[cur][hf][i + 1]}, -dq[i / 2]));
                    pp[4 * hf + i] = p.x;
                    pp[4 * hf + i + 1] = p.y;
                    ds[4 * hf + i] = d.x;
                    ds[4 * hf + i + 1] = d.y;
                }
            }
            const typename E::Frag pf = pack8<E>(pp), dsf = pack8<E>(ds);
#pragma unroll
            for (int dt = 0; dt < HD / 16; ++dt) {
                dv[dt] = mma(colfrag_at<E>(Dc[dt], 0, st), pf, dv[dt]);     // dV^T
                dk[dt] = mma(colfrag_at<E>(Qc[dt], 0, st), dsf, dk[dt]);    // dK^T
            }
        }
        // dk / dv[dt][i] = dK / dV[k0 + fr][16 dt + 4 fg + i]
        const int key = k0 + fr;
        {
            T* row = dqkv + ((size_t)b * L + key) * D3 + h * HD;
            store8_pair<E>(row + D, key < L, dk[0], dk[1], scale, scale, 0, 1);
            store8_pair<E>(row + D, key < L, dk[2], dk[3], scale, scale, 2, 3);
            store8_pair<E>(row + 2 * D, key < L, dv[0], dv[1], 1.0f, 1.0f, 0, 1);
            store8_pair<E>(row + 2 * D, key < L, dv[2], dv[3], 1.0f, 1.0f, 2, 3);
        }
    }
    if (touch.n) touch_wait(tsink);
    EBC_ATTN_STAMP(2);
}

// ------------------------------------------------------------------------------ sequences longer than LP
// The reference interpolates the positional embedding to any grid (models/clip/_clip/image_encoder.py:183-198); the
// trainer's default input_size 448 makes 1 + 32 + 28*28 = 817 tokens.  Past LP rows a (crop, head)'s K / V (forward,
// dQ) or Q / dO (dK / dV) no longer fit LDS, so these kernels stream them through it in chunks of LP rows: 8-wave
// workgroups of 128 queries (keys), the next chunk's global loads issued right after the current chunk is staged, so
// they fly under its MFMAs.  The forward keeps a running row maximum m and sum l per query (online softmax: O and l
// rescaled by 2^((m_old - m_new) c) when a chunk raises m); the backward kernels are the two-role pair (dQ publishes
// delta = rowsum(dO * O), dK / dV reads it), accumulating over the chunks in registers.  Per chunk the arithmetic is
// the LP-resident kernels'.
constexpr int LNW = 8;                  // waves per workgroup
constexpr int L_MAX = 16384;            // 1 + prompts + (H/16)(W/16) up to 2048x2048 inputs

template <class E>
__global__ __launch_bounds__(64 * LNW) void attn_fwd_long_kernel(const typename E::T* __restrict__ qkv,
                                                                typename E::T* __restrict__ out, float* __restrict__ lse,
                                                                int B, int L, int H, float scale)
{
    using T = typename E::T;
    using C = AttnCfg<E>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* Ks = reinterpret_cast<T*>(smem);
    T* Vs = reinterpret_cast<T*>(smem + C::TILE_BYTES);
    constexpr int QB = 16 * LNW;
    const int nqb = (L + QB - 1) / QB;
    const int bid = attn_block();
    const int bh = bid / nqb, qb = bid % nqb;
    const int b = bh / H, h = bh % H;
    const int D3 = 3 * H * HD, D = H * HD;
    const T* base = qkv + (size_t)b * L * D3 + h * HD;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, fg = lane >> 4;
    const int q0 = qb * QB + w * 16, qme = q0 + fr;           // waves past L still stage chunks (barriers)
    RowFetch<E, LNW> fk, fv;
    rows_fetch<E, LNW>(fk, base + D, D3, min(L, LP));
    rows_fetch<E, LNW>(fv, base + 2 * D, D3, min(L, LP));
    typename E::Frag qf[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) qf[ks] = gload8<E>(base + (size_t)qme * D3 + 32 * ks + 8 * fg, qme < L);
    const float c2 = scale * LOG2E;
    float m = -INFINITY, sum = 0.f;
    f32x4 o[HD / 16];
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nch = (L + LP - 1) / LP;
    for (int ch = 0; ch < nch; ++ch) {
        const int c0 = ch * LP, Lc = min(LP, L - c0);
        if (ch) __syncthreads();                               // every wave is done with the previous chunk
        rows_store<E, LNW>(Ks, fk);
        rows_store<E, LNW>(Vs, fv);
        __syncthreads();
        if (ch + 1 < nch) {
            const int n1 = min(LP, L - c0 - LP);
            rows_fetch<E, LNW>(fk, base + (size_t)(c0 + LP) * D3 + D, D3, n1);
            rows_fetch<E, LNW>(fv, base + (size_t)(c0 + LP) * D3 + 2 * D, D3, n1);
        }
        // s[kt][i] = S[q = q0 + fr][key = c0 + 16 kt + 4 fg + i]; keys past the chunk's end masked
        const int nkt = (Lc + 15) >> 4;
        // (all products first, then the mask and the maximum: the LP kernel's order -- reading each tile's maximum
        // right behind its MFMA pair measured wrong maxima on gfx950 for some query lanes)
        f32x4 s[NKT];
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt) {
            s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (kt < nkt) {
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) s[kt] = mma(lds_rowfrag<E>(Ks, 16 * kt + fr, 32 * ks + 8 * fg), qf[ks], s[kt]);
            }
        }
        float mc = -INFINITY;
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt) {
            if (kt < nkt) {
                if (kt == nkt - 1) {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if (16 * kt + 4 * fg + i >= Lc) s[kt][i] = -INFINITY;
                }
                mc = fmaxf(mc, fmaxf(fmaxf(s[kt][0], s[kt][1]), fmaxf(s[kt][2], s[kt][3])));
            }
        }
        mc = fmaxf(mc, __shfl_xor(mc, 16, 64));
        mc = fmaxf(mc, __shfl_xor(mc, 32, 64));
        const float mn = fmaxf(m, mc);
        const float alpha = __builtin_amdgcn_exp2f((m - mn) * c2);   // first chunk: 2^-inf = 0
        const float mcn = mn * c2;
        float cs = 0.f;
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt) {
            if (kt < nkt) {
#pragma unroll
                for (int i = 0; i < 4; ++i) { s[kt][i] = __builtin_amdgcn_exp2f(fmaf(s[kt][i], c2, -mcn)); cs += s[kt][i]; }
            }
        }
        cs += __shfl_xor(cs, 16, 64);
        cs += __shfl_xor(cs, 32, 64);
        sum = sum * alpha + cs;
        m = mn;
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt)
#pragma unroll
            for (int i = 0; i < 4; ++i) o[dt][i] *= alpha;
#pragma unroll
        for (int st = 0; st < NKT / 2; ++st) {
            if (2 * st >= nkt) continue;
            const float pv[8] = {s[2 * st][0], s[2 * st][1], s[2 * st][2], s[2 * st][3],
                                 s[2 * st + 1][0], s[2 * st + 1][1], s[2 * st + 1][2], s[2 * st + 1][3]};
            const typename E::Frag pf = pack8<E>(pv);
#pragma unroll
            for (int dt = 0; dt < HD / 16; ++dt) o[dt] = mma(attn_colfrag<E>(Vs, 32 * st, 16 * dt), pf, o[dt]);
        }
    }
    // o[dt][i] = O[q = q0 + fr][d = 16 dt + 4 fg + i]
    if (qme < L) {
        const float inv = 1.0f / sum;
        T* orow = out + ((size_t)b * L + qme) * D + h * HD + 4 * fg;
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt)
            store4<E>(orow + 16 * dt, o[dt][0] * inv, o[dt][1] * inv, o[dt][2] * inv, o[dt][3] * inv);
        if (fg == 0 && lse) lse[((size_t)b * H + h) * L + qme] = m * scale + logf(sum);   // natural-log units
    }
}

template <class E>
__global__ __launch_bounds__(64 * LNW) void attn_bwd_dq_long_kernel(const typename E::T* __restrict__ qkv,
                                                                   const typename E::T* __restrict__ dout,
                                                                   const typename E::T* __restrict__ out,
                                                                   const float* __restrict__ lse, float* __restrict__ delta,
                                                                   typename E::T* __restrict__ dqkv, int B, int L, int H,
                                                                   float scale)
{
    using T = typename E::T;
    using C = AttnCfg<E>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* Ks = reinterpret_cast<T*>(smem);
    T* Vs = reinterpret_cast<T*>(smem + C::TILE_BYTES);
    constexpr int QB = 16 * LNW;
    const int nqb = (L + QB - 1) / QB;
    const int bid = attn_block();
    const int bh = bid / nqb, qb = bid % nqb;
    const int b = bh / H, h = bh % H;
    const int D3 = 3 * H * HD, D = H * HD;
    const T* base = qkv + (size_t)b * L * D3 + h * HD;
    RowFetch<E, LNW> fk, fv;
    rows_fetch<E, LNW>(fk, base + D, D3, min(L, LP));
    rows_fetch<E, LNW>(fv, base + 2 * D, D3, min(L, LP));
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, fg = lane >> 4;
    const int q0 = qb * QB + w * 16, qme = q0 + fr;
    const bool qv = qme < L;
    typename E::Frag qf[2], df[2], of[2];
    const T* drow = dout + ((size_t)b * L + qme) * D + h * HD;
    const T* orow = out + ((size_t)b * L + qme) * D + h * HD;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
        qf[ks] = gload8<E>(base + (size_t)qme * D3 + 32 * ks + 8 * fg, qv);
        df[ks] = gload8<E>(drow + 32 * ks + 8 * fg, qv);
        of[ks] = gload8<E>(orow + 32 * ks + 8 * fg, qv);
    }
    const float lq = qv ? lse[((size_t)b * H + h) * L + qme] : INFINITY;
    float dq;                                                  // delta = rowsum(dO * O), published for dK / dV
    {
        float dd = 0.f;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
            for (int j = 0; j < 8; ++j) dd = fmaf((float)df[ks][j], (float)of[ks][j], dd);
        }
        dd += __shfl_xor(dd, 16, 64);
        dd += __shfl_xor(dd, 32, 64);
        dq = qv ? dd : 0.f;
        if (fg == 0 && qv) delta[((size_t)b * H + h) * L + qme] = dd;
    }
    const float c2 = scale * LOG2E, lq2 = lq * LOG2E;
    f32x4 dq_acc[HD / 16];
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) dq_acc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nch = (L + LP - 1) / LP;
    for (int ch = 0; ch < nch; ++ch) {
        const int c0 = ch * LP, Lc = min(LP, L - c0);
        if (ch) __syncthreads();
        rows_store<E, LNW>(Ks, fk);
        rows_store<E, LNW>(Vs, fv);
        __syncthreads();
        if (ch + 1 < nch) {
            const int n1 = min(LP, L - c0 - LP);
            rows_fetch<E, LNW>(fk, base + (size_t)(c0 + LP) * D3 + D, D3, n1);
            rows_fetch<E, LNW>(fv, base + (size_t)(c0 + LP) * D3 + 2 * D, D3, n1);
        }
        const int nkt = (Lc + 15) >> 4;
#pragma unroll
        for (int st = 0; st < NKT / 2; ++st) {
            if (2 * st >= nkt) continue;
            float ds[8];
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
                const int kt = 2 * st + hf;
                if (kt >= nkt) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) ds[4 * hf + i] = 0.f;
                    continue;
                }
                f32x4 sv = f32x4{0.f, 0.f, 0.f, 0.f}, pv = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
                    sv = mma(lds_rowfrag<E>(Ks, 16 * kt + fr, 32 * ks + 8 * fg), qf[ks], sv);
                    pv = mma(lds_rowfrag<E>(Vs, 16 * kt + fr, 32 * ks + 8 * fg), df[ks], pv);
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float p = __builtin_amdgcn_exp2f(fmaf(sv[i], c2, -lq2));
                    if (kt == nkt - 1 && 16 * kt + 4 * fg + i >= Lc) p = 0.f;
                    ds[4 * hf + i] = p * (pv[i] - dq);
                }
            }
            const typename E::Frag dsf = pack8<E>(ds);
#pragma unroll
            for (int dt = 0; dt < HD / 16; ++dt) dq_acc[dt] = mma(dsf, attn_colfrag<E>(Ks, 32 * st, 16 * dt), dq_acc[dt]);
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int q = q0 + 4 * fg + i;
        if (q < L) {
            T* row = dqkv + ((size_t)b * L + q) * D3 + h * HD;
#pragma unroll
            for (int dt = 0; dt < HD / 16; ++dt) row[16 * dt + fr] = E::from(dq_acc[dt][i] * scale);
        }
    }
}

template <class E>
__global__ __launch_bounds__(64 * LNW) void attn_bwd_dkv_long_kernel(const typename E::T* __restrict__ qkv,
                                                                    const typename E::T* __restrict__ dout,
                                                                    const float* __restrict__ lse,
                                                                    const float* __restrict__ delta,
                                                                    typename E::T* __restrict__ dqkv, int B, int L, int H,
                                                                    float scale)
{
    using T = typename E::T;
    using C = AttnCfg<E>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* Qs = reinterpret_cast<T*>(smem);
    T* Ds = reinterpret_cast<T*>(smem + C::TILE_BYTES);
    float* ls = reinterpret_cast<float*>(smem + 2 * C::TILE_BYTES);
    float* dl = ls + LP;
    constexpr int QB = 16 * LNW;
    const int nkb = (L + QB - 1) / QB;
    const int bid = attn_block();
    const int bh = bid / nkb, kb = bid % nkb;
    const int b = bh / H, h = bh % H;
    const int D3 = 3 * H * HD, D = H * HD;
    const T* base = qkv + (size_t)b * L * D3 + h * HD;
    const T* dob = dout + (size_t)b * L * D + h * HD;
    const float* lrow = lse + ((size_t)b * H + h) * L;
    const float* drw = delta + ((size_t)b * H + h) * L;
    RowFetch<E, LNW> fq, fd;
    rows_fetch<E, LNW>(fq, base, D3, min(L, LP));
    rows_fetch<E, LNW>(fd, dob, D, min(L, LP));
    const int t = threadIdx.x;
    // this thread's lse (pre-scaled by log2 e) and delta of chunk row t; padding rows: p = 0
    float lsv = INFINITY, dlv = 0.f;
    if (t < LP && t < L) { lsv = lrow[t] * LOG2E; dlv = drw[t]; }
    const int lane = t & 63, w = t >> 6, fr = lane & 15, fg = lane >> 4;
    const int k0 = kb * QB + w * 16, kme = k0 + fr;
    const bool kv = kme < L;
    typename E::Frag kf[2], vf[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
        kf[ks] = gload8<E>(base + (size_t)kme * D3 + D + 32 * ks + 8 * fg, kv);
        vf[ks] = gload8<E>(base + (size_t)kme * D3 + 2 * D + 32 * ks + 8 * fg, kv);
    }
    const float c2 = scale * LOG2E;
    f32x4 dk[HD / 16], dv[HD / 16];
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) { dk[dt] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[dt] = f32x4{0.f, 0.f, 0.f, 0.f}; }
    const int nch = (L + LP - 1) / LP;
    for (int ch = 0; ch < nch; ++ch) {
        const int c0 = ch * LP, Lc = min(LP, L - c0);
        if (ch) __syncthreads();
        rows_store<E, LNW>(Qs, fq);
        rows_store<E, LNW>(Ds, fd);
        if (t < LP) { ls[t] = lsv; dl[t] = dlv; }
        __syncthreads();
        if (ch + 1 < nch) {
            const int c1 = c0 + LP, n1 = min(LP, L - c1);
            rows_fetch<E, LNW>(fq, base + (size_t)c1 * D3, D3, n1);
            rows_fetch<E, LNW>(fd, dob + (size_t)c1 * D, D, n1);
            lsv = INFINITY; dlv = 0.f;
            if (t < n1) { lsv = lrow[c1 + t] * LOG2E; dlv = drw[c1 + t]; }
        }
        const int nqt = (Lc + 15) >> 4;                        // query rows past the chunk's end: lse = +inf, p = 0
#pragma unroll 2
        for (int st = 0; st < NKT / 2; ++st) {
            if (2 * st >= nqt) break;
            float pp[8], ds[8];
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
                const int qt = 2 * st + hf;
                f32x4 sv = f32x4{0.f, 0.f, 0.f, 0.f}, pv = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
                    sv = mma(lds_rowfrag<E>(Qs, 16 * qt + fr, 32 * ks + 8 * fg), kf[ks], sv);   // S^T[q][key]
                    pv = mma(lds_rowfrag<E>(Ds, 16 * qt + fr, 32 * ks + 8 * fg), vf[ks], pv);   // dP^T[q][key]
                }
                const float4 l4 = *reinterpret_cast<const float4*>(ls + 16 * qt + 4 * fg);
                const float4 d4 = *reinterpret_cast<const float4*>(dl + 16 * qt + 4 * fg);
                const float lq[4] = {l4.x, l4.y, l4.z, l4.w}, dq[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float p = __builtin_amdgcn_exp2f(fmaf(sv[i], c2, -lq[i]));
                    pp[4 * hf + i] = p;
                    ds[4 * hf + i] = p * (pv[i] - dq[i]);
                }
            }
            const typename E::Frag pf = pack8<E>(pp), dsf = pack8<E>(ds);
#pragma unroll
            for (int dt = 0; dt < HD / 16; ++dt) {
                dv[dt] = mma(pf, attn_colfrag<E>(Ds, 32 * st, 16 * dt), dv[dt]);
                dk[dt] = mma(dsf, attn_colfrag<E>(Qs, 32 * st, 16 * dt), dk[dt]);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int key = k0 + 4 * fg + i;
        if (key < L) {
            T* row = dqkv + ((size_t)b * L + key) * D3 + h * HD;
#pragma unroll
            for (int dt = 0; dt < HD / 16; ++dt) {
                row[D + 16 * dt + fr] = E::from(dk[dt][i] * scale);
                row[2 * D + 16 * dt + fr] = E::from(dv[dt][i]);
            }
        }
    }
}

template <class E> int attn_fwd_long(const void* qkv, void* out, float* lse, int B, int L, int H, hipStream_t st)
{
    using C = AttnCfg<E>;
    const size_t lds = 2 * C::TILE_BYTES;
    if (!ensure_lds<attn_fwd_long_kernel<E>>((int)lds, st)) return EBC_E_LAUNCH;
    const int grid = B * H * ((L + 16 * LNW - 1) / (16 * LNW));
    hipLaunchKernelGGL((attn_fwd_long_kernel<E>), dim3(grid), dim3(64 * LNW), lds, st, (const typename E::T*)qkv,
                       (typename E::T*)out, lse, B, L, H, 0.125f);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

template <class E> int attn_bwd_long(const void* qkv, const void* dout, const void* out, const float* lse, float* delta,
                                     void* dqkv, int B, int L, int H, hipStream_t st)
{
    using C = AttnCfg<E>;
    const size_t lds_dq = 2 * C::TILE_BYTES, lds_kv = 2 * C::TILE_BYTES + 2 * LP * sizeof(float);
    if (!ensure_lds<attn_bwd_dq_long_kernel<E>>((int)lds_dq, st) || !ensure_lds<attn_bwd_dkv_long_kernel<E>>((int)lds_kv, st))
        return EBC_E_LAUNCH;
    const int grid = B * H * ((L + 16 * LNW - 1) / (16 * LNW));
    hipLaunchKernelGGL((attn_bwd_dq_long_kernel<E>), dim3(grid), dim3(64 * LNW), lds_dq, st, (const typename E::T*)qkv,
                       (const typename E::T*)dout, (const typename E::T*)out, lse, delta, (typename E::T*)dqkv, B, L, H,
                       0.125f);
    EBC_CHECK_LAUNCH();
    hipLaunchKernelGGL((attn_bwd_dkv_long_kernel<E>), dim3(grid), dim3(64 * LNW), lds_kv, st, (const typename E::T*)qkv,
                       (const typename E::T*)dout, lse, (const float*)delta, (typename E::T*)dqkv, B, L, H, 0.125f);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

// 16 waves (one workgroup per (crop, head), K / V staged once) while the (crop, head) units fit one pass of the 256 CUs;
// with more units (32 crops: 384, 1.5 passes of 16-wave workgroups, one a CU) the forward takes 8-wave workgroups of
// 128 queries, two a CU (768 halves: 1.5 passes of the 512 slots, each half half the work)
constexpr int ATTN_CUS = 256;
int attn_waves(int L) { return L > 128 ? 16 : 8; }

// Weight touch mode (ebc_set_weight_touch): 1 (default) in the attention kernels, 0 off.  (r05 measured a third mode, a
// touch kernel on a side stream whose workgroups reserve enough LDS to land only on the 64 CUs a 16-crop attention
// launch leaves idle: 4.58 ms a step against 4.39 in-kernel and 4.55 with no touch, same box -- the fork / join events
// around 24 launches a step cost more than the touch; removed.)
int g_touch_mode = 1;
int attn_fwd_waves(int B, int L, int H) { return attn_waves(L) == 16 && B * H <= ATTN_CUS ? 16 : 8; }

// the CLIP ViT-B/16 + 32-prompt sequence (1 + 32 + 196 tokens) gets kernels compiled for it
constexpr int L_VPT32 = 229;

template <class E, int NW, int LFIX, int QT = 1> int attn_fwd_nw(const void* qkv, void* out, float* lse, int B, int L, int H,
                                                                hipStream_t st, const TouchList* touch = nullptr)
{
    using C = AttnCfg<E>;
    const size_t lds = 2 * C::TILE_BYTES;
    if (!ensure_lds<attn_fwd_kernel<E, NW, LFIX, QT>>((int)lds, st)) return EBC_E_LAUNCH;
    const int grid = B * H * ((L + 16 * NW * QT - 1) / (16 * NW * QT));
    const TouchList t = touch && g_touch_mode == 1 ? *touch : TouchList{};
    const int pi = probe_on() ? probe_start(EBC_PROBE_ATTN_FWD, 0, 0, 0, 0, B, L, H, st) : -1;
    hipLaunchKernelGGL((attn_fwd_kernel<E, NW, LFIX, QT>), dim3(grid), dim3(64 * NW), lds, st, (const typename E::T*)qkv,
                       (typename E::T*)out, lse, B, L, H, 0.125f, t);
    probe_stop(pi, st);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}
template <class E> int attn_fwd_t(const void* qkv, void* out, float* lse, int B, int L, int H, hipStream_t st,
                                  const TouchList* touch)
{
    if (attn_fwd_waves(B, L, H) == 16)
        return L == L_VPT32 ? attn_fwd_nw<E, 16, L_VPT32>(qkv, out, lse, B, L, H, st, touch)
                            : attn_fwd_nw<E, 16, 0>(qkv, out, lse, B, L, H, st, touch);
    return L == L_VPT32 ? attn_fwd_nw<E, 8, L_VPT32>(qkv, out, lse, B, L, H, st, touch)
                        : attn_fwd_nw<E, 8, 0>(qkv, out, lse, B, L, H, st, touch);
}

template <class E, int NW, int LFIX> int attn_bwd_nw(const void* qkv, const void* dout, const void* out, const float* lse,
                                                     float* delta, void* dqkv, int B, int L, int H, hipStream_t st)
{
    using C = AttnCfg<E>;
    const size_t lds_dq = 2 * C::TILE_BYTES, lds_kv = 2 * C::TILE_BYTES + 2 * LP * sizeof(float);
    if (!ensure_lds<attn_bwd_dq_kernel<E, NW, LFIX>>((int)lds_dq, st) || !ensure_lds<attn_bwd_dkv_kernel<E, NW, LFIX>>((int)lds_kv, st))
        return EBC_E_LAUNCH;
    const int grid = B * H * ((L + 16 * NW - 1) / (16 * NW));
    int pi = probe_on() ? probe_start(EBC_PROBE_ATTN_BWD_DQ, 0, 0, 0, 0, B, L, H, st) : -1;
    hipLaunchKernelGGL((attn_bwd_dq_kernel<E, NW, LFIX>), dim3(grid), dim3(64 * NW), lds_dq, st, (const typename E::T*)qkv,
                       (const typename E::T*)dout, (const typename E::T*)out, lse, delta, (typename E::T*)dqkv, B, L, H,
                       0.125f);
    probe_stop(pi, st);
    EBC_CHECK_LAUNCH();
    pi = probe_on() ? probe_start(EBC_PROBE_ATTN_BWD_DKV, 0, 0, 0, 0, B, L, H, st) : -1;
    hipLaunchKernelGGL((attn_bwd_dkv_kernel<E, NW, LFIX>), dim3(grid), dim3(64 * NW), lds_kv, st, (const typename E::T*)qkv,
                       (const typename E::T*)dout, lse, delta, (typename E::T*)dqkv, B, L, H, 0.125f);
    probe_stop(pi, st);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}
template <class E, int LFIX> int attn_bwd_one(const void* qkv, const void* dout, const void* out, const float* lse,
                                              void* dqkv, int B, int L, int H, hipStream_t st, int rows, const TouchList* touch)
{
    using C = AttnCfg<E>;
    const size_t lds = 4 * C::TILE_BYTES + 2 * LP * sizeof(float);
    if (!ensure_lds<attn_bwd_one_kernel<E, LFIX>>((int)lds, st)) return EBC_E_LAUNCH;
    const TouchList t = touch && g_touch_mode == 1 ? *touch : TouchList{};
    const int pi = probe_on() ? probe_start(EBC_PROBE_ATTN_BWD_DQ, 1, 0, 0, 0, B, L, H, st) : -1;
    hipLaunchKernelGGL((attn_bwd_one_kernel<E, LFIX>), dim3(B * H), dim3(1024), lds, st, (const typename E::T*)qkv,
                       (const typename E::T*)dout, (const typename E::T*)out, lse, (typename E::T*)dqkv, B, L, H, 0.125f,
                       rows, t);
    probe_stop(pi, st);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

// 16-bit backward: one workgroup per (crop, head) (r03: the two-role grid of 8-wave dQ and dK/dV workgroups fetched
// 2.2x the bytes and ran 388 vs 367 us per step); f32 (parity mode): the dQ and dK/dV kernels one after the other

template <class E> int attn_bwd_t(const void* qkv, const void* dout, const void* out, const float* lse, float* delta,
                                  void* dqkv, int B, int L, int H, hipStream_t st, int rows, const TouchList* touch)
{
    if constexpr (E::BYTES == 2) {
        return L == L_VPT32 ? attn_bwd_one<E, L_VPT32>(qkv, dout, out, lse, dqkv, B, L, H, st, rows, touch)
                            : attn_bwd_one<E, 0>(qkv, dout, out, lse, dqkv, B, L, H, st, rows, touch);
    }
    if (attn_waves(L) == 16)
        return L == L_VPT32 ? attn_bwd_nw<E, 16, L_VPT32>(qkv, dout, out, lse, delta, dqkv, B, L, H, st)
                            : attn_bwd_nw<E, 16, 0>(qkv, dout, out, lse, delta, dqkv, B, L, H, st);
    return attn_bwd_nw<E, 8, 0>(qkv, dout, out, lse, delta, dqkv, B, L, H, st);
}

}  // namespace

namespace ebc {
bool touch_enabled() { return g_touch_mode == 1; }
}  // namespace ebc

extern "C" int ebc_set_weight_touch(int mode)
{
    if (mode < 0 || mode > 1) return EBC_E_ARG;
    g_touch_mode = mode;
    return EBC_OK;
}

namespace ebc {
int attention_fwd(int dtype, const void* qkv, void* out, float* lse, int B, int L, int H, hipStream_t st,
                  const TouchList* touch)
{
    if (L <= 0 || L > L_MAX || B <= 0 || H <= 0) return EBC_E_UNSUPPORTED;
    if (L > LP) {                                  // K / V streamed through LDS in chunks (no weight touch)
        switch (dtype) {
            case EBC_F32: return attn_fwd_long<EF32>(qkv, out, lse, B, L, H, st);
            case EBC_F16: return attn_fwd_long<EF16>(qkv, out, lse, B, L, H, st);
            case EBC_BF16: return attn_fwd_long<EBF16>(qkv, out, lse, B, L, H, st);
        }
        return EBC_E_ARG;
    }
    switch (dtype) {
        case EBC_F32: return attn_fwd_t<EF32>(qkv, out, lse, B, L, H, st, nullptr);
        case EBC_F16: return attn_fwd_t<EF16>(qkv, out, lse, B, L, H, st, touch);
        case EBC_BF16: return attn_fwd_t<EBF16>(qkv, out, lse, B, L, H, st, touch);
    }
    return EBC_E_ARG;
}
int attention_bwd(int dtype, const void* qkv, const void* dout, const void* out, const float* lse, float* delta,
                  void* dqkv, int B, int L, int H, hipStream_t st, int rows, const TouchList* touch)
{
    if (L <= 0 || L > L_MAX || B <= 0 || H <= 0 || rows < 0) return EBC_E_UNSUPPORTED;
    if (L > LP) {                                  // the two-role chunked pair; rows > 0 computes every row (a superset)
        if (!delta || !lse) return EBC_E_ARG;
        switch (dtype) {
            case EBC_F32: return attn_bwd_long<EF32>(qkv, dout, out, lse, delta, dqkv, B, L, H, st);
            case EBC_F16: return attn_bwd_long<EF16>(qkv, dout, out, lse, delta, dqkv, B, L, H, st);
            case EBC_BF16: return attn_bwd_long<EBF16>(qkv, dout, out, lse, delta, dqkv, B, L, H, st);
        }
        return EBC_E_ARG;
    }
    switch (dtype) {
        case EBC_F32: return attn_bwd_t<EF32>(qkv, dout, out, lse, delta, dqkv, B, L, H, st, rows, nullptr);
        case EBC_F16: return attn_bwd_t<EF16>(qkv, dout, out, lse, delta, dqkv, B, L, H, st, rows, touch);
        case EBC_BF16: return attn_bwd_t<EBF16>(qkv, dout, out, lse, delta, dqkv, B, L, H, st, rows, touch);
    }
    return EBC_E_ARG;
}
}  // namespace ebc
