// Host-side orchestration of the CLIP ViT-B/16 + deep-VPT encoder (forward, and dX-only backward
// with the per-layer VPT gradients), plus the C-ABI wrappers of the individual kernels.
//
// Reference: CLIP_EBC._forward_vpt   models/clip/model.py:142-189
//            ResidualAttentionBlock  models/clip/_clip/blocks.py:22-42
//
// Layout in HBM (M = B * L rows, L = 1 + NV + G tokens, row-major [B][L][768]):
//   X_l   f32 [M,768]  residual stream entering block l (rows 1..NV hold vpt_l)   l = 0..layers
//   X1_l  f32 [M,768]  after the attention half of block l
//   QKV_l T   [M,2304] packed in-projection output,  O_l T [M,768] attention output
//   A_l   T   [M,3072] MLP pre-activation (for QuickGELU')
//   mean/rstd of ln_1, ln_2 per row; lse_l [B,H,L] softmax log-normalisers
// The persistent [B, L, 768] buffer replaces the reference's 24 torch.cat per step: VPT rows are
// overwritten in place before each block (and their gradient rows reduced + zeroed in backward).
#include <vector>

#include <algorithm>

#include "ebc_common.h"
#include "kernels.h"


namespace {

constexpr int WIDTH = 768, HEADS = 12, MLP = 3072, QKVW = 3 * WIDTH;

inline size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

struct Carver {
    char* base; size_t off = 0; bool dry;
    Carver(void* b, bool d) : base((char*)b), dry(d) {}
    template <class P> P* take(size_t bytes) {
        P* p = dry ? nullptr : reinterpret_cast<P*>(base + off);
        off += align_up(bytes);
        return p;
    }
};

struct LayerSave {
    float *X1, *m1, *r1, *m2, *r2, *lse;
    void *QKV, *O, *A;
};

struct Layout {
    std::vector<float*> X;          // layers + 1
    std::vector<LayerSave> s;       // layers
    void *H, *G, *patch_t;          // transient
    float *patch_f, *mpost, *rpost;
    // backward transients
    float *dXa, *dXb, *delta;
    float* vpt_rows;                // [layers][B][NV][768] per-crop prompt gradients (summed over crops at the end)
    void *dXt, *dH, *dA, *dO, *dQKV;
    float* rpart;                   // LayerNorm folding: [M][parts][2] row partials (sum, sum of squares) of X1 / X_l+1
    int parts_out, parts_proj;      //   written by the out-proj / c_proj residual products (gemm_rowstat_parts)
    float* bpart;                   // LayerNorm-backward folding: [M][parts_gelu][2] partials of the GELU' products
    int parts_gelu;
    void* gws;                      // split-K GEMM workspace (leading counter block zeroed per call)
    size_t gws_bytes;
    size_t bytes;
};

Layout carve(void* ws, int B, int L, int G, int layers, int dtype, int training)
{
    const size_t M = (size_t)B * L;
    const size_t es = dtype == EBC_F32 ? 4 : 2;
    Carver c(ws, ws == nullptr);
    Layout lay;
    const int nsave = training ? layers : 1;
    lay.X.resize(layers + 1);
    for (int l = 0; l <= layers; ++l)
        lay.X[l] = (training || l < 2) ? c.take<float>(M * WIDTH * 4) : lay.X[l & 1];
    if (!training) for (int l = 2; l <= layers; ++l) lay.X[l] = lay.X[l & 1];
    lay.s.resize(layers);
    for (int l = 0; l < layers; ++l) {
        LayerSave& s = lay.s[l];
        if (l < nsave) {
            s.X1 = c.take<float>(M * WIDTH * 4);
            s.m1 = c.take<float>(M * 4); s.r1 = c.take<float>(M * 4);
            s.m2 = c.take<float>(M * 4); s.r2 = c.take<float>(M * 4);
            s.lse = c.take<float>((size_t)B * HEADS * L * 4);
            s.QKV = c.take<void>(M * QKVW * es);
            s.O = c.take<void>(M * WIDTH * es);
            s.A = c.take<void>(M * MLP * es);
        } else {
            s = lay.s[0];
        }
    }
    lay.H = c.take<void>(M * WIDTH * es);
    lay.G = c.take<void>(M * MLP * es);
    lay.patch_t = c.take<void>((size_t)B * G * WIDTH * es);
    lay.patch_f = c.take<float>((size_t)B * G * WIDTH * 4);
    lay.mpost = c.take<float>((size_t)B * G * 4);
    lay.rpost = c.take<float>((size_t)B * G * 4);
    if (training) {
        lay.dXa = c.take<float>(M * WIDTH * 4);
        lay.dXb = c.take<float>(M * WIDTH * 4);
        lay.delta = c.take<float>((size_t)B * HEADS * L * 4);
        lay.dXt = c.take<void>(M * WIDTH * es);
        lay.dH = c.take<void>(M * WIDTH * es);
        lay.dA = c.take<void>(M * MLP * es);
        lay.dO = c.take<void>(M * WIDTH * es);
        lay.dQKV = c.take<void>(M * QKVW * es);
        const int NV = L - 1 - G;
        lay.vpt_rows = NV > 0 ? c.take<float>((size_t)layers * B * NV * WIDTH * 4) : nullptr;
    } else {
        lay.vpt_rows = nullptr;
        lay.dXa = lay.dXb = lay.delta = nullptr;
        lay.dXt = lay.dH = lay.dA = lay.dO = lay.dQKV = nullptr;
    }
    lay.bpart = nullptr;
    lay.parts_gelu = 0;
    if (dtype != EBC_F32 && training) {
        lay.parts_gelu = ebc::gemm_rowstat_parts(dtype, (int)M, MLP, WIDTH);
        if (lay.parts_gelu <= ebc::GEMM_LN_PMAX_B) lay.bpart = c.take<float>(M * lay.parts_gelu * 2 * 4);
    }
    if (dtype != EBC_F32) {
        lay.parts_out = ebc::gemm_rowstat_parts(dtype, (int)M, WIDTH, WIDTH);
        lay.parts_proj = ebc::gemm_rowstat_parts(dtype, (int)M, WIDTH, MLP);
        lay.rpart = c.take<float>(M * std::max(lay.parts_out, lay.parts_proj) * 2 * 4);
    } else {
        lay.parts_out = lay.parts_proj = 0;
        lay.rpart = nullptr;
    }
    // the largest split-K workspace any of the encoder GEMMs asks for
    size_t g = ebc::gemm_workspace_bytes(dtype, B * G, WIDTH, WIDTH);          // patch embedding
    const int Mi = (int)M;
    const int shapes[][2] = {{QKVW, WIDTH}, {WIDTH, WIDTH}, {MLP, WIDTH}, {WIDTH, MLP}, {WIDTH, QKVW}};
    for (const auto& sh : shapes) g = std::max(g, ebc::gemm_workspace_bytes(dtype, Mi, sh[0], sh[1]));
    lay.gws_bytes = g;
    lay.gws = g ? c.take<void>(g) : nullptr;
    lay.bytes = c.off;
    return lay;
}

bool check_weights(const EbcVitWeights* w) {
    return w && w->layers > 0 && w->layer && w->width == WIDTH && w->heads == HEADS && w->patch == 16 && w->num_vpt >= 0;
}

}  // namespace

extern "C" size_t ebc_vit_workspace_bytes(int B, int H, int W, int layers, int num_vpt, int dtype, int training)
{
    const int G = (H / 16) * (W / 16), L = 1 + num_vpt + G;
    return carve(nullptr, B, L, G, layers, dtype, training).bytes;
}

extern "C" int ebc_vit_forward(const EbcVitWeights* w, const float* image, int B, int H, int W,
                               const float* const* vpt, long vpt_bstride, int dtype, int training,
                               void* ws, size_t ws_bytes, float* feat, ebc_stream_t stream)
{
    if (!check_weights(w) || !image || !ws || !feat || B <= 0 || H % 16 || W % 16) return EBC_E_ARG;
    hipStream_t st = (hipStream_t)stream;
    const int NV = w->num_vpt, G = (H / 16) * (W / 16), L = 1 + NV + G, layers = w->layers;
    if (L > 16384) return EBC_E_UNSUPPORTED;                 // attention.hip L_MAX
    Layout lay = carve(ws, B, L, G, layers, dtype, training);
    if (lay.bytes > ws_bytes) return EBC_E_ARG;
    if (NV > 0 && (!vpt || !vpt[0])) return EBC_E_ARG;
    if (lay.gws && hipMemsetAsync(lay.gws, 0, std::min<size_t>(lay.gws_bytes, 16 * 1024), st) != hipSuccess)
        return EBC_E_LAUNCH;
    auto gemm = [&](int epi, int out_f32, const void* A, const void* Bm, void* C, const float* bias, const float* resid,
                    void* aux, int m, int n, int k) {
        return ebc::gemm_nt(dtype, epi, out_f32, A, Bm, C, bias, resid, aux, m, n, k, st, lay.gws, lay.gws_bytes);
    };

    // patch embedding: im2col + GEMM with conv1 weight [768, 3*16*16] (image_encoder.py:141)
    EBC_TRY(ebc::im2col(dtype, image, lay.patch_t, B, H, W, 16, st));
    EBC_TRY(gemm(EBC_EPI_STORE, 1, lay.patch_t, w->w_patch, lay.patch_f, nullptr, nullptr, nullptr, B * G, WIDTH, WIDTH));
    // CLS + pos + ln_pre, VPT_0 rows (model.py:150-168)
    EBC_TRY(ebc::embed_tokens(lay.patch_f, w->cls, w->pos, w->ln_pre_g, w->ln_pre_b, NV ? vpt[0] : nullptr,
                              vpt_bstride, lay.X[0], B, L, G, NV, WIDTH, st));
    // one block on crops [b0, b0 + nb) (rows r0 = b0 * L of every [B][L][*] buffer) on stream sx
    const size_t es = dtype == EBC_F32 ? 4 : 2;
    // The frozen weights were last read a step ago (HBM).  Block l's attention reads onto the die (Infinity Cache) the
    // weights of the GEMMs after it -- its out-proj, c_fc and c_proj, and block l+1's QKV -- while it computes
    // (attention.hip touch_issue): those GEMMs then start with their B operand on-die.  16-bit path only.
    // LayerNorm folding (16-bit, every layer carrying the folded weights): ln_2 of every block and ln_1 of blocks
    // 1.. run inside the QKV / c_fc products' epilogues.  The residual products before them (out-proj; c_proj of the
    // block below) also write a compute-dtype copy of their output rows into H and per-row partial sums / sums of
    // squares into rpart; the product reads H as its A operand, the folded weight W diag(gamma) as B, and finishes
    // rstd * (acc - mean * W'.1) + b + W beta (gemm.hip EPI_LN), writing the row's mean / rstd for the backward.
    // Saves the two LayerNorm launches' read of X and write of H per block; the backward is unchanged.
    bool fold = dtype != EBC_F32 && lay.rpart && std::max(lay.parts_out, lay.parts_proj) <= ebc::GEMM_LN_PMAX;
    for (int l = 0; l < layers && fold; ++l) {
        const EbcVitLayer& p = w->layer[l];
        fold = p.w_qkv_ln && p.b_qkv_ln && p.s_qkv_ln && p.w_fc_ln && p.b_fc_ln && p.s_fc_ln;
    }
    auto touch_fwd = [&](int l) {
        ebc::TouchList t{};
        const EbcVitLayer& p = w->layer[l];
        t.add(p.w_out, (size_t)WIDTH * WIDTH * es);
        t.add(fold ? p.w_fc_ln : p.w_fc, (size_t)MLP * WIDTH * es);
        t.add(p.w_proj, (size_t)WIDTH * MLP * es);
        if (l + 1 < layers) t.add(fold ? w->layer[l + 1].w_qkv_ln : w->layer[l + 1].w_qkv, (size_t)QKVW * WIDTH * es);
        return t;
    };
    auto block = [&](int l, int b0, int nb, hipStream_t sx) -> int {
        const EbcVitLayer& p = w->layer[l];
        const LayerSave& s = lay.s[training ? l : 0];
        const size_t r0 = (size_t)b0 * L;
        const int m = nb * L;
        float* X = lay.X[l] + r0 * WIDTH;
        float* Xn = lay.X[l + 1] + r0 * WIDTH;
        float* X1 = s.X1 + r0 * WIDTH;
        char* QKV = (char*)s.QKV + r0 * QKVW * es;
        char* O = (char*)s.O + r0 * WIDTH * es;
        char* A = training ? (char*)s.A + r0 * MLP * es : nullptr;
        char* Hn = (char*)lay.H + r0 * WIDTH * es;
        char* Gm = (char*)lay.G + r0 * MLP * es;
        float* lse = s.lse + (size_t)b0 * HEADS * L;
        auto gemm = [&](int epi, int out_f32, const void* Am, const void* Bm, void* C, const float* bias,
                        const float* resid, void* aux, int n, int k) {
            return ebc::gemm_nt(dtype, epi, out_f32, Am, Bm, C, bias, resid, aux, m, n, k, sx, lay.gws, lay.gws_bytes);
        };
        auto gemm_ln = [&](int epi, int out_f32, const void* Am, const void* Bm, void* C, const float* bias,
                           const float* resid, void* aux, int n, int k, const ebc::GemmLn& ln) {
            return ebc::gemm_nt_ln(dtype, epi, out_f32, Am, Bm, C, bias, resid, aux, m, n, k, sx, lay.gws, lay.gws_bytes, ln);
        };
        // x = x + out_proj(attn(ln_1(x))); deep VPT: the prompt rows come from vpt_l (written into X)
        const bool vrows = l > 0 && NV > 0 && vpt[l];
        if (fold && l > 0) {
            // X_l's rows (the prompt rows already replaced by vpt_l), their H copy and partials came from block
            // l-1's c_proj
            ebc::GemmLn ln;
            ln.lnp = lay.rpart + r0 * lay.parts_proj * 2; ln.lnparts = lay.parts_proj; ln.lnw = p.s_qkv_ln;
            ln.mean = s.m1 + r0; ln.rstd = s.r1 + r0;
            EBC_TRY(gemm_ln(ebc::GEMM_EPI_LN, 0, Hn, p.w_qkv_ln, QKV, p.b_qkv_ln, nullptr, nullptr, QKVW, WIDTH, ln));
        } else {
            if (vrows)
                EBC_TRY(ebc::layernorm_fwd_vpt(dtype, X, vpt[l] + (size_t)b0 * vpt_bstride, vpt_bstride, L, NV, p.ln1_g,
                                               p.ln1_b, Hn, s.m1 + r0, s.r1 + r0, m, WIDTH, sx));
            else
                EBC_TRY(ebc::layernorm_fwd(dtype, X, 0, 0, 0, p.ln1_g, p.ln1_b, Hn, nullptr, s.m1 + r0, s.r1 + r0, m, WIDTH, sx));
            EBC_TRY(gemm(EBC_EPI_STORE, 0, Hn, p.w_qkv, QKV, p.b_qkv, nullptr, nullptr, QKVW, WIDTH));
        }
        const ebc::TouchList tl = touch_fwd(l);
        EBC_TRY(ebc::attention_fwd(dtype, QKV, O, lse, nb, L, HEADS, sx, &tl));
        // x = x + c_proj(QuickGELU(c_fc(ln_2(x))))
        if (fold) {
            ebc::GemmLn res;
            res.xh = Hn; res.rpart = lay.rpart + r0 * lay.parts_out * 2;
            EBC_TRY(gemm_ln(EBC_EPI_RESID, 1, O, p.w_out, X1, p.b_out, X, nullptr, WIDTH, WIDTH, res));
            ebc::GemmLn ln;
            ln.lnp = res.rpart; ln.lnparts = lay.parts_out; ln.lnw = p.s_fc_ln;
            ln.mean = s.m2 + r0; ln.rstd = s.r2 + r0;
            EBC_TRY(gemm_ln(ebc::GEMM_EPI_LN_GELU, 0, Hn, p.w_fc_ln, Gm, p.b_fc_ln, nullptr, A, MLP, WIDTH, ln));
        } else {
            EBC_TRY(gemm(EBC_EPI_RESID, 1, O, p.w_out, X1, p.b_out, X, nullptr, WIDTH, WIDTH));
            EBC_TRY(ebc::layernorm_fwd(dtype, X1, 0, 0, 0, p.ln2_g, p.ln2_b, Hn, nullptr, s.m2 + r0, s.r2 + r0, m, WIDTH, sx));
            EBC_TRY(gemm(EBC_EPI_GELU, 0, Hn, p.w_fc, Gm, p.b_fc, nullptr, A, MLP, WIDTH));
        }
        if (fold && l + 1 < layers) {
            ebc::GemmLn res;
            res.xh = Hn; res.rpart = lay.rpart + r0 * lay.parts_proj * 2;
            if (NV > 0 && vpt[l + 1]) {
                // deep VPT: block l+1's prompt rows written in place of this product's (copy, H rows and partials)
                res.vrep = vpt[l + 1] + (size_t)b0 * vpt_bstride; res.vrep_bs = vpt_bstride;
                res.vrep_L = L; res.vrep_nv = NV;
            }
            EBC_TRY(gemm_ln(EBC_EPI_RESID, 1, Gm, p.w_proj, Xn, p.b_proj, X1, nullptr, WIDTH, MLP, res));
        } else {
            EBC_TRY(gemm(EBC_EPI_RESID, 1, Gm, p.w_proj, Xn, p.b_proj, X1, nullptr, WIDTH, MLP));
        }
        return EBC_OK;
    };
    // (the two crop halves on two streams, overlapping one half's GEMM store phases with the other's main loops,
    // measured 2.9 % slower per train step, r01: the half-batch GEMMs lose more tile efficiency than the overlap wins)
    for (int l = 0; l < layers; ++l) EBC_TRY(block(l, 0, B, st));
    // ln_post on the patch rows only (CLS and prompt rows are dropped, model.py:185-188)
    EBC_TRY(ebc::layernorm_fwd(EBC_F32, lay.X[layers], G, L, 1 + NV, w->ln_post_g, w->ln_post_b, feat, nullptr,
                               lay.mpost, lay.rpost, B * G, WIDTH, st));
    return EBC_OK;
}

extern "C" int ebc_vit_backward(const EbcVitWeights* w, int B, int H, int W, int dtype, void* ws, size_t ws_bytes,
                                const float* dfeat, float* const* dvpt, long vpt_bstride, int flags, ebc_stream_t stream)
{
    if (!check_weights(w) || !ws || !dfeat) return EBC_E_ARG;
    hipStream_t st = (hipStream_t)stream;
    const int NV = w->num_vpt, G = (H / 16) * (W / 16), L = 1 + NV + G, layers = w->layers;
    const int M = B * L;
    Layout lay = carve(ws, B, L, G, layers, dtype, 1);
    if (lay.bytes > ws_bytes) return EBC_E_ARG;
    const int per_batch = vpt_bstride != 0;

    // ln_post backward into the patch rows of dX_L; CLS / prompt rows get zero gradient
    float* dX = lay.dXa;
    float* dXo = lay.dXb;
    if (lay.gws && hipMemsetAsync(lay.gws, 0, std::min<size_t>(lay.gws_bytes, 16 * 1024), st) != hipSuccess)
        return EBC_E_LAUNCH;
    auto gemm = [&](int epi, const void* A, const void* Bm, void* C, void* aux, int m, int n, int k) {
        return ebc::gemm_nt(dtype, epi, 0, A, Bm, C, nullptr, nullptr, aux, m, n, k, st, lay.gws, lay.gws_bytes);
    };
    // ln_2's backward folded into the c_fc dX product (16-bit, every layer carrying (W_fc')^T): the GELU' product also
    // writes, per row, the partial sums sum_k dA_k s_k and sum_k dA_k (A_k - c_k) over its columns (s = W_fc'.1, c = the
    // folded c_fc bias; A = the saved pre-activation = xhat W_fc'^T + c): these are sum_j g_j and sum_j g_j xhat_j of
    // ln_2's backward, g = dLN2 (.) gamma_2.  The c_fc dX product then multiplies by (W_fc')^T, so its accumulator IS g,
    // and finishes dX1 = dX + rstd (g - mean(g) - xhat mean(g xhat)) in its epilogue (gemm.hip EPI_LN_BWD): no dH write
    // and re-read, no LayerNorm launch.
    bool fold_b = dtype != EBC_F32 && lay.bpart && !(flags & EBC_VIT_BWD_NO_LN_FOLD) &&
                  ebc::gemm_ln_bwd_fold_pays(dtype, M, WIDTH, MLP);
    for (int l = 0; l < layers && fold_b; ++l) {
        const EbcVitLayer& p = w->layer[l];
        fold_b = p.wt_fc_ln && p.s_fc_ln && p.b_fc_ln;
    }
    // block l's attention backward reads onto the die the transposed weights of the dX products after it: its QKV dX
    // and block l-1's c_proj / c_fc / out-proj ones (see ebc_vit_forward)
    const size_t es = dtype == EBC_F32 ? 4 : 2;
    auto touch_bwd = [&](int l) {                  // l == layers: the last block's dX weights alone
        ebc::TouchList t{};
        if (l < layers) t.add(w->layer[l].wt_qkv, (size_t)WIDTH * QKVW * es);
        if (l > 0) {
            const EbcVitLayer& q = w->layer[l - 1];
            t.add(q.wt_proj, (size_t)MLP * WIDTH * es);
            t.add(fold_b ? q.wt_fc_ln : q.wt_fc, (size_t)WIDTH * MLP * es);
            t.add(q.wt_out, (size_t)WIDTH * WIDTH * es);
        }
        return t;
    };
    // (the CLS / prompt rows of dX, dXt are written as zeros by the same launch: no memsets); it reads onto the die
    // the last block's c_proj / c_fc / out-proj dX weights, which no attention backward precedes
    const ebc::TouchList tl_top = touch_bwd(layers);
    EBC_TRY(ebc::layernorm_bwd_fill(dtype, dfeat, lay.X[layers], G, L, 1 + NV, lay.mpost, lay.rpost, w->ln_post_g, dX,
                                    lay.dXt, B * G, WIDTH, st, dtype != EBC_F32 ? &tl_top : nullptr));
    for (int l = layers - 1; l >= 0; --l) {
        const EbcVitLayer& p = w->layer[l];
        LayerSave& s = lay.s[l];
        const ebc::TouchList tl = touch_bwd(l);
        // MLP half: dA = (dX . W_proj) * QuickGELU'(A);  dH2 = dA . W_fc;  dX1 = dX + LN2'(dH2)
        if (fold_b) {
            ebc::GemmLn gb;
            gb.bpart = lay.bpart; gb.lnb_s = p.s_fc_ln; gb.lnb_c = p.b_fc_ln;
            EBC_TRY(ebc::gemm_nt_ln(dtype, EBC_EPI_GELU_BWD, 0, lay.dXt, p.wt_proj, lay.dA, nullptr, nullptr, s.A, M, MLP,
                                    WIDTH, st, lay.gws, lay.gws_bytes, gb));
            ebc::GemmLn lb;
            lb.xh = lay.dXt; lb.lnx = s.X1; lb.lnp = lay.bpart; lb.lnparts = lay.parts_gelu; lb.mean = s.m2; lb.rstd = s.r2;
            EBC_TRY(ebc::gemm_nt_ln(dtype, ebc::GEMM_EPI_LN_BWD, 1, lay.dA, p.wt_fc_ln, dXo, nullptr, dX, nullptr, M, WIDTH,
                                    MLP, st, lay.gws, lay.gws_bytes, lb));
        } else {
            EBC_TRY(gemm(EBC_EPI_GELU_BWD, lay.dXt, p.wt_proj, lay.dA, s.A, M, MLP, WIDTH));
            EBC_TRY(gemm(EBC_EPI_STORE, lay.dA, p.wt_fc, lay.dH, nullptr, M, WIDTH, MLP));
            EBC_TRY(ebc::layernorm_bwd(dtype, 0, lay.dH, s.X1, 0, 0, 0, s.m2, s.r2, p.ln2_g, dX, dXo, lay.dXt, M, WIDTH, st));
        }
        { float* t = dX; dX = dXo; dXo = t; }
        // attention half: dO = dX1 . W_out;  dQKV = attn'(...);  dH = dQKV . W_qkv;  dX = dX1 + LN1'(dH)
        EBC_TRY(gemm(EBC_EPI_STORE, lay.dXt, p.wt_out, lay.dO, nullptr, M, WIDTH, WIDTH));
        if (l == 0 && NV > 0 && dvpt && dvpt[0] && !(flags & EBC_VIT_BWD_FULL_LAYER0)) {
            // layer 0: the frozen encoder below (ln_pre, embeddings, conv1) takes no gradient, so only the prompt
            // rows' input gradient is wanted -- dQ / dK / dV of the first query and key block (rows 1..NV), dH on
            // the B*NV prompt rows (row-mapped A operand), ln_1's backward of those rows straight into the prompt
            // rows (same values as the full backward's rows: every kept element is summed in the same order)
            EBC_TRY(ebc::attention_bwd(dtype, s.QKV, lay.dO, s.O, s.lse, lay.delta, lay.dQKV, B, L, HEADS, st, 1 + NV, &tl));
            EBC_TRY(ebc::gemm_nt(dtype, EBC_EPI_STORE, 0, lay.dQKV, p.wt_qkv, lay.dH, nullptr, nullptr, nullptr, B * NV,
                                 WIDTH, QKVW, st, lay.gws, lay.gws_bytes, NV, L, 1));
            float* rows = per_batch ? dvpt[0] : lay.vpt_rows;
            EBC_TRY(ebc::layernorm_bwd_rows(dtype, lay.dH, lay.X[0], NV, L, 1, s.m1, s.r1, p.ln1_g, dX, rows, B * NV,
                                            WIDTH, st));
            break;
        }
        EBC_TRY(ebc::attention_bwd(dtype, s.QKV, lay.dO, s.O, s.lse, lay.delta, lay.dQKV, B, L, HEADS, st, 0, &tl));
        EBC_TRY(gemm(EBC_EPI_STORE, lay.dQKV, p.wt_qkv, lay.dH, nullptr, M, WIDTH, QKVW));
        // prompt rows (deep VPT; shallow VPT: layer 0 only): ln_1's backward routes their gradient to the
        // per-crop rows (straight into dvpt_l when it is per crop) and zeroes them in the token stream,
        // since the prompt replaced them at this block's input
        if (NV > 0 && dvpt && dvpt[l]) {
            float* rows = per_batch ? dvpt[l] : lay.vpt_rows + (size_t)l * B * NV * WIDTH;
            EBC_TRY(ebc::layernorm_bwd_vpt(dtype, lay.dH, lay.X[l], s.m1, s.r1, p.ln1_g, dX, dXo, lay.dXt, M, WIDTH,
                                           rows, L, NV, st));
        } else {
            EBC_TRY(ebc::layernorm_bwd(dtype, 0, lay.dH, lay.X[l], 0, 0, 0, s.m1, s.r1, p.ln1_g, dX, dXo, lay.dXt, M, WIDTH, st));
        }
        { float* t = dX; dX = dXo; dXo = t; }
    }
    // dvpt_l = sum over crops of the prompt rows, every layer in one launch (shared prompts)
    if (NV > 0 && dvpt && !per_batch) EBC_TRY(ebc::vpt_sum(lay.vpt_rows, dvpt, layers, B, NV, WIDTH, st));
    return EBC_OK;
}

// ---------------------------------------------------------------------------- kernel C-ABI
extern "C" int ebc_layernorm_fwd(int dtype, const float* x, int rows_per_group, int group_stride, int group_offset,
                                 const float* gamma, const float* beta, void* out, float* out_f32, float* mean,
                                 float* rstd, int M, int D, ebc_stream_t stream)
{
    return ebc::layernorm_fwd(dtype, x, rows_per_group, group_stride, group_offset, gamma, beta, out, out_f32, mean,
                              rstd, M, D, (hipStream_t)stream);
}
extern "C" int ebc_layernorm_bwd(int dtype, int dy_f32, const void* dy, const float* x, int rows_per_group,
                                 int group_stride, int group_offset, const float* mean, const float* rstd,
                                 const float* gamma, const float* dx_in, float* dx_out, void* dx_out_t, int M, int D,
                                 ebc_stream_t stream)
{
    return ebc::layernorm_bwd(dtype, dy_f32, dy, x, rows_per_group, group_stride, group_offset, mean, rstd, gamma,
                              dx_in, dx_out, dx_out_t, M, D, (hipStream_t)stream);
}
extern "C" int ebc_attention_fwd(int dtype, const void* qkv, void* out, float* lse, int B, int L, int H, ebc_stream_t stream)
{
    return ebc::attention_fwd(dtype, qkv, out, lse, B, L, H, (hipStream_t)stream);
}
extern "C" int ebc_attention_bwd(int dtype, const void* qkv, const void* dout, const void* out, const float* lse,
                                 float* delta_ws, void* dqkv, int B, int L, int H, ebc_stream_t stream)
{
    return ebc::attention_bwd(dtype, qkv, dout, out, lse, delta_ws, dqkv, B, L, H, (hipStream_t)stream);
}
extern "C" int ebc_head_fwd(int dtype_z, const void* Z, const float* text, const float* logit_scale, const float* anchors,
                            float* logits, float* expo, int P, int HW, int NB, int embed, ebc_stream_t stream)
{
    return ebc::head_fwd(dtype_z, Z, text, logit_scale, anchors, logits, expo, P, HW, NB, embed, (hipStream_t)stream);
}
extern "C" size_t ebc_head_bwd_workspace_bytes(int P, int embed)
{
    return ebc::head_bwd_ws_bytes(P, embed);
}
extern "C" int ebc_head_bwd(int dtype_z, int dtype_dz, const void* Z, const float* text, const float* logit_scale,
                            const float* anchors, const float* dlogits, const float* dexp, const float* gscale, void* dZ,
                            float* dbias, float* dscale, int P, int HW, int NB, int embed, void* workspace,
                            size_t workspace_bytes, ebc_stream_t stream)
{
    return ebc::head_bwd(dtype_z, dtype_dz, Z, text, logit_scale, anchors, dlogits, dexp, gscale, dZ, dbias, dscale, P, HW,
                         NB, embed, workspace, workspace_bytes, (hipStream_t)stream);
}
extern "C" int ebc_cast_f32(int dtype, const float* in, void* out, size_t n, ebc_stream_t stream)
{
    return ebc::cast_f32(dtype, in, out, n, (hipStream_t)stream);
}
