// Internal launchers shared by the C-ABI entry points and the ViT orchestrator.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace ebc {
// Device buffers an attention launch reads onto the die while it computes (the next GEMMs' frozen weights, last read
// a step ago): every wave of the launch reads a dword of its share of their 128-B lines (attention.hip touch_issue),
// so the later GEMMs' L2 misses are served by the Infinity Cache instead of HBM.
struct TouchList {
    const void* ptr[8];
    size_t bytes[8];
    int n;
    void add(const void* p, size_t b) { if (p && b >= 128 && n < 8) { ptr[n] = p; bytes[n] = b; ++n; } }
};
// ebc_set_weight_touch: the touch lists are issued (attention.hip g_touch_mode == 1)
bool touch_enabled();
// in-step launch timing (probe.hip): probe_start returns a record index (or -1 when not armed)
bool probe_on();
int probe_start(int kind, int epi, int bm, int bn, int mode, int m, int n, int k, hipStream_t st);
void probe_stop(int idx, hipStream_t st);
int gemm_nt(int dtype, int epi, int out_f32, const void* A, const void* B, void* C, const float* bias,
            const float* resid, void* aux, int M, int N, int K, hipStream_t st, void* ws = nullptr,
            size_t ws_bytes = 0, int a_rpg = 0, int a_gstride = 0, int a_goff = 0);
// LayerNorm folded into the encoder GEMMs (gemm.hip GemmArgs, vit.hip; 16-bit): a RESID product that also writes a
// compute-dtype copy of its rows (xh) and per-row partial sums / sums of squares (rpart [M][parts][2],
// parts = gemm_rowstat_parts), and GEMM_EPI_LN / GEMM_EPI_LN_GELU products normalising their A rows from them
struct GemmLn {
    void* xh = nullptr;
    float* rpart = nullptr;
    const float* lnp = nullptr;
    int lnparts = 0;
    const float* lnw = nullptr;
    float* mean = nullptr;
    float* rstd = nullptr;
    // RESID: replace the deep-VPT prompt rows (1 <= r % vrep_L <= vrep_nv) of the output by vrep (crop stride vrep_bs)
    const float* vrep = nullptr;
    long vrep_bs = 0;
    int vrep_L = 0, vrep_nv = 0;
    // LayerNorm backward folded into the encoder's dX products (r05).  GELU_BWD with bpart: per row and (tile column,
    // wave column) the partial sums  sum_k dA_k s_k  and  sum_k dA_k (A_k - c_k)  over the product's columns, s = W'.1
    // and c = b + W beta of the folded forward product (lnb_s, lnb_c): with g = dX_ln (.) gamma these are sum_j g_j and
    // sum_j g_j xhat_j of the LayerNorm the forward folded, read in A's space (A = xhat W'^T + c).  EPI_LN_BWD: the next
    // dX product, B = (W')^T, so acc = g; out = rstd (g - sum g / N - xhat sum(g xhat) / N) + resid (f32, xhat from lnx
    // and the row's mean / rstd), also written to xh in the compute dtype -- the LayerNorm backward without its launch.
    const float* lnb_s = nullptr;
    const float* lnb_c = nullptr;
    float* bpart = nullptr;
    const float* lnx = nullptr;
};
constexpr int GEMM_EPI_LN = 6, GEMM_EPI_LN_GELU = 7, GEMM_EPI_LN_BWD = 8;
constexpr int GEMM_LN_PMAX = 16;   // most row partials an EPI_LN product reads (gemm_rowstat_parts of its producer)
constexpr int GEMM_LN_PMAX_B = 32; // ... and an EPI_LN_BWD product (the GELU' product's: 3072 / 192 x 2)
int gemm_nt_ln(int dtype, int epi, int out_f32, const void* A, const void* B, void* C, const float* bias,
               const float* resid, void* aux, int M, int N, int K, hipStream_t st, void* ws, size_t ws_bytes,
               const GemmLn& ln);
int gemm_rowstat_parts(int dtype, int M, int N, int K);
// whether the c_fc dX product (M x N = 768 x K = 3072) runs the LayerNorm-backward epilogue without losing occupancy
bool gemm_ln_bwd_fold_pays(int dtype, int M, int N, int K);
// split-K workspace the heuristic wants for this shape (0: no split); zero-filled counter block first
size_t gemm_workspace_bytes(int dtype, int M, int N, int K);
// implicit-GEMM 3x3 convolution geometry (gemm.hip MODE 1 / MODE 2)
struct ConvGeom {
    int H, W, C;      // output image (stride 1, pad 1), channels per tap
    int Hp, Wp;       // MODE 1: padded NHWC operand image [B][Hp][Wp][C]
    int HWp;          // MODE 2: K columns per image (H*W rounded up to 8)
    long Qs, Pimg;    // MODE 2: row stride of dz^T / x^T (elements), positions per row-padded x^T image ((H+2)*W)
    int nimg;         // images (B): the algorithmic K of a weight gradient is nimg * H * W
};
// mode 1: C[M = B*H*W, N] = conv(A = padded NHWC image, B = weights [N][9*C]), epi 0 store / 4 + BN stats
//         (per-tile column partials at ws + 16 KiB: [stats_tiles][2][N]);
// mode 2: C[M, N = 9*C] f32 = A^T-image . B^T-images (weight gradient), split-K through ws
// epi 5 (mode 1): C = conv + gy * (y > 0)   (decoder: conv1 input gradient + residual-branch gradient)
int conv_gemm(int dtype, int mode, int epi, const void* A, const void* B, void* C, const ConvGeom& geo, int M, int N,
              int K, void* ws, size_t wsb, int* stats_tiles, hipStream_t st, const void* gy = nullptr,
              const void* y = nullptr);
size_t conv_gemm_workspace_bytes(int dtype, int mode, int M, int N, int K);
constexpr size_t CONV_WS_STATS_OFFSET = 16 * 1024;
int layernorm_fwd(int dtype, const float* x, int rpg, int gstride, int goff, const float* gamma, const float* beta,
                  void* out, float* outf, float* mean, float* rstd, int M, int D, hipStream_t st);
int layernorm_bwd_fill(int dtype, const float* dy, const float* x, int rpg, int gstride, int goff, const float* mean,
                       const float* rstd, const float* gamma, float* dx_out, void* dx_out_t, int M, int D, hipStream_t st,
                       const TouchList* touch = nullptr);
int layernorm_bwd(int dtype, int dy_f32, const void* dy, const float* x, int rpg, int gstride, int goff,
                  const float* mean, const float* rstd, const float* gamma, const float* dx_in, float* dx_out,
                  void* dx_out_t, int M, int D, hipStream_t st);
int im2col(int dtype, const float* x, void* out, int B, int H, int W, int P, hipStream_t st);
int embed_tokens(const float* patch, const float* cls, const float* pos, const float* gamma, const float* beta,
                 const float* vpt, long vpt_bstride, float* X, int B, int L, int G, int NVPT, int D, hipStream_t st);
// ln_1 with the deep-VPT rows taken from the prompt (and written into X): replaces insert_vpt + layernorm_fwd
int layernorm_fwd_vpt(int dtype, float* X, const float* vpt, long vpt_bstride, int L, int NVPT, const float* gamma,
                      const float* beta, void* out, float* mean, float* rstd, int M, int D, hipStream_t st);
// ln_1 backward that routes the prompt rows' gradient to vpt_rows [B][NVPT][D] (and zeroes them in dx_out /
// dx_out_t): replaces layernorm_bwd + vpt_grad; vpt_sum then reduces the per-crop rows over the batch for
// every layer in one launch
int layernorm_bwd_vpt(int dtype, const void* dy, const float* x, const float* mean, const float* rstd,
                      const float* gamma, const float* dx_in, float* dx_out, void* dx_out_t, int M, int D, float* vpt_rows,
                      int L, int NVPT, hipStream_t st);
int vpt_sum(const float* rows, float* const* dst, int layers, int B, int NVPT, int D, hipStream_t st);
int insert_vpt(float* X, const float* vpt, long vpt_bstride, int B, int L, int NVPT, int D, hipStream_t st);
int vpt_grad(int dtype, float* dX, void* dXt, float* dvpt, int B, int L, int NVPT, int D, int per_batch, int accumulate,
             hipStream_t st);
int head_fwd(int dtype_z, const void* Z, const float* text, const float* logit_scale, const float* anchors,
             float* logits, float* expo, int P, int HW, int NB, int embed, hipStream_t st);
// d bias / d logit_scale as per-block partials (ws: head_bwd_ws_bytes) summed in block order by a second launch
size_t head_bwd_ws_bytes(int P, int embed);
int head_bwd(int dtype_z, int dtype_dz, const void* Z, const float* text, const float* logit_scale, const float* anchors,
             const float* dlogits, const float* dexp, const float* gscale, void* dZ, float* dbias, float* dscale,
             int P, int HW, int NB, int embed, void* ws, size_t wsb, hipStream_t st);
int attn_delta(int dtype, const void* dO, const void* O, float* delta, int B, int L, int H, hipStream_t st);
int cast_f32(int dtype, const float* in, void* out, size_t n, hipStream_t st);
int attention_fwd(int dtype, const void* qkv, void* out, float* lse, int B, int L, int H, hipStream_t st,
                  const TouchList* touch = nullptr);
// delta (FA2 D_i = rowsum(dO * O)) is computed by the dQ kernel and written to `delta` [B,H,L]
// rows > 0: only dQ of the queries and dK / dV of the keys below `rows` are needed (16-bit: the launch covers
// the first ceil(rows / 128) blocks of each (crop, head); the other dqkv rows are left unwritten)
int attention_bwd(int dtype, const void* qkv, const void* dout, const void* out, const float* lse, float* delta,
                  void* dqkv, int B, int L, int H, hipStream_t st, int rows = 0,
                  const TouchList* touch = nullptr);
// LayerNorm backward of the mapped rows into a dense output: dx_out[r] = dx_in[map r] + LN'(dy[r]) with x, mean,
// rstd at map r (layer 0's prompt rows: r = (b, j) -> b * gstride + goff + j)
int layernorm_bwd_rows(int dtype, const void* dy, const float* x, int rpg, int gstride, int goff, const float* mean,
                       const float* rstd, const float* gamma, const float* dx_in, float* dx_out, int M, int D,
                       hipStream_t st);
}  // namespace ebc

#define EBC_TRY(x)                  \
    do {                            \
        int _rc = (x);              \
        if (_rc != 0) return _rc;   \
    } while (0)
