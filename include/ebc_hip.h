/*
 * libebc_hip.so — C-ABI of the MI355X-native CLIP-EBC hot path (gfx950 / CDNA4).
 *
 * The reference (Yiming-M/CLIP-EBC) is pure Python on PyTorch; it has no FFI.  Its boundary
 * is the Python API.  These entry points are what that API binds to through
 * ctypes (clip-ebc_amd/ebc_amd/_lib.py); each cites the reference interface it replaces.
 *
 * Conventions (all entry points):
 *   - every pointer is caller-owned DEVICE memory (torch-allocated), except where noted;
 *   - no allocation, no host<->device synchronisation, no device sync inside a call; work is
 *     enqueued on `stream` (a hipStream_t passed as void*), so calls are graph-capturable;
 *   - return 0 (EBC_OK) or a negative EBC_E_* code; numerical roll-backs are reported per
 *     crop through `status`, never as an error;
 *   - `dtype` selects the GEMM/attention input type: EBC_F32 (parity mode, exact-f32 MFMA),
 *     EBC_F16 (the reference's AMP dtype) or EBC_BF16.
 */
#ifndef EBC_HIP_H
#define EBC_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* ebc_stream_t;

enum { EBC_F32 = 0, EBC_F16 = 1, EBC_BF16 = 2 };
enum { EBC_OK = 0, EBC_E_ARG = -1, EBC_E_LAUNCH = -2, EBC_E_UNSUPPORTED = -3 };
enum { EBC_COUNT_DMCOUNT = 0, EBC_COUNT_MAE = 1, EBC_COUNT_MSE = 2, EBC_COUNT_OT_ONLY = 3 };

/* Library version / self-description (host-only, no device work). */
int ebc_version(void);

/* ------------------------------------------------------------------------------------------
 * DACE loss with DMCount, fused, one workgroup per crop, all Sinkhorn iterations on device.
 *
 * Replaces DACELoss.forward (losses/dace_loss.py:49-70) with its DMLoss
 * (losses/dm_loss.py:99-124), OTLoss (losses/dm_loss.py:38-79) and
 * sinkhorn (losses/bregman_pytorch.py:11-144), forward AND backward:
 *   pred_class     [B, N, g, g] f32 logits      (g = size / reduction)
 *   pred_density   [B, 1, g, g] f32
 *   target_density [B, 1, size, size] f32 dot map (or already [B,1,g,g] if target_is_reduced)
 *   points         [sum(n_b), 2] f32 (x, y) pixels, packed;  offsets [B+1] int32 (device)
 *   bins_lo/hi     [N] f32 (device), inclusive bins; hi may be +inf
 *   order          [B] int32 (device) crop processing order (heaviest first), or NULL
 * Outputs:
 *   grad_class   [B, N, g, g]  d loss / d pred_class  (for upstream grad 1)
 *   grad_density [B, 1, g, g]  d loss / d pred_density
 *   losses       [5] f32: loss, ot_loss, tv_loss, count_loss, ce_loss (loss_info keys)
 *   crop_stats   [B, 8] f32: ce_b, tv_b*n_b, count_b, ot_b, wd_b, iters, rolled_back, err_last
 *   beta_out     [B, g*g] f32 or NULL;  status [B] int32 or NULL (iterations, negative = rollback)
 * count_mode: EBC_COUNT_DMCOUNT / _MAE / _MSE (DACELoss count_loss="dmcount"/"mae"/"mse"), or
 *   EBC_COUNT_OT_ONLY: OTLoss.forward alone (losses/dm_loss.py:38-79): grad_density = the OT gradient
 *   (weight_count_loss * weight_ot times it), losses[1] = sum of the crops' OT losses, no TV / count terms.
 * size / reduction (the density grid g) may be any integer up to 64 (e.g. 28 / 14 / 7 for 224 crops at reduction
 * 8 / 16 / 32, 56 / 28 / 14 for 448, 48 for 384 at 8, 64 for 512 at 8; the kernel runs on an LDS grid
 * G in {8,16,24,28,32,40,48,56,64} >= g whose extra cells are dead); EBC_E_UNSUPPORTED above 64.
 * grid cell k sits at k * reduction + reduction / 2 (dm_loss.py:31).
 * norm_cood: OTLoss norm_cood (dm_loss.py:31-34,51): coordinates mapped to [-1, 1].
 * workspace: ebc_dace_workspace_bytes(...) bytes of device memory.
 */
size_t ebc_dace_workspace_bytes(int B, int total_points, int size, int reduction);
/* a_out[i] = a[i] * *s, b_out[i] = b[i] * *s (s a device scalar): the loss gradients times the upstream gradient of the
 * loss (GradScaler's scale) in one launch */
int ebc_scale2(const float* s, const float* a, float* a_out, long na, const float* b, float* b_out, long nb,
               ebc_stream_t stream);
int ebc_dace_loss(const float* pred_class, const float* pred_density, const float* target_density,
                  int target_is_reduced, const float* points, const int* offsets, const int* order,
                  const float* bins_lo, const float* bins_hi, int B, int N, int size, int reduction,
                  int count_mode, int norm_cood, float weight_count_loss, float weight_ot, float weight_tv,
                  float reg, int max_iter, float stop_thr, int eval_freq,
                  float* grad_class, float* grad_density, float* losses, float* crop_stats,
                  float* beta_out, int* status, void* workspace, size_t workspace_bytes,
                  ebc_stream_t stream);
/* The same with the crop offsets [B+1] and order [B] in HOST memory (B <= 64): passed to the kernel as launch
 * arguments, so the label metadata needs no host-to-device copy. */
int ebc_dace_loss_h(const float* pred_class, const float* pred_density, const float* target_density,
                    int target_is_reduced, const float* points, const int* offsets_host, const int* order_host,
                    const float* bins_lo, const float* bins_hi, int B, int N, int size, int reduction,
                    int count_mode, int norm_cood, float weight_count_loss, float weight_ot, float weight_tv,
                    float reg, int max_iter, float stop_thr, int eval_freq,
                    float* grad_class, float* grad_density, float* losses, float* crop_stats,
                    float* beta_out, int* status, void* workspace, size_t workspace_bytes,
                    ebc_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * General dense Sinkhorn-Knopp, one problem: replaces sinkhorn(a, b, C, reg, maxIter, stopThr, verbose,
 * log, eval_freq, print_freq) (losses/bregman_pytorch.py:11-144) for callers of that function itself
 * (the DMCount path uses ebc_dace_loss, whose cost is separable).  a [na], b [nb], C [na, nb] f32.
 * Outputs (each may be NULL except info): P [na, nb] = u K v; u [na], v [nb]; alpha = reg log(u + 1e-16),
 * beta = reg log(v + 1e-16); err [ceil(max_iter / eval_freq)] (the log's err list, only when log != 0);
 * info [2] int32 = {iterations run (negative: NaN/Inf rollback at that iteration), err entries}.
 * workspace: ebc_sinkhorn_workspace_bytes(na, nb) bytes (0 when K fits LDS).  EBC_E_UNSUPPORTED when
 * u and v together exceed LDS (na + nb beyond ~20000). */
size_t ebc_sinkhorn_workspace_bytes(int na, int nb);
int ebc_sinkhorn(const float* a, const float* b, const float* C, int na, int nb, float reg, int max_iter,
                 float stop_thr, int eval_freq, int log, float* P, float* u, float* v, float* alpha, float* beta,
                 float* err, int* info, void* workspace, size_t workspace_bytes, ebc_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * GEMM  C[M,N] = A[M,K] . B[N,K]^T (+bias[N]) with a fused epilogue.  A, B of `dtype`; K % 64 == 0
 * (K % 32 for f32), N % 64 == 0.  Replaces the nn.Linear / nn.MultiheadAttention projections of
 * ResidualAttentionBlock (models/clip/_clip/blocks.py:22-42), the patch-embed conv1
 * (image_encoder.py:141, as im2col-GEMM) and the 1x1 projection (models/clip/model.py:91-95).
 *   epilogue 0 STORE:    C = acc + bias                      (C of dtype, or f32 if out_f32)
 *   epilogue 1 GELU:     aux = acc + bias; C = QuickGELU(aux) (blocks.py:17-19)
 *   epilogue 2 RESID:    C = resid(f32) + acc + bias          (C f32: the residual stream, may be in place;
 *                                                              C in dtype when !out_f32)
 *   epilogue 3 GELU_BWD: C = acc * QuickGELU'(aux)           (MLP backward, dX only)
 */
enum { EBC_EPI_STORE = 0, EBC_EPI_GELU = 1, EBC_EPI_RESID = 2, EBC_EPI_GELU_BWD = 3 };
int ebc_gemm(int dtype, int epilogue, int out_f32, const void* A, const void* B, void* C,
             const float* bias, const float* resid, void* aux, int M, int N, int K, ebc_stream_t stream);
/* The tile configuration ebc_gemm / ebc_gemm_ws dispatch for this shape (host-only, no device work):
 * returns the configuration id (> 0; EBC_GEMM_CFG overrides are honoured as in the launch) and writes
 * out[3] = {tile rows, tile columns, split-K factor}.  Lets tests pin which kernel instance a shape runs. */
int ebc_gemm_tile_config(int dtype, int M, int N, int K, int* out);
/* Same, allowed to split K over workgroups (16-bit dtypes) when the output has too few 256-wide
 * tiles to fill the GPU.  `workspace` (>= ebc_gemm_workspace_bytes; 0 = no split for this shape)
 * must be zero-filled before its first use and is then owned by the stream: every call leaves
 * its leading counter block zero again, the rest is scratch. */
size_t ebc_gemm_workspace_bytes(int dtype, int M, int N, int K);
int ebc_gemm_ws(int dtype, int epilogue, int out_f32, const void* A, const void* B, void* C,
                const float* bias, const float* resid, void* aux, int M, int N, int K,
                void* workspace, size_t workspace_bytes, ebc_stream_t stream);
/* Weight-gradient GEMM for a long reduction (K = pixels), f32 output:  C[M,N] = A[M,K] . B[N,K]^T
 * with A, B in `dtype` (K-contiguous: the transposed activations / output gradients).  Replaces the
 * projection's dW = dZ^T Y of models/clip/model.py:91-95 (nn.Conv2d 1x1 backward).  Splits K over
 * workgroups (deterministic last-arriver sum); `workspace` as for ebc_gemm_ws. */
size_t ebc_gemm_wgrad_workspace_bytes(int dtype, int M, int N, int K);
int ebc_gemm_wgrad(int dtype, const void* A, const void* B, float* C, int M, int N, int K,
                   void* workspace, size_t workspace_bytes, ebc_stream_t stream);
/* out[c][r] = in[r][c] for in [R][C] (16-bit or f32 elements; C and the output row stride ld_out >= R
 * multiples of 8, any R): the K-contiguous operand copies for ebc_gemm_wgrad. */
int ebc_transpose(int dtype, const void* in, void* out, int R, int C, long ld_out, ebc_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * CLIP ViT-B/16 + deep VPT encoder: CLIP_EBC._forward_vpt (models/clip/model.py:142-189), whole
 * forward and dX-only backward (frozen encoder: gradients reach the VPT tokens only), one call each.
 * Weight pointers are device memory of `dtype` (matrices, nn.Linear [out, in] layout) or f32
 * (biases, LayerNorm, embeddings); wt_* are the transposed matrices [in, out] used by backward.
 * The EbcVitWeights / EbcVitLayer structs themselves live in HOST memory.
 */
typedef struct {
    const void* w_qkv;  const float* b_qkv;    /* attn.in_proj_weight [2304,768], in_proj_bias */
    const void* w_out;  const float* b_out;    /* attn.out_proj [768,768] */
    const void* w_fc;   const float* b_fc;     /* mlp.c_fc [3072,768] */
    const void* w_proj; const float* b_proj;   /* mlp.c_proj [768,3072] */
    const float* ln1_g; const float* ln1_b; const float* ln2_g; const float* ln2_b;
    const void* wt_qkv; const void* wt_out; const void* wt_fc; const void* wt_proj;   /* transposes */
    /* optional (16-bit; all null: ln_1 / ln_2 run as LayerNorm launches): ln_1 / ln_2 folded into the QKV / c_fc
     * products -- the weight rows pre-scaled by gamma (W' = W diag(gamma), [out, 768] in dtype), the folded bias
     * b + W beta and the row sums W'.1 (f32 [out]); the layer's input rows are then normalised in those products'
     * epilogues from row statistics the previous residual product writes */
    const void* w_qkv_ln; const float* b_qkv_ln; const float* s_qkv_ln;
    const void* w_fc_ln;  const float* b_fc_ln;  const float* s_fc_ln;
    /* optional (16-bit, with the fold above; null: LayerNorm-backward launches): the transposes of the folded weights,
     * (W')^T [768, out], so the dX products after the GELU' / attention backward produce g = dX_ln (.) gamma and finish
     * the LayerNorm backward in their epilogues (row sums from the GELU' product's partials, vit.hip) */
    const void* wt_qkv_ln; const void* wt_fc_ln;
} EbcVitLayer;

typedef struct {
    int layers, width, heads, patch, num_vpt;
    const void* w_patch;                        /* conv1.weight as [768, 3*16*16] */
    const float* cls;                           /* class_embedding [768] */
    const float* pos;                           /* positional_embedding [G+1, 768] for this input size */
    const float* ln_pre_g; const float* ln_pre_b; const float* ln_post_g; const float* ln_post_b;
    const EbcVitLayer* layer;                   /* host array [layers] */
} EbcVitWeights;

/* Workspace (device bytes) holding the saved activations (training) or the ping-pong buffers. */
size_t ebc_vit_workspace_bytes(int B, int H, int W, int layers, int num_vpt, int dtype, int training);
/* image [B,3,H,W] f32 -> feat [B, (H/16)*(W/16), 768] f32 (= ln_post of the patch tokens, NHWC).
 * vpt: host array [layers] of device pointers ([num_vpt,768] f32, or [B,num_vpt,768] with
 * vpt_bstride = num_vpt*768 elements for per-crop prompts); vpt[l] == NULL for l > 0 keeps the
 * previous block's prompt outputs (shallow VPT, model.py:177-178). */
int ebc_vit_forward(const EbcVitWeights* w, const float* image, int B, int H, int W,
                    const float* const* vpt, long vpt_bstride, int dtype, int training,
                    void* workspace, size_t workspace_bytes, float* feat, ebc_stream_t stream);
/* dfeat [B, G, 768] f32 -> dvpt[l] ([num_vpt,768] f32, summed over crops; per crop if vpt_bstride).
 * Layer 0's backward stops at its prompt rows (the frozen embedding below takes no gradient: dQ/dK/dV of the first
 * query/key block, dH and ln_1' of the prompt rows only); flags & EBC_VIT_BWD_FULL_LAYER0 runs it over every row
 * instead, which must give bit-identical prompt gradients (a parity hook for tests/test_gpu_model.py).
 * flags & EBC_VIT_BWD_NO_LN_FOLD runs ln_2's backward as a LayerNorm launch even when wt_fc_ln is set (A/B, tests). */
enum { EBC_VIT_BWD_FULL_LAYER0 = 1, EBC_VIT_BWD_NO_LN_FOLD = 2 };
int ebc_vit_backward(const EbcVitWeights* w, int B, int H, int W, int dtype, void* workspace,
                     size_t workspace_bytes, const float* dfeat, float* const* dvpt, long vpt_bstride, int flags,
                     ebc_stream_t stream);

/* LayerNorm over 768 channels (models/clip/_clip/blocks.py:8-14, fp32 math, eps 1e-5).
 * Row r of the output reads input row (r / rows_per_group) * group_stride + group_offset +
 * r % rows_per_group (rows_per_group = 0: identity), e.g. ln_post on the patch rows only. */
int ebc_layernorm_fwd(int dtype, const float* x, int rows_per_group, int group_stride, int group_offset,
                      const float* gamma, const float* beta, void* out, float* out_f32, float* mean,
                      float* rstd, int M, int D, ebc_stream_t stream);
int ebc_layernorm_bwd(int dtype, int dy_f32, const void* dy, const float* x, int rows_per_group,
                      int group_stride, int group_offset, const float* mean, const float* rstd,
                      const float* gamma, const float* dx_in, float* dx_out, void* dx_out_t, int M, int D,
                      ebc_stream_t stream);
/* Multi-head attention on the packed qkv [B*L, 3*H*64] (nn.MultiheadAttention, need_weights=False,
 * blocks.py:35-37): out [B*L, H*64], lse [B,H,L]; backward writes dqkv [B*L, 3*H*64].
 * L <= 256: K/V (and Q/dO) resident in LDS, one workgroup per (crop, head); 256 < L <= 16384 (the position
 * embedding interpolated for larger inputs, image_encoder.py:183-198): K/V streamed through LDS in 256-row chunks
 * with an online softmax; longer sequences return EBC_E_UNSUPPORTED. */
int ebc_attention_fwd(int dtype, const void* qkv, void* out, float* lse, int B, int L, int H, ebc_stream_t stream);
int ebc_attention_bwd(int dtype, const void* qkv, const void* dout, const void* out, const float* lse,
                      float* delta_ws, void* dqkv, int B, int L, int H, ebc_stream_t stream);
/* Blockwise image-text similarity head (models/clip/model.py:200-217):
 * Z [P=B*HW, embed] projected features (NHWC rows) -> logits [B,NB,HW], exp [B,1,HW]; text [NB, embed];
 * embed = the CLIP joint width: 512 (ViT-B/16) or 1024 (ResNet-50), NB <= 16.
 * Backward: dZ (element type dtype_dz), d projection bias (column sums), d logit_scale; gscale (device scalar) scales the
 * upstream gradients (NULL = 1).  d bias / d logit_scale are summed deterministically (per-block partials in `workspace`,
 * ebc_head_bwd_workspace_bytes(P, embed) bytes, reduced in block order); workspace may be NULL when both are NULL.
 * Replaces the autograd backward of model.py:198-217 (F.normalize, cosine logits x exp(logit_scale), softmax, expectation)
 * and the projection bias's column sum. */
int ebc_head_fwd(int dtype_z, const void* Z, const float* text, const float* logit_scale, const float* anchors,
                 float* logits, float* expo, int P, int HW, int NB, int embed, ebc_stream_t stream);
size_t ebc_head_bwd_workspace_bytes(int P, int embed);
int ebc_head_bwd(int dtype_z, int dtype_dz, const void* Z, const float* text, const float* logit_scale,
                 const float* anchors, const float* dlogits, const float* dexp, const float* gscale, void* dZ,
                 float* dbias, float* dscale, int P, int HW, int NB, int embed, void* workspace, size_t workspace_bytes,
                 ebc_stream_t stream);
int ebc_cast_f32(int dtype, const float* in, void* out, size_t n, ebc_stream_t stream);

/* Sliding-window evaluation (utils/eval_utils.py:26-96).  Tiles t = i*cols + j, rows/cols =
 * ceil((H-wh)/sh)+1, last row/column snapped to the border.
 * gather:   tiles [tile_count, C, wh, ww] <- image [C, H, W], tiles tile_begin .. +tile_count
 * assemble: out [Cp, H/r, W/r] = per-pixel mean of preds [rows*cols, Cp, wh/r, ww/r] */
int ebc_tile_gather(const float* image, float* tiles, int C, int H, int W, int wh, int ww, int sh, int sw,
                    int tile_begin, int tile_count, ebc_stream_t stream);
int ebc_tile_assemble(const float* preds, float* out, int Cp, int H, int W, int wh, int ww, int sh, int sw,
                      int reduction, ebc_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Training-crop augmentation on device (the reference runs it on CPU in
 * DataLoader workers, utils/data_utils.py:14-26).  One descriptor per output crop (device array);
 * the host samples the random parameters with the reference's RNG calls:
 *   crop window + resize  RandomResizedCrop / _crop / _resize (datasets/transforms.py:9-43,133-171):
 *                         torch F.interpolate(bicubic, antialias=True) taps; src == NULL skips it
 *   flip                  RandomHorizontalFlip (transforms.py:174-187), on the resize store
 *   jitter_ops            ColorJitter order (transforms.py:190-201 -> torchvision ColorJitter):
 *                         3 bits per slot (up to 4 slots), 1 brightness, 2 contrast, 3 saturation, 4 hue
 *                         (torchvision adjust_hue: _rgb2hsv, h = (h + hue) % 1, _hsv2rgb, per pixel)
 *   blur                  GaussianBlur(kernel_size, sigma=(sx, sy)) (transforms.py:217-223), reflect pad
 *   noise                 PepperSaltNoise (transforms.py:242-255) over uniforms u[3][out_h][out_w]:
 *                         noise_off >= 0: u = noise + noise_off, a field the host drew with the reference's own
 *                         `torch.rand_like(image)` (transforms.py:252), so the host RNG stream stays the reference's;
 *                         noise_off < 0: u = counter-based uniforms from `seed` (no host draw, no upload)
 *   normalize             Normalize(ImageNet mean/std) (datasets/crowd.py:64,162)
 * workspace: per crop tmp_off .. + max(3*crop_h*out_w, 3*out_h*out_w) floats (caller-assigned).
 * noise: the device uniform fields noise_off indexes; NULL = every crop takes the counter-based uniforms. */
#define EBC_AUG_MAX_BLUR 31
typedef struct {
    int64_t src_off, out_off, tmp_off;   /* element offsets: source image [3][src_h][src_w], output [3][out_h][out_w], scratch */
    int64_t noise_off;                   /* element offset of this crop's uniform field in `noise`, or -1 (hash of seed) */
    int32_t src_h, src_w, top, left, crop_h, crop_w, out_h, out_w;
    int32_t flip, jitter_ops;
    float brightness, contrast, saturation;
    int32_t blur, noise;
    float saltiness, spiciness;
    uint32_t seed;
    int32_t normalize;
    float hue;                           /* ColorJitter hue factor in [-0.5, 0.5] (op 4) */
} EbcCropDesc;
typedef struct {
    float mean[3], std[3];
    int32_t blur_k;                      /* odd, <= EBC_AUG_MAX_BLUR */
    float sigma_x, sigma_y;
} EbcAugConst;
/* max_crop_h / max_out_h: maxima over the descriptors (grid sizing) */
int ebc_augment_crops(const float* src, const EbcCropDesc* desc, int n, int max_crop_h, int max_out_h, float* out,
                      float* workspace, const float* noise, EbcAugConst k, ebc_stream_t stream);
/* generate_density_map(label, H, W, sigma=None) (datasets/utils.py:11-28) for B crops: out [B][1][H][W]
 * = 1 at (clamp(int y), clamp(int x)) of points [sum n, 2] (x, y), offsets [B+1] (device) */
int ebc_point_map(const float* points, const int* offsets, int B, int H, int W, int max_points, float* out,
                  ebc_stream_t stream);


/* ------------------------------------------------------------------------------------------
 * Decoder BasicBlock (models/utils.py:254-303, cfg [768] for vit_b_16, models/clip/model.py:250-251)
 * with the reduction adapt F.interpolate(x2, bilinear, align_corners=False) (model.py:195-196),
 * training-mode BatchNorm2d (batch statistics, running stats; SyncBatchNorm = caller all-reduces
 * `colsum` / `sums` between the two calls that bracket them) and the whole backward.
 * Layouts (T = dtype): feat [B][h][w][C] f32; padded NHWC images [Q][C] T with Q = B*Hp*Wp;
 * z / dx / y [B*H*W][C] T; transposed images xT3 [3][C][Qs], dzT [N][Qs] T; conv weights
 * [N][3][3][C] T (forward) and [C][3][3][N] T (flipped, data gradient); dw [N][C][3][3] f32 (nn.Conv2d layout).
 * ebc_dec_geometry writes {Hp, Wp, G, kpi, Q, Qs}.  The workspace's first 16 KiB must be zero before
 * the first call (split-K arrival counters, re-armed by every call); it is stream-owned scratch. */
int ebc_dec_geometry(int dtype, int B, int H, int W, int C, long* out6);
size_t ebc_dec_workspace_bytes(int dtype, int B, int H, int W, int C, int N);
/* xpad = zero-padded bilinear x`up` upsample of feat (H = h*up) */
int ebc_dec_upsample_pad(int dtype, const float* feat, void* xpad, int B, int h, int w, int C, int up,
                         ebc_stream_t stream);
/* out[B*H*W][N] = conv3x3(xpad, weight) (nn.Conv2d(C, N, 3, padding=1, bias=False)); colsum != NULL:
 * also the f64 column sums [2][N] (sum, sum of squares) for BatchNorm; add_gy/add_y != NULL (data
 * gradient of conv1): out += add_gy * (add_y > 0), the residual branch's gradient through the final ReLU */
int ebc_conv3x3_fwd(int dtype, const void* xpad, const void* weight, void* out, double* colsum, const void* add_gy,
                    const void* add_y, void* ws, size_t wsb, int B, int H, int W, int C, int N, ebc_stream_t stream);
/* The implicit-GEMM tile configuration of a decoder conv product (mode 1: forward / data gradient,
 * M = B*H*W rows, N output channels, K = 9*C; mode 2: weight gradient, M = N channels, N = 9*C,
 * K = interior pixel rows): returns its id, out[3] = {tile rows, tile columns, split-K ways}; out[2] = -G: stream-K,
 * G workgroups share the k-tiles of the tiles past the last whole wave of 256 (those run first as a plain
 * launch). Host-only. */
int ebc_conv_tile_config(int dtype, int mode, int M, int N, int K, int* out);
/* dw[N][C][3][3] f32 = weight gradient from dzT and xT3 */
int ebc_conv3x3_wgrad(int dtype, const void* dzT, const void* xT3, float* dw, void* ws, size_t wsb, int B, int H,
                      int W, int C, int N, ebc_stream_t stream);
/* BatchNorm2d statistics -> mean, rstd, scale = gamma*rstd, shift = beta - mean*scale; running stats
 * updated (momentum, unbiased variance) when colsum != NULL, read (eval) when colsum == NULL.
 * count < 0: the element count is the DEVICE value colsum[2*C] (SyncBatchNorm: each rank stores its own
 * count there and all-reduces it with the sums, so ranks may hold different batch sizes, as
 * torch.nn.SyncBatchNorm allows); num_batches_tracked (int64, may be NULL) is incremented by the same launch */
int ebc_bn_finalize(const double* colsum, double count, float eps, float momentum, const float* gamma,
                    const float* beta, float* mean, float* rstd, float* scale, float* shift, float* running_mean,
                    float* running_var, long long* num_batches_tracked, int C, ebc_stream_t stream);
/* ebc_conv3x3_fwd with the BatchNorm statistics epilogue + ebc_bn_finalize (count = B*H*W, running stats updated,
 * num_batches_tracked incremented when non-NULL) for BatchNorms with no SyncBatchNorm exchange between the two: the
 * conv's per-tile column sums are reduced and finalized in one launch; colsum_out (may be NULL) gets the f64 sums */
int ebc_conv3x3_fwd_bn(int dtype, const void* xpad, const void* weight, void* out, void* ws, size_t wsb, int B, int H,
                       int W, int C, int N, float eps, float momentum, const float* gamma, const float* beta,
                       float* mean, float* rstd, float* scale, float* shift, float* running_mean, float* running_var,
                       long long* num_batches_tracked, double* colsum_out, ebc_stream_t stream);
/* hpad = zero-padded relu(z*scale + shift) */
int ebc_bn_relu_pad(int dtype, const void* z, const float* scale, const float* shift, void* hpad, int B, int H,
                    int W, int C, ebc_stream_t stream);
/* y = relu(z*scale + shift + bilinear_up(feat)) */
int ebc_bn_add_relu(int dtype, const void* z, const float* scale, const float* shift, const float* feat, int up,
                    void* y, int B, int H, int W, int C, ebc_stream_t stream);
/* sums[2][C] f64 = (sum g, sum g*xhat), g = gy * relu'(mask_y, or z*scale+shift when mask_y == NULL) */
int ebc_bn_bwd_reduce(int dtype, const void* gy, const void* mask_y, const void* z, const float* mean,
                      const float* rstd, const float* scale, const float* shift, double* sums, void* ws, size_t wsb,
                      long P, int C, ebc_stream_t stream);
/* dgamma, dbeta (may be NULL) and coef[3][C] for ebc_bn_bwd_apply; count < 0: device count at sums[2*C] */
int ebc_bn_bwd_finalize(const double* sums, double count, const float* gamma, const float* rstd, float* dgamma,
                        float* dbeta, float* coef, int C, ebc_stream_t stream);
/* dz = BatchNorm input gradient -> dzpad (padded NHWC) and dzT (transposed) */
int ebc_bn_bwd_apply(int dtype, const void* gy, const void* mask_y, const void* z, const float* mean,
                     const float* rstd, const float* scale, const float* shift, const float* coef, void* dzpad,
                     void* dzT, int B, int H, int W, int C, ebc_stream_t stream);
/* xT3 = kx-shifted transposed copies of a padded NHWC image (weight-gradient operand) */
int ebc_dec_transpose3(int dtype, const void* xpad, void* xT3, int B, int H, int W, int C, ebc_stream_t stream);
/* conv weight [N][C][3][3] f32 -> wk [N][3][3][C] (forward) and wf [C][3][3][N] (flipped, data gradient) */
int ebc_dec_prep_weights(int dtype, const float* w, void* wk, void* wf, int N, int C, ebc_stream_t stream);
/* dfeat [B][h][w][C] f32 = bilinear_up^T(g), g [B*H*W][C] (up = 1 or 2) */
int ebc_dec_upsample_bwd(int dtype, const void* g, float* dfeat, int B, int h, int w, int C, int up,
                         ebc_stream_t stream);
/* Flat-layout helpers of the ResNet-50 decoder Bottleneck (models/utils.py:306-363 with expansion 1, cfg [2048],
 * models/clip/model.py:234-246): its 1x1 convs are ebc_gemm products on unpadded rows [P = B*H*W][C]; the middle
 * 3x3 conv uses ebc_conv3x3_* above.
 *   ebc_dec_upsample:      x [P][C] T = bilinear x`up` upsample of feat [B][h][w][C] f32 (unpadded)
 *   ebc_bn_stats:          colsum [2][C] f64 = (sum z, sum z*z) over the P rows of z (BatchNorm batch statistics);
 *                          workspace as ebc_bn_bwd_reduce's (>= ebc_dec_workspace_bytes for that geometry)
 *   ebc_bn_relu:           out [P][C] T = relu(z*scale + shift)
 *   ebc_bn_bwd_apply_flat: dz [P][C] T = BatchNorm input gradient (coef from ebc_bn_bwd_finalize), g = gy * relu'(mask_y,
 *                          or z*scale+shift when mask_y == NULL); gmask != NULL also receives g [P][C] f32 (the
 *                          identity branch's gradient). */
int ebc_dec_upsample(int dtype, const float* feat, void* x, int B, int h, int w, int C, int up, ebc_stream_t stream);
int ebc_bn_stats(int dtype, const void* z, double* colsum, void* ws, size_t wsb, long P, int C, ebc_stream_t stream);
/* ebc_bn_stats + ebc_bn_finalize (count = P) in two launches instead of three, for BatchNorms whose statistics need no
 * SyncBatchNorm exchange between the two (models/utils.py / _clip/image_encoder.py BatchNorm2d, train mode);
 * colsum_out (may be NULL) receives the f64 sums ebc_bn_stats would. */
int ebc_bn_stats_finalize(int dtype, const void* z, void* ws, size_t wsb, long P, int C, float eps, float momentum,
                          const float* gamma, const float* beta, float* mean, float* rstd, float* scale, float* shift,
                          float* running_mean, float* running_var, double* colsum_out, long long* num_batches_tracked,
                          ebc_stream_t stream);
/* ebc_bn_bwd_reduce + ebc_bn_bwd_finalize (count = P) in two launches instead of three (no SyncBatchNorm exchange) */
int ebc_bn_bwd_reduce_finalize(int dtype, const void* gy, const void* mask_y, const void* z, const float* mean,
                               const float* rstd, const float* scale, const float* shift, const float* gamma,
                               float* dgamma, float* dbeta, float* coef, void* ws, size_t wsb, long P, int C,
                               ebc_stream_t stream);
int ebc_bn_relu(int dtype, const void* z, const float* scale, const float* shift, void* out, long P, int C,
                ebc_stream_t stream);
int ebc_bn_bwd_apply_flat(int dtype, const void* gy, const void* mask_y, const void* z, const float* mean,
                          const float* rstd, const float* scale, const float* shift, const float* coef, void* dz,
                          float* gmask, long P, int C, ebc_stream_t stream);
/* ModifiedResNet encoder blocks on HIP (models/clip/_clip/image_encoder.py:10-115, blocks.py:56-101: 1x1 -> 3x3 ->
 * avgpool(stride) -> 1x1, downsample = avgpool + 1x1 + BN), NHWC rows [B*H*W][C], C % 8 == 0, H, W even:
 *   ebc_bn_relu_avgpool:  out [B][H/2][W/2][C] = AvgPool2d(2)(relu(z*scale + shift))      (bn2 -> relu2 -> avgpool)
 *   ebc_avgpool2:         out = AvgPool2d(2)(x), same element type                        (downsample "-1" pool)
 *   ebc_avgpool2_bwd:     gx [B][H][W][C] = g[b][y/2][x/2] / 4 (g f32 or the compute dtype -> gx in dtype_out)
 *   ebc_bn_add_relu_flat: y = relu(z*scale + shift + idt*iscale + ishift) (iscale == NULL: + idt)  (bn3 + identity) */
int ebc_bn_relu_avgpool(int dtype, const void* z, const float* scale, const float* shift, void* out, int B, int H, int W,
                        int C, ebc_stream_t stream);
int ebc_avgpool2(int dtype_in, int dtype_out, const void* x, void* out, int B, int H, int W, int C, ebc_stream_t stream);
int ebc_avgpool2_bwd(int dtype_in, int dtype_out, const void* g, void* gx, int B, int H, int W, int C, ebc_stream_t stream);
int ebc_bn_add_relu_flat(int dtype, const void* z, const float* scale, const float* shift, const void* idt,
                         const float* iscale, const float* ishift, void* y, long P, int C, ebc_stream_t stream);
/* 1x1 conv weight [N][K] f32 (nn.Conv2d [N][K][1][1]) -> wk [N][K] and wt [K][N] in dtype (the GEMM operands of the
 * forward and of the data gradient), one launch; N, K multiples of 32 */
int ebc_prep_weights_1x1(int dtype, const float* w, void* wk, void* wt, int N, int K, ebc_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Optimizer step: Adam with the GradScaler folded in.  Replaces the reference's
 * Adam(params, lr, weight_decay) (utils/train_utils.py:80-85) driven under GradScaler (trainer.py:123) as
 * grad_scaler.step(optimizer); grad_scaler.update() (train.py:54-57), i.e. torch.optim.Adam (L2 weight decay,
 * no amsgrad / maximize) + torch.amp.GradScaler's inf check, unscale, skip and scale update.
 * tensors[n]: HOST array of f32 device tensors (param, grad, exp_avg, exp_avg_sq, numel), any n.
 * step: DEVICE float[2], the optimizer's step count; scaler: DEVICE float[2][3] = {scale, growth_tracker,
 *   found_inf} x 2, or NULL (no loss scaling: bf16 / fp32 training).  A call reads entry [parity] of each and
 *   writes entry [1 - parity] (the next step count; the next scale and tracker and a cleared found_inf), so the
 *   caller flips each parity after every call.
 * With a scaler, any non-finite gradient skips the update (params, moments and step count unchanged) and backs
 *   the scale off; otherwise the gradients are divided by the scale (and, write_unscaled_grad = 1, written back
 *   unscaled as GradScaler.unscale_ leaves them) and the scale grows by growth_factor every growth_interval
 *   applied steps.
 * Two launches (check, update) per 32 tensors; arithmetic as torch's fused Adam (tests/test_gpu_optim.py). */
typedef struct {
    float* param;
    float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    long numel;
} EbcAdamTensor;
int ebc_adam_step(const EbcAdamTensor* tensors, int n, float* step, int step_parity, float* scaler, int scaler_parity,
                  double lr, double beta1, double beta2, double eps, double weight_decay, double growth_factor,
                  double backoff_factor, int growth_interval, int write_unscaled_grad, ebc_stream_t stream);
/* The same step in two calls, for several parameter groups sharing one GradScaler (torch skips the WHOLE optimizer
 * step when any group has a non-finite gradient): ebc_amp_check over every group's tensors first (found_inf of entry
 * [scaler_parity]), then ebc_adam_update per group (the update launch alone; each call writes the same next scaler
 * state). */
int ebc_amp_check(const EbcAdamTensor* tensors, int n, float* scaler, int scaler_parity, ebc_stream_t stream);
int ebc_adam_update(const EbcAdamTensor* tensors, int n, float* step, int step_parity, float* scaler, int scaler_parity,
                    double lr, double beta1, double beta2, double eps, double weight_decay, double growth_factor,
                    double backoff_factor, int growth_interval, int write_unscaled_grad, ebc_stream_t stream);

/* Weight touch (performance only; the results do not change): the encoder's attention launches read onto the die the
 * frozen weights of the GEMMs after them (attention.hip touch_issue).  mode 1 (default): on; 0: off (A/B, tests). */
int ebc_set_weight_touch(int mode);

/* ------------------------------------------------------------------------------------------
 * Measurement (bench.py): in-step kernel durations and profile windows.  Not on the reference's
 * surface; the reference has no instrumentation.
 * ebc_probe_begin(capacity): from now on every launch of the instrumented kernels is bracketed by HIP
 *   events on its own stream (at most `capacity` launches recorded).
 * ebc_probe_end(out, capacity): stops recording, waits for the last event and writes one record per
 *   launch (returns the number recorded; records beyond `capacity` are dropped).
 * ebc_marker(id, stream): launches the named empty kernel `ebc_marker_kernel` (profile window edges). */
enum { EBC_PROBE_GEMM = 1, EBC_PROBE_DACE = 2, EBC_PROBE_ATTN_FWD = 3, EBC_PROBE_ATTN_BWD_DQ = 4,
       EBC_PROBE_ATTN_BWD_DKV = 5, EBC_PROBE_LN_FWD = 6, EBC_PROBE_LN_BWD = 7 };
typedef struct {
    int kind;                 /* EBC_PROBE_* */
    int epi, bm, bn, mode;    /* GEMM: epilogue, tile, MODE (0 plain, 1 implicit 3x3 conv, 2 conv weight gradient) */
    int m, n, k;              /* GEMM: problem; DACE: B, total points, grid g; attention: B, L, heads; LN: rows */
    float ms;                 /* measured duration */
} EbcProbeRecord;
int ebc_probe_begin(int capacity);
int ebc_probe_end(EbcProbeRecord* out, int capacity);
int ebc_marker(int id, ebc_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* EBC_HIP_H */
