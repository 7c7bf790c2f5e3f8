/*
 * vit_hip.h — C-ABI of libvit_hip.so, the MI355X (gfx950 / CDNA4) compute library behind the drop-in
 * `VisionTransformer` package (vision-transformer_amd/VisionTransformer).
 *
 * The reference (SiddhantSKarki/Vision-Transformer) has no FFI: its boundary is the torch.nn.Module API and every op
 * below replaces an ATen call site on the training hot path (SURVEY.md §2 table "ATen op call sites").  Each entry
 * point cites the reference line(s) whose arithmetic it replaces.
 *
 * Conventions (all entry points):
 *   - plain device pointers + int64 sizes; no torch types; dtype enums below;
 *   - `stream` is a hipStream_t passed as void*; every launch is asynchronous on it; no device sync, no allocation
 *     (callers own all buffers and workspaces — the PyTorch caching allocator in the host package);
 *   - return 0 on success, a nonzero vit_status on failure with a thread-local message in vit_last_error();
 *   - re-entrant; the only process-wide state is the option table of vit_set_option (below), whose defaults are the
 *     shipped configuration.  The library never reads the environment.
 */
#ifndef VIT_HIP_H
#define VIT_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VIT_ABI_VERSION 14

typedef enum { VIT_OK = 0, VIT_ERR_INVALID = 1, VIT_ERR_LAUNCH = 2 } vit_status;
typedef enum { VIT_F32 = 0, VIT_BF16 = 1, VIT_MASK4 = 2 } vit_dtype;

/* VIT_MASK4: a bit mask of an [m][n] tensor (ReLU / dropout masks saved by the forward for the backward): byte
 * ((i/4)*ceil(n/4) + j/4)*4 + i%4, bit j%4; 4*ceil(m/4)*ceil(n/4) bytes.  One byte = 4 columns of a row; one dword =
 * a 4 x 4 block (byte = row).  8x smaller than the bf16 tensor it replaces as a mask source. */
typedef enum { VIT_ACT_NONE = 0, VIT_ACT_RELU = 1, VIT_ACT_GELU = 2 } vit_act;

/* Launch flags (vit_gemm_desc.flags, vit_attn_bwd `flags`).
 * VIT_FLAG_SHARED_CUS: other kernels may hold compute units while this launch runs — RCCL all-reduce kernels of the
 *   data-parallel backward overlap it.  Kernels that otherwise run a persistent one-workgroup-per-CU grid with a
 *   static item assignment (the bf16 GEMM's wide-epilogue kinds, the fused attention backward) then launch one
 *   workgroup per item, so the hardware places work on whichever CUs are free instead of a workgroup waiting for a
 *   CU a collective holds.  Same arithmetic, bitwise-identical results. */
#define VIT_FLAG_SHARED_CUS 1

int vit_abi_version(void);
const char* vit_last_error(void);

/* Launch options (process-wide; every name's default is the shipped configuration).  They choose between kernel
 * variants that compute the same function — A/B runs and the per-variant tests use them — and are the only switches
 * the library has: nothing is read from the environment, so a user's environment cannot change which kernels run.
 *   "gemm_impl"          0 automatic (default); 1 / 2 / 4 force the bf16 GEMM kernel generation (register-staged
 *                        128x128 / LDS-DMA 128x128 / LDS-DMA 256x256 ping-pong)
 *   "gemm_tail"          0 (default since round 5): 1 = split-K tail for a last round of 256x256 tiles that fills at
 *                        most half the CUs.  With the package's two-stream forward and backward the other stream
 *                        fills those CUs instead: the tails measured 0.18 ms/step slower at C2
 *   "gemm_tail_min_kt"   40: minimum k-tiles (K / 64) for that tail (with the tail on and the weight gradients on their
 *                        own stream, the QKV input gradient's tail at K = 2304 (36) measured 0.35 ms/step slower)
 *   "splitk_min_kt"      0 (automatic): minimum k-tiles per K-slice in vit_gemm_split_k_hint
 *   "gemm_group_m"       0 (automatic): tile-row group size of the 256x256 tile order
 *   "gemm_epi_general"   0: 1 forces the general (unspecialised) GEMM epilogue
 *   "gemm_persist"       1: persistent one-workgroup-per-CU grid for the wide-epilogue GEMM kinds (0: one per tile)
 *   "attn_fwd_split"     0: 1 forces the tiled attention forward for T <= 256
 *   "attn_bwd_split"     0: 1 forces the tiled attention backward for T <= 256
 *   "attn_bwd_grid"      0 (automatic): workgroups of the persistent attention backward
 *   "ln16"               1: the 16-B-per-lane LayerNorm forward where the layout allows it
 *   "ln_al"              1: LayerNorm backward accumulators in LDS (0: registers)
 *   "attn_fwd_ring"      1: the persistent ring attention forward for T <= 256 (0: one workgroup per (image, head))
 *   "gemm_tail_v2"       0: 1 runs the tile rows of a last round of 256x256 tiles at most half full that the split-K
 *                        tail does not take as 128x128 tiles (two workgroups per CU) in a second launch (measured
 *                        slower at C2: 33.0 vs 31.6 ms/step)
 *   "splitk_rounds"      1: rounds of 256 workgroups the weight-gradient K split aims at (vit_gemm_split_k_hint)
 *   "attn_fwd_grid"      0 (automatic: one workgroup per CU): workgroups of the persistent ring attention forward
 *                        when the call's own max_wgs is 0
 * vit_set_option returns VIT_ERR_INVALID for an unknown name; vit_get_option returns INT64_MIN for one. */
int vit_set_option(const char* name, int64_t value);
int64_t vit_get_option(const char* name);

/* ------------------------------------------------------------------------------------------------------------
 * GEMM with fused epilogue:  C[i][j] = epi( alpha * sum_r A(i,r) * B(j,r) )
 *   A(i,r) at a[i*lda + r] when a_kcontig, else a[r*lda + i]   (same for B with ldb / b_kcontig)
 *   epi(v): v += beta*C_old (f32 out only); v += bias[j]; act; v *= (aux(i,j) > 0) when aux (aux_dtype VIT_MASK4:
 *           v *= aux bit);
 *           dropout(p, seed, index i*n + j) with 1/(1-p) scale; v += res(row(i), j) where row(i) = i % res_rowmod
 *           (res_rowmod == 0: i); stored at C[orow(i)*ldc + j], orow(i) = (i/G)*Gs + i%G when out_group_rows = G > 0.
 * Replaces: nn.Linear (transformer.py:12-18,38,56,58; vit.py:70,73), the conv-as-GEMM (vit.py:21-28), and all their
 * autograd dgrad/wgrad GEMMs; dropout (transformer.py:47,59); residual adds (transformer.py:77-78); ReLU (:57).
 * bf16 inputs run on v_mfma_f32_16x16x32_bf16 (fp32 accumulate); f32 inputs on v_mfma_f32_32x32x2_f32 (exact fp32).
 * ------------------------------------------------------------------------------------------------------------ */
typedef struct vit_gemm_desc {
  const void* a;
  const void* b;
  void* c;
  int64_t lda, ldb, ldc;
  int64_t m, n, k;
  int32_t a_kcontig, b_kcontig;
  int32_t in_dtype;   /* vit_dtype of A and B */
  int32_t out_dtype;  /* vit_dtype of C */
  float alpha, beta;
  const float* bias;  /* [n] or NULL */
  int32_t act;        /* vit_act */
  int32_t aux_dtype;
  const void* aux;    /* relu-backward mask source (keep where aux > 0) or NULL */
  int64_t ldaux;
  const void* res;    /* residual added last, or NULL */
  int64_t ldres;
  int64_t res_rowmod;
  int32_t res_dtype;
  float dropout_p;    /* 0 disables */
  uint32_t dropout_seed;
  int32_t split_k;    /* >1: K split over workgroups, fp32 slabs in workspace, deterministic reduce */
  int64_t out_group_rows, out_group_stride;
  void* workspace;
  int64_t workspace_bytes;
  /* NULL, or [ceil(m/256)][n] f32: per-256-row-block column sums of C as stored (after the epilogue and the
   * out_dtype rounding) — the bias gradient of the layer whose input gradient C is (transformer.py Linear backward),
   * finished by vit_colsum_finish.  Requires out_group_rows == 0. */
  float* colsum_part;
  /* NULL, or a VIT_MASK4 buffer for C: the dropout keep bits when the epilogue applies dropout (transformer.py:47,59),
   * else (C as stored > 0) — the ReLU-backward mask (transformer.py:57).  Requires out_group_rows == 0. */
  void* mask_out;
  /* 0/1, or S: the dropout index of output row i is (i * S) * n + j — C computes rows i*S of a larger [m*S][n] tensor
   * (the last block's token-0 rows, ldA = S*K), and its dropout draws the same bits as the full tensor's rows. */
  int64_t dropout_row_stride;
  int32_t flags;      /* VIT_FLAG_* */
  /* 0, or R0: C's row i is row i + R0 of the tensor its dropout indices refer to ((i + R0) * S * n + j with S the
   * row stride above): a GEMM over a row range of a larger tensor (one half-batch chain of the forward) draws the
   * same bits as the whole tensor's rows (ABI 13). */
  int64_t dropout_row0;
} vit_gemm_desc;

/* Workspace vit_gemm can use: split_k > 1: the K-split fp32 slabs (required).  split_k <= 1: the slabs of the split-K
 * tail (when the 256x256 tiles leave the last round of the 256 CUs at most half full, those tile rows run split-K
 * over the idle CUs; option "gemm_tail" 0 disables it), or 0.  Without it (NULL / too small) the GEMM runs unsplit. */
int64_t vit_gemm_workspace_bytes(const vit_gemm_desc* d);
/* Recommended split_k for C[m][n] with reduction depth k and input dtype (VIT_BF16 / VIT_F32) on the kernel vit_gemm
 * will pick: fills one round of the 256 CUs with output tiles x K-slices, each slice >= 4 (bf16) / 8 (f32)
 * k-tiles deep.  Used for the weight-gradient GEMMs (reduction over B*T rows; transformer.py Linear backward). */
int vit_gemm_split_k_hint(int64_t m, int64_t n, int64_t k, int in_dtype);
int vit_gemm(const vit_gemm_desc* d, void* stream);

/* ------------------------------------------------------------------------------------------------------------
 * Patch embedding (vit.py:21-29,39-42).
 *   vit_im2col: x[B][C][H][W] (x_dtype) -> cols[B*N][C*P*P] (dtype), column order (c, kh, kw) = conv weight order,
 *               patch order row-major over (H/P, W/P).  The GEMM epilogue then adds conv bias + pos (res_rowmod = N)
 *               and writes rows (b, n) to x0[b*T + n] (out_group_rows = N, out_group_stride = T).
 *   vit_embed_cls: x0[b*T + N][:] = cls[b][:] + pos[N][:]   (CLS appended LAST, vit.py:41)
 * ------------------------------------------------------------------------------------------------------------ */
int vit_im2col(const void* x, int32_t x_dtype, void* cols, int32_t dtype, int64_t B, int64_t C, int64_t H,
               int64_t W, int64_t P, void* stream);
/* vit_col2im: the inverse permutation of vit_im2col (k = s = P): x[B][C][H][W] (x_dtype) <- cols[B*N][C*P*P] (dtype).
 * Used for the input-image gradient (conv dgrad, vit.py:21-28 backward) when the caller's input requires grad. */
int vit_col2im(const void* cols, int32_t dtype, void* x, int32_t x_dtype, int64_t B, int64_t C, int64_t H, int64_t W,
               int64_t P, void* stream);
int vit_embed_cls(const float* cls, const float* pos, void* x0, int32_t dtype, int64_t B, int64_t T, int64_t D,
                  void* stream);

/* ------------------------------------------------------------------------------------------------------------
 * LayerNorm (nn.LayerNorm, transformer.py:71-72,77-78; vit.py:72), fp32 statistics.
 *   fwd: y = (x - mean) * rstd * gamma + beta; saves mean/rstd [rows].
 *   bwd: dx = rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dy * gamma;
 *        dx_out = dx (+ dres when dres != NULL)                    — fused residual-gradient add (transformer.py:77-78)
 *        drop_out = dx_out * keep(drop_seed, i*cols + j)            — fused dropout backward of the producer branch,
 *                   WITHOUT the 1/(1-p) scale (exact in bf16: the consumers apply it, e.g. as GEMM alpha); with
 *                   drop_mask (VIT_MASK4 [rows][cols], the producing GEMM's mask_out) the keep bits are read from it
 *                   instead of re-hashed
 *        dgamma/dbeta: per-workgroup partials in `partial` [2][nparts][cols], reduced by vit_colsum_finish
 *        (deterministic); with `osum` != 0 also partial [2] = column sums of the stored gradient output (drop_out
 *        / (1-p) when drop_out is given, else dx_out) — the bias gradient of the Linear that consumes it, so
 *        [3][nparts][cols].
 * ------------------------------------------------------------------------------------------------------------ */
int vit_layernorm_fwd(const void* x, int64_t ldx, const float* gamma, const float* beta, void* y, int64_t ldy,
                      float* mean, float* rstd, int64_t rows, int64_t cols, float eps, int32_t dtype, void* stream);
int64_t vit_layernorm_bwd_parts(int64_t rows, int64_t cols);
int vit_layernorm_bwd(const void* dy, int64_t lddy, const void* x, int64_t ldx, const float* gamma,
                      const float* mean, const float* rstd, const void* dres, void* dx_out, void* drop_out,
                      float drop_p, uint32_t drop_seed, const void* drop_mask, float* partial, int32_t osum,
                      int64_t rows, int64_t cols, int32_t dtype, void* stream);

/* ------------------------------------------------------------------------------------------------------------
 * Multi-head self-attention (transformer.py:9-31 per head, :44-45 concat): qkv[B*T][3*D] with Q at columns
 * h*hd, K at D + h*hd, V at 2D + h*hd; o[B*T][D] (heads concatenated, same column order as torch.cat).
 *   o = softmax(scale * Q K^T) V with scale = sqrt(hd) in the reference (multiplied, transformer.py:24);
 *   lse[B][H][T] (natural log of the row softmax denominator, scaled-logit domain) saved for backward;
 *   probs [B][H][T][T] f32 optional (the `.attention_probs` side attribute, transformer.py:48).
 * bf16 & hd == 64: flash-style MFMA kernels (K/V tiles in LDS, online softmax); otherwise a generic VALU kernel.
 * Under the reference's x sqrt(hd) logit scale most softmax rows saturate and dS = P (dP - delta) becomes a small
 *   difference, so delta = rowsum(dO * O) must be exact to fp32 rounding:
 *   - the fused backward (bf16, hd == 64, T <= 256: every ViT-B/L 224^2 config) forms delta = rowsum(P * dP) itself
 *     from the fp32 P and dP it computes anyway; it reads neither `o` nor `o32`;
 *   - the tiled backward (T > 256) takes delta from o32 when given: the forward then also stores O unrounded,
 *     [B*T][D] f32 (o32 == NULL: the bf16 O, standard flash-attention practice, cheaper but inexact).
 *   vit_attn_bwd_uses_o32() says which one a shape runs (1: pass o32 to the forward and the backward).
 * fwd max_wgs (ABI 14): 0 = automatic (one workgroup per CU, or option "attn_fwd_grid"); > 0 = the persistent ring
 *   forward (T <= 256) runs at most max_wgs workgroups — per call, so two callers on two threads or streams never
 *   share the choice (the package's two-stream forward gives one chain 3/4 of the CUs this way).  Other forms ignore it.
 * bwd: dqkv[B*T][3*D]; workspace = vit_attn_bwd_workspace_bytes.
 * ------------------------------------------------------------------------------------------------------------ */
int vit_attn_fwd(const void* qkv, void* o, float* o32, float* lse, float* probs, int64_t B, int64_t T, int64_t H,
                 int64_t hd, float scale, int32_t dtype, int64_t max_wgs, void* stream);
int vit_attn_bwd_uses_o32(int64_t B, int64_t T, int64_t H, int64_t hd, int32_t dtype);
int64_t vit_attn_bwd_workspace_bytes(int64_t B, int64_t T, int64_t H, int64_t hd, int32_t dtype);
int vit_attn_bwd(const void* qkv, const void* o, const float* o32, const void* d_o, const float* lse, void* dqkv,
                 int64_t B, int64_t T, int64_t H, int64_t hd, float scale, int32_t dtype, void* workspace,
                 int32_t flags, void* stream);

/* Query 0 only (round 5): the last encoder block, whose output the classifier reads at token 0 only (vit.py:80), needs
 * attention output row 0 of every image (queries 1..T-1 feed rows nothing reads) and, in the backward, has a nonzero
 * output gradient on row 0 only; every softmax row is independent, so row 0 alone is the same function, in O(T hd) per
 * (image, head) instead of O(T^2 hd).
 *   fwd: o[b*T][D] (row 0 of every image; other rows untouched), lse[b][h][0].
 *   bwd: from d_o0[b][D] (image b's row-0 output gradient, row stride ldo): dQ row 0, every row of dK and dV into
 *        dqkv[B*T][3*D] (dQ rows 1..T-1 untouched).  P is recomputed as the forward forms it (row max, exp2, 1/sum;
 *        no log-sum-exp round trip: a one-key row has P = 1, dS = 0 exactly); delta = sum_k P dP from fp32 P and dP.
 *   fp32 arithmetic, outputs rounded once; hd <= 128, hd % 4 == 0, T <= 4096. */
int vit_attn_fwd_row0(const void* qkv, void* o, float* lse, int64_t B, int64_t T, int64_t H, int64_t hd, float scale,
                      int32_t dtype, void* stream);
int vit_attn_bwd_row0(const void* qkv, const void* d_o0, int64_t ldo, void* dqkv, int64_t B, int64_t T, int64_t H,
                      int64_t hd, float scale, int32_t dtype, void* stream);

/* ------------------------------------------------------------------------------------------------------------
 * Reductions / elementwise.
 *   vit_colsum: out[j] = beta*out[j] + alpha * sum_i x[i*ldx + j]  (bias / pos / LN-affine gradients); deterministic.
 *   vit_colsum_finish: outs[s][j] = beta*outs[s][j] + sum_p part[s][p][j] for s < nsets (<= 3), summed in a fixed
 *               order — second stage of the column sums fused into vit_gemm (colsum_part) / vit_layernorm_bwd.
 *   vit_copy2d: dst[orow(i)*ldd + j] = beta*dst + src[irow(i)*lds + j] with optional row grouping on the source
 *               (irow(i) = (i/G)*Gs + i%G) — token-0 gather (vit.py:80), CLS-gradient copy, dropout-free casts.
 *   vit_dropout_bwd: y = x * keep(seed, i) * scale  (transformer.py:47,59 backward: scale = 1/(1-p); the engine
 *                    passes 1 and folds 1/(1-p) into the consumers, so the stored masked gradient is exact).
 *   vit_gelu_fwd/bwd: exact-erf GELU (vit.py:71) on f32.
 *   vit_softmax_xent: per-row softmax cross entropy (train.py:81,93): loss = mean_i(-log p[i][y_i]) and
 *                     dlogits = (softmax - onehot) / rows, in one pass.
 * ------------------------------------------------------------------------------------------------------------ */
int64_t vit_colsum_workspace_bytes(int64_t rows, int64_t cols);
int vit_colsum(const void* x, int64_t ldx, int32_t dtype, int64_t rows, int64_t cols, float* out, float alpha,
               float beta, void* workspace, void* stream);
int vit_colsum_finish(const float* part, int64_t nparts, int64_t cols, int32_t nsets, float* out0, float* out1,
                      float* out2, float beta, void* stream);
/* vit_colsum_finish_batch: up to 8 vit_colsum_finish jobs in one launch (the bias / LN-affine gradients of one encoder
 * block), each job's result bitwise that of its own vit_colsum_finish. */
typedef struct {
  const float* part;  /* [nsets][nparts][cols] */
  int64_t nparts, cols;
  int32_t nsets;      /* 1..3 */
  float* out[3];
  float beta;
} vit_colsum_job;
int vit_colsum_finish_batch(const vit_colsum_job* jobs, int32_t njobs, void* stream);
int vit_copy2d(const void* src, int64_t lds, int32_t src_dtype, void* dst, int64_t ldd, int32_t dst_dtype,
               int64_t rows, int64_t cols, int64_t src_group_rows, int64_t src_group_stride, float beta,
               void* stream);
int vit_dropout_bwd(const void* x, void* y, int32_t dtype, int64_t n, float p, uint32_t seed, float scale,
                    void* stream);
/* dx = dy * (y > 0): ReLU backward for the module-level FeedForward path (transformer.py:57). */
int vit_relu_bwd(const void* dy, const void* y, void* dx, int32_t dtype, int64_t n, void* stream);
/* y[i][j] = x[i][j] * bit(mask, i, j) * scale — a dropout backward from the forward's saved VIT_MASK4 keep bits
 * (transformer.py:59 backward at the head, where the gradient covers the token-0 rows only). */
int vit_mask4_apply(const void* x, int64_t ldx, int32_t x_dtype, void* y, int64_t ldy, int32_t y_dtype,
                    const void* mask, int64_t rows, int64_t cols, float scale, void* stream);
int vit_gelu_fwd(const float* x, float* y, int64_t n, void* stream);
int vit_gelu_bwd(const float* x, const float* dy, float* dx, int64_t n, void* stream);
int vit_softmax_xent(const float* logits, const int64_t* labels, int64_t rows, int64_t classes, float* loss,
                     float* dlogits, float* workspace, void* stream);

/* ------------------------------------------------------------------------------------------------------------
 * Image pipeline of the training loader (train.py:151-155: convert('RGB') -> transforms.Resize((S, S)) ->
 * ToTensor; BrainTumorDataset.py:35-39 / CIFAR10 :157-159 feed it PIL images).  A batch of raw uint8 HWC images of
 * any sizes (ragged allowed), packed into one byte buffer `src`, described by meta[B][4] = (byte offset, H, W, C)
 * (int64, DEVICE memory; C in {1: L, 2: LA, 3: RGB, 4: RGBA} -> RGB as PIL converts), becomes out[B][3][S_h][S_w]
 * (VIT_F32 or VIT_BF16) = PIL-bilinear-resized pixel / 255, bit-exact with Pillow's 8-bit two-pass resampler.
 *   vit_resize_ksize: taps per output sample for one axis (in_size -> out_size); pass the max over the batch and axes.
 *   workspace: vit_resize_workspace_bytes(B, S_h, S_w, ksize) bytes (per-image coefficient tables).
 * ------------------------------------------------------------------------------------------------------------ */
int vit_resize_ksize(int64_t in_size, int64_t out_size);
int64_t vit_resize_workspace_bytes(int64_t B, int64_t out_h, int64_t out_w, int64_t ksize);
int vit_resize_to_tensor(const void* src, const int64_t* meta, int64_t B, int64_t out_h, int64_t out_w, int64_t ksize,
                         void* out, int32_t out_dtype, void* workspace, int64_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------------------------
 * Optimizer (train.py:66,96: torch.optim.AdamW(lr, weight_decay=1e-4), betas (0.9, 0.999), eps 1e-8) as ONE
 * multi-tensor launch over a device-resident chunk table; also refreshes the compute-dtype shadow weights.
 *   p *= 1 - lr*wd;  m = b1*m + (1-b1)*g*gs;  v = b2*v + (1-b2)*(g*gs)^2;
 *   p -= (lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps);  shadow = (dtype) p   (gs = grad_scale, e.g. 1/world_size)
 * vit_pack: shadow = (dtype) src over the same table layout (used after external writes to the fp32 params).
 * ------------------------------------------------------------------------------------------------------------ */
typedef struct vit_tensor_chunk {
  float* p;
  const float* g;
  float* m;
  float* v;
  void* shadow; /* NULL: no shadow for this chunk */
  int64_t n;
} vit_tensor_chunk;

int vit_adamw(const vit_tensor_chunk* table_dev, int64_t nchunks, float lr, float beta1, float beta2, float eps,
              float weight_decay, float bias_corr1, float bias_corr2, float grad_scale, int32_t shadow_dtype,
              void* stream);
int vit_pack(const vit_tensor_chunk* table_dev, int64_t nchunks, int32_t shadow_dtype, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* VIT_HIP_H */
