/*
 * mtts_decoder.h -- C ABI of the CFM decoder operators in libmtts_hip.so (gfx950).
 *
 * Same conventions as mtts.h (caller-owned buffers, negative mtts_status on error, thread-local
 * mtts_last_error(), stream-ordered, no host synchronisation).  Activations are TOKEN-MAJOR:
 * [rows = batch*time, channels], channels contiguous, fp32 in HBM.
 *
 * Reference operators replaced (matcha/models/components/..., relative to the reference root):
 *   mtts_conv_gemm / mtts_conv_wgrad  <- nn.Conv1d k3/k1, stride-2 Downsample1D, ConvTranspose1d
 *                                        Upsample1D (decoder.py:51-116, 189-251) and the Linear layers
 *                                        of BasicTransformerBlock / FeedForward (transformer.py:105-188,
 *                                        diffusers Attention to_q/k/v/to_out), forward and backward
 *   mtts_gn_mish_fwd / _bwd           <- Block1D's GroupNorm(8) + Mish + mask (decoder.py:58-66) with
 *                                        Resnet1D's time-embedding add (decoder.py:82-83) and the final
 *                                        GroupNorm + Mish (decoder.py:366-368)
 *   mtts_layernorm_fwd / _bwd         <- BasicTransformerBlock norm1 / norm3 (transformer.py:316, 345)
 *   mtts_attention_fwd / _bwd         <- diffusers AttnProcessor2_0 scaled_dot_product_attention with
 *                                        the float 0/1 mask as an additive key bias (transformer.py:320-328)
 *   mtts_cfm_pack_fwd / _bwd          <- phi_t (flow_matching.py:138) + pack([x, mu], "b * t") (decoder.py:288)
 *   mtts_time_embedding               <- SinusoidalPosEmb.forward (decoder.py:8-31)
 *   mtts_rows_linear_fwd / _bwd       <- TimeStepEmbeddingNet (decoder.py:33-49: Linear -> SiLU -> Linear) and
 *                                        every Resnet1D.mlp (decoder.py:71-72, 80-81: Mish -> Linear) on the B
 *                                        time-embedding rows, forward and backward
 */
#ifndef MTTS_DECODER_H_
#define MTTS_DECODER_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MTTS_PREC_FP32 0 /* fp32 operands, v_mfma_f32_32x32x2_f32 (parity mode)            */
#define MTTS_PREC_BF16 1 /* bf16 operands, v_mfma_f32_32x32x16_bf16, fp32 accumulation      */

#define MTTS_ACT_NONE 0
#define MTTS_ACT_GELU 1  /* erf GELU (diffusers GELU, approximate="none") */
#define MTTS_ACT_DGELU 2 /* multiply by GELU'(aux[row, n]) -- backward through a GELU */
#define MTTS_ACT_RELU 3  /* max(x, 0) */
#define MTTS_ACT_DRELU 4 /* zero where aux[row, n] <= 0 -- backward through a ReLU (aux: its output) */

#define MTTS_CONV_MAX_TAPS 8
#define MTTS_GEMM_GLDS 32  /* schedule ids 32.. : bf16 LDS-DMA kernels (csrc/conv_gemm_glds.hip)   */
#define MTTS_GEMM_WREG 96  /* schedule id 96: bf16 weight-stationary kernel, K <= 256 linears (csrc/conv_gemm_wreg.hip) */

/*
 * Implicit GEMM  C[row(b,u), n] = epi( sum_{j<ntaps} sum_{c<cin} A[b*Ti + u*in_stride + off[j], c]
 *                                                               * a_scale[...] * W[n, j*cin + c] )
 * for b < nb, u < To; input rows outside [0, Ti) read as zero.  epi = (+ bias[n]) -> [C_pre <- value]
 * -> act -> (+ residual[row, n]) -> (* c_scale[row]);  row(b,u) = b*To_full + u*out_stride + out_off.
 * act MTTS_ACT_DGELU / MTTS_ACT_DRELU multiply by GELU'(aux) / [aux > 0] instead (aux/ldaux: the saved
 * pre-activation / activation output).
 * W is packed [N][Kp] (bf16 for MTTS_PREC_BF16, fp32 otherwise), K = ntaps*cin, Kp >= K, Kp % 8 == 0.
 * Requirements: cin % 8 == 0, lda % 4 == 0, A and W 16-byte aligned, and off[] an arithmetic
 * progression (off[j] = off[0] + j*(off[1]-off[0]): every conv, dgrad and stride-phase GEMM is one).
 */
typedef struct mtts_conv_gemm_args {
    const float *A;
    const float *a_scale; /* [nb*Ti] or NULL */
    int32_t lda, Ti, To, nb, in_stride, ntaps;
    int32_t off[MTTS_CONV_MAX_TAPS];
    int32_t cin;
    const void *W;
    int32_t N, K, Kp;
    const float *bias; /* [N] or NULL */
    int32_t act;
    const float *residual; /* rows addressed like C, or NULL */
    int32_t ldr;
    const float *c_scale; /* [nb*To_full] or NULL */
    float *C;
    int32_t ldc, To_full, out_stride, out_off;
    float *C_pre;      /* optional: pre-activation values (rows addressed like C, ld = ldc) */
    const float *aux;  /* MTTS_ACT_DGELU: pre-activation input (rows addressed like C) */
    int32_t ldaux;
    float dropout_p;       /* > 0: inverted dropout after act (before residual)                  */
    const uint32_t *seed;  /* device pointer to 2 words: the dropout stream (graph-replay safe)   */
    int32_t flags;         /* MTTS_GEMM_F_* */
} mtts_conv_gemm_args;

/* mtts_conv_gemm_args.flags */
#define MTTS_GEMM_F_BINARY_SCALE 0x1 /* a_scale holds only 0 / 1 (a sequence mask): lets the bf16 path
                                        stage A rows by LDS-DMA, reading zeros for masked rows */
#define MTTS_GEMM_F_A_BF16 0x2       /* A holds bf16 (lda in elements, lda % 8 == 0, cin % 8 == 0; bf16
                                        precision only, LDS-DMA schedules) */
#define MTTS_GEMM_F_C_BF16 0x4       /* C (not C_pre) is written as bf16 (ldc in elements) */
#define MTTS_GEMM_F_FAST_ACT 0x8     /* GELU / GELU' with a 5e-7 (fp32-evaluated) erf approximation (bf16-mixed) */
#define MTTS_GEMM_F_PRE_BF16 0x10    /* C_pre is written and aux read as bf16 (bf16-mixed: the saved pre-activation,
                                        half the bytes; ldc / ldaux in elements, % 4 == 0 for the vector epilogue) */
#define MTTS_GEMM_F_W_SPLIT 0x40     /* bf16 precision: W holds TWO bf16 planes, hi = bf16(w) at W and lo =
                                        bf16(w - hi) at W + N*Kp (elements); every product is A*hi + A*lo (two
                                        MFMAs), i.e. the weights enter with ~16 significant bits instead of 8:
                                        the fp32 weights' rounding -- a STATIC perturbation of the model, the
                                        dominant bf16-mixed loss error -- drops out (mtts_pack_job.lo_off packs it) */
#define MTTS_GEMM_F_A_SPLIT 0x80     /* with MTTS_GEMM_F_W_SPLIT and an fp32 A: A is split on the fly into
                                        hi = bf16(a) and lo = bf16(a - hi) and every product is
                                        A_hi*W_hi + A_hi*W_lo + A_lo*W_hi (three bf16 MFMAs, fp32 accumulate):
                                        ~16 significant bits per operand, the bf16x3 emulation of an fp32 GEMM
                                        (register-staged schedules; the text encoder's forward in the parity
                                        policy) */

#define MTTS_GEMM_F_SPLIT3 0x100     /* bf16 precision, fp32 A, LDS-DMA schedules (round 4): W holds THREE bf16 planes
                                        hi / mid / lo at W, W + N*Kp, W + 2*N*Kp (hi + mid + lo = w exactly; mtts_pack_job
                                        with MTTS_PACK_THREE_PLANES), A is split the same way in the kernel and every
                                        product is the six terms of combined order <= 2^-16 (bf16x6): fp32-faithful
                                        results at bf16 MFMA rates (the parity policy's text encoder forward) */

int mtts_conv_gemm(const mtts_conv_gemm_args *args, int32_t precision, void *hip_stream);
/* Same, with an explicit schedule: 0..17 = register-staged tile configs (csrc/conv_gemm.hip kCfgs;
 * 8..17 bf16-only: 64-wide K steps, two K steps in flight), MTTS_GEMM_GLDS + i = the bf16 LDS-DMA schedules
 * (csrc/conv_gemm_glds.hip), MTTS_GEMM_WREG = the weight-stationary schedule (csrc/conv_gemm_wreg.hip), -1 = heuristic.
 * For tuning and tests; mtts_conv_gemm picks the configuration itself. */
int mtts_conv_gemm_tile(const mtts_conv_gemm_args *args, int32_t precision, int32_t tile_cfg, void *hip_stream);
/* With a caller-owned workspace: lets the bf16 LDS-DMA schedules split K over several workgroups
 * (fp32 partial slabs, combined in a fixed order by a second kernel that also runs the epilogue) when
 * the output alone cannot fill the chip (e.g. the text encoder's 3840-row GEMMs).  tile_cfg as above
 * (-1 = heuristic); splits: 0 = heuristic, 1 = never, >= 2 = that many (LDS-DMA schedules only).
 * mtts_conv_gemm_workspace_size returns the bytes the same (args, precision, tile_cfg, splits) needs
 * (0: no split); a smaller workspace runs the GEMM unsplit. */
size_t mtts_conv_gemm_workspace_size(const mtts_conv_gemm_args *args, int32_t precision, int32_t tile_cfg,
                                     int32_t splits);
int mtts_conv_gemm_ws(const mtts_conv_gemm_args *args, int32_t precision, int32_t tile_cfg, int32_t splits,
                      void *workspace, size_t workspace_bytes, void *hip_stream);

/*
 * Weight gradient of the same implicit GEMM:
 *   dW[n, j*cin + c] = sum_{b,u} dY[row(b,u), n] * A[b*Ti + u*in_stride + off[j], c] * a_scale[...]
 *   db[n]            = sum_{b,u} dY[row(b,u), n]                      (when db != NULL)
 * written (or added, accumulate != 0) to dw[n*sn + c*sc + j*sj] -- any layout of [N, cin, ntaps].
 * Deterministic: split over rows into fp32 partial slabs in the workspace, reduced in a fixed order.
 */
typedef struct mtts_conv_wgrad_args {
    const float *dY;
    int32_t ldy, To_full, out_stride, out_off;
    const float *A;
    const float *a_scale;
    int32_t lda, Ti, To, nb, in_stride, ntaps;
    int32_t off[MTTS_CONV_MAX_TAPS];
    int32_t cin;
    int32_t N, K;
    int32_t flags; /* MTTS_GEMM_F_A_BF16: A holds bf16 (lda in elements; bf16 precision only);
                      MTTS_GEMM_F_BINARY_SCALE: a_scale holds only 0 / 1 (lets the bf16 LDS-DMA schedule
                      drop masked rows by address selection); MTTS_WGRAD_F_DY_BF16: dY holds bf16 (ldy in
                      elements, rows 8-byte aligned; bf16 precision, default schedule) */
} mtts_conv_wgrad_args;
#define MTTS_WGRAD_F_DY_BF16 0x20

size_t mtts_conv_wgrad_workspace_size(const mtts_conv_wgrad_args *args);
int mtts_conv_wgrad(const mtts_conv_wgrad_args *args, int32_t precision, float *dw, int64_t sn, int64_t sc,
                    int64_t sj, float *db, int32_t accumulate, void *workspace, size_t workspace_bytes,
                    void *hip_stream);
/* Same, with an explicit schedule: rows_per_step 32 (or 64, bf16), target_blocks 64..1024 for the
 * row split, depth 1 (or 2, bf16) row steps in flight (-1 = defaults).  For tuning;
 * mtts_conv_wgrad_workspace_size covers every schedule. */
int mtts_conv_wgrad_tile(const mtts_conv_wgrad_args *args, int32_t precision, int32_t rows_per_step,
                         int32_t target_blocks, int32_t depth, float *dw, int64_t sn, int64_t sc, int64_t sj,
                         float *db, int32_t accumulate, void *workspace, size_t workspace_bytes, void *hip_stream);
/* Inside the reduction deferral (mtts_defer_reductions below) the weight-gradient GEMMs are queued too
 * (unless MTTS_DEFER_WGRAD=0) and mtts_flush_reductions launches them batched -- up to 12 per launch, each
 * with its own row split -- before their sums; a queued gradient takes a split plan with fewer, longer
 * splits (the batch fills the chip).  mode 0: that plan for queued gradients only (default); 1: for every
 * call (an immediate call then equals a queued one bitwise); 2: the per-launch plan for every call. */
void mtts_wgrad_plan_mode(int32_t mode);
/* Caps the grid of the weight-gradient launches that follow at `blocks` workgroups, each walking several
 * (tile, split) blocks -- bitwise the same results; 0 (default) = one workgroup per block.  The side-stream
 * flush sets it so the batched gradients leave CUs to the latency-bound work on the main stream. */
void mtts_wgrad_flush_cap(int32_t blocks);

/*
 * y[b,t,c] = mish(GN(h)[b,t,c]) * mask[b,t] + add[b,c]      (mask / add optional)
 * GroupNorm statistics per (b, group) over all T rows x C/G channels (the full padded length, as the
 * reference).  mean/rstd [B,G] are saved for the backward.  C % G == 0, (C/G) % 4 == 0.
 */
int mtts_gn_mish_fwd(const float *h, const float *gamma, const float *beta, const float *mask, const float *add,
                     float *y, float *mean, float *rstd, int32_t B, int32_t T, int32_t C, int32_t G, float eps,
                     void *hip_stream);
size_t mtts_gn_mish_bwd_workspace_size(int32_t B, int32_t C);
/* dh (and dgamma, dbeta [C], dadd [B,C] when non-NULL) from dy and the forward's inputs/statistics;
 * C/G <= 256. */
int mtts_gn_mish_bwd(const float *dy, const float *h, const float *gamma, const float *beta, const float *mask,
                     const float *mean, const float *rstd, float *dh, float *dgamma, float *dbeta, float *dadd,
                     int32_t B, int32_t T, int32_t C, int32_t G, void *workspace, size_t workspace_bytes,
                     void *hip_stream);
/* The same with the activation storage chosen by flags (bf16-mixed mode: the conv output h and the
 * Block1D output y are only GEMM operands and GroupNorm inputs, stored as autocast holds them):
 * forward MTTS_NORM_F_X_BF16 (h bf16) | MTTS_NORM_F_Y_BF16 (y bf16); backward MTTS_NORM_F_X_BF16 |
 * MTTS_NORM_F_Y_BF16 (h and dh bf16) [| MTTS_NORM_F_DY_BF16 (dy bf16)], or 0.  Statistics and sums in
 * fp32; bf16 values are widened exactly and the outputs rounded once. */
int mtts_gn_mish_fwd_ex(const void *h, const float *gamma, const float *beta, const float *mask, const float *add,
                        void *y, float *mean, float *rstd, int32_t B, int32_t T, int32_t C, int32_t G, float eps,
                        int32_t flags, void *hip_stream);
int mtts_gn_mish_bwd_ex(const void *dy, const void *h, const float *gamma, const float *beta, const float *mask,
                        const float *mean, const float *rstd, void *dh, float *dgamma, float *dbeta, float *dadd,
                        int32_t B, int32_t T, int32_t C, int32_t G, int32_t flags, void *workspace,
                        size_t workspace_bytes, void *hip_stream);

/*
 * Counter-based dropout (train mode, nn.Dropout semantics: keep with prob 1-p, scale 1/(1-p)).
 * keep(row, col) is a hash of (seed[0], seed[1], row, col); `seed` is a DEVICE pointer (2 words) so a
 * captured HIP graph draws a fresh mask on every replay, and a backward pass regenerates the exact
 * mask the forward used without storing it.  y = x * keep / (1-p) over [rows, cols], leading dim ld.
 */
int mtts_dropout_apply(const float *x, float *y, int32_t rows, int32_t cols, int32_t ld, float p,
                       const uint32_t *seed, void *hip_stream);
/* Backward of an epilogue "act -> dropout" from the forward OUTPUT y: dx = dy * [y > 0] (act
 * MTTS_ACT_RELU) * keep(seed, r, c) / (1-p) (p > 0).  Rows/cols index like mtts_dropout_apply. */
int mtts_act_dropout_bwd(const float *dy, const float *y, float *dx, int32_t rows, int32_t cols, int32_t ld,
                         int32_t act, float p, const uint32_t *seed, void *hip_stream);
/* mtts_act_dropout_bwd with the output's row scale first: dx = (dy * row_scale[r]) -> act' -> dropout
 * (row_scale [rows] or NULL).  The text encoder FFN's backward through its masked output
 * (text_encoder.py:253, `* x_mask`) without materialising dy * mask. */
int mtts_act_dropout_bwd_scaled(const float *dy, const float *y, const float *row_scale, float *dx, int32_t rows,
                                int32_t cols, int32_t ld, int32_t act, float p, const uint32_t *seed,
                                void *hip_stream);

/* LayerNorm over the last dim of x [M, C]; mean/rstd [M] saved.  C % 4 == 0, C <= 1024.  Optional
 * fused tail applied to the normalized output: act MTTS_ACT_RELU, then dropout(p) with the
 * counter-based mask keyed (seed, row, channel) -- the text encoder's LN -> ReLU -> Dropout
 * (text_encoder.py:48-55) and LN -> Dropout (:81-95).  act = MTTS_ACT_NONE, p = 0: plain LayerNorm.
 * act | MTTS_NORM_F_Y_BF16: y is written as bf16 (a GEMM operand in bf16-mixed mode, half the bytes). */
#define MTTS_NORM_F_Y_BF16 0x100
#define MTTS_NORM_F_X_BF16 0x200  /* GroupNorm: the input h (forward and backward) holds bf16           */
#define MTTS_NORM_F_DY_BF16 0x400 /* GroupNorm backward: dy holds bf16 (with X_BF16 | Y_BF16)            */
int mtts_layernorm_fwd(const float *x, const float *w, const float *b, float *y, float *mean, float *rstd,
                       int32_t M, int32_t C, float eps, int32_t act, float dropout_p, const uint32_t *seed,
                       void *hip_stream);
size_t mtts_layernorm_bwd_workspace_size(int32_t M, int32_t C);
/* dx (and dw, db when non-NULL) from dy w.r.t. the forward's (tail) output; the same act / p / seed as
 * the forward (b is needed for the ReLU gate). */
int mtts_layernorm_bwd(const float *dy, const float *x, const float *w, const float *b, const float *mean,
                       const float *rstd, float *dx, float *dw, float *db, int32_t M, int32_t C, int32_t act,
                       float dropout_p, const uint32_t *seed, void *workspace, size_t workspace_bytes,
                       void *hip_stream);
/* Plain LayerNorm backward plus a residual branch's gradient: dx = LN'(dy) + dres (a pre-LN transformer
 * sub-block, transformer.py:316-358, where x feeds both the norm and the residual add). */
int mtts_layernorm_bwd_res(const float *dy, const float *x, const float *w, const float *b, const float *mean,
                           const float *rstd, const float *dres, float *dx, float *dw, float *db, int32_t M,
                           int32_t C, void *workspace, size_t workspace_bytes, void *hip_stream);

/*
 * Batched weight packing (csrc/pack.hip): each job is one affine gather of an fp32 torch weight into
 * (a column block of) a GEMM operand with row stride ld (bf16 or fp32 per `precision`), K ordered
 * tap-major / channel-minor:
 *     dst[r*ld + j*C + c] = src[r*sr + c*sc + (j0 + j*js)*sj]  for j < ntaps, c < C;
 *     dst[r*ld + k'] = 0 for C*ntaps <= k' < Kp  (Kp = columns this job writes).
 * Covers Conv1d forward / dgrad / stride-2 phase layouts, ConvTranspose1d phases and stacked Linear
 * weights (row blocks, or column blocks of the transposed stack).  Kp % 8 == 0, ld % 8 == 0, dst
 * 16-byte aligned.  `jobs` is a HOST array.
 */
typedef struct mtts_pack_job {
    const float *src;
    void *dst;
    int32_t rows, C, ntaps, Kp, ld;
    int64_t sr, sc, sj;
    int32_t j0, js;
    int64_t lo_off; /* bf16 only: > 0 also writes lo = bf16(w - bf16(w)) at dst + lo_off (elements): the
                       second plane of an MTTS_GEMM_F_W_SPLIT operand; 0 = hi plane only.  With
                       MTTS_PACK_THREE_PLANES or'ed in: mid = bf16(w - hi) at dst + off and lo = bf16(w - hi - mid)
                       at dst + 2 * off (off = lo_off without the flag): an MTTS_GEMM_F_SPLIT3 operand */
} mtts_pack_job;
#define MTTS_PACK_THREE_PLANES (1ll << 62)

int mtts_pack_weights(const mtts_pack_job *jobs, int32_t njobs, int32_t precision, void *hip_stream);

/*
 * Flash attention of the decoder's transformer blocks (transformer.py:191-370: diffusers Attention,
 * 4 heads x 64, AttnProcessor2_0 -> F.scaled_dot_product_attention with the FLOAT 0/1 mask, i.e. an
 * additive per-key bias).  scores[b,h,i,j] = scale * q_i.k_j + key_bias[b,j]; o = softmax(scores) v.
 * Token-major rows (row = b*T + t), head h at columns [h*D, h*D+D): q/k/v may be column slices of one
 * fused QKV buffer (shared row stride ldq).  D: a multiple of 8 up to 96 (the decoder uses 64).  lse [B,H,T] receives log2(sum_j 2^(scores*log2 e))
 * for the backward.  Rows and strides: 16-byte aligned pointers, strides multiples of 4 floats.
 */
typedef struct mtts_attn_args {
    const float *q, *k, *v;
    int32_t ldq;
    const float *key_bias; /* [B*T] or NULL (no bias) */
    float *o;
    int32_t ldo;
    float *lse;
    int32_t B, T, H, D;
    float scale;
    float dropout_p;      /* dropout on the probabilities (text encoder, text_encoder.py:222); 0 = off */
    const uint32_t *seed; /* device pointer (2 words), keyed (seed, (b*H+h)*T + q, key) */
    int32_t flags;        /* MTTS_ATTN_F_IO_BF16: q/k/v/o and the gradients' dout/dq/dk/dv hold bf16
                             (bf16 precision; strides in elements); lse / Drow stay fp32 */
} mtts_attn_args;
#define MTTS_ATTN_F_IO_BF16 0x1

typedef struct mtts_attn_grads {
    const float *dout; /* dL/do, row stride lddo */
    int32_t lddo;
    float *dq, *dk, *dv; /* written (not accumulated), shared row stride ldd */
    int32_t ldd;
} mtts_attn_grads;

int mtts_attention_fwd(const mtts_attn_args *args, int32_t precision, void *hip_stream);
size_t mtts_attention_bwd_workspace_size(int32_t B, int32_t T, int32_t H);
/* Deterministic backward (no atomics): a dQ pass (also forms rowsum(dO*O)) then a dK/dV pass. */
int mtts_attention_bwd(const mtts_attn_args *args, const mtts_attn_grads *grads, int32_t precision,
                       void *workspace, size_t workspace_bytes, void *hip_stream);

/* Rotary position embedding of the text encoder's attention (text_encoder.py:99-143): on the q and
 * k column blocks of a fused token-major projection x [rows = B*T, 3C] (H heads of C/H dims), the first
 * rope_dims dims of every head are rotated by position t = row % T in rotate-half form with
 * cos_t/sin_t [T][rope_dims/2]; the v block is copied.  inverse = 1 applies R^T (the backward).
 * Out of place (x != y). */
int mtts_rope_qk(const float *x, float *y, int32_t rows, int32_t T, int32_t C, int32_t H, int32_t rope_dims,
                 const float *cos_t, const float *sin_t, int32_t inverse, void *hip_stream);

/* ---------------------------------------------------------------------------------------------
 * Optimizer step: gradient-norm clipping + AdamW (train.py gradient_clip_val=1.0 ->
 * torch.nn.utils.clip_grad_norm_; baselightningmodule.py:59-65 torch.optim.AdamW) over a flat fp32
 * parameter array and its two flat moment arrays.  Gradients are read through a chunk table: chunk i
 * covers grad[0 .. n) at flat offset `offset` (n <= 65536 recommended: one 256-thread block each).
 *   coef = min(max_norm / (||g||_2 + 1e-6), 1) (max_norm <= 0: no clipping); t = *step + 1;
 *   p *= 1 - lr*wd; m += (1-b1)(g*coef - m); v = b2 v + (1-b2)(g*coef)^2;
 *   p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps);  *step = t.
 * lr (fp64) and step (fp32) are device scalars (graph-replay safe); the norm is reduced in a fixed order.
 * betas / eps / weight decay / lr are doubles as in torch: every derived scalar (1-b1, 1-b2, lr/(1-b1^t),
 * sqrt(1-b2^t), 1-lr*wd) is formed in double and rounded to fp32 once, then each torch op rounds once.
 * ------------------------------------------------------------------------------------------- */
typedef struct mtts_adamw_chunk {
    const float *grad;
    int64_t offset;
    int32_t n;
    int32_t pad_;
} mtts_adamw_chunk;

size_t mtts_clip_adamw_workspace_size(int32_t nchunks);
int mtts_clip_adamw(const mtts_adamw_chunk *chunks, int32_t nchunks, float *params, float *exp_avg,
                    float *exp_avg_sq, const double *lr, float *step, float max_norm, double beta1, double beta2,
                    double eps, double weight_decay, void *workspace, size_t workspace_bytes, void *hip_stream);
/* The same on g * grad_scale: the data-parallel step all-reduces gradient SUMS (ncclSum: RCCL's one-rank
 * all-reduce is then no kernel at all, and no pre-multiply pass at N > 1) and folds DDP's mean, 1 / world, in
 * here -- exact for a power-of-two world (the norm is sqrt(sum g^2) * grad_scale, the same value). */
int mtts_clip_adamw_scaled(const mtts_adamw_chunk *chunks, int32_t nchunks, float *params, float *exp_avg,
                           float *exp_avg_sq, const double *lr, float *step, float max_norm, double beta1,
                           double beta2, double eps, double weight_decay, float grad_scale, void *workspace,
                           size_t workspace_bytes, void *hip_stream);

/* ---------------------------------------------------------------------------------------------
 * Partial-sum reductions of the parameter gradients, batched.
 *
 * The weight-gradient GEMMs (mtts_conv_wgrad*) and the norm backwards (mtts_layernorm_bwd,
 * mtts_gn_mish_bwd) produce fp32 partial slabs and sum them in a fixed order (deterministic, no
 * float atomics).  One job:
 *     out[map(i)] (+)= sum_{s < splits} part[s * stride + i]      for i < n
 * with map(i) = i (cols == 0), or for cols > 0 the weight-gradient layout: i = r*cols + k,
 * k = j*cin + c -> r*sr + c*sc + j*sj.  mtts_reduce_partials runs the jobs now (one launch per 32).
 *
 * Deferral: between mtts_defer_reductions(1) and mtts_defer_reductions(0) the backward entry points
 * queue their reduction jobs instead of launching them; mtts_flush_reductions(stream) then runs the
 * whole queue as ONE batched launch (the ~120 per-layer reduce launches of a training step become a
 * few), mtts_discard_reductions() drops it.  The caller keeps the producers' workspaces alive and
 * reads none of the outputs until the flush, on a stream ordered after every producer.  Process-wide
 * state (autograd runs backward functions on its own thread).
 * ------------------------------------------------------------------------------------------- */
typedef struct mtts_reduce_job {
    const float *part;
    float *out;
    int64_t stride; /* floats between consecutive slabs, >= n */
    int64_t n;      /* elements per slab */
    int32_t splits;
    int32_t accumulate;
    int32_t cols, cin; /* cols == 0: out[i]; else the weight layout above */
    int64_t sr, sc, sj;
} mtts_reduce_job;

int mtts_reduce_partials(const mtts_reduce_job *jobs, int32_t njobs, void *hip_stream);
/* out[c] (+)= sum_r x[r * ld + c] for c < n (a bias gradient): one partials launch over 128-row chunks
 * (workspace: mtts_colsum_workspace_size bytes, kept alive by the caller until the sums ran) + one
 * reduce job, queued when deferral is on.  Fixed order (deterministic). */
size_t mtts_colsum_workspace_size(int64_t rows, int32_t n);
int mtts_colsum(const float *x, int64_t rows, int32_t n, int32_t ld, float *out, int32_t accumulate, float *workspace,
                size_t workspace_bytes, void *hip_stream);
void mtts_defer_reductions(int32_t on);
int32_t mtts_pending_reductions(void);
int mtts_flush_reductions(void *hip_stream);
void mtts_discard_reductions(void);

/* ---------------------------------------------------------------------------------------------
 * CFM decoder input (flow_matching.py:130-145, decoder.py:8-31 and :288), csrc/cfm_prep.hip
 * ------------------------------------------------------------------------------------------- */
/* packed[b,t,0:C] = (1 - (1 - sigma_min) t_b) z[b,:,t] + t_b x1[b,:,t];  packed[b,t,C:2C] = mu[b,:,t]
 * (x1, z, mu channel-major [B,C,T]; t [B]; packed token-major [B,T,2C]; C <= 128; torch's fp32 order). */
int mtts_cfm_pack_fwd(const float *x1, const float *z, const float *t, const float *mu, int32_t B, int32_t C,
                      int32_t T, float sigma_min, float *packed, void *hip_stream);
/* d_mu[b,c,t] = d_packed[b,t,C+c] */
int mtts_cfm_pack_bwd(const float *d_packed, int32_t B, int32_t C, int32_t T, float *d_mu, void *hip_stream);
/* SinusoidalPosEmb: out[b,k] = sin(scale t_b f_k), out[b,dim/2+k] = cos(...), f_k = exp(-k ln(1e4)/(dim/2-1)) */
int mtts_time_embedding(const float *t, int32_t B, int32_t dim, float scale, float *out, void *hip_stream);

/* ---------------------------------------------------------------------------------------------
 * Token embedding (text_encoder.py:341-342 nn.Embedding, :389 `embedding(x) * sqrt(C)`), csrc/embedding.hip
 * ------------------------------------------------------------------------------------------- */
/* out[r,:] = weight[ids[r],:] * scale; ids int64 [rows] in [0, V); weight [V,C], out [rows,C] fp32.  An
 * out-of-range id (torch: a device assert) writes a NaN row, so the step's losses turn NaN. */
int mtts_embedding_fwd(const int64_t *ids, const float *weight, int64_t rows, int32_t V, int32_t C, float scale,
                       float *out, void *hip_stream);
/* dweight[v,:] = sum over rows r with ids[r]==v of dout[r,:] * scale in a fixed order (overwrites; deterministic,
 * unlike torch's atomic embedding backward). */
int mtts_embedding_bwd(const int64_t *ids, const float *dout, int64_t rows, int32_t V, int32_t C, float scale,
                       float *dweight, void *hip_stream);

/* ---------------------------------------------------------------------------------------------
 * Rows linear: skinny fp32 Linear layers on B rows (the decoder's time MLP, csrc/time_mlp.hip)
 * ------------------------------------------------------------------------------------------- */
#define MTTS_ROWS_MAX_MATS 8
#define MTTS_ROWS_ACT_NONE 0
#define MTTS_ROWS_ACT_SILU 1 /* x / (1 + exp(-x)) */
#define MTTS_ROWS_ACT_MISH 2 /* x tanh(softplus(x)) */
/* For each of nmat (<= 8) matrices W_i [N_i, K] (fp32, 16-byte aligned rows)
 * sharing the input x [B, K]:
 *   out_i[b, n] = sum_k x[b, k] W_i[n, k] + bias_i[n]   (bias table or its entries may be NULL)
 *   out_act_i = act(out_i)                              (out_act table or entries may be NULL)
 * K % 4 == 0.  Exact fp32 MFMA; the reduction is split over workgroups (256 indices each) and summed in a
 * fixed order by the last workgroup of each output tile: deterministic.  workspace: at least
 * mtts_rows_linear_workspace_size(B, K, nmat, N) bytes, 256-byte aligned, its first (counter) region
 * ZEROED once by the caller before first use -- the kernels leave it zeroed (graph replays reuse it);
 * one workspace serves the forward and backward calls of the same (B, K, nmat, N) on one stream. */
size_t mtts_rows_linear_workspace_size(int32_t B, int32_t K, int32_t nmat, const int32_t *N);
int mtts_rows_linear_fwd(const float *x, int32_t B, int32_t K, int32_t nmat, const float *const *W,
                         const float *const *bias, const int32_t *N, float *const *out, float *const *out_act,
                         int32_t act, void *workspace, size_t workspace_bytes, void *hip_stream);
/* Backward of out_i = a W_i^T + bias_i with a = act(pre) the layer's input rows [B, K]:
 *   dx[b, k]   = (sum_i sum_n dy_i[b, n] W_i[n, k]) * act'(pre[b, k])   (dx may be NULL; N_i % 4 == 0)
 *   dW_i[n, k] = sum_b dy_i[b, n] a[b, k] ; db_i[n] = sum_b dy_i[b, n]    (dW NULL: neither; db table may be NULL)
 * All outputs are overwritten.  act NONE: pre unused (dx is the plain input gradient).  Workspace as above. */
int mtts_rows_linear_bwd(const float *a, const float *pre, int32_t act, int32_t B, int32_t K, int32_t nmat,
                         const float *const *W, const int32_t *N, const float *const *dy, float *dx,
                         float *const *dW, float *const *db, void *workspace, size_t workspace_bytes,
                         void *hip_stream);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* MTTS_DECODER_H_ */
