/*
 * mtts.h -- C ABI of libmtts_hip.so, the MI355X (gfx950) hot path of the Matcha-TTS training step.
 *
 * Every entry point takes plain device pointers, sizes and a hipStream_t passed as void*.
 * No torch types cross this boundary.  Conventions:
 *   - Ownership: the caller allocates every input, output and workspace buffer
 *     (query sizes with the *_workspace_size functions).  The library keeps no global state
 *     beyond the lazily loaded code objects.
 *   - Errors: 0 (MTTS_OK) on success, a negative mtts_status otherwise; mtts_last_error() returns a
 *     thread-local message describing the last failure on the calling thread.  Never aborts.
 *   - Threading: calls are stream-ordered and asynchronous (no host synchronisation), re-entrant
 *     across streams and threads; the device is the current device of the calling thread.
 *
 * Reference interfaces replaced (paths relative to the reference repository root):
 *   mtts_maximum_path_f32          <- matcha/utils/monotonic_align/__init__.py:40-55  maximum_path(value, mask)
 *   mtts_prior_maximum_path        <- matcha/models/matcha_tts.py:276-288 (log-prior lattice + maximum_path +
 *                                     the duration target), fused
 *   mtts_expand_rows_fwd / _bwd    <- matcha/models/matcha_tts.py:314-315  mu_y = attn^T @ mu_x
 *   mtts_compute_batch_alignments  <- matcha/utils/monotonic_align/core.pyx:101-128   compute_batch_alignments(...)
 *                                     (bound as maximum_path_c, __init__.py:4-8)
 *   mtts_losses_fwd / _bwd         <- flow_matching.py:145-149 (CFM loss) + matcha_tts.py:319-323 (prior loss)
 *   mtts_mel_log_fwd               <- matcha/utils/audio_process.py:62-72  MelSpectrogram.__call__ (after the STFT)
 *   mtts_sequence_mask_f32         <- matcha/utils/model.py:13-34 sequence_mask(...).to(float) (matcha_tts.py:259,
 *                                     text_encoder.py:398) and text_encoder.py:300-303 masked_fill(-1e4) as a key bias
 *   mtts_duration_loss_fwd / _bwd  <- matcha_tts.py:287-288 + utils/model.py:117-135 duration_loss
 *   mtts_loss_sum                  <- baselightningmodule.py:121-128 (dur + prior + diff, the logged values)
 * Decoder / CFM operators (matcha/models/components/{decoder,transformer,flow_matching}.py) are
 * declared in mtts_decoder.h.
 */
#ifndef MTTS_H_
#define MTTS_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MTTS_ABI_VERSION 1

typedef enum mtts_status {
    MTTS_OK = 0,
    MTTS_ERR_INVALID_ARG = -1, /* null pointer, negative size, bad flag */
    MTTS_ERR_SHAPE = -2,       /* shape outside what the kernels support (e.g. Tx > 4096) */
    MTTS_ERR_WORKSPACE = -3,   /* workspace too small */
    MTTS_ERR_HIP = -4,         /* a HIP runtime call failed (launch, attribute) */
    MTTS_ERR_UNSUPPORTED = -5  /* feature not built into this library */
} mtts_status;

/* Library identity / diagnostics. */
int mtts_abi_version(void);
const char *mtts_last_error(void);

/* ---------------------------------------------------------------------------------------------
 * Monotonic Alignment Search (Viterbi max-path over the [T_text x T_mel] log-likelihood lattice)
 * ------------------------------------------------------------------------------------------- */

/* flags for mtts_maximum_path_f32 */
#define MTTS_MAS_VALUE_PREMASKED 0x1 /* value already holds value*mask: skip the multiply      */
#define MTTS_MAS_NO_DENSE_PATH 0x2   /* only row_start_out/lengths_out: do not write `path`    */

/* Maximum text length (Tx) the kernels accept. */
#define MTTS_MAS_MAX_TX 8192 /* maximum_path / the fused prior path (transposed lattice): 8 waves x 16 text rows per lane of
                                the multi-wave DP (round 6; 4096 in rounds 4-5; 2048 with MTTS_MAS_MW=0) */
#define MTTS_MAS_MAX_TX_ROW_MAJOR 4096 /* mtts_compute_batch_alignments (the row-major lattice it mutates): 8 x 8 rows */

/* Bytes of device workspace mtts_maximum_path_f32 / mtts_compute_batch_alignments need. */
size_t mtts_maximum_path_workspace_size(int32_t B, int32_t Tx, int32_t Ty);

/*
 * maximum_path(value, mask)                         (reference: monotonic_align/__init__.py:40-55)
 *   value, mask : float32 [B, Tx, Ty], C-contiguous, device memory.
 *   path        : float32 [B, Tx, Ty] output, fully written: exactly one 1.0 per column y < t_y[b],
 *                 zeros elsewhere (unless MTTS_MAS_NO_DENSE_PATH).
 *   t_x[b] = (int)sum_x mask[b, x, 0],  t_y[b] = (int)sum_y mask[b, 0, y]   (__init__.py:52-53)
 *   The DP runs on value*mask (one fp32 multiply per cell, __init__.py:45) with the Cython's tie rule
 *   (`from_prev >= from_same` -> diagonal, core.pyx:73) and `best + score` as one fp32 add (:80):
 *   the path is bit-identical to the compiled Cython for 1 <= t_x <= t_y.
 *   Defined behaviour where the reference is undefined: t_x == 0, t_y == 0 or t_x > t_y produce an
 *   all-zero path for that utterance (its row starts are -1).
 *   lengths_out   : optional int32 [B, 2] = (t_x, t_y) per utterance.
 *   row_start_out : optional int32 [B, Tx]; row x of utterance b covers columns
 *                   [row_start[b,x], row_start[b,x+1]-1] (the last row ends at t_y-1); -1 = no path.
 *   The caller's value and mask are not modified.
 */
int mtts_maximum_path_f32(const float *value, const float *mask, float *path, int32_t B, int32_t Tx,
                          int32_t Ty, int32_t flags, int32_t *lengths_out, int32_t *row_start_out,
                          void *workspace, size_t workspace_bytes, void *hip_stream);

/*
 * compute_batch_alignments(paths, values, t_xs, t_ys, max_neg_val)   (reference: core.pyx:101-128)
 *   paths  : int32 [B, Tx, Ty]; ones are SET on the path, other entries are left untouched (:88).
 *   values : float32 [B, Tx, Ty]; MUTATED exactly like the Cython (:83-85): for y < t_y, x < t_x the
 *            cell receives the DP value (in-band: cumulative best + score; out-of-band: max_neg_val);
 *            cells outside the [t_x, t_y] rectangle are untouched.
 *   t_xs, t_ys : int32 [B] device arrays.
 */
int mtts_compute_batch_alignments(int32_t *paths, float *values, const int32_t *t_xs,
                                  const int32_t *t_ys, int32_t B, int32_t Tx, int32_t Ty,
                                  float max_neg_val, void *workspace, size_t workspace_bytes,
                                  void *hip_stream);

/*
 * Fused alignment of the training forward (matcha_tts.py:276-288):
 *   lattice[b,i,j] = (log N(y[b,:,j]; mu_x[b,:,i], I)) * x_mask[b,i] * y_mask[b,j]   (matcha_tts.py:277-282,
 *                    maximum_path's value*mask) with the masks from x_lengths / y_lengths (int64 [B]),
 *   then the DP and backtrack of mtts_maximum_path_f32 on it (t_x = x_lengths, t_y = y_lengths).
 *   mu_x : float32 [B, C, Tx], y : float32 [B, C, Ty] (channel-major, C-contiguous, device memory).
 *   Outputs (each optional): path float32 [B,Tx,Ty] (dense hard attention), lengths_out int32 [B,2],
 *   row_start_out int32 [B,Tx] (as mtts_maximum_path_f32), dur_out float32 [B,Tx] = sum_j path[b,i,j],
 *   col_row_out int32 [B,Ty] = the text row of frame j (-1 past t_y), lattice_out float32 [B,Tx,Ty]
 *   (the masked lattice; otherwise it lives in the workspace).
 *   The lattice sums run in ascending channel order, one fp32 operation each (bit-reproducible on the
 *   host); the reference's torch matmuls use an implementation-defined order.
 */
size_t mtts_prior_maximum_path_workspace_size(int32_t B, int32_t Tx, int32_t Ty);
int mtts_prior_maximum_path(const float *mu_x, const float *y, const int64_t *x_lengths, const int64_t *y_lengths,
                            int32_t B, int32_t C, int32_t Tx, int32_t Ty, float *path, int32_t *lengths_out,
                            int32_t *row_start_out, float *dur_out, int32_t *col_row_out, float *lattice_out,
                            void *workspace, size_t workspace_bytes, void *hip_stream);

/*
 * mu_y = attn^T @ mu_x for a hard alignment (matcha_tts.py:314-315) as a gather, and its backward:
 *   fwd: dst[b,c,j] = src[b,c,col_row[b,j]] (0 where col_row < 0); src [B,C,Tx], dst [B,C,Ty] float32.
 *   bwd: dx[b,c,i] = sum over the frames j of row i (row_start / lengths of mtts_maximum_path_f32) of
 *        dy[b,c,j]: 16 strided partial sums (j = start + l + 16k, ascending k) combined by a fixed
 *        xor tree (deterministic, no atomics).
 */
int mtts_expand_rows_fwd(const float *src, const int32_t *col_row, int32_t B, int32_t C, int32_t Tx, int32_t Ty,
                         float *dst, void *hip_stream);
int mtts_expand_rows_bwd(const float *dy, const int32_t *row_start, const int32_t *lengths, int32_t B, int32_t C,
                         int32_t Tx, int32_t Ty, float *dx, void *hip_stream);

/* ---------------------------------------------------------------------------------------------
 * Log-mel features of the data path (matcha/utils/audio_process.py:32-81, MelSpectrogram.__call__)
 * ------------------------------------------------------------------------------------------- */
/*
 * out[b,m,f] = log(max(sum_{k in [band_lo[m], band_hi[m])} mel_w[m,k] * sqrt(re^2 + im^2 + 1e-9), clip))
 *   spec : float32 [B, n_freq, F, 2] (torch.stft's complex output viewed as real, C-contiguous)
 *   mel_w: float32 [n_mels, n_freq] (the librosa slaney basis); band_lo/hi int32 [n_mels]: the nonzero
 *          bins of each filter (zero weights outside are skipped -- exact, they add +0).
 *   out  : float32 [B, n_mels, F].  Bins are summed in ascending k (fixed order, deterministic).
 */
int mtts_mel_log_fwd(const float *spec, const float *mel_w, const int32_t *band_lo, const int32_t *band_hi,
                     int32_t B, int32_t n_freq, int32_t F, int32_t n_mels, float clip_val, float *out,
                     void *hip_stream);

/* ---------------------------------------------------------------------------------------------
 * Training losses (flow_matching.py:145-149 CFM loss, matcha_tts.py:319-323 prior loss), fused
 * ------------------------------------------------------------------------------------------- */
/*
 * out[0] = sum((u_pred - (x1 - (1 - sigma_min) z))^2) / D         (unmasked numerator, reference quirk)
 * out[1] = sum(0.5 ((y - mu_y)^2 + log 2pi) * y_mask) / D,  D = out[2] = sum(y_mask) * C
 *   u_pred token-major [B,T,C]; x1, z, y, mu_y channel-major [B,C,T]; y_mask float [B,T] (float32, device).  u_pred = NULL
 *   skips the CFM term (out[0] = 0); mu_y = NULL skips the prior term.  C <= 128.  Deterministic.
 * Backward: du_pred = 2 g_diff / D (u_pred - u) (token-major), dmu_y = -g_prior / D (y - mu_y) * y_mask
 *   (channel-major); either output may be NULL.  fwd_out is the forward's out (D read from out[2]).
 */
size_t mtts_losses_workspace_size(int32_t B, int32_t T);
int mtts_losses_fwd(const float *u_pred, const float *x1, const float *z, const float *y, const float *mu_y,
                    const float *y_mask, int32_t B, int32_t C, int32_t T, float sigma_min, float *out,
                    void *workspace, size_t workspace_bytes, void *hip_stream);
int mtts_losses_bwd(const float *g_diff, const float *g_prior, const float *fwd_out, const float *u_pred, const float *x1, const float *z,
                    const float *y, const float *mu_y, const float *y_mask, int32_t B, int32_t C, int32_t T,
                    float sigma_min, float *du_pred, float *dmu_y, void *hip_stream);

/* ---------------------------------------------------------------------------------------------
 * Step glue: sequence masks, the duration loss, the loss sum (csrc/losses.hip)
 * ------------------------------------------------------------------------------------------- */
/* mask[b, t] = t < lengths[b] ? 1 : 0 (fp32 [B, T]); key_bias[b, t] = (mask - 1) * 1e4 when non-NULL
 * (either output may be NULL, not both).  lengths int64 [B]. */
int mtts_sequence_mask_f32(const int64_t *lengths, int32_t B, int32_t T, float *mask, float *key_bias,
                           void *hip_stream);
/* logw_ = log(1e-8 + dur) * x_mask (x_mask from lengths);  out[0] = sum((logw - logw_)^2) / sum(lengths),
 * out[1] = sum(lengths) as fp32.  logw, dur fp32 [B, T] (dur: the MAS durations); fixed-order sum.
 * Backward: dlogw = (g / out[1]) * (2 (logw - logw_)). */
int mtts_duration_loss_fwd(const float *logw, const float *dur, const int64_t *lengths, int32_t B, int32_t T,
                           float *out, void *hip_stream);
int mtts_duration_loss_bwd(const float *g, const float *fwd_out, const float *logw, const float *dur,
                           const int64_t *lengths, int32_t B, int32_t T, float *dlogw, void *hip_stream);
/* total = (dur + prior) + diff; logged (optional, 4 floats) = [dur, prior, diff, total].  prior may be NULL (0). */
int mtts_loss_sum(const float *dur, const float *prior, const float *diff, float *total, float *logged,
                  void *hip_stream);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* MTTS_H_ */
