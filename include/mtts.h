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
 *   mtts_compute_batch_alignments  <- matcha/utils/monotonic_align/core.pyx:101-128   compute_batch_alignments(...)
 *                                     (bound as maximum_path_c, __init__.py:4-8)
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
    MTTS_ERR_SHAPE = -2,       /* shape outside what the kernels support (e.g. Tx > 512) */
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
#define MTTS_MAS_MAX_TX 512

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

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* MTTS_H_ */
