/*
 * oracle/mas_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * CPU restatement of the reference Monotonic Alignment Search:
 *   /root/reference/matcha/utils/monotonic_align/core.pyx
 *     compute_single_alignment   core.pyx:16-96
 *     compute_batch_alignments   core.pyx:101-128  (OpenMP prange over utterances, :121)
 *   /root/reference/matcha/utils/monotonic_align/__init__.py
 *     maximum_path               __init__.py:40-55  (value*mask, lengths from mask sums)
 *
 * Parity: pinned against golden vectors produced by the compiled reference Cython
 * (tests/golden/make_golden.py builds oracle/_ref/ from core.pyx and records its outputs);
 * tests/test_oracle_golden.py checks this file against every fixture.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 *
 * Numerics: compiled with -ffp-contract=off so `best + score` is one fp32 add
 * (core.pyx:80) and `value * mask` is one fp32 multiply (__init__.py:45).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* core.pyx:16-96.  score is [t_x_stride rows][ty_stride cols] of ONE utterance.
 * Mutates score in place exactly like the Cython (:83-85) and sets ones in align (:88).
 * Returns 0, or -1 when the scratch allocation fails (Cython silently returns, :43-50). */
static int single_alignment(int32_t *align, float *score, int ty_stride,
                            int t_x, int t_y, float neg)
{
    if (t_x <= 0 || t_y <= 0) return 0; /* Cython: UB (writes row -1); defined here as no-op */
    float *dp_prev = (float *)malloc((size_t)t_x * sizeof(float));
    float *dp_cur = (float *)malloc((size_t)t_x * sizeof(float));
    /* calloc: the Cython mallocs (garbage). Only read in-band (t_x<=t_y) where it is written. */
    unsigned char *take_diag = (unsigned char *)calloc((size_t)t_x * (size_t)t_y, 1);
    if (!dp_prev || !dp_cur || !take_diag) {
        free(dp_prev); free(dp_cur); free(take_diag);
        return -1;
    }
    for (int x = 0; x < t_x; ++x) dp_prev[x] = neg;                  /* :52-53 */
    for (int y = 0; y < t_y; ++y) {                                   /* :55 */
        for (int x = 0; x < t_x; ++x) dp_cur[x] = neg;               /* :56-57 */
        int x_min = t_x + y - t_y; if (x_min < 0) x_min = 0;          /* :59 */
        int x_max = y + 1; if (x_max > t_x) x_max = t_x;              /* :60 */
        for (int x = x_min; x < x_max; ++x) {                         /* :62 */
            float from_prev = (x == 0) ? ((y == 0) ? 0.0f : neg) : dp_prev[x - 1]; /* :63-66 */
            float from_same = (x == y) ? neg : ((y > 0) ? dp_prev[x] : neg);      /* :68-71 */
            float best;
            if (from_prev >= from_same || x == y) {                   /* :73 tie -> diagonal */
                best = from_prev;
                take_diag[(size_t)x * t_y + y] = 1;
            } else {
                best = from_same;
                take_diag[(size_t)x * t_y + y] = 0;
            }
            dp_cur[x] = best + score[(size_t)x * ty_stride + y];      /* :80 */
        }
        for (int x = 0; x < t_x; ++x) {                               /* :83-85 */
            dp_prev[x] = dp_cur[x];
            score[(size_t)x * ty_stride + y] = dp_prev[x];
        }
    }
    int idx = t_x - 1;                                                /* :37 */
    for (int y = t_y - 1; y >= 0; --y) {                              /* :87 */
        align[(size_t)idx * ty_stride + y] = 1;                       /* :88 */
        if (y == 0) break;                                            /* :89-90 */
        if (idx > 0 && (idx == y || take_diag[(size_t)idx * t_y + y] == 1)) idx -= 1; /* :91-92 */
    }
    free(dp_prev); free(dp_cur); free(take_diag);
    return 0;
}

/* core.pyx:101-128 (compute_batch_alignments): paths int32[B,Tx,Ty], values float32[B,Tx,Ty]
 * (mutated), per-utterance lengths.  nthreads<=0 -> OpenMP default. */
int mtts_oracle_mas_batch(int32_t *paths, float *values, const int32_t *t_xs,
                          const int32_t *t_ys, int B, int Tx, int Ty, float neg, int nthreads)
{
    int rc = 0;
#ifdef _OPENMP
    if (nthreads > 0) {
#pragma omp parallel for schedule(static) num_threads(nthreads) reduction(| : rc)
        for (int b = 0; b < B; ++b)
            rc |= single_alignment(paths + (size_t)b * Tx * Ty, values + (size_t)b * Tx * Ty,
                                   Ty, t_xs[b], t_ys[b], neg);
    } else {
#pragma omp parallel for schedule(static) reduction(| : rc)
        for (int b = 0; b < B; ++b)
            rc |= single_alignment(paths + (size_t)b * Tx * Ty, values + (size_t)b * Tx * Ty,
                                   Ty, t_xs[b], t_ys[b], neg);
    }
#else
    (void)nthreads;
    for (int b = 0; b < B; ++b)
        rc |= single_alignment(paths + (size_t)b * Tx * Ty, values + (size_t)b * Tx * Ty,
                               Ty, t_xs[b], t_ys[b], neg);
#endif
    return rc;
}

/* __init__.py:40-55 (maximum_path): path_out float32[B,Tx,Ty] (fully written),
 * scratch float32[B,Tx,Ty] receives value*mask and then the DP lattice,
 * iscratch int32[B,Tx,Ty] receives the int path.  t_x = mask.sum(1)[:,0], t_y = mask.sum(2)[:,0]. */
int mtts_oracle_maximum_path(const float *value, const float *mask, float *path_out,
                             float *scratch, int32_t *iscratch, int32_t *t_out,
                             int B, int Tx, int Ty, int nthreads)
{
    size_t n = (size_t)B * Tx * Ty;
    for (size_t i = 0; i < n; ++i) scratch[i] = value[i] * mask[i];   /* :45 */
    memset(iscratch, 0, n * sizeof(int32_t));                          /* :49 np.zeros */
    int32_t *txs = (int32_t *)malloc((size_t)B * sizeof(int32_t) * 2);
    if (!txs) return -1;
    int32_t *tys = txs + B;
    for (int b = 0; b < B; ++b) {
        const float *m = mask + (size_t)b * Tx * Ty;
        float sx = 0.0f, sy = 0.0f;
        for (int x = 0; x < Tx; ++x) sx += m[(size_t)x * Ty];          /* :52 mask.sum(1)[:,0] */
        for (int y = 0; y < Ty; ++y) sy += m[y];                        /* :53 mask.sum(2)[:,0] */
        txs[b] = (int32_t)sx;
        tys[b] = (int32_t)sy;
        if (t_out) { t_out[2 * b] = txs[b]; t_out[2 * b + 1] = tys[b]; }
    }
    int rc = mtts_oracle_mas_batch(iscratch, scratch, txs, tys, B, Tx, Ty, -1e9f, nthreads);
    for (size_t i = 0; i < n; ++i) path_out[i] = (float)iscratch[i];   /* :55 .to(dtype) */
    free(txs);
    return rc;
}
