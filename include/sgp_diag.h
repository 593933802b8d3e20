/*
 * sgp_diag.h -- diagnostic entry points of libsgp.so.
 *
 * Not part of the drop-in boundary (the reference has no counterpart): they let the GPU tests
 * and bench.py pin, on the hardware, claims the fused evaluations make internally.  Plain C,
 * host buffers, same status codes and sgp_last_error() as sgp.h.
 */
#ifndef SGP_DIAG_H
#define SGP_DIAG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* The two m x m SPD inverses of a VI evaluation's phase 2 (the Gauss-Jordan chains that replace
 * R's chol / solve of Sigma22 and Sigma22 + t(Sigma12) %*% ZSig12, R/vi_functions.R:87-103,
 * 231-239), launched together as the evaluation launches them: inv(A) in place on a second
 * stream (K22's chain on `aux`) and inv(A + beta B) formed as the chain reads it on the first
 * (Bm's chain on the launch stream).  per_step = 0: the persistent one-launch chains (m <= 4096,
 * what the evaluations run); 1: one launch per 64-wide pivot step (the pre-round-5 chain, and
 * the product's chain above m = 4096).  The two must agree bit for bit (k_dense.hip).
 * A, B: m x m column-major, symmetric; invA, invS: m x m column-major; logdet[0] = log det A,
 * logdet[1] = log det(A + beta B).  SGP_ENOTPD as the evaluations (R's chol() message);
 * SGP_EHIP naming the watchdog when a chain's inter-workgroup wait expired. */
int sgp_diag_gj_pair(int device, int64_t m, const double* A, const double* B, double beta,
                     int per_step, double* invA, double* invS, double* logdet);

/* The HBM store ceiling of this device for the K12 builder's roofline: `reps` passes of plain
 * 16-byte non-temporal vector stores over `bytes` bytes, laid out as the builder stores (per
 * wave instruction 4 rows x 256 B of a row-major matrix with 1024-double rows; pattern 1) or as
 * one linear stream (pattern 0).  *gbs = the best pass in GB/s (1e9 B/s). */
int sgp_diag_store_bw(int device, int64_t bytes, int reps, int pattern, double* gbs);

#ifdef __cplusplus
}
#endif
#endif /* SGP_DIAG_H */
