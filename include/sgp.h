/*
 * sgp.h -- C ABI of the MI355X-native sparse-GP objective+gradient path.
 *
 * Drop-in boundary for luisdamiano/sparseRGPs' native layer and hot path.
 * Plain C: pointers, sizes and enums only; no torch/HIP types in signatures
 * (streams are passed as `void*` = hipStream_t).  Matrices use R's layout:
 * column-major fp64 with an explicit leading dimension.
 *
 * Layer 1 (elementwise fillers, host buffers) replaces the Rcpp .Call routines
 * registered in src/RcppExports.cpp:284-311:
 *   sgp_make_cov      <- make_cov_matC     src/covariance_functionsC.cpp:72-169
 *                        make_cov_mat_ardC src/covariance_functionsC.cpp:191-252
 *   sgp_dsig_dtheta   <- dsig_dthetaC      src/covariance_function_derivativesC.cpp:307-552
 *                        dsig_dtheta_ardC  src/covariance_function_derivativesC.cpp:555-722
 *   sgp_kernel_pair / sgp_dkernel_pair <- the per-pair exports cov_fun_*C, dsqexp_*C
 *                        (covariance_functionsC.cpp:5-52, covariance_function_derivativesC.cpp:35-171)
 *
 * Layer 2 (fused evaluation over a device-resident context) replaces the R-level
 * hot path that calls those routines once per optimizer iteration:
 *   sgp_eval_vi     <- elbo_fun (R/vi_functions.R:64-121) + delbo_dcov_par (126-602),
 *                      with K12/K22/Z built as in norm_grad_ascent_vi (vi_functions.R:1089-1128)
 *   sgp_eval_fitc   <- obj_fun_norm (R/laplace_approx_obj_funs.R:6-52) + dlogp_dcov_par
 *                      (R/laplace_approx_gradient.R:720-1135), Z as in norm_grad_ascent
 *                      (R/laplace_gradient_ascent.R:1568-1593)
 *   sgp_vi_phase1/2, sgp_vi_finish: the same VI evaluation split at its two
 *                      row-sum reductions so a caller can all-reduce across GPUs.
 *   sgp_eval_laplace <- newtrap_sparseGP (R/newtrap_sparseGP.R:6-186) + dlogq_dcov_par
 *                      (R/laplace_approx_gradient.R:25-553), Poisson likelihood
 *
 * Hyperparameters are passed as `theta` laid out [sigma, l_1..l_L, tau] with
 * L = 1 (sqexp, exp) or L = d (ard).  Gradients are d/d log(theta) in that order
 * (the reference's trans_par scale, R/laplace_approx_gradient.R:850-853).
 *
 * Errors: every entry point returns an sgp_status; sgp_last_error() gives a
 * thread-local message.  A failed Cholesky returns SGP_ENOTPD (R's chol() error,
 * caught by try() in R/knot_proposal_functions.R:641-642).
 */
#ifndef SGP_H
#define SGP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SGP_ABI_VERSION 1

typedef enum {
  SGP_OK = 0,
  SGP_EINVAL = 1,  /* bad argument: unknown kernel/parameter, size, NULL        */
  SGP_ENOTPD = 2,  /* Cholesky pivot <= 0 or non-finite; see sgp_last_error()    */
  SGP_EHIP = 3,    /* HIP runtime failure                                        */
  SGP_ENOMEM = 4   /* device allocation failed                                   */
} sgp_status;

typedef enum {
  SGP_KERNEL_SQEXP = 0, /* "sqexp": sigma^2 exp(-|x-u|^2/(2 l^2))                */
  SGP_KERNEL_ARD = 1,   /* "ard":   sigma^2 exp(-sum_c ((x_c-u_c)/l_c)^2 / 2)      */
  SGP_KERNEL_EXP = 2    /* "exp":   sigma^2 exp(-sum_c |x_c-u_c| / l)  (L1)        */
} sgp_kernel;

/* flags for the fused evaluations */
#define SGP_FLAG_R_DET 1u /* reproduce R's det() overflow in log(det(K22)) */
/* objective only (elbo_fun, obj_fun_norm, newtrap_sparseGP without dlogq_dcov_par): every
 * gradient pass is skipped and grad may be NULL; the knot posterior stays available */
#define SGP_FLAG_OBJ_ONLY 2u

const char* sgp_last_error(void);
int sgp_abi_version(void);
int sgp_device_count(int* count);

/* number of hyperparameters for a kernel and input dimension d: 3 or d + 2 */
int sgp_num_params(int kernel, int d);

/* ---------------- Layer 1: elementwise fillers (host in/out) ---------------- */

/* K(x_i, x'_j) for all pairs.  x: n x d (ldx >= n), xp: np x d (ldxp >= np) or NULL for the
 * symmetric mode (R's x_pred = matrix()), which adds tau^2 + delta on the diagonal.
 * out: n x np column-major (ldo >= n).  Runs on `device` (HIP). */
int sgp_make_cov(int device, int kernel, const double* x, int64_t n, int64_t ldx,
                 const double* xp, int64_t np, int64_t ldxp, int d,
                 const double* theta, double delta, double* out, int64_t ldo);

/* d K / d log(theta_p) for all pairs; param indexes theta's layout.  Reproduces the
 * reference's quirks: tau -> 2 tau^2 iff all coordinates equal; "exp" derivatives use the
 * L2 distance; "exp" cross-mode tau returns zeros. */
int sgp_dsig_dtheta(int device, int kernel, const double* x, int64_t n, int64_t ldx,
                    const double* xp, int64_t np, int64_t ldxp, int d,
                    const double* theta, int param, double* out, int64_t ldo);

/* per-pair scalar forms (host-only, for the R shim's cov_fun_*C / dsqexp_*C exports) */
double sgp_kernel_pair(int kernel, const double* x1, const double* x2, int d, const double* theta);
double sgp_dkernel_pair(int kernel, const double* x1, const double* x2, int d,
                        const double* theta, int param);

/* ---------------- Layer 2: device-resident context + fused evaluation ---------------- */

typedef struct sgp_ctx sgp_ctx;

/* Copy X (n x d, column-major, ldx >= n), y and mu (n) to HBM on `device`; reserve work
 * space for up to m_max inducing points.  The context owns all device memory; nothing is
 * allocated per evaluation.  A context is externally synchronized (one host thread). */
int sgp_ctx_create(sgp_ctx** out, int device, const double* X, int64_t n, int64_t ldx, int d,
                   const double* y, const double* mu, int64_t m_max);
int sgp_ctx_destroy(sgp_ctx* ctx);

/* Row-sharded context over several GPUs of one node (config C4; BASELINE north_star: "sharding
 * the n observation rows across the 8 GPUs of one node with an RCCL all-reduce", SURVEY 8(b)'s
 * sgp_ctx_create(X, y, mu, n, d, ngpus)).  Shard k (k < nshards) holds the contiguous row block
 * [k*n/N + min(k, n%N), ...) -- sparsergps_amd.dist.shard_rows -- on device devices[k] (NULL:
 * device k).  The library drives the shards itself: one host thread per distinct device, the
 * row-sum reductions of every evaluation (VI and FITC: two; Laplace: two per NR iteration and
 * two for the gradient) summed on each device over its shards (fixed order) and then over the
 * devices by an in-process RCCL all-reduce (ncclCommInitAll over the distinct devices, on each
 * device's stream, in place).  A device may repeat (several shards on one GPU).
 * The handle is used with the ordinary entry points: sgp_eval_vi / sgp_eval_fitc /
 * sgp_eval_laplace / sgp_lap_nr, sgp_lap_set_f / sgp_lap_set_expo / sgp_lap_get_f /
 * sgp_lap_get_grad_psi (n values
 * in the global row order) / sgp_lap_objective_values, sgp_posterior_u, sgp_ctx_enable_knot_grad,
 * sgp_knot_gradient (bounds NULL = the knot bounds of ALL rows), sgp_ctx_row_bounds (all rows),
 * sgp_ctx_set_data, sgp_ctx_rows (all rows), the three candidate scorers (each VI candidate as an
 * objective-only evaluation at [U; cand_t], m + 1 <= m_max), the timing calls (shard 0's
 * record) and sgp_ctx_destroy.  The phase-level entry points (sgp_vi_phase1 ... sgp_lap_step),
 * sgp_ctx_set_stream, sgp_ctx_set_packed_reduction and sgp_eval_full return SGP_EINVAL.
 * 1 <= nshards <= min(n, 64). */
int sgp_ctx_create_multi(sgp_ctx** out, const int* devices, int nshards, const double* X,
                         int64_t n, int64_t ldx, int d, const double* y, const double* mu,
                         int64_t m_max);
/* shards and distinct devices of a context (1 and 1 for sgp_ctx_create's) */
int sgp_ctx_shards(const sgp_ctx* ctx, int* nshards, int* ndevices);
/* launch on this hipStream_t; NULL selects the context's own (non-blocking) stream */
int sgp_ctx_set_stream(sgp_ctx* ctx, void* hip_stream);
/* replace y / mu (e.g. Laplace pseudo-data); host buffers of length n */
int sgp_ctx_set_data(sgp_ctx* ctx, const double* y, const double* mu);
int64_t sgp_ctx_rows(const sgp_ctx* ctx);

/* Titsias ELBO and d ELBO / d log theta at knots U (m x d column-major, ldu >= m).
 * K22 = Kuu + delta I, Z = tau^2 + delta (vi_functions.R:733-753).  grad: num_params. */
int sgp_eval_vi(sgp_ctx* ctx, int kernel, const double* theta, const double* U, int64_t m,
                int64_t ldu, double delta, unsigned flags, double* obj, double* grad);

/* FITC log marginal likelihood and gradient (obj_fun_norm + dlogp_dcov_par). */
int sgp_eval_fitc(sgp_ctx* ctx, int kernel, const double* theta, const double* U, int64_t m,
                  int64_t ldu, double delta, unsigned flags, double* obj, double* grad);

/* Multi-GPU VI: each rank owns a row block of X.  phase1 writes its partial first
 * reduction (sgp_vi_red1_count doubles) to the DEVICE buffer red1; the caller sums red1
 * over ranks in place (e.g. RCCL all-reduce); phase2 consumes the reduced red1 and writes
 * its partial second reduction (sgp_vi_red2_count doubles) to red2; after summing red2 over
 * ranks, sgp_vi_finish returns the objective and gradient.  n_global = total rows. */
int64_t sgp_vi_red1_count(int64_t m);
int64_t sgp_vi_red2_count(int kernel, int d);
int sgp_vi_phase1(sgp_ctx* ctx, int kernel, const double* theta, const double* U, int64_t m,
                  int64_t ldu, double delta, double* red1);
int sgp_vi_phase2(sgp_ctx* ctx, const double* red1, int64_t n_global, unsigned flags, double* red2);
int sgp_vi_finish(sgp_ctx* ctx, const double* red2, double* obj, double* grad);
/* Packed first reduction (multi-GPU VI): with packing on, phase1 writes S as its lower 64 x 64
 * blocks only -- the (mp/64)(mp/64 + 1)/2 blocks of 4096 doubles, block (r, c) with r >= c
 * at index r (r + 1) / 2 + c, row-major inside -- followed by t (mp) and r'r, i.e.
 * sgp_vi_red1_packed_count(m) doubles instead of sgp_vi_red1_count(m) (53 % of it at
 * m = 1024), and phase2 unpacks the summed buffer on the device.  Only the all-reduce between
 * the phases sees the layout; the result is the same. */
int64_t sgp_vi_red1_packed_count(int64_t m);
int sgp_ctx_set_packed_reduction(sgp_ctx* ctx, int enable);

/* Multi-GPU FITC (three steps, two all-reduces): red1 = [S_D, t, r'D^-1 r, sum log Z],
 * red2 = [S_omega, ..., sum omega, contraction records]; sgp_fitc_finish runs the replicated
 * m x m tail on the device and returns the objective and gradient. */
int64_t sgp_fitc_red1_count(int64_t m);
int64_t sgp_fitc_red2_count(int kernel, int d, int64_t m);
int sgp_fitc_phase1(sgp_ctx* ctx, int kernel, const double* theta, const double* U, int64_t m,
                    int64_t ldu, double delta, double* red1);
int sgp_fitc_phase2(sgp_ctx* ctx, const double* red1, int64_t n_global, unsigned flags,
                    double* red2);
int sgp_fitc_finish(sgp_ctx* ctx, const double* red2, double* obj, double* grad);

/* Poisson sparse Laplace (config 5): one evaluation = newtrap_sparseGP warm-started from the
 * context's latent vector f (R/newtrap_sparseGP.R:6-186, obj_fun_pois
 * R/laplace_approx_obj_funs.R:108-174) followed by dlogq_dcov_par at the mode
 * (R/laplace_approx_gradient.R:25-553), exactly as one iteration of laplace_grad_ascent
 * (R/laplace_gradient_ascent.R:510-541).  K22 = Kuu + (tau^2 + delta) I (quirk Q1).
 * expo = the Poisson exposure `m` of the reference's likelihood helpers
 * (R/derivative_functions_of_data_likelihoods.R:7-61): a positive scalar for every row, or
 * SGP_EXPO_ROWS for the per-row exposure of sgp_lap_set_expo; tol/maxit = tol_nr/maxit_nr.
 * The mode f stays resident in the context and warm-starts the next evaluation; its value
 * at context creation is 0, the reference starts at log(mean(y)) - log(expo)
 * (R/optimize_gp.R:480): set it with sgp_lap_set_f.  obj = the last NR objective value
 * (log q(y | theta, xu, f_hat)); nr_iters = length(objective_function_values).
 * maxit = 0 skips the NR loop: objective and dlogq_dcov_par at the resident f as given. */
int sgp_lap_set_f(sgp_ctx* ctx, const double* f /* n host values, or NULL */, double fill);
/* Per-row Poisson exposure: the reference's `m` is "a vector of the areas of each grid cell"
 * (R/derivative_functions_of_data_likelihoods.R:38), passed through unchanged from
 * optimize_gp's `a` (R/optimize_gp.R:461-468) and used element-wise (-m * exp(ff), y * log(m)).
 * a = n host values (each > 0 and finite; SGP_EINVAL names the first that is not), or NULL for
 * every row = fill.  The vector stays resident; a Laplace evaluation (sgp_eval_laplace,
 * sgp_lap_nr, sgp_lap_begin, sgp_lap_candidates) called with expo = SGP_EXPO_ROWS uses it, and
 * a positive expo keeps meaning that exposure on every row.  Multi-device contexts take the n
 * values in the global row order. */
#define SGP_EXPO_ROWS 0.0
int sgp_lap_set_expo(sgp_ctx* ctx, const double* a /* n host values, or NULL */, double fill);
int sgp_lap_get_f(sgp_ctx* ctx, double* f /* n host values */);
/* grad psi of the last Newton-Raphson step (n host values): the `gradient` element
 * newtrap_sparseGP returns (R/newtrap_sparseGP.R:183-184) -- evaluated at the mode estimate
 * that step started from, as the reference's loop leaves it.  SGP_EINVAL unless an NR step
 * has run since the last NR run began (sgp_lap_begin; a maxit = 0 evaluation takes no step),
 * and after sgp_lap_set_f or OAT candidate scoring. */
int sgp_lap_get_grad_psi(sgp_ctx* ctx, double* grad_psi);
/* objective_function_values of the last NR run (first min(count, max_n) copied; *count = all) */
int sgp_lap_objective_values(sgp_ctx* ctx, double* out, int max_n, int* count);
int sgp_eval_laplace(sgp_ctx* ctx, int kernel, const double* theta, const double* U, int64_t m,
                     int64_t ldu, double delta, double expo, double tol, int maxit,
                     double* obj, double* grad, int* nr_iters);

/* Multi-GPU Laplace as a reduction state machine.  sgp_lap_begin writes this rank's partial
 * sums (count doubles) to the DEVICE buffer red_out; the caller sums them over ranks in place,
 * then calls sgp_lap_step(red_in = the summed buffer, red_out = a different buffer) until
 * *done; each step reports the next count.  Every rank takes identical decisions (they
 * are functions of the summed buffers only).  Buffers hold sgp_lap_red_count doubles. */
int64_t sgp_lap_red_count(int kernel, int d, int64_t m);
int sgp_lap_begin(sgp_ctx* ctx, int kernel, const double* theta, const double* U, int64_t m,
                  int64_t ldu, double delta, double expo, double tol, int maxit, unsigned flags,
                  double* red_out, int64_t* count);
int sgp_lap_step(sgp_ctx* ctx, const double* red_in, double* red_out, int64_t* count,
                 int* done, double* obj, double* grad, int* nr_iters);
/* newtrap_sparseGP alone (R/newtrap_sparseGP.R:6-186): the NR loop from the resident f, f left
 * at the mode; obj = the last entry of objective_function_values (= sgp_lap_begin with
 * SGP_FLAG_OBJ_ONLY driven to completion) */
int sgp_lap_nr(sgp_ctx* ctx, int kernel, const double* theta, const double* U, int64_t m,
               int64_t ldu, double delta, double expo, double tol, int maxit, double* obj,
               int* nr_iters);

/* Full (non-sparse) Gaussian GP over the context's n rows (config 1; requires m_max >= n):
 * obj = log dmvnorm(y; mu, Sigma11) (obj_fun_norm_full, R/laplace_approx_obj_funs.R:56-61) and
 * grad = dlogp_dcov_par_full (R/laplace_approx_gradient.R:1140-1269; its alpha is Sigma11^-1 y,
 * not Sigma11^-1 (y - mu)), Sigma11 = k(xy, xy) + (tau^2 + delta) I.  SGP_FLAG_OBJ_ONLY skips
 * the gradient (grad may be NULL). */
int sgp_eval_full(sgp_ctx* ctx, int kernel, const double* theta, double delta, unsigned flags,
                  double* obj, double* grad);

/* Posterior of the knot values u at the end of a fit, from the context's last completed
 * evaluation (VI: vi_functions.R:1161-1180; FITC: laplace_gradient_ascent.R:1635-1655;
 * Laplace: newtrap_sparseGP.R:137-176).  muu, u_mean: m host values; u_var: m x m host,
 * column-major (ld m). */
int sgp_posterior_u(sgp_ctx* ctx, const double* muu, double* u_mean, double* u_var);

/* Sparse prediction at x_pred (np x d, column-major, ld ldxp) from a knot posterior:
 *   SGP_PRED_VI      predict_vi      (R/vi_functions.R:1222-1333; gaussian only)
 *   SGP_PRED_LAPLACE predict_laplace (R/laplace_approx_prediction.R:3-123; FITC or Laplace fits,
 *                    gaussian != 0 selects the family == "gaussian" Sigma22)
 *   SGP_PRED_FULL    predict_gp_full (R/laplace_approx_prediction.R:281-405): a full Gaussian
 *                    GP -- U = xy, u_mean = y, muu = mu, u_var unused (may be NULL)
 * as dispatched by predict_gp (R/laplace_approx_prediction.R:408-542).  u_var is m x m
 * column-major (ld ldv).  pred_var: np values, or with full_cov the np x np matrix
 * (column-major, ld ldpv).  Host buffers; device work space is allocated per call. */
enum { SGP_PRED_VI = 0, SGP_PRED_LAPLACE = 1, SGP_PRED_FULL = 2 };
int sgp_predict(int device, int kernel, const double* theta, double delta, int method,
                int gaussian, const double* U, int64_t m, int64_t ldu, const double* u_mean,
                const double* muu, const double* u_var, int64_t ldv, const double* x_pred,
                int64_t np, int64_t ldxp, int d, const double* mu_pred, int full_cov,
                double* pred_mean, double* pred_var, int64_t ldpv);

/* Knot gradients (xu_opt = "simultaneous"; the knot branches of delbo_dcov_par
 * R/vi_functions.R:425-593, dlogp_dcov_par R/laplace_approx_gradient.R:973-1126 and
 * dlogq_dcov_par 341-543, with dsqexp_dx2 / dsqexp_dx2_ard
 * R/covariance_function_derivatives.R:178-302 as dcov_fun_dknot).  When enabled,
 * every evaluation also contracts G against dK12/du in the same GEMM epilogue, and the
 * multi-GPU second reduction buffers grow by sgp_knot_red_extra(d, m) doubles (VI, FITC;
 * sgp_lap_red_count already has room).  sgp_knot_gradient then returns, row-major
 * (knot-major, quirk Q16), d obj / d u_kc times the reference's factor
 * (ub - lb) / ((u - lb)(ub - u) + 1e-4) (quirk Q8) with bounds = d x 2 column-major
 * [lower | upper], or NULL for the reference's knot_bounds from this context's rows
 * (vi_functions.R:175-178; multi-GPU callers pass the global bounds, see
 * sgp_ctx_row_bounds). */
int sgp_ctx_enable_knot_grad(sgp_ctx* ctx, int enable);
int64_t sgp_knot_red_extra(int d, int64_t m);
int sgp_knot_gradient(sgp_ctx* ctx, const double* bounds, double* grad_knot);
int sgp_ctx_row_bounds(sgp_ctx* ctx, double* col_min, double* col_max);

/* OAT knot proposal scoring (VI): the ELBO at knots [U; cand_t] for each of T candidate knots
 * (cand: T x d, column-major, ld ldc) at fixed theta -- the meta-model y values of
 * knot_prop_random_norm_vi / knot_prop_ego_norm_vi (R/vi_functions.R:2196-2300, 1584-) --
 * from bordered Schur complements instead of T rebuilds of K12.  NaN marks a candidate whose
 * bordered K22 or Bm is not positive definite (the reference's try-error). */
int sgp_vi_candidates(sgp_ctx* ctx, int kernel, const double* theta, const double* U, int64_t m,
                      int64_t ldu, double delta, unsigned flags, const double* cand, int64_t T,
                      int64_t ldc, double* obj_out);

/* OAT knot proposal scoring for FITC (knot_prop_random_norm / knot_prop_ego_norm,
 * R/knot_proposal_functions.R:1176-1363, 498-): obj_fun_norm at knots [U; cand_t] with
 * Sigma22 = Kuu + delta I, for each of T candidates (m + 1 <= m_max).  NaN = try-error. */
int sgp_fitc_candidates(sgp_ctx* ctx, int kernel, const double* theta, const double* U,
                        int64_t m, int64_t ldu, double delta, unsigned flags, const double* cand,
                        int64_t T, int64_t ldc, double* obj_out);

/* OAT knot proposal scoring for Poisson Laplace (knot_prop_random / knot_prop_ego,
 * R/knot_proposal_functions.R:1001-1173, 46-): for each candidate, newtrap_sparseGP at knots
 * [U; cand_t] warm-started from the resident f (the fit's fmax); obj_out[t] = its last
 * objective value.  The resident f is restored afterwards.  NaN = try-error. */
int sgp_lap_candidates(sgp_ctx* ctx, int kernel, const double* theta, const double* U, int64_t m,
                       int64_t ldu, double delta, double expo, double tol, int maxit,
                       const double* cand, int64_t T, int64_t ldc, double* obj_out);

/* Per-phase timing (HIP events on the launch stream).  Enabling clears the record; every
 * evaluation after it appends its phases, and sgp_ctx_timings returns the per-phase totals
 * over those sgp_ctx_timing_evals() evaluations (names: '\n'-separated phase names; ms: their
 * total durations, max n entries).  Nothing is read back while evaluations run. */
int sgp_ctx_enable_timing(sgp_ctx* ctx, int enable);
/* record only the phase called `name` (NULL: every phase) -- bench.py times its dominant
 * kernel inside the timed region this way, with no other event records in the stream */
int sgp_ctx_timing_filter(sgp_ctx* ctx, const char* name);
int64_t sgp_ctx_timing_evals(const sgp_ctx* ctx);
int sgp_ctx_timings(sgp_ctx* ctx, char* names, int64_t names_len, double* ms, int max_n, int* count);

#ifdef __cplusplus
}
#endif
#endif /* SGP_H */
