// Internal declarations shared by the HIP translation units of libsgp.so.
// Device code targets gfx950 (MI355X / CDNA4) only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SGP_MAXD 32          // largest input dimension d supported by the fused kernels
#define SGP_TILE 128         // n x m tile edge of the MFMA kernels (rows and knots padded to it)
#define SGP_DB 64            // block edge of the m x m dense routines
#define SGP_GJ_SYNC_WORDS (128 + 2 * 64 * 64)   // k_dense.hip: ticket, exits, flags (nb <= 64)

typedef double d4 __attribute__((ext_vector_type(4)));

// exp(x) for x <= 0 (the only range a covariance exponent takes): Cody-Waite reduction
// x = k ln2 + r, |r| <= ln2/2, degree-13 Taylor polynomial (truncation < 5e-18), ldexp.
// Branch-free; < 2 ulp; returns 0 below -745.13 (where exp underflows).
__device__ __forceinline__ double sgp_exp_nonpos(double x) {
  constexpr double c2 = 1.0 / 2, c3 = 1.0 / 6, c4 = 1.0 / 24, c5 = 1.0 / 120, c6 = 1.0 / 720,
                   c7 = 1.0 / 5040, c8 = 1.0 / 40320, c9 = 1.0 / 362880, c10 = 1.0 / 3628800,
                   c11 = 1.0 / 39916800, c12 = 1.0 / 479001600, c13 = 1.0 / 6227020800.0;
  const double k = __builtin_rint(x * 1.4426950408889634074);
  double r = __builtin_fma(-k, 6.93147180369123816490e-01, x);
  r = __builtin_fma(-k, 1.90821492927058770002e-10, r);
  double p = c13;
  p = __builtin_fma(p, r, c12);
  p = __builtin_fma(p, r, c11);
  p = __builtin_fma(p, r, c10);
  p = __builtin_fma(p, r, c9);
  p = __builtin_fma(p, r, c8);
  p = __builtin_fma(p, r, c7);
  p = __builtin_fma(p, r, c6);
  p = __builtin_fma(p, r, c5);
  p = __builtin_fma(p, r, c4);
  p = __builtin_fma(p, r, c3);
  p = __builtin_fma(p, r, c2);
  p = __builtin_fma(p, r, 1.0);
  p = __builtin_fma(p, r, 1.0);
  const double v = __builtin_ldexp(p, (int)fmax(k, -2000.0));
  return (x < -745.13321910194110842) ? 0.0 : v;
}

// Covariance-function parameters in the form the kernels use.
//   sqexp: K = sig2 * exp(coef * sum_c d_c^2),            coef = -1/(2 l^2)
//   ard:   K = sig2 * exp(-0.5 * sum_c (d_c * rl_c)^2),    rl_c = 1/l_c
//   exp:   K = sig2 * exp(coef * sum_c |d_c|),             coef = -1/l
// d_c = x_c - u_c on the raw coordinates (so exact coincidence stays exact).
struct KernParams {
  int kernel;            // 0 sqexp, 1 ard, 2 exp
  int d;
  int L;                 // number of length scales: 1 or d
  int P;                 // number of hyperparameters: L + 2
  double sigma, sig2, tau, tau2, delta;
  double coef;
  double l[SGP_MAXD];
  double rl[SGP_MAXD];   // 1/l_c (sqexp/exp: rl[0] = 1/l)
  double rl2[SGP_MAXD];  // 1/l_c^2
  // Origin the K12 builder's GEMM-form exponent is centred on (the knots' mean; any point
  // gives the same K up to rounding -- centring keeps |x~|^2 + |u~|^2 small, see k_cov.hip)
  double ctr[SGP_MAXD];
  // Upper bound on |x~|^2 over the knots and the rows the builder sees (x~ = (x - ctr) * rl):
  // the GEMM-form exponent's absolute rounding is ~eps (|x~|^2 + |u~|^2), so above
  // SGP_MFMA_SPAN2_MAX the direct-difference VALU builder is used instead (knm_mfma_ok).
  double span2;
  double lsig2;          // log(sig2): folded into the builder's GEMM-form exponent
  // sgp_exp_kp's constants as kernel arguments, so they sit in SGPRs and each Horner step is
  // one v_fma_f64 (as literals the compiler pairs every step with a v_mov_b64): log2(e),
  // ln2 hi/lo, then the degree-13 Taylor coefficients 1/13! .. 1/2!
  double ec[16];
  // sgp_exp_tab's constants: 32 log2(e), ln2/32 hi/lo, 1/6! .. 1/2!, and the table 2^(j/32)
  double xt[8];
  double et[32];
};
void set_exp_consts(KernParams* kp);

// |x~|^2 bound below which the matrix-core K12 builder keeps K within ~1e-12 relative of the
// direct-difference form (1e4 * 2^-52 * a few); the C2 / C3 / C5 workloads sit below 100.
constexpr double SGP_MFMA_SPAN2_MAX = 1.0e4;
inline bool knm_mfma_ok(const KernParams& kp) {
  return kp.d <= 32 && kp.kernel != 2 && kp.span2 <= SGP_MFMA_SPAN2_MAX;
}

// exp(x) for x already clamped to [-746, log(DBL_MAX)] by a 32-entry table: x = (32 e + j) ln2/32
// + r, |r| <= ln2/64, exp(x) = 2^e T_j (1 + p(r)) with p the degree-6 Taylor polynomial of
// e^r - 1 (truncation < 2e-18 relative).  etab = kp.et staged in LDS: 32 doubles span the 64
// banks once, so a wave's lookups never conflict.  Below -745.13 ldexp underflows to 0.
__device__ __forceinline__ double sgp_exp_tab(double x, const KernParams& kp,
                                              const double* etab) {
  const double k = __builtin_rint(x * kp.xt[0]);
  double r = __builtin_fma(-k, kp.xt[1], x);
  r = __builtin_fma(-k, kp.xt[2], r);
  double p = kp.xt[3];
  p = __builtin_fma(p, r, kp.xt[4]);
  p = __builtin_fma(p, r, kp.xt[5]);
  p = __builtin_fma(p, r, kp.xt[6]);
  p = __builtin_fma(p, r, kp.xt[7]);
  p = __builtin_fma(p, r, 1.0);
  p = p * r;
  const int ki = (int)k;
  const double t = etab[ki & 31];
  return __builtin_ldexp(__builtin_fma(t, p, t), ki >> 5);
}

// exp(x) for x already clamped to [-746, log(DBL_MAX)]: the same reduction and polynomial as
// sgp_exp_nonpos with the constants read from kp (SGPRs).  Below -745.13 ldexp underflows to
// 0, as exp does.
__device__ __forceinline__ double sgp_exp_kp(double x, const KernParams& kp) {
  const double k = __builtin_rint(x * kp.ec[0]);
  double r = __builtin_fma(-k, kp.ec[1], x);
  r = __builtin_fma(-k, kp.ec[2], r);
  double p = kp.ec[3];
#pragma unroll
  for (int q = 4; q < 15; ++q) p = __builtin_fma(p, r, kp.ec[q]);
  p = __builtin_fma(p, r, 1.0);
  p = __builtin_fma(p, r, 1.0);
  return __builtin_ldexp(p, (int)k);
}


// ---------------------------------------------------------------- k_cov.hip
// Layer-1 fillers, column-major output (R layout).  x/xp are column-major on device.
hipError_t launch_fill_cov(const KernParams& kp, const double* x, int64_t n, int64_t ldx,
                           const double* xp, int64_t np, int64_t ldxp, bool sym, double* out,
                           int64_t ldo, hipStream_t s);
hipError_t launch_fill_dcov(const KernParams& kp, const double* x, int64_t n, int64_t ldx,
                            const double* xp, int64_t np, int64_t ldxp, bool sym, int param,
                            double* out, int64_t ldo, hipStream_t s);
// t partials of the builder (VI): *t_rows rows tslab[q][j] (q < t_rows <= n_pad / 64) whose
// column sums are t_j = sum_i K_ij r_i; reduce with launch_knot_reduce(tslab, *t_rows, mp, 1, ...).
hipError_t launch_build_knm_t(const KernParams& kp, const double* X, int64_t ldx, int64_t n,
                              int64_t n_pad, const double* U, int64_t ldu, int64_t m, int64_t mp,
                              double* K, const double* r, double* tslab, int64_t* t_rows,
                              hipStream_t s, bool beside_chain = true);
// K12 (n_pad x mp, row-major, ld = mp).  Rows >= n and columns >= m are written as 0.
// beside_chain: the K22 chain runs concurrently on the aux stream (phase 1), so the first row
// blocks are built at reduced occupancy to leave it room (launch_build_knm_t always does).
hipError_t launch_build_knm(const KernParams& kp, const double* X, int64_t ldx, int64_t n,
                            int64_t n_pad, const double* U, int64_t ldu, int64_t m, int64_t mp,
                            double* K, hipStream_t s, bool beside_chain = false);
// K22 = Kuu + diag_add on the diagonal, padded with identity (mp x mp, row-major).
// diag value = ((sig2 + tau2 + delta) - diag_sub) exactly like R's make_cov(...) - tau^2 I.
hipError_t launch_build_kmm(const KernParams& kp, const double* U, int64_t ldu, int64_t m,
                            int64_t mp, double diag_sub, double* K22, hipStream_t s,
                            double* K22_copy = nullptr);   // also written when non-null
// sum_{j,k<m} G22_jk * dK22^p_jk for every parameter p != tau, where
// G22 = a*u u^T + b*(Ainv - Binv) + c*M3.  Writes P partial sums per block into slab.
// records per block: P (sigma, length scales, tau-coincidence sum of G22)
hipError_t launch_contract_kmm(const KernParams& kp, const double* U, int64_t ldu, int64_t m,
                               int64_t mp, const double* uvec, const double* Ainv,
                               const double* Binv, const double* M3, double a, double b,
                               double c, const double* vvec, const double* wvec, double e2,
                               double* slab, int64_t slab_cap, int* nblocks, hipStream_t s);

// ---------------------------------------------------------------- k_mfma.hip
// S_aug partials: S = K^T diag(w) K (lower 128-tiles), t = K^T diag(w) r, rr = r^T diag(w) r.
// w == nullptr means w = 1.  Writes per-(split,tile) slabs, then reduces into
// red = [S (mp x mp, full symmetric), t (mp), rr, n_local].
// With tv set, t = K^T tv and rr = tv^T r instead (w still weights S).
hipError_t launch_syrk_aug(const double* K, int64_t n_pad, int64_t mp, const double* r,
                           const double* w, double* slab, int64_t slab_cap, double* red,
                           hipStream_t s, int part = 3,  // part: 1 = main kernel, 2 = reduce
                           const double* tv = nullptr,
                           int with_t = 1,               // 0: S only (red[mm..] untouched)
                           const double* rr_src = nullptr,    // part 2: copy *rr_src to rr's slot
                           bool packed = false,    // part 2: S as its packed lower 64-blocks
                           bool w_nonneg = false,  // w >= 0: sqrt(w) scales the staged rows
                           // part 2, many splits, one slab region: the two reduction passes in
                           // one launch (the last group of each 256-element slice sums the group
                           // totals); SGP_SYRK_RSYNC_WORDS zeroed words, left zeroed
                           unsigned* rsync = nullptr);
#define SGP_SYRK_RSYNC_WORDS 4096
// doubles of S's packed lower 64-blocks, and the full S from them (sgp_ctx_set_packed_reduction)
int64_t syrk_packed_doubles(int64_t mp);
hipError_t launch_unpack_lower64(const double* packed, int64_t mp, double* S, hipStream_t s);
int64_t syrk_slab_doubles(int64_t n_pad, int64_t mp);
// true when launch_syrk_aug uses the fragment-balanced mp = 256 kernel (S only)
bool syrk_use_s256(int64_t mp, bool with_t);
// Gradient contraction on T = K M (K: n_pad x mp, M: mp x mp):
//   G_ij = alpha_i u_j + rs_i T_ij,  alpha_i = (r_i - K_i u) * iz_i computed in the same pass
//   (iz_i = invz_vec ? invz_vec[i] : invz; uvec == nullptr -> alpha = u = 0;
//   rs_i = rs_vec ? rs * rs_vec[i] : rs).  Per 128x128 tile record (L + 5 doubles):
//   [sum G*K, sum G*K*w_c (c < L), tau-coincidence sum G, count, sum diag_j, alpha^T alpha
//   (only if count_a2)].  coinc_diag may be nullptr.
// Epilogue operands of the K12 contraction (k_mfma.hip k_contract):
//   G_ij = alpha_i u_j + beta_i v_j + rs_i T_ij,  T = K M,  rs_i = rs * (rs_vec ? rs_vec[i] : 1)
//   alpha_i = alpha_in[i] when alpha_in is set, else (r_i - K_i u) * iz_i fused into the k-loop
//   when u is set (iz_i = invz_vec ? invz_vec[i] : invz), else 0.
struct ConArgs {
  const double* r = nullptr;
  double invz = 0.0;
  const double* invz_vec = nullptr;
  const double* uvec = nullptr;
  const double* alpha_in = nullptr;
  const double* beta_in = nullptr;
  const double* vvec = nullptr;
  const double* rs_vec = nullptr;
  double rs = 1.0;
  const double* cdiag = nullptr;
  int count_a2 = 0;
  double* alpha_out = nullptr;
  // knot gradient partials (d <= 8): per 128-row tile ti and column j, sum_i G_ij K_ij t_ijc
  // with t = scaled coordinate difference (ARD: (x_c - u_c)/l_c; sqexp/exp: x_c - u_c),
  // written to knot_slab[(ti * mp + j) * d + c]
  double* knot_slab = nullptr;
  // stored products T = K M (row-major n_pad x mp): a row-quadratic pass writes T to tstore; a
  // gradient pass with tin set reads T instead of running the MFMA k-loop (alpha must then come
  // from alpha_in; d <= 8)
  double* tstore = nullptr;
  const double* tin = nullptr;
  // a second stored product folded into the same pass (FITC / Laplace: the K Bm^-1 and
  // K K22^-1 gradient terms summed in one read of K): G_ij += rs2_i (K M2)_ij with
  // rs2_i = rs2 * rs_vec2[i] (or rs2), T2 = K M2 read from tin2; M2 serves the coincidence sums
  const double* tin2 = nullptr;
  const double* M2 = nullptr;
  const double* rs_vec2 = nullptr;
  double rs2 = 0.0;
  // the balanced (Stream-K) launch of VI's gradient contraction (k_contract_sk): hand-over
  // slots (sgp_con_sk_doubles), per-slot flags (sk_slots words, zero at allocation), this
  // launch's epoch (> 0, new per launch), the resident-workgroup count and a status word (-1:
  // a hand-over wait expired).  sk_ws == nullptr: always the one-tile-per-workgroup grid
  double* sk_ws = nullptr;
  unsigned* sk_flags = nullptr;
  unsigned sk_epoch = 0;
  int sk_slots = 0;
  int* sk_status = nullptr;
  int sk_dp = -1;   // whole rounds run as the grid before the balanced part (-1: all but the last)
};
// hand-over workspace (doubles) of a balanced contraction over `slots` workgroups
int64_t sgp_con_sk_doubles(int slots);
hipError_t launch_contract_args(const KernParams& kp, const double* K, const double* M,
                                const double* X, int64_t ldx, int64_t n, int64_t n_pad,
                                const double* U, int64_t ldu, int64_t m, int64_t mp,
                                const ConArgs& ca, double* slab, int64_t* nrec_out,
                                int64_t* nwg_out, hipStream_t s);
hipError_t launch_contract_knm(const KernParams& kp, const double* K, const double* M,
                               const double* X, int64_t ldx, int64_t n, int64_t n_pad,
                               const double* U, int64_t ldu, int64_t m, int64_t mp,
                               const double* r, double invz, const double* invz_vec,
                               const double* uvec, const double* rs_vec, double rs,
                               const double* coinc_diag, int count_a2, double* slab,
                               int64_t* nrec_out, int64_t* nwg_out, hipStream_t s);
// out_i = sum_j K_ij (K M)_ij = diag(K M K^T) (n_pad); optional fused alpha as above.
// rowq_slab: (mp/128) x n_pad work.  tstore (optional, n_pad x mp row-major): keeps T = K M for a
// later gradient pass with ConArgs::tin = tstore.
hipError_t launch_rowquad_knm(const KernParams& kp, const double* K, const double* M, int64_t n,
                              int64_t n_pad, int64_t m, int64_t mp, const double* r,
                              double invz, const double* invz_vec, const double* uvec,
                              double* alpha_out, double* rowq_slab, double* out,
                              hipStream_t s, double* tstore = nullptr);
// generic m x m GEMM on f64 MFMA: C = alpha*op(A)*op(B) + beta*C, sizes multiples of 64.
hipError_t launch_gemm64(bool transA, bool transB, bool lower_only, int64_t M, int64_t N,
                         int64_t K, double alpha, const double* A, int64_t lda,
                         const double* B, int64_t ldb, double beta, double* C, int64_t ldc,
                         hipStream_t s);

// ---------------------------------------------------------------- k_dense.hip
// In-place inverse of an SPD matrix A (mp x mp, full storage) by blocked Gauss-Jordan with
// 64-wide pivots; logd[k] = sum log L_ii of the k-th pivot block's Cholesky factor, so
// log det A = 2 * sum_k logd[k].  Work: R (64 x mp), Cb (mp x 64), P (64 x 64).
// In-place SPD inverse (blocked Gauss-Jordan) of the mp x mp matrix A.  P: mp x 64 pivot
// inverses; logd: mp / 64 block log-determinant halves; sync: SGP_GJ_SYNC_WORDS words, zero
// when the chain is launched (and zero again when it has finished), one area per chain that may
// run at the same time; R: mp x mp scratch (only for mp > 64 * 64)
hipError_t dense_spd_inverse(double* A, int64_t mp, double* R, double* P, double* logd,
                             int* status, unsigned* sync, hipStream_t s);
// out = inv(A0 + beta B0), the sum formed by the chain as it reads it (out, R distinct from A0
// and B0)
hipError_t dense_spd_inverse_sum(const double* A0, double beta, const double* B0, double* out,
                                 int64_t mp, double* R, double* P, double* logd, int* status,
                                 unsigned* sync, hipStream_t s);
// the same with the chain chosen by the caller: the persistent one-launch chain (per_step false;
// nb <= 64) or one launch per pivot step (any nb) -- bit-identical results (sgp_diag_gj_pair)
hipError_t dense_spd_inverse_chain(double* A, int64_t mp, double* R, double* P, double* logd,
                                   int* status, unsigned* sync, hipStream_t s, bool per_step);
hipError_t dense_spd_inverse_sum_chain(const double* A0, double beta, const double* B0,
                                       double* out, int64_t mp, double* R, double* P, double* logd,
                                       int* status, unsigned* sync, hipStream_t s, bool per_step);
// C = a*A + b*B elementwise over mp x mp
hipError_t dense_axpby(double a, const double* A, double b, const double* B, double* C,
                       int64_t count, hipStream_t s);
// VI phase 2's m-vectors: the row pass u = invz Binv t, P = a K22inv + b Binv, part_j =
// sum_k Binv_jk S_jk (part: mp doubles), and the scalars *tu_out = t.u, *trbs_out = sum part
// (= tr(Binv S)), *rr_out = *rr (one block; only the finish reads them, so they can run on
// another stream behind the row pass)
hipError_t launch_vi_mm_rows(const double* Binv, const double* K22inv, const double* S,
                             const double* t, int64_t mp, double invz, double a, double b,
                             double* u, double* P, double* part, hipStream_t s);
hipError_t launch_vi_mm_scalars(const double* t, const double* u, const double* part, int64_t mp,
                                const double* rr, double* tu_out, double* trbs_out,
                                double* rr_out, hipStream_t s);
// y = scale * A x  (A: mp x mp row-major)
hipError_t dense_gemv(const double* A, int64_t mp, const double* x, double scale, double* y,
                      hipStream_t s);
// out[0] = sum_i a_i * b_i over count (b == nullptr: sum a_i); deterministic two-stage.
hipError_t launch_dot(const double* a, const double* b, int64_t count, double* partial,
                      double* out, hipStream_t s);
// out[k] = sum over rows r < nrows of slab[r*ncol + k], k < ncol; deterministic.
hipError_t launch_colsum(const double* slab, int64_t nrows, int64_t ncol, double* out,
                         hipStream_t s);
// diag extraction: out[j] = A[j*lda + j]
hipError_t launch_diag(const double* A, int64_t mp, int64_t lda, double* out, hipStream_t s);
// sum of per-block logs -> out
hipError_t launch_sum_small(const double* v, int64_t count, double* out, hipStream_t s);
// launch_sum_small and launch_diag in one launch (sum over v[0..count), out diag of A)
hipError_t launch_sum_and_diag(const double* v, int64_t count, double* sum, const double* A,
                               int64_t mp, int64_t lda, double* diag, hipStream_t s);

// FITC per-row helpers (k_dense.hip).
// w_i = 1 / (c0 - q_i) for i < n (0 for padded rows); per-block sums of log(c0 - q_i) -> slab.
hipError_t launch_fitc_z(const double* q, int64_t n, int64_t n_pad, double c0, double* w,
                         double* slab, int* nblocks, hipStream_t s);
// omega_i = alpha_i^2 - (w_i - w_i^2 p_i) for i < n (0 otherwise); per-block sums -> slab.
hipError_t launch_fitc_omega(const double* alpha, const double* w, const double* p, int64_t n,
                             int64_t n_pad, double* omega, double* slab, int* nblocks,
                             hipStream_t s);

// ---------------------------------------------------------------- k_lap.hip
// K12 matrix-vector passes (HBM-bound, one read of K each).
// y1 = K x1 (and y2 = K x2 if x2 != nullptr), n_pad rows.
hipError_t launch_gemv_rows(const double* K, int64_t n_pad, int64_t mp, const double* x1,
                            const double* x2, double* y1, double* y2, hipStream_t s);
// out[v*mp + j] = sum_i K_ij V[v*ldv + i] for v < nv (<= 4); part = slab of
// lap_gemv_cols_slab(n_pad, mp, nv) doubles (row-chunk partials, deterministic reduce).
hipError_t launch_gemv_cols(const double* K, int64_t n_pad, int64_t mp, const double* V,
                            int64_t ldv, int nv, double* part, int64_t part_cap, double* out,
                            hipStream_t s);
int64_t lap_gemv_cols_slab(int64_t n_pad, int64_t mp, int nv);
// Poisson-Laplace per-row steps (see k_lap.hip for the formulas and reference lines).  av: the
// per-row exposure (n_pad values) or nullptr for the scalar expo on every row.
hipError_t launch_lap_z(const double* q, int64_t n, int64_t n_pad, double c0, double* Z,
                        double* zinv, hipStream_t s);
hipError_t launch_lap_obj(int64_t n, int64_t n_pad, const double* f, const double* y,
                          const double* mu, const double* Z, const double* zinv, double expo,
                          const double* av, double* B, double* rf, double* tv, double* slab,
                          int* nblocks, hipStream_t s);
hipError_t launch_lap_nr_a(int64_t n, int64_t n_pad, const double* f, const double* y,
                           const double* mu, const double* Z, const double* zinv, double expo,
                           const double* av, const double* y1, double tol, double* g,
                           double* omzw, double* v, double* gpsi, double* slab, int* nblocks,
                           hipStream_t s);
// NR part a as one K pass (y1 = K x1, the row update above, out = K^T v, out_cnt = stop-rule
// count); mp <= 2048; part: lap_rowpass_slab(n_pad, mp) doubles.
hipError_t launch_lap_nr_a_fused(const double* K, int64_t n, int64_t n_pad, int64_t mp,
                                 const double* x1, const double* f, const double* y,
                                 const double* mu, const double* Z, const double* zinv,
                                 double expo, const double* av, double tol, double* y1, double* g,
                                 double* omzw, double* v, double* gpsi, double* part,
                                 int64_t part_cap, double* out, double* out_cnt, hipStream_t s);
// NR part b + the next objective's t as one K pass: f updated in place (y2 = K x2), out_t =
// K^T tv and out_rr = sum tv (f - mu) at the new f, tv = (f - mu)/Z.  mp <= 2048.
hipError_t launch_lap_nr_b_t_fused(const double* K, int64_t n, int64_t n_pad, int64_t mp,
                                   const double* x2, double* f, const double* y,
                                   const double* mu, const double* Z, const double* zinv,
                                   const double* g, const double* omzw, const double* y1,
                                   double* part, int64_t part_cap, double* out_t, double* out_rr,
                                   hipStream_t s);
// work space of both fused passes (doubles)
int64_t lap_rowpass_slab(int64_t n_pad, int64_t mp);
hipError_t launch_lap_nr_b(int64_t n, int64_t n_pad, double* f, const double* mu, const double* Z,
                           const double* g, const double* omzw, const double* y1,
                           const double* y2, hipStream_t s);
hipError_t launch_lap_grad_a(int64_t n, int64_t n_pad, const double* f, const double* y,
                             const double* mu, const double* Z, const double* zinv, double expo,
                             const double* av, const double* y1, const double* p, double* c2,
                             double* g, double* B, double* dMt, double* sv, double* bsv,
                             hipStream_t s);
hipError_t launch_lap_grad_b(int64_t n, int64_t n_pad, const double* B, const double* sv,
                             const double* y3, const double* dMt, const double* c2,
                             const double* g, double* h, double* a, double* slab, int* nblocks,
                             hipStream_t s);

// knot gradients (k_mfma.hip / k_cov.hip)
// out[j*d + c] (+)= sum over row tiles of knot_slab (deterministic two-level reduction);
// part: 64 * mp * d doubles of work space
hipError_t launch_knot_reduce(const double* knot_slab, int64_t ntiles, int64_t mp, int d,
                              double* part, int64_t part_cap, double* out, bool accumulate,
                              hipStream_t s);
// out[k*d + c] = 2 sum_l G22_kl K22_kl (u_lc - u_kc), G22 as in launch_contract_kmm
hipError_t launch_knot_kmm(const KernParams& kp, const double* U, int64_t ldu, int64_t m,
                           int64_t mp, const double* uvec, const double* Ainv,
                           const double* Binv, const double* M3, double a, double b, double c,
                           const double* vvec, const double* wvec, double e2, double* out,
                           hipStream_t s);

// C = A^T B over n_pad rows (A: n_pad x ma, ld lda; B: n_pad x mb, ld ldb; ma, mb multiples of
// 128), f64 MFMA split-K; C row-major ma x mb.  slab: gemm_tn_slab_doubles(n_pad, ma, mb).
int64_t gemm_tn_slab_doubles(int64_t n_pad, int64_t ma, int64_t mb);
hipError_t launch_gemm_tn(const double* A, int64_t lda, int64_t ma, const double* B, int64_t ldb,
                          int64_t mb, int64_t n_pad, double* slab, int64_t slab_cap, double* C,
                          hipStream_t s);
// candidate knots (VI, k_lap.hip): per column t < T of the mp x Tp row-major blocks, the
// bordered-system scalars -> obj[t] (NaN when a Schur complement is not positive)
hipError_t launch_vi_cand_scalars(int64_t m, int64_t mp, int64_t T, int64_t Tp,
                                  const double* K22c, const double* W, const double* SW,
                                  const double* P, const double* Bt, const double* BB,
                                  const double* u, const double* rk, const double* cc,
                                  const double* base, double* out, hipStream_t s);
// column sums of squares: out[j] = sum_i K_ij^2 (deterministic two-level, part as gemv_cols)
hipError_t launch_colnorm2(const double* K, int64_t n_pad, int64_t mp, double* part,
                           int64_t part_cap, double* out, hipStream_t s);

// One contraction pass's records, in two launches (k_mfma.hip k_rec_pass1 / k_rec_pass2):
// rec[c] = sum_k slab[c * len + k] for c < nrow (field-major per-tile records), plus tau's
// coincidence sums {sum G_ij, #pairs, sum cdiag_j} over the pairs x_i == u_j added to
// rec[coff + 0..2]; alpha = the pass's alpha_i (alpha_in, or the fused alpha written through
// alpha_out).  part: nrow * 32 + 3 * 1024 doubles (both passes' partials).
// With defer != nullptr the second launch is only described in *defer, for the end-of-evaluation
// readback kernel to run first (launch_rec_gather: one launch fewer on the critical path).
struct RecPass2 {
  const double* part_r = nullptr;
  const double* part_c = nullptr;
  double* rec = nullptr;   // nullptr: nothing deferred
  int G = 0, nrow = 0, nbc = 0, coff = 0;
};
hipError_t launch_records(const double* slab, int64_t nrow, int64_t len, const double* X,
                          int64_t ldx, int64_t n, int d, const double* U, int64_t ldu, int64_t m,
                          const uint64_t* khash, const int* kidx, const double* K, int64_t mp,
                          const double* M, const ConArgs& cg, const double* alpha, double* part,
                          int64_t part_cap, int coff, double* rec, uint8_t* cflag, int flag_mode,
                          hipStream_t s, RecPass2* defer = nullptr);
// The end-of-evaluation readback, one block: a deferred records pass 2 (p2.rec set) and then
// dst[off[q] + i] = src[q][i] for each segment (dst: pinned host memory, device-visible).
constexpr int SGP_RB_SEGS = 4;
struct GatherSegs {
  const double* src[SGP_RB_SEGS];
  int off[SGP_RB_SEGS];   // destination offset (doubles)
  int n[SGP_RB_SEGS];     // doubles
  int count;
};
hipError_t launch_rec_gather(const RecPass2& p2, const GatherSegs& g, double* dst, hipStream_t s);
