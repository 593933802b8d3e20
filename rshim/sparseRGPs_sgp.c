/*
 * sparseRGPs_sgp.c -- the R side of the drop-in boundary: libsgp.so (include/sgp.h) behind
 * the native routines luisdamiano/sparseRGPs registers.
 *
 * Part 1 replaces src/RcppExports.cpp + src/covariance_functionsC.cpp +
 * src/covariance_function_derivativesC.cpp: the 20 `.Call` routines of
 * src/RcppExports.cpp:284-306 under the same symbol names and arities, registered by
 * R_init_sparseRGPs exactly like RcppExports.cpp:309-312, so R/RcppExports.R:1-127 and every
 * R caller stay unchanged.  Plain R C API (no Rcpp).  Argument meaning and error behaviour
 * follow the Rcpp originals:
 *   - cov_par is a named list; a missing name is Rcpp's "Index out of bounds" error;
 *   - x_pred = matrix() (a 1x1 NA) selects the symmetric mode (NumericMatrix::is_na(x_pred(0,0)));
 *   - an unknown covariance function / parameter name prints the reference's Rcerr message
 *     and returns a 0x0 matrix;
 *   - the per-pair exports return the same named lists (derivative, trans_par, inv_trans_par),
 *     including inv_trans_par = real_to_pos(sigma) = exp(sigma) as the originals compute it.
 *
 * Part 2 is the fused hot path for the R drivers (rshim/R/sgp_hotpath.R): a device-resident
 * context per fit (external pointer with a finalizer) and one call per optimizer iteration.
 *
 * Build: see rshim/Makevars (links -lsgp).  R itself is absent from this repository's
 * environments, so the file is compiled (gcc -Werror) against tests/r_api/'s declarations of
 * the R API it uses and linked with a mock R runtime (tests/r_api/mock_rt.c):
 * tests/test_rshim_exec.py calls every registered routine by name and arity, checks PROTECT
 * balance after each call and compares the results with fixtures and the oracle;
 * tests/test_rshim.py checks the registry against the reference's RcppExports.cpp.
 */
#include <R.h>
#include <Rinternals.h>
#include <R_ext/Rdynload.h>

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "sgp.h"

/* ------------------------------------------------------------------ helpers */

static int sgp_dev(void) {
  const char* s = getenv("SGP_DEVICE");
  return s ? atoi(s) : 0;
}

/* cov_par[[name]] as Rcpp's as<double>(cov_par[name]) -- error text as Rcpp's */
static double list_num(SEXP lst, const char* name) {
  SEXP nms = Rf_getAttrib(lst, R_NamesSymbol);
  if (!Rf_isNull(nms))
    for (R_len_t i = 0; i < Rf_length(lst); ++i)
      if (!strcmp(CHAR(STRING_ELT(nms, i)), name)) return Rf_asReal(VECTOR_ELT(lst, i));
  Rf_error("Index out of bounds: [index='%s'].", name);
  return 0.0;
}

static int list_has(SEXP lst, const char* name) {
  SEXP nms = Rf_getAttrib(lst, R_NamesSymbol);
  if (Rf_isNull(nms)) return 0;
  for (R_len_t i = 0; i < Rf_length(lst); ++i)
    if (!strcmp(CHAR(STRING_ELT(nms, i)), name)) return 1;
  return 0;
}

static const char* str0(SEXP s) {
  if (!Rf_isString(s) || Rf_length(s) < 1) Rf_error("expecting a string");
  return CHAR(STRING_ELT(s, 0));
}

/* theta = [sigma, l (or cov_par[[lnames[c]]], c < d), tau]; tau = 0 when not needed and absent */
static void theta_from(SEXP cov_par, int ard, SEXP lnames, int d, int need_tau, double* theta) {
  theta[0] = list_num(cov_par, "sigma");
  if (ard) {
    if (Rf_length(lnames) < d) Rf_error("lnames has fewer than %d names", d);
    for (int c = 0; c < d; ++c) theta[1 + c] = list_num(cov_par, CHAR(STRING_ELT(lnames, c)));
  } else {
    theta[1] = list_num(cov_par, "l");
  }
  const int L = ard ? d : 1;
  theta[L + 1] = (need_tau || list_has(cov_par, "tau")) ? list_num(cov_par, "tau") : 0.0;
}

static void check(int st) {
  if (st != SGP_OK) Rf_error("%s", sgp_last_error());
}

static SEXP empty_matrix(void) { return Rf_allocMatrix(REALSXP, 0, 0); }

/* NumericMatrix::is_na(x_pred(0,0)): matrix() is a 1x1 logical NA */
static int is_sym(SEXP xr) {
  if (Rf_length(xr) < 1) Rf_error("x_pred has no elements (use matrix() for the symmetric mode)");
  return ISNAN(REAL(xr)[0]);
}

static SEXP as_real(SEXP x) { return Rf_coerceVector(x, REALSXP); }

static int ncols_of(SEXP x) { return Rf_isMatrix(x) ? Rf_ncols(x) : 1; }
static int nrows_of(SEXP x) { return Rf_isMatrix(x) ? Rf_nrows(x) : Rf_length(x); }

/* list(name1 = v1, ...) */
static SEXP named_list(int n, const char** names, SEXP* vals) {
  SEXP out = PROTECT(Rf_allocVector(VECSXP, n));
  SEXP nm = PROTECT(Rf_allocVector(STRSXP, n));
  for (int i = 0; i < n; ++i) {
    SET_VECTOR_ELT(out, i, vals[i]);
    SET_STRING_ELT(nm, i, Rf_mkChar(names[i]));
  }
  Rf_setAttrib(out, R_NamesSymbol, nm);
  UNPROTECT(2);
  return out;
}

/* ------------------------------------------------- Part 1: the 20 registered routines */

/* real_to_pos / pos_to_real: covariance_function_derivativesC.cpp:10-20 */
SEXP _sparseRGPs_real_to_pos(SEXP x) {
  SEXP xr = PROTECT(as_real(x));
  const R_xlen_t n = XLENGTH(xr);
  SEXP out = PROTECT(Rf_allocVector(REALSXP, n));
  for (R_xlen_t i = 0; i < n; ++i) REAL(out)[i] = exp(REAL(xr)[i]);
  UNPROTECT(2);
  return out;
}

SEXP _sparseRGPs_pos_to_real(SEXP x) {
  SEXP xr = PROTECT(as_real(x));
  const R_xlen_t n = XLENGTH(xr);
  SEXP out = PROTECT(Rf_allocVector(REALSXP, n));
  for (R_xlen_t i = 0; i < n; ++i) REAL(out)[i] = log(REAL(xr)[i]);
  UNPROTECT(2);
  return out;
}

/* real_to_bounded: covariance_function_derivativesC.cpp:25-28, (ub e^x + lb) / (e^x + 1).
 * Rcpp sugar does not recycle: the expression's length is its leftmost operand's, ub, and
 * element i reads x[i] and lb[i] (past their end when they are shorter -- undefined there, an
 * R error here). */
static double bounded(double x, double ub, double lb) { return (ub * exp(x) + lb) / (exp(x) + 1.0); }

SEXP _sparseRGPs_real_to_bounded(SEXP x, SEXP ub, SEXP lb) {
  SEXP xr = PROTECT(as_real(x)), ur = PROTECT(as_real(ub)), lr = PROTECT(as_real(lb));
  const R_xlen_t n = XLENGTH(ur);
  if (XLENGTH(xr) < n || XLENGTH(lr) < n)
    Rf_error("x and lb need at least length(ub) = %ld values", (long)n);
  SEXP out = PROTECT(Rf_allocVector(REALSXP, n));
  for (R_xlen_t i = 0; i < n; ++i) REAL(out)[i] = bounded(REAL(xr)[i], REAL(ur)[i], REAL(lr)[i]);
  UNPROTECT(4);
  return out;
}

/* two equal-length coordinate vectors of one pair */
typedef struct {
  SEXP a, b;
  int d;
} Pair;

static Pair pair_of(SEXP x1, SEXP x2) {
  Pair p;
  p.a = PROTECT(as_real(x1));
  p.b = PROTECT(as_real(x2));
  p.d = Rf_length(p.a);
  if (Rf_length(p.b) != p.d) Rf_error("x1 and x2 differ in length (%d vs %d)", p.d, Rf_length(p.b));
  return p; /* caller UNPROTECTs 2 */
}

/* derivative list: derivative, trans_par, inv_trans_par */
static SEXP deriv_list(SEXP deriv, SEXP trans, SEXP inv) {
  static const char* nm[3] = {"derivative", "trans_par", "inv_trans_par"};
  SEXP v[3] = {deriv, trans, inv};
  return named_list(3, nm, v);
}

/* scalar per-pair derivative through sgp_dkernel_pair, wrapped like the Rcpp originals:
 * trans_par = log(par), inv_trans_par = real_to_pos(par) */
static SEXP pair_deriv(int kernel, SEXP x1, SEXP x2, SEXP cov_par, SEXP lnames, int param_kind,
                       int comp) {
  Pair p = pair_of(x1, x2);
  const int ard = kernel == SGP_KERNEL_ARD;
  const int L = ard ? p.d : 1;
  double theta[40];
  if (p.d < 1 || p.d > 32) Rf_error("input dimension %d outside [1, 32]", p.d);
  if (param_kind == 2) {
    /* d*_dtauC read only cov_par$tau (covariance_function_derivativesC.cpp:148) */
    for (int i = 0; i <= L; ++i) theta[i] = 1.0;
    theta[L + 1] = list_num(cov_par, "tau");
  } else {
    theta_from(cov_par, ard, lnames, p.d, 0, theta);
  }
  int param = param_kind == 0 ? 0 : param_kind == 2 ? L + 1 : 1 + comp;
  if (param_kind == 1 && (comp < 0 || comp >= L)) Rf_error("comp %d outside 1..%d", comp + 1, L);
  const double par = theta[param];
  const double dv = sgp_dkernel_pair(kernel, REAL(p.a), REAL(p.b), p.d, theta, param);
  if (ISNAN(dv) && !ISNAN(par)) check(SGP_EINVAL);
  SEXP out = PROTECT(deriv_list(PROTECT(Rf_ScalarReal(dv)), PROTECT(Rf_ScalarReal(log(par))),
                                PROTECT(Rf_ScalarReal(exp(par)))));
  UNPROTECT(6);
  return out;
}

/* covariance_function_derivativesC.cpp:35-55 */
SEXP _sparseRGPs_dsqexp_dsigmaC(SEXP x1, SEXP x2, SEXP cov_par) {
  return pair_deriv(SGP_KERNEL_SQEXP, x1, x2, cov_par, R_NilValue, 0, 0);
}
/* :58-85 */
SEXP _sparseRGPs_dsqexp_dsigma_ardC(SEXP x1, SEXP x2, SEXP cov_par, SEXP lnames) {
  return pair_deriv(SGP_KERNEL_ARD, x1, x2, cov_par, lnames, 0, 0);
}
/* :88-107 */
SEXP _sparseRGPs_dsqexp_dlC(SEXP x1, SEXP x2, SEXP cov_par) {
  return pair_deriv(SGP_KERNEL_SQEXP, x1, x2, cov_par, R_NilValue, 1, 0);
}
/* :110-140, comp is 1-based */
SEXP _sparseRGPs_dsqexp_dl_ardC(SEXP x1, SEXP x2, SEXP cov_par, SEXP lnames, SEXP comp) {
  return pair_deriv(SGP_KERNEL_ARD, x1, x2, cov_par, lnames, 1, (int)Rf_asReal(comp) - 1);
}
/* :143-172: 2 tau^2 iff all(x1 == x2) */
SEXP _sparseRGPs_dsqexp_dtauC(SEXP x1, SEXP x2, SEXP cov_par) {
  return pair_deriv(SGP_KERNEL_SQEXP, x1, x2, cov_par, R_NilValue, 2, 0);
}
/* :229-247 ("exp" derivatives use the L2 distance, quirk Q12) */
SEXP _sparseRGPs_dexp_dsigmaC(SEXP x1, SEXP x2, SEXP cov_par) {
  return pair_deriv(SGP_KERNEL_EXP, x1, x2, cov_par, R_NilValue, 0, 0);
}
/* :250-267 */
SEXP _sparseRGPs_dexp_dlC(SEXP x1, SEXP x2, SEXP cov_par) {
  return pair_deriv(SGP_KERNEL_EXP, x1, x2, cov_par, R_NilValue, 1, 0);
}
/* :270-298 */
SEXP _sparseRGPs_dexp_dtauC(SEXP x1, SEXP x2, SEXP cov_par) {
  return pair_deriv(SGP_KERNEL_EXP, x1, x2, cov_par, R_NilValue, 2, 0);
}

/* knot derivatives, covariance_function_derivativesC.cpp:175-226: per coordinate c
 *   (x1_c - x2_c) / l_c^2 * k(x1, x2) * dx2/dtx2_c,  tx2 = log((x2 - lb) / (ub - x2)),
 *   dx2/dtx2 = e^tx2 (ub - lb) / (e^tx2 + 1)^2;  trans_par = tx2,
 *   inv_trans_par = real_to_bounded(x2, ub, lb).  Every sugar expression there has x2's length
 *   d and reads lb[c], ub[c] for c < d (no recycling): lb and ub need at least d values. */
static SEXP knot_deriv(int kernel, SEXP x1, SEXP x2, SEXP cov_par, SEXP lb, SEXP ub, SEXP lnames) {
  Pair p = pair_of(x1, x2);
  SEXP lr = PROTECT(as_real(lb)), ur = PROTECT(as_real(ub));
  const int d = p.d, ard = kernel == SGP_KERNEL_ARD;
  if (d < 1 || d > 32) Rf_error("input dimension %d outside [1, 32]", d);
  if (Rf_length(lr) < d || Rf_length(ur) < d) Rf_error("lb and ub need at least %d values", d);
  double theta[40];
  theta_from(cov_par, ard, lnames, d, 0, theta);
  const double k = sgp_kernel_pair(kernel, REAL(p.a), REAL(p.b), d, theta);
  if (ISNAN(k)) check(SGP_EINVAL);
  SEXP dv = PROTECT(Rf_allocVector(REALSXP, d));
  SEXP tr = PROTECT(Rf_allocVector(REALSXP, d));
  SEXP iv = PROTECT(Rf_allocVector(REALSXP, d));
  for (int c = 0; c < d; ++c) {
    const double x2c = REAL(p.b)[c], lbc = REAL(lr)[c], ubc = REAL(ur)[c];
    const double l = ard ? theta[1 + c] : theta[1];
    const double t = log((x2c - lbc) / (ubc - x2c));
    const double et = exp(t);
    const double dxdt = (et * (ubc - lbc)) / ((et + 1.0) * (et + 1.0));
    REAL(dv)[c] = (1.0 / (l * l)) * (REAL(p.a)[c] - x2c) * k * dxdt;
    REAL(tr)[c] = t;
    REAL(iv)[c] = bounded(x2c, ubc, lbc);
  }
  SEXP out = PROTECT(deriv_list(dv, tr, iv));
  UNPROTECT(8);
  return out;
}

SEXP _sparseRGPs_dsqexp_dx2C(SEXP x1, SEXP x2, SEXP cov_par, SEXP lb, SEXP ub) {
  return knot_deriv(SGP_KERNEL_SQEXP, x1, x2, cov_par, lb, ub, R_NilValue);
}

SEXP _sparseRGPs_dsqexp_dx2_ardC(SEXP x1, SEXP x2, SEXP cov_par, SEXP lb, SEXP ub, SEXP lnames) {
  return knot_deriv(SGP_KERNEL_ARD, x1, x2, cov_par, lb, ub, lnames);
}

/* cov_fun_sqrd_expC / cov_fun_sqrd_exp_ardC / cov_fun_expC: covariance_functionsC.cpp:5-52 */
static SEXP pair_value(int kernel, SEXP x1, SEXP x2, SEXP cov_par, SEXP lnames) {
  Pair p = pair_of(x1, x2);
  if (p.d < 1 || p.d > 32) Rf_error("input dimension %d outside [1, 32]", p.d);
  double theta[40];
  theta_from(cov_par, kernel == SGP_KERNEL_ARD, lnames, p.d, 0, theta);
  const double v = sgp_kernel_pair(kernel, REAL(p.a), REAL(p.b), p.d, theta);
  if (ISNAN(v)) check(SGP_EINVAL);
  UNPROTECT(2);
  return Rf_ScalarReal(v);
}

SEXP _sparseRGPs_cov_fun_sqrd_expC(SEXP x1, SEXP x2, SEXP cov_par) {
  return pair_value(SGP_KERNEL_SQEXP, x1, x2, cov_par, R_NilValue);
}
SEXP _sparseRGPs_cov_fun_sqrd_exp_ardC(SEXP x1, SEXP x2, SEXP cov_par, SEXP lnames) {
  return pair_value(SGP_KERNEL_ARD, x1, x2, cov_par, lnames);
}
SEXP _sparseRGPs_cov_fun_expC(SEXP x1, SEXP x2, SEXP cov_par) {
  return pair_value(SGP_KERNEL_EXP, x1, x2, cov_par, R_NilValue);
}

/* One HIP fill (sgp_make_cov when param < 0, else sgp_dsig_dtheta) into a fresh R matrix. */
static SEXP fill(int kernel, SEXP x, SEXP x_pred, SEXP cov_par, SEXP lnames, double delta,
                 int param) {
  SEXP xr = PROTECT(as_real(x));
  SEXP pr = PROTECT(as_real(x_pred));
  const int sym = is_sym(pr);
  const int n = nrows_of(xr), d = ncols_of(xr);
  const int np = sym ? n : nrows_of(pr);
  if (!sym && ncols_of(pr) != d) Rf_error("x and x_pred differ in columns");
  const int L = kernel == SGP_KERNEL_ARD ? d : 1;
  double theta[40];
  if (d < 1 || d > 32) Rf_error("input dimension %d outside [1, 32]", d);
  theta_from(cov_par, kernel == SGP_KERNEL_ARD, lnames, d, sym || param == L + 1, theta);
  SEXP out = PROTECT(Rf_allocMatrix(REALSXP, n, np));
  int st;
  if (param < 0)
    st = sgp_make_cov(sgp_dev(), kernel, REAL(xr), n, n, sym ? NULL : REAL(pr), np, np, d, theta,
                      delta, REAL(out), n);
  else
    st = sgp_dsig_dtheta(sgp_dev(), kernel, REAL(xr), n, n, sym ? NULL : REAL(pr), np, np, d,
                         theta, param, REAL(out), n);
  check(st);
  UNPROTECT(3);
  return out;
}

/* make_cov_matC: covariance_functionsC.cpp:72-169 ("sqexp" / "exp") */
SEXP _sparseRGPs_make_cov_matC(SEXP x, SEXP x_pred, SEXP cov_par, SEXP cov_fun, SEXP delta) {
  const char* f = str0(cov_fun);
  const int kernel = !strcmp(f, "sqexp") ? SGP_KERNEL_SQEXP : !strcmp(f, "exp") ? SGP_KERNEL_EXP : -1;
  if (kernel < 0) {
    REprintf("Error: invalid covariance function");
    return empty_matrix();
  }
  return fill(kernel, x, x_pred, cov_par, R_NilValue, Rf_asReal(delta), -1);
}

/* make_cov_mat_ardC: covariance_functionsC.cpp:191-252 ("ard" only) */
SEXP _sparseRGPs_make_cov_mat_ardC(SEXP x, SEXP x_pred, SEXP cov_par, SEXP cov_fun, SEXP delta,
                                   SEXP lnames) {
  if (strcmp(str0(cov_fun), "ard")) {
    REprintf("Error: invalid covariance function");
    return empty_matrix();
  }
  return fill(SGP_KERNEL_ARD, x, x_pred, cov_par, lnames, Rf_asReal(delta), -1);
}

/* dsig_dthetaC: covariance_function_derivativesC.cpp:307-552.  The message / fall-through
 * rules of the original's branches:
 *   sqexp, symmetric, unknown name  -> falls out of the branch: "Error: invalid covariance
 *                                      function" (l.545-546), 0x0
 *   sqexp, cross, unknown name      -> "Error: invalid parameter name ..." (l.420), 0x0
 *   exp, cross, tau or unknown name -> `return mat;` of zeros before the tau branch (quirk Q13)
 *   exp, symmetric, unknown name    -> "Error" (l.550), 0x0 */
SEXP _sparseRGPs_dsig_dthetaC(SEXP x, SEXP x_pred, SEXP cov_par, SEXP cov_fun, SEXP par_name) {
  const char* f = str0(cov_fun);
  const char* pn = str0(par_name);
  const int idx = !strcmp(pn, "sigma") ? 0 : !strcmp(pn, "l") ? 1 : !strcmp(pn, "tau") ? 2 : -1;
  SEXP pr = PROTECT(as_real(x_pred));
  const int sym = is_sym(pr);
  SEXP out;
  if (!strcmp(f, "sqexp")) {
    if (idx < 0) {
      REprintf(sym ? "Error: invalid covariance function"
                   : "Error: invalid parameter name for chosen covariance function");
      out = empty_matrix();
    } else {
      out = fill(SGP_KERNEL_SQEXP, x, x_pred, cov_par, R_NilValue, 0.0, idx);
    }
  } else if (!strcmp(f, "exp")) {
    if (!sym && (idx < 0 || idx == 2)) {
      out = PROTECT(Rf_allocMatrix(REALSXP, nrows_of(x), nrows_of(pr)));
      memset(REAL(out), 0, sizeof(double) * (size_t)XLENGTH(out));
      UNPROTECT(1);
    } else if (idx < 0) {
      REprintf("Error");
      out = empty_matrix();
    } else {
      out = fill(SGP_KERNEL_EXP, x, x_pred, cov_par, R_NilValue, 0.0, idx);
    }
  } else {
    REprintf("Error: invalid covariance function");
    out = empty_matrix();
  }
  UNPROTECT(1);
  return out;
}

/* dsig_dtheta_ardC: covariance_function_derivativesC.cpp:555-722 (sigma, any of lnames, tau) */
SEXP _sparseRGPs_dsig_dtheta_ardC(SEXP x, SEXP x_pred, SEXP cov_par, SEXP cov_fun,
                                  SEXP par_name, SEXP lnames) {
  if (strcmp(str0(cov_fun), "ard")) {
    REprintf("Error: invalid covariance function");
    return empty_matrix();
  }
  const char* pn = str0(par_name);
  const int d = ncols_of(x);
  SEXP pr = PROTECT(as_real(x_pred));
  const int sym = is_sym(pr);
  UNPROTECT(1);
  int idx = -1;
  if (!strcmp(pn, "sigma")) idx = 0;
  for (int c = 0; idx < 0 && c < Rf_length(lnames) && c < d; ++c)
    if (!strcmp(pn, CHAR(STRING_ELT(lnames, c)))) idx = 1 + c;
  if (idx < 0 && !strcmp(pn, "tau")) idx = d + 1;
  if (idx < 0) {
    REprintf(sym ? "Error" : "Error: invalid parameter name for chosen covariance function");
    return empty_matrix();
  }
  return fill(SGP_KERNEL_ARD, x, x_pred, cov_par, lnames, 0.0, idx);
}

/* ------------------------------------------------- Part 2: fused hot path for the drivers */

static void ctx_finalize(SEXP p) {
  sgp_ctx* c = (sgp_ctx*)R_ExternalPtrAddr(p);
  if (c) {
    sgp_ctx_destroy(c);
    R_ClearExternalPtr(p);
  }
}

static sgp_ctx* ctx_of(SEXP p) {
  if (TYPEOF(p) != EXTPTRSXP) Rf_error("not an sgp context");
  sgp_ctx* c = (sgp_ctx*)R_ExternalPtrAddr(p);
  if (!c) Rf_error("sgp context already destroyed");
  return c;
}

static int kernel_of(SEXP cov_fun) {
  const char* f = str0(cov_fun);
  if (!strcmp(f, "sqexp")) return SGP_KERNEL_SQEXP;
  if (!strcmp(f, "ard")) return SGP_KERNEL_ARD;
  if (!strcmp(f, "exp")) return SGP_KERNEL_EXP;
  Rf_error("invalid covariance function '%s'", f);
  return -1;
}

/* sgp_R_ctx_create(xy, y, mu, m_max, devices): X, y, mu to HBM once per fit.
 * devices = NULL or length 0: one device (SGP_DEVICE, default 0; sgp_ctx_create);
 * otherwise the device index of each row shard (sgp_ctx_create_multi: the rows split into
 * length(devices) contiguous blocks, the reductions of every evaluation summed inside libsgp
 * over the devices by an RCCL all-reduce -- north star C4).  rshim/R/sgp_hotpath.R picks them
 * (from the R options ngpus / devices). */
SEXP sgp_R_ctx_create(SEXP xy, SEXP y, SEXP mu, SEXP m_max, SEXP devices) {
  SEXP xr = PROTECT(as_real(xy)), yr = PROTECT(as_real(y)), mr = PROTECT(as_real(mu));
  SEXP dr = PROTECT(Rf_isNull(devices) ? R_NilValue : as_real(devices));
  const int n = nrows_of(xr), d = ncols_of(xr);
  if (Rf_length(yr) != n || Rf_length(mr) != n) Rf_error("y and mu must have nrow(xy) values");
  const int nsh = Rf_isNull(dr) ? 0 : Rf_length(dr);
  if (nsh > 64) Rf_error("at most 64 row shards (got %d devices)", nsh);
  sgp_ctx* c = NULL;
  if (nsh == 0) {
    check(sgp_ctx_create(&c, sgp_dev(), REAL(xr), n, n, d, REAL(yr), REAL(mr),
                         (int64_t)Rf_asInteger(m_max)));
  } else {
    int dv[64];
    for (int k = 0; k < nsh; ++k) {
      const double v = REAL(dr)[k];
      if (!(v >= 0.0) || v != floor(v)) Rf_error("devices must be non-negative integers");
      dv[k] = (int)v;
    }
    check(sgp_ctx_create_multi(&c, dv, nsh, REAL(xr), n, n, d, REAL(yr), REAL(mr),
                               (int64_t)Rf_asInteger(m_max)));
  }
  SEXP p = PROTECT(R_MakeExternalPtr(c, R_NilValue, R_NilValue));
  R_RegisterCFinalizerEx(p, ctx_finalize, TRUE);
  UNPROTECT(5);
  return p;
}

/* visible HIP devices (0 without any) */
SEXP sgp_R_device_count(void) {
  int cnt = 0;
  if (sgp_device_count(&cnt) != SGP_OK) cnt = 0;
  return Rf_ScalarInteger(cnt);
}

/* c(row shards, distinct devices) of a context */
SEXP sgp_R_ctx_shards(SEXP ctx) {
  int ns = 0, nd = 0;
  check(sgp_ctx_shards(ctx_of(ctx), &ns, &nd));
  SEXP out = PROTECT(Rf_allocVector(REALSXP, 2));
  REAL(out)[0] = ns;
  REAL(out)[1] = nd;
  UNPROTECT(1);
  return out;
}

SEXP sgp_R_ctx_destroy(SEXP ctx) {
  ctx_finalize(ctx);
  return R_NilValue;
}

/* new y / mu on the same rows (sgp_ctx_set_data) */
SEXP sgp_R_set_data(SEXP ctx, SEXP y, SEXP mu) {
  sgp_ctx* c = ctx_of(ctx);
  SEXP yr = PROTECT(as_real(y)), mr = PROTECT(as_real(mu));
  if (Rf_length(yr) != sgp_ctx_rows(c) || Rf_length(mr) != sgp_ctx_rows(c))
    Rf_error("y and mu must have one value per context row");
  check(sgp_ctx_set_data(c, REAL(yr), REAL(mr)));
  UNPROTECT(2);
  return R_NilValue;
}

static SEXP obj_grad(double obj, SEXP grad) {
  static const char* nm[2] = {"objective", "gradient"};
  SEXP v[2] = {PROTECT(Rf_ScalarReal(obj)), grad};
  SEXP out = named_list(2, nm, v);
  UNPROTECT(1);
  return out;
}

/* sgp_R_eval(ctx, method, cov_fun, theta, xu, delta, flags): one fused evaluation.
 * method 0 = VI (elbo_fun + delbo_dcov_par), 1 = FITC (obj_fun_norm + dlogp_dcov_par).
 * flags: SGP_FLAG_R_DET (R's det() overflow, quirk Q4), SGP_FLAG_OBJ_ONLY.
 * -> list(objective, gradient [theta layout, d/dlog theta]) */
SEXP sgp_R_eval(SEXP ctx, SEXP method, SEXP cov_fun, SEXP theta, SEXP xu, SEXP delta, SEXP flags) {
  sgp_ctx* c = ctx_of(ctx);
  SEXP th = PROTECT(as_real(theta)), ur = PROTECT(as_real(xu));
  const unsigned fl = (unsigned)Rf_asInteger(flags);
  const int m = nrows_of(ur);
  SEXP grad = PROTECT(Rf_allocVector(REALSXP, Rf_length(th)));
  double obj = 0.0;
  const int kernel = kernel_of(cov_fun);
  if (Rf_length(th) != sgp_num_params(kernel, ncols_of(ur))) Rf_error("theta has the wrong length");
  const int st = Rf_asInteger(method) == 1
                     ? sgp_eval_fitc(c, kernel, REAL(th), REAL(ur), m, m, Rf_asReal(delta), fl,
                                     &obj, (fl & SGP_FLAG_OBJ_ONLY) ? NULL : REAL(grad))
                     : sgp_eval_vi(c, kernel, REAL(th), REAL(ur), m, m, Rf_asReal(delta), fl,
                                   &obj, (fl & SGP_FLAG_OBJ_ONLY) ? NULL : REAL(grad));
  check(st); /* SGP_ENOTPD carries R's chol() message: try() in knot proposals still works */
  SEXP out = obj_grad(obj, grad);
  UNPROTECT(3);
  return out;
}

/* the Poisson exposure argument `m` (R/derivative_functions_of_data_likelihoods.R:7-61, "a vector
 * of the areas of each grid cell", l.38): one value -> that exposure on every row; one value per
 * context row -> made resident (sgp_lap_set_expo) and passed as SGP_EXPO_ROWS */
static double expo_arg(sgp_ctx* c, SEXP expo) {
  SEXP er = PROTECT(as_real(expo));
  double v = 0.0;
  if (Rf_length(er) == 1) {
    v = REAL(er)[0];
  } else if (Rf_length(er) == sgp_ctx_rows(c)) {
    check(sgp_lap_set_expo(c, REAL(er), 0.0));
    v = SGP_EXPO_ROWS;
  } else {
    Rf_error("the exposure m must have length 1 or one value per row");
  }
  UNPROTECT(1);
  return v;
}

/* sgp_R_eval_laplace(ctx, cov_fun, theta, xu, delta, expo, tol, maxit, grad):
 * newtrap_sparseGP from the resident f + (grad != 0) dlogq_dcov_par at the mode.
 * maxit = 0: objective and gradient at the resident f (no NR step).  expo: length 1 or n.
 * -> list(objective, gradient, nr_iter) */
SEXP sgp_R_eval_laplace(SEXP ctx, SEXP cov_fun, SEXP theta, SEXP xu, SEXP delta, SEXP expo,
                        SEXP tol, SEXP maxit, SEXP want_grad) {
  sgp_ctx* c = ctx_of(ctx);
  SEXP th = PROTECT(as_real(theta)), ur = PROTECT(as_real(xu));
  const int m = nrows_of(ur), kernel = kernel_of(cov_fun);
  SEXP grad = PROTECT(Rf_allocVector(REALSXP, Rf_length(th)));
  double obj = 0.0;
  int it = 0;
  const double ex = expo_arg(c, expo);
  if (Rf_asLogical(want_grad))
    check(sgp_eval_laplace(c, kernel, REAL(th), REAL(ur), m, m, Rf_asReal(delta), ex,
                           Rf_asReal(tol), Rf_asInteger(maxit), &obj, REAL(grad), &it));
  else
    check(sgp_lap_nr(c, kernel, REAL(th), REAL(ur), m, m, Rf_asReal(delta), ex,
                     Rf_asReal(tol), Rf_asInteger(maxit), &obj, &it));
  static const char* nm[3] = {"objective", "gradient", "nr_iter"};
  SEXP v[3] = {PROTECT(Rf_ScalarReal(obj)), grad, PROTECT(Rf_ScalarInteger(it))};
  SEXP out = named_list(3, nm, v);
  UNPROTECT(5);
  return out;
}

/* the resident latent vector f (sgp_lap_set_f / sgp_lap_get_f) */
SEXP sgp_R_lap_set_f(SEXP ctx, SEXP f) {
  sgp_ctx* c = ctx_of(ctx);
  SEXP fr = PROTECT(as_real(f));
  if (Rf_length(fr) == 1)
    check(sgp_lap_set_f(c, NULL, REAL(fr)[0]));
  else if (Rf_length(fr) == sgp_ctx_rows(c))
    check(sgp_lap_set_f(c, REAL(fr), 0.0));
  else
    Rf_error("f must have length 1 or one value per context row");
  UNPROTECT(1);
  return R_NilValue;
}

SEXP sgp_R_lap_get_f(SEXP ctx) {
  sgp_ctx* c = ctx_of(ctx);
  SEXP f = PROTECT(Rf_allocVector(REALSXP, (R_xlen_t)sgp_ctx_rows(c)));
  check(sgp_lap_get_f(c, REAL(f)));
  UNPROTECT(1);
  return f;
}

/* grad psi of the last NR step: newtrap_sparseGP's `gradient` (newtrap_sparseGP.R:183-184) */
SEXP sgp_R_lap_get_grad_psi(SEXP ctx) {
  sgp_ctx* c = ctx_of(ctx);
  SEXP g = PROTECT(Rf_allocVector(REALSXP, (R_xlen_t)sgp_ctx_rows(c)));
  check(sgp_lap_get_grad_psi(c, REAL(g)));
  UNPROTECT(1);
  return g;
}

/* objective_function_values of the last NR run */
SEXP sgp_R_lap_objective_values(SEXP ctx) {
  sgp_ctx* c = ctx_of(ctx);
  int cnt = 0;
  check(sgp_lap_objective_values(c, NULL, 0, &cnt));
  SEXP out = PROTECT(Rf_allocVector(REALSXP, cnt));
  check(sgp_lap_objective_values(c, REAL(out), cnt, &cnt));
  UNPROTECT(1);
  return out;
}

SEXP sgp_R_enable_knot_grad(SEXP ctx, SEXP enable) {
  check(sgp_ctx_enable_knot_grad(ctx_of(ctx), Rf_asLogical(enable)));
  return R_NilValue;
}

/* knot gradient of the last evaluation, row-major (quirk Q16); bounds = d x 2 [lower, upper]
 * (the reference's knot_bounds, vi_functions.R:175-178) or NULL for this context's rows */
SEXP sgp_R_knot_gradient(SEXP ctx, SEXP bounds, SEXP m, SEXP d) {
  sgp_ctx* c = ctx_of(ctx);
  const R_xlen_t len = (R_xlen_t)Rf_asInteger(m) * Rf_asInteger(d);
  SEXP br = PROTECT(Rf_isNull(bounds) ? R_NilValue : as_real(bounds));
  if (!Rf_isNull(br) && Rf_length(br) != 2 * Rf_asInteger(d)) Rf_error("bounds must be d x 2");
  SEXP g = PROTECT(Rf_allocVector(REALSXP, len));
  check(sgp_knot_gradient(c, Rf_isNull(br) ? NULL : REAL(br), REAL(g)));
  UNPROTECT(2);
  return g;
}

/* knot posterior of the last evaluation (sgp_posterior_u) -> list(u_mean, u_var) */
SEXP sgp_R_posterior_u(SEXP ctx, SEXP muu) {
  sgp_ctx* c = ctx_of(ctx);
  SEXP mr = PROTECT(as_real(muu));
  const int m = Rf_length(mr);
  SEXP um = PROTECT(Rf_allocVector(REALSXP, m));
  SEXP uv = PROTECT(Rf_allocMatrix(REALSXP, m, m));
  check(sgp_posterior_u(c, REAL(mr), REAL(um), REAL(uv)));
  static const char* nm[2] = {"u_mean", "u_var"};
  SEXP v[2] = {um, uv};
  SEXP out = named_list(2, nm, v);
  UNPROTECT(3);
  return out;
}

/* sgp_R_predict(method, gaussian, cov_fun, theta, delta, xu, u_mean, muu, u_var, x_pred,
 *               mu_pred, full_cov) -> list(pred_mean, pred_var) (predict_gp's two outputs) */
SEXP sgp_R_predict(SEXP method, SEXP gaussian, SEXP cov_fun, SEXP theta, SEXP delta, SEXP xu,
                   SEXP u_mean, SEXP muu, SEXP u_var, SEXP x_pred, SEXP mu_pred, SEXP full_cov) {
  SEXP th = PROTECT(as_real(theta)), ur = PROTECT(as_real(xu)), um = PROTECT(as_real(u_mean));
  SEXP mr = PROTECT(as_real(muu)), xp = PROTECT(as_real(x_pred)), mp = PROTECT(as_real(mu_pred));
  SEXP uv = PROTECT(Rf_isNull(u_var) ? R_NilValue : as_real(u_var));
  const int m = nrows_of(ur), d = ncols_of(ur), np = nrows_of(xp), fc = Rf_asLogical(full_cov);
  if (ncols_of(xp) != d) Rf_error("x_pred and xu differ in columns");
  if (Rf_length(um) != m || Rf_length(mr) != m || Rf_length(mp) != np)
    Rf_error("u_mean/muu need one value per knot and mu_pred one per prediction row");
  SEXP pm = PROTECT(Rf_allocVector(REALSXP, np));
  SEXP pv = PROTECT(fc ? Rf_allocMatrix(REALSXP, np, np) : Rf_allocVector(REALSXP, np));
  check(sgp_predict(sgp_dev(), kernel_of(cov_fun), REAL(th), Rf_asReal(delta),
                    Rf_asInteger(method), Rf_asLogical(gaussian), REAL(ur), m, m, REAL(um),
                    REAL(mr), Rf_isNull(uv) ? NULL : REAL(uv), m, REAL(xp), np, np, d, REAL(mp),
                    fc, REAL(pm), REAL(pv), fc ? np : 1));
  static const char* nm[2] = {"pred_mean", "pred_var"};
  SEXP v[2] = {pm, pv};
  SEXP out = named_list(2, nm, v);
  UNPROTECT(9);
  return out;
}

/* OAT candidate scoring: objective at knots [xu; cand_t] per candidate row (NaN = try-error).
 * method 0 = VI ELBO, 1 = FITC obj_fun_norm, 2 = Poisson Laplace (newtrap from the resident f) */
SEXP sgp_R_candidates(SEXP ctx, SEXP method, SEXP cov_fun, SEXP theta, SEXP xu, SEXP delta,
                      SEXP cand, SEXP expo, SEXP tol, SEXP maxit) {
  sgp_ctx* c = ctx_of(ctx);
  SEXP th = PROTECT(as_real(theta)), ur = PROTECT(as_real(xu)), cr = PROTECT(as_real(cand));
  const int m = nrows_of(ur), T = nrows_of(cr), kernel = kernel_of(cov_fun);
  if (ncols_of(cr) != ncols_of(ur)) Rf_error("cand and xu differ in columns");
  SEXP out = PROTECT(Rf_allocVector(REALSXP, T));
  const int meth = Rf_asInteger(method);
  int st;
  if (meth == 0)
    st = sgp_vi_candidates(c, kernel, REAL(th), REAL(ur), m, m, Rf_asReal(delta), 0u, REAL(cr),
                           T, T, REAL(out));
  else if (meth == 1)
    st = sgp_fitc_candidates(c, kernel, REAL(th), REAL(ur), m, m, Rf_asReal(delta), 0u,
                             REAL(cr), T, T, REAL(out));
  else
    st = sgp_lap_candidates(c, kernel, REAL(th), REAL(ur), m, m, Rf_asReal(delta),
                            expo_arg(c, expo), Rf_asReal(tol), Rf_asInteger(maxit), REAL(cr), T,
                            T, REAL(out));
  check(st);
  UNPROTECT(4);
  return out;
}

/* full Gaussian GP (config 1): list(objective, gradient) of obj_fun_norm_full +
 * dlogp_dcov_par_full over the context's rows (m_max >= n) */
SEXP sgp_R_eval_full(SEXP ctx, SEXP cov_fun, SEXP theta, SEXP delta, SEXP flags) {
  sgp_ctx* c = ctx_of(ctx);
  SEXP th = PROTECT(as_real(theta));
  const unsigned fl = (unsigned)Rf_asInteger(flags);
  SEXP grad = PROTECT(Rf_allocVector(REALSXP, Rf_length(th)));
  double obj = 0.0;
  check(sgp_eval_full(c, kernel_of(cov_fun), REAL(th), Rf_asReal(delta), fl, &obj,
                      (fl & SGP_FLAG_OBJ_ONLY) ? NULL : REAL(grad)));
  SEXP out = obj_grad(obj, grad);
  UNPROTECT(2);
  return out;
}

/* ------------------------------------------------- registration */

static const R_CallMethodDef CallEntries[] = {
    /* src/RcppExports.cpp:284-306, same names and arities */
    {"_sparseRGPs_real_to_pos", (DL_FUNC)&_sparseRGPs_real_to_pos, 1},
    {"_sparseRGPs_pos_to_real", (DL_FUNC)&_sparseRGPs_pos_to_real, 1},
    {"_sparseRGPs_real_to_bounded", (DL_FUNC)&_sparseRGPs_real_to_bounded, 3},
    {"_sparseRGPs_dsqexp_dsigmaC", (DL_FUNC)&_sparseRGPs_dsqexp_dsigmaC, 3},
    {"_sparseRGPs_dsqexp_dsigma_ardC", (DL_FUNC)&_sparseRGPs_dsqexp_dsigma_ardC, 4},
    {"_sparseRGPs_dsqexp_dlC", (DL_FUNC)&_sparseRGPs_dsqexp_dlC, 3},
    {"_sparseRGPs_dsqexp_dl_ardC", (DL_FUNC)&_sparseRGPs_dsqexp_dl_ardC, 5},
    {"_sparseRGPs_dsqexp_dtauC", (DL_FUNC)&_sparseRGPs_dsqexp_dtauC, 3},
    {"_sparseRGPs_dsqexp_dx2C", (DL_FUNC)&_sparseRGPs_dsqexp_dx2C, 5},
    {"_sparseRGPs_dsqexp_dx2_ardC", (DL_FUNC)&_sparseRGPs_dsqexp_dx2_ardC, 6},
    {"_sparseRGPs_dexp_dsigmaC", (DL_FUNC)&_sparseRGPs_dexp_dsigmaC, 3},
    {"_sparseRGPs_dexp_dlC", (DL_FUNC)&_sparseRGPs_dexp_dlC, 3},
    {"_sparseRGPs_dexp_dtauC", (DL_FUNC)&_sparseRGPs_dexp_dtauC, 3},
    {"_sparseRGPs_dsig_dthetaC", (DL_FUNC)&_sparseRGPs_dsig_dthetaC, 5},
    {"_sparseRGPs_dsig_dtheta_ardC", (DL_FUNC)&_sparseRGPs_dsig_dtheta_ardC, 6},
    {"_sparseRGPs_cov_fun_sqrd_expC", (DL_FUNC)&_sparseRGPs_cov_fun_sqrd_expC, 3},
    {"_sparseRGPs_cov_fun_sqrd_exp_ardC", (DL_FUNC)&_sparseRGPs_cov_fun_sqrd_exp_ardC, 4},
    {"_sparseRGPs_cov_fun_expC", (DL_FUNC)&_sparseRGPs_cov_fun_expC, 3},
    {"_sparseRGPs_make_cov_matC", (DL_FUNC)&_sparseRGPs_make_cov_matC, 5},
    {"_sparseRGPs_make_cov_mat_ardC", (DL_FUNC)&_sparseRGPs_make_cov_mat_ardC, 6},
    /* the fused hot path (rshim/R/sgp_hotpath.R) */
    {"sgp_R_ctx_create", (DL_FUNC)&sgp_R_ctx_create, 5},
    {"sgp_R_device_count", (DL_FUNC)&sgp_R_device_count, 0},
    {"sgp_R_ctx_shards", (DL_FUNC)&sgp_R_ctx_shards, 1},
    {"sgp_R_ctx_destroy", (DL_FUNC)&sgp_R_ctx_destroy, 1},
    {"sgp_R_set_data", (DL_FUNC)&sgp_R_set_data, 3},
    {"sgp_R_eval", (DL_FUNC)&sgp_R_eval, 7},
    {"sgp_R_eval_laplace", (DL_FUNC)&sgp_R_eval_laplace, 9},
    {"sgp_R_lap_set_f", (DL_FUNC)&sgp_R_lap_set_f, 2},
    {"sgp_R_lap_get_f", (DL_FUNC)&sgp_R_lap_get_f, 1},
    {"sgp_R_lap_objective_values", (DL_FUNC)&sgp_R_lap_objective_values, 1},
    {"sgp_R_lap_get_grad_psi", (DL_FUNC)&sgp_R_lap_get_grad_psi, 1},
    {"sgp_R_enable_knot_grad", (DL_FUNC)&sgp_R_enable_knot_grad, 2},
    {"sgp_R_knot_gradient", (DL_FUNC)&sgp_R_knot_gradient, 4},
    {"sgp_R_posterior_u", (DL_FUNC)&sgp_R_posterior_u, 2},
    {"sgp_R_predict", (DL_FUNC)&sgp_R_predict, 12},
    {"sgp_R_candidates", (DL_FUNC)&sgp_R_candidates, 10},
    {"sgp_R_eval_full", (DL_FUNC)&sgp_R_eval_full, 5},
    {NULL, NULL, 0}};

/* RcppExports.cpp:309-312 */
void R_init_sparseRGPs(DllInfo* dll) {
  R_registerRoutines(dll, NULL, CallEntries, NULL, NULL);
  R_useDynamicSymbols(dll, FALSE);
}
