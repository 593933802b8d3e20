/* Host-side sanitizer driver for libsgp's C ABI ("race detection /
 * sanitizers"): built with AddressSanitizer + UndefinedBehaviorSanitizer on the HOST code of
 * every csrc/*.hip translation unit (device code is compiled as usual and never runs here),
 * it drives the entry points that need no GPU:
 *   - the per-pair kernels sgp_kernel_pair / sgp_dkernel_pair (the R shim's cov_fun_*C and
 *     dsqexp_*C exports) over every kernel, parameter index and d in 1..SGP_MAXD, including
 *     invalid kernels / parameter indices (NaN + sgp_last_error);
 *   - the reduction-size queries (sgp_vi_red1_count, ...), sgp_num_params, sgp_abi_version;
 *   - the argument checks of every context entry point with a NULL context and of the
 *     fillers / sgp_predict / sgp_ctx_create with invalid shapes (all must return
 *     SGP_EINVAL before touching the device, with a readable sgp_last_error()).
 * Values are checked against a plain C restatement of covariance_functionsC.cpp's per-pair
 * forms.  Exit status 0 = all checks passed and no sanitizer report (reports abort). */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sgp.h"

static int failures = 0;
#define CHECK(cond, ...)                                  \
  do {                                                    \
    if (!(cond)) {                                        \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                       \
      fprintf(stderr, "\n");                              \
      ++failures;                                         \
    }                                                     \
  } while (0)

static double urand(unsigned* s) {
  *s = *s * 1664525u + 1013904223u;
  return (double)(*s >> 8) / 16777216.0;
}

/* covariance_functionsC.cpp:5-52 restated: theta = [sigma, l.., tau] */
static double ref_pair(int kernel, const double* a, const double* b, int d, const double* th) {
  const double s2 = th[0] * th[0];
  double s = 0.0;
  if (kernel == SGP_KERNEL_SQEXP) {
    for (int c = 0; c < d; ++c) s += (a[c] - b[c]) * (a[c] - b[c]);
    return s2 * exp(-s / (2.0 * th[1] * th[1]));
  }
  if (kernel == SGP_KERNEL_ARD) {
    for (int c = 0; c < d; ++c) s += (a[c] - b[c]) * (a[c] - b[c]) / (th[1 + c] * th[1 + c]);
    return s2 * exp(-s / 2.0);
  }
  for (int c = 0; c < d; ++c) s += fabs(a[c] - b[c]);
  return s2 * exp(-s / th[1]);
}

static void pair_checks(void) {
  unsigned seed = 12345u;
  double x1[64], x2[64], th[64];
  for (int kernel = 0; kernel <= 2; ++kernel) {
    for (int d = 1; d <= 32; ++d) {
      const int P = sgp_num_params(kernel, d);
      CHECK(P == (kernel == SGP_KERNEL_ARD ? d + 2 : 3), "num_params(%d, %d) = %d", kernel, d, P);
      for (int rep = 0; rep < 4; ++rep) {
        for (int c = 0; c < d; ++c) {
          x1[c] = urand(&seed) * 2.0 - 1.0;
          x2[c] = (rep == 3) ? x1[c] : urand(&seed) * 2.0 - 1.0;   /* rep 3: coincident */
        }
        for (int p = 0; p < P; ++p) th[p] = 0.5 + urand(&seed);
        const double v = sgp_kernel_pair(kernel, x1, x2, d, th);
        const double r = ref_pair(kernel, x1, x2, d, th);
        CHECK(fabs(v - r) <= 1e-13 * fabs(r) + 1e-300, "kernel_pair k=%d d=%d: %g vs %g", kernel,
              d, v, r);
        for (int p = 0; p < P; ++p) {
          const double g = sgp_dkernel_pair(kernel, x1, x2, d, th, p);
          CHECK(isfinite(g), "dkernel_pair k=%d d=%d p=%d not finite", kernel, d, p);
          if (p == P - 1)   /* tau: 2 tau^2 iff the points coincide (quirk Q5) */
            CHECK(g == (rep == 3 ? 2.0 * th[P - 1] * th[P - 1] : 0.0), "tau derivative %g", g);
        }
        CHECK(isnan(sgp_dkernel_pair(kernel, x1, x2, d, th, P)), "param P accepted");
        CHECK(isnan(sgp_dkernel_pair(kernel, x1, x2, d, th, -1)), "param -1 accepted");
      }
    }
    CHECK(sgp_num_params(kernel, 0) < 0, "d = 0 accepted");
  }
  CHECK(isnan(sgp_kernel_pair(3, x1, x2, 2, th)), "kernel 3 accepted");
  CHECK(strlen(sgp_last_error()) > 0, "no error message after an invalid kernel");
  CHECK(sgp_num_params(-1, 2) < 0, "kernel -1 accepted");
}

static void count_checks(void) {
  for (int64_t m = 1; m <= 3000; m += 37) {
    CHECK(sgp_vi_red1_count(m) > m, "vi red1(%lld)", (long long)m);
    CHECK(sgp_fitc_red1_count(m) > m, "fitc red1(%lld)", (long long)m);
    for (int d = 1; d <= 32; d += 7) {
      for (int k = 0; k <= 2; ++k) {
        CHECK(sgp_vi_red2_count(k, d) > 0, "vi red2");
        CHECK(sgp_fitc_red2_count(k, d, m) > 0, "fitc red2");
        CHECK(sgp_lap_red_count(k, d, m) > m, "lap red");
      }
      CHECK(sgp_knot_red_extra(d, m) >= m * d, "knot red extra");
    }
  }
  CHECK(sgp_abi_version() > 0, "abi version");
}

static void einval_checks(void) {
  double th[8] = {1.0, 0.5, 0.1, 0, 0, 0, 0, 0}, buf[64] = {0}, o = 0.0;
  double x[8] = {0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8};
  int64_t cnt = 0;
  int it = 0, done = 0, ci = 0;
  char names[64];
#define EINVAL_(call) CHECK((call) == SGP_EINVAL, "%s did not return SGP_EINVAL", #call)
  EINVAL_(sgp_device_count(NULL));
  CHECK(sgp_ctx_destroy(NULL) == SGP_OK, "sgp_ctx_destroy(NULL) is a no-op like free(NULL)");
  EINVAL_(sgp_ctx_set_stream(NULL, NULL));
  EINVAL_(sgp_ctx_set_data(NULL, buf, buf));
  EINVAL_(sgp_eval_vi(NULL, 1, th, buf, 1, 1, 1e-6, 0u, &o, buf));
  EINVAL_(sgp_eval_fitc(NULL, 1, th, buf, 1, 1, 1e-6, 0u, &o, buf));
  EINVAL_(sgp_vi_phase1(NULL, 1, th, buf, 1, 1, 1e-6, buf));
  EINVAL_(sgp_vi_phase2(NULL, buf, 1, 0u, buf));
  EINVAL_(sgp_vi_finish(NULL, buf, &o, buf));
  EINVAL_(sgp_fitc_phase1(NULL, 1, th, buf, 1, 1, 1e-6, buf));
  EINVAL_(sgp_fitc_phase2(NULL, buf, 1, 0u, buf));
  EINVAL_(sgp_fitc_finish(NULL, buf, &o, buf));
  EINVAL_(sgp_lap_set_f(NULL, buf, 0.0));
  EINVAL_(sgp_lap_set_expo(NULL, buf, 1.0));
  EINVAL_(sgp_lap_get_f(NULL, buf));
  EINVAL_(sgp_lap_objective_values(NULL, buf, 4, &ci));
  EINVAL_(sgp_eval_laplace(NULL, 1, th, buf, 1, 1, 1e-6, 1.0, 1e-5, 10, &o, buf, &it));
  EINVAL_(sgp_lap_begin(NULL, 1, th, buf, 1, 1, 1e-6, 1.0, 1e-5, 10, 0u, buf, &cnt));
  EINVAL_(sgp_lap_step(NULL, buf, buf, &cnt, &done, &o, buf, &it));
  EINVAL_(sgp_lap_nr(NULL, 1, th, buf, 1, 1, 1e-6, 1.0, 1e-5, 10, &o, &it));
  EINVAL_(sgp_eval_full(NULL, 1, th, 1e-6, 0u, &o, buf));
  EINVAL_(sgp_posterior_u(NULL, buf, buf, buf));
  EINVAL_(sgp_ctx_enable_knot_grad(NULL, 1));
  EINVAL_(sgp_knot_gradient(NULL, NULL, buf));
  EINVAL_(sgp_ctx_row_bounds(NULL, buf, buf));
  EINVAL_(sgp_vi_candidates(NULL, 1, th, buf, 1, 1, 1e-6, 0u, x, 1, 1, buf));
  EINVAL_(sgp_fitc_candidates(NULL, 1, th, buf, 1, 1, 1e-6, 0u, x, 1, 1, buf));
  EINVAL_(sgp_lap_candidates(NULL, 1, th, buf, 1, 1, 1e-6, 1.0, 1e-5, 10, x, 1, 1, buf));
  EINVAL_(sgp_ctx_enable_timing(NULL, 1));
  EINVAL_(sgp_ctx_timing_filter(NULL, "contract_knm"));
  EINVAL_(sgp_ctx_timings(NULL, names, sizeof names, buf, 4, &ci));
  CHECK(sgp_ctx_rows(NULL) < 0, "sgp_ctx_rows(NULL)");
  CHECK(sgp_ctx_timing_evals(NULL) < 0 || sgp_ctx_timing_evals(NULL) == 0, "timing_evals(NULL)");
  /* invalid shapes: rejected before any device call */
  sgp_ctx* ctx = NULL;
  EINVAL_(sgp_ctx_create(&ctx, 0, x, 0, 1, 1, x, x, 4));
  EINVAL_(sgp_ctx_create(&ctx, 0, x, 4, 2, 1, x, x, 4));
  EINVAL_(sgp_ctx_create(&ctx, 0, x, 4, 4, 33, x, x, 4));
  EINVAL_(sgp_ctx_create(&ctx, 0, x, 4, 4, 1, NULL, x, 4));
  EINVAL_(sgp_ctx_create(NULL, 0, x, 4, 4, 1, x, x, 4));
  {
    const int dv[3] = {0, -1, 0};
    EINVAL_(sgp_ctx_create_multi(&ctx, NULL, 0, x, 4, 4, 1, x, x, 4));
    EINVAL_(sgp_ctx_create_multi(&ctx, NULL, 5, x, 4, 4, 1, x, x, 4));
    EINVAL_(sgp_ctx_create_multi(&ctx, dv, 3, x, 4, 4, 1, x, x, 4));
    EINVAL_(sgp_ctx_create_multi(&ctx, NULL, 2, x, 4, 4, 33, x, x, 4));
    EINVAL_(sgp_ctx_create_multi(NULL, NULL, 2, x, 4, 4, 1, x, x, 4));
    EINVAL_(sgp_ctx_shards(NULL, NULL, NULL));
  }
  CHECK(ctx == NULL, "ctx written on failure");
  EINVAL_(sgp_make_cov(0, 1, x, 4, 2, NULL, 0, 0, 2, th, 1e-6, buf, 4));
  EINVAL_(sgp_make_cov(0, 1, x, -1, 1, NULL, 0, 0, 2, th, 1e-6, buf, 4));
  EINVAL_(sgp_make_cov(0, 1, x, 4, 4, NULL, 0, 0, 2, th, 1e-6, NULL, 4));
  EINVAL_(sgp_make_cov(0, 7, x, 4, 4, NULL, 0, 0, 2, th, 1e-6, buf, 4));
  EINVAL_(sgp_dsig_dtheta(0, 1, x, 4, 4, NULL, 0, 0, 2, th, 9, buf, 4));
  EINVAL_(sgp_dsig_dtheta(0, 0, x, 4, 4, x, 2, 1, 2, th, 0, buf, 4));
  EINVAL_(sgp_predict(0, 0, th, 1e-6, 0, 1, NULL, 1, 1, buf, buf, buf, 1, x, 1, 1, 1, buf, 0,
                      buf, buf, 1));
  EINVAL_(sgp_predict(0, 0, th, 1e-6, 0, 1, x, 2, 1, buf, buf, buf, 2, x, 1, 1, 1, buf, 0, buf,
                      buf, 1));
  EINVAL_(sgp_predict(0, 0, th, 1e-6, 9, 1, x, 1, 1, buf, buf, buf, 1, x, 1, 1, 1, buf, 0, buf,
                      buf, 1));
#undef EINVAL_
  CHECK(strlen(sgp_last_error()) > 0, "no error message after EINVAL");
}

int main(void) {
  pair_checks();
  count_checks();
  einval_checks();
  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("host ABI sanitizer driver: all checks passed\n");
  return 0;
}
