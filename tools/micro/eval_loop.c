/* Evaluation rate of sgp_eval_vi from a plain C loop (no Python between evaluations): the
 * library's own host path, for comparison with bench.py's (tools/c2_loop.py).
 * build: gcc -O2 -I include -o tools/micro/eval_loop tools/micro/eval_loop.c \
 *        -L sparsergps_amd/lib -lsgp -Wl,-rpath,$PWD/sparsergps_amd/lib -lm
 * usage: eval_loop N M D KERNEL(0 sqexp, 1 ard) EVALS  (C2 / C3 generator shapes, uniform data) */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "sgp.h"

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 100000, m = argc > 2 ? atol(argv[2]) : 256;
  const int d = argc > 3 ? atoi(argv[3]) : 3, kernel = argc > 4 ? atoi(argv[4]) : 0;
  const int evals = argc > 5 ? atoi(argv[5]) : 300;
  double *X = malloc(sizeof(double) * n * d), *y = malloc(sizeof(double) * n);
  double *mu = malloc(sizeof(double) * n), *U = malloc(sizeof(double) * m * d);
  srand(7);
  for (long i = 0; i < n * d; ++i) X[i] = 10.0 * rand() / RAND_MAX;
  for (long j = 0; j < m * d; ++j) U[j] = 10.0 * rand() / RAND_MAX;
  double ym = 0.0;
  for (long i = 0; i < n; ++i) {
    double s = 0.0;
    for (int c = 0; c < d; ++c) s += sin(X[i + c * n]);
    y[i] = s + 0.5 * (2.0 * rand() / RAND_MAX - 1.0);
    ym += y[i] / n;
  }
  for (long i = 0; i < n; ++i) mu[i] = ym;
  const int P = sgp_num_params(kernel, d);
  double* th = malloc(sizeof(double) * P);
  double* g = malloc(sizeof(double) * P);
  sgp_ctx* c = NULL;
  if (sgp_ctx_create(&c, 0, X, n, n, d, y, mu, m)) { fprintf(stderr, "%s\n", sgp_last_error()); return 1; }
  double obj = 0.0, t0 = 0.0;
  for (int k = 0; k < evals + 20; ++k) {
    if (k == 20) t0 = now();
    for (int p = 0; p < P; ++p) th[p] = (p == 0 ? 1.0 : p == P - 1 ? 0.5 : (kernel ? 3.0 : 1.0)) * exp(1e-3 * sin(p + k));
    if (sgp_eval_vi(c, kernel, th, U, m, m, 1e-6, 0, &obj, g)) { fprintf(stderr, "%s\n", sgp_last_error()); return 1; }
  }
  const double dt = now() - t0;
  printf("n=%ld m=%ld d=%d kernel=%d: %.1f evals/s (%.1f us per evaluation), obj %.6f\n", n, m, d,
         kernel, evals / dt, 1e6 * dt / evals, obj);
  sgp_ctx_destroy(c);
  return 0;
}
