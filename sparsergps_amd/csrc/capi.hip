// C ABI of libsgp.so (include/sgp.h): context management and the fused VI evaluation.
//
// One evaluation of sgp_eval_vi == one optimizer-iteration body of the reference's
// norm_grad_ascent_vi (R/vi_functions.R:1089-1128): build K12/K22 at (theta, U), the ELBO
// (elbo_fun, vi_functions.R:64-121) and its gradient w.r.t. log(theta)
// (delbo_dcov_par, vi_functions.R:126-602).  The reference evaluates the gradient as
// P separate n x m^2 pipelines; this implementation uses the adjoint form
//     S = K^T K, t = K^T r (one SYRK)              -> every m x m quantity
//     G = alpha u^T + K P (one GEMM) contracted with dK/dtheta in the epilogue
// which is algebraically identical and needs ~3 n m^2 flops in total.
#include <math.h>

#include <cmath>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/sgp.h"
#include "../../include/sgp_diag.h"
#include "sgp_internal.h"

#ifdef SGP_HOST_PROBE
// entry, before the readback's synchronisation, after it, exit of the last sgp_eval_vi
// (CLOCK_MONOTONIC seconds: Python's time.perf_counter reads the same clock)
extern "C" __attribute__((visibility("default"))) double sgp_probe_t[4] = {0.0, 0.0, 0.0, 0.0};
#endif
#include "sgp_probe.h"
#include "sgp_multi.h"

namespace {

thread_local std::string g_err;

void set_err(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
}

#define HIPCHK(expr)                                                                       \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess) {                                                                \
      set_err("HIP error '%s' at %s:%d", hipGetErrorString(e_), __FILE__, __LINE__);      \
      return SGP_EHIP;                                                                     \
    }                                                                                      \
  } while (0)

// Entry points a multi-device context (sgp_ctx_create_multi) answers through multi.hip, and the
// ones it refuses (their reductions and streams are internal to it)
#define MULTI_FWD(c, call)                   \
  do {                                       \
    if ((c) && (c)->multi) return (call);    \
  } while (0)
#define MULTI_REFUSE(c, name)                                                                  \
  do {                                                                                         \
    if ((c) && (c)->multi) {                                                                   \
      set_err("%s is not available on a multi-device context (sgp_ctx_create_multi runs its " \
              "reductions inside the library)", name);                                         \
      return SGP_EINVAL;                                                                       \
    }                                                                                          \
  } while (0)

int multi_bad_args() {
  set_err("invalid arguments");
  return SGP_EINVAL;
}

inline int64_t round_up(int64_t v, int64_t q) { return (v + q - 1) / q * q; }

int num_ls(int kernel, int d) { return kernel == SGP_KERNEL_ARD ? d : 1; }

int make_params(int kernel, int d, const double* theta, double delta, KernParams* kp) {
  if (kernel < 0 || kernel > 2) {
    set_err("invalid covariance function (kernel=%d)", kernel);
    return SGP_EINVAL;
  }
  if (d < 1 || d > SGP_MAXD) {
    set_err("input dimension d=%d outside [1, %d]", d, SGP_MAXD);
    return SGP_EINVAL;
  }
  if (!theta) {
    set_err("theta is NULL");
    return SGP_EINVAL;
  }
  memset(kp, 0, sizeof(*kp));
  kp->kernel = kernel;
  kp->d = d;
  kp->L = num_ls(kernel, d);
  kp->P = kp->L + 2;
  kp->sigma = theta[0];
  kp->sig2 = theta[0] * theta[0];
  kp->tau = theta[kp->L + 1];
  kp->tau2 = kp->tau * kp->tau;
  kp->delta = delta;
  for (int c = 0; c < kp->L; ++c) {
    const double l = theta[1 + c];
    if (!(l > 0.0)) {
      set_err("length scale %d is not positive (%g)", c + 1, l);
      return SGP_EINVAL;
    }
    kp->l[c] = l;
    kp->rl[c] = 1.0 / l;
    kp->rl2[c] = 1.0 / (l * l);
  }
  if (kernel == SGP_KERNEL_SQEXP) kp->coef = -1.0 / (2.0 * (theta[1] * theta[1]));
  else if (kernel == SGP_KERNEL_ARD) kp->coef = -0.5;
  else kp->coef = -1.0 / theta[1];
  if (kernel != SGP_KERNEL_ARD)
    for (int c = 1; c < d; ++c) { kp->l[c] = kp->l[0]; kp->rl[c] = kp->rl[0]; kp->rl2[c] = kp->rl2[0]; }
  kp->lsig2 = log(kp->sig2);
  set_exp_consts(kp);
  return SGP_OK;
}

}  // namespace

void set_exp_consts(KernParams* kp) {
  kp->ec[0] = 1.4426950408889634074;
  kp->ec[1] = 6.93147180369123816490e-01;
  kp->ec[2] = 1.90821492927058770002e-10;
  double f = 1.0;
  for (int q = 2; q <= 13; ++q) f *= (double)q;   // 13!
  for (int q = 13; q >= 2; --q) {                 // ec[3] = 1/13!, ..., ec[14] = 1/2!
    kp->ec[3 + (13 - q)] = 1.0 / f;
    f /= (double)q;
  }
  kp->ec[15] = 0.0;
  kp->xt[0] = 46.166241308446828384;                 // 32 / ln2
  kp->xt[1] = 6.93147180369123816490e-01 / 32.0;      // fdlibm ln2_hi (low 21 bits zero) / 32
  kp->xt[2] = 1.90821492927058770002e-10 / 32.0;      // ln2_lo / 32
  kp->xt[3] = 1.0 / 720.0;
  kp->xt[4] = 1.0 / 120.0;
  kp->xt[5] = 1.0 / 24.0;
  kp->xt[6] = 1.0 / 6.0;
  kp->xt[7] = 0.5;
  for (int j = 0; j < 32; ++j) kp->et[j] = (double)exp2l((long double)j / 32.0L);
}

namespace {

// kp->ctr = column means of the m x d knot matrix U (column-major, ld ldu; host memory), and
// kp->span2 = a bound on |x~|^2 over the knots and the data box [xlo, xhi] (per coordinate;
// NULL = knots only) that the matrix-core builder's accuracy guard reads (knm_mfma_ok).
// extra (T points, column-major, ld ldx; NULL = none): further points the same parameters will
// be built against (OAT candidate knots, which may lie outside the data box): they widen
// span2 but do not move the centre.
void set_center(KernParams* kp, const double* U, int64_t m, int64_t ldu, const double* xlo,
                const double* xhi, const double* extra = nullptr, int64_t T = 0,
                int64_t ldx = 0) {
  double span2 = 0.0;
  for (int c = 0; c < kp->d; ++c) {
    double s = 0.0, lo = U[c * ldu], hi = U[c * ldu];
    for (int64_t j = 0; j < m; ++j) {
      const double v = U[j + c * ldu];
      s += v;
      lo = v < lo ? v : lo;
      hi = v > hi ? v : hi;
    }
    kp->ctr[c] = m > 0 ? s / (double)m : 0.0;
    if (xlo && xhi) {
      lo = xlo[c] < lo ? xlo[c] : lo;
      hi = xhi[c] > hi ? xhi[c] : hi;
    }
    for (int64_t j = 0; extra && j < T; ++j) {
      const double v = extra[j + c * ldx];
      lo = v < lo ? v : lo;
      hi = v > hi ? v : hi;
    }
    const double e = fmax(fabs(lo - kp->ctr[c]), fabs(hi - kp->ctr[c])) * kp->rl[c];
    span2 += e * e;
  }
  kp->span2 = span2 == span2 ? span2 : INFINITY;   // NaN coordinates: the VALU form
}

// column ranges of an n x d column-major host matrix
void col_range(const double* X, int64_t n, int64_t ldx, int d, std::vector<double>* lo,
               std::vector<double>* hi) {
  lo->assign((size_t)d, 0.0);
  hi->assign((size_t)d, 0.0);
  for (int c = 0; c < d; ++c) {
    double a = n > 0 ? X[c * ldx] : 0.0, b = a;
    for (int64_t i = 1; i < n; ++i) {
      const double v = X[i + c * ldx];
      a = v < a ? v : a;
      b = v > b ? v : b;
    }
    (*lo)[(size_t)c] = a;
    (*hi)[(size_t)c] = b;
  }
}

struct Timer {
  std::string name;
  hipEvent_t a, b;
};

}  // namespace

struct sgp_ctx {
  // a row-sharded multi-device context (sgp_ctx_create_multi): the entry points below forward
  // to multi.hip, and none of the members after this one is used
  MultiCtx* multi = nullptr;
  int device = 0;
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
  int64_t n = 0, n_pad = 0, m_max = 0, mp_max = 0;
  int d = 0;
  // per-row data (HBM-resident for the context's lifetime)
  double* X = nullptr;      // n_pad x d, column-major, ld = n_pad
  double* r = nullptr;      // y - mu, n_pad
  double* K = nullptr;      // n_pad x mp (row-major, ld = mp)
  double* alpha = nullptr;  // n_pad
  double* zinv = nullptr;   // n_pad (FITC weights 1/Z)
  double* omega = nullptr;  // n_pad (FITC 2 W_ii)
  double* pvec = nullptr;   // n_pad (row quadratic forms)
  double* rowq = nullptr;   // (mp_max/128) x n_pad row-partial work
  double* red2f = nullptr;  // internal FITC second reduction
  // knots and m x m work
  double* U = nullptr;      // mp_max x d, column-major, ld = mp_max
  double *K22 = nullptr, *K22inv = nullptr, *Bm = nullptr, *Binv = nullptr, *Pm = nullptr;
  double *Xt = nullptr, *T1 = nullptr, *M3 = nullptr;
  double *Xt22 = nullptr, *T22 = nullptr;  // K22-stage temporaries (aux stream)
  // sync words of the two Gauss-Jordan chains that can run together: [0] main stream (Bm),
  // [SGP_GJ_SYNC_WORDS] the aux stream's K22 chain (dense_spd_inverse: zero between launches)
  unsigned* gjs = nullptr;
  double *dinv = nullptr, *dinv22 = nullptr, *logd22 = nullptr, *logdB = nullptr;
  double *uvec = nullptr, *cdiag = nullptr;
  int* status = nullptr;
  double *red1 = nullptr, *red2 = nullptr;
  double *slab_syrk = nullptr, *slab_con = nullptr, *slab_small = nullptr, *sc = nullptr;
  // the balanced gradient contraction's hand-over slots and flags (k_contract_sk)
  double* sk_ws = nullptr;
  unsigned* sk_flags = nullptr;
  unsigned sk_epoch = 0;
  int sk_slots = 0;
  double* tslab = nullptr;                // builder t = K^T r partials (VI), n_pad/64 x mp
  // stored products of the FITC / Laplace row-quadratic passes (n_pad x mp each, allocated on
  // first use): tq = K K22^-1, tp = K Bm^-1 (FITC) or K C (Laplace).  The gradient
  // contraction passes read them instead of recomputing the same 2 n m^2 GEMMs.
  double *tq = nullptr, *tp = nullptr;
  int tstore_state = 0;                   // 0 untried, 1 allocated, -1 unavailable
  int64_t slab_syrk_cap = 0, slab_con_cap = 0, slab_small_cap = 0;
  // state carried between phases
  KernParams kp;
  int64_t m = 0, mp = 0, n_global = 0;
  double delta = 0.0;
  unsigned flags = 0;
  // knot gradients (opt-in)
  bool knot_on = false;
  double *knot_slab = nullptr, *knot_part = nullptr, *knot_kmm = nullptr;
  std::vector<double> knot_raw;           // d F / d u (m x d, row-major), before the chain factor
  std::vector<double> hU;                 // host copy of the knots (m x d, column-major)
  double* pin = nullptr;                  // pinned staging for knot uploads
  hipEvent_t ev_pin = nullptr;            // the last upload's copies have been issued before it
  bool knots_valid = false;               // c->U / khash / kidx hold hU (layout knots_mp)
  int64_t knots_mp = 0;
  uint64_t* khash = nullptr;              // sorted knot coordinate hashes (k_coinc)
  int* kidx = nullptr;                    // knot index of each sorted hash
  uint8_t* cflag = nullptr;               // per data row: equals some knot (k_coinc)
  int64_t knots_gen = 0;                  // bumped whenever the resident knot set changes
  int64_t cflag_gen = -1;                 // knot set cflag was computed for
  std::vector<double> xmin, xmax;         // column ranges of this context's rows
  int phase = 0;
  int last_mode = 0;   // 1 VI, 2 FITC, 3 Laplace: the evaluation sgp_posterior_u refers to
  // K22 stage runs on `aux` concurrently with phase 1 (it depends only on U and theta)
  hipStream_t aux = nullptr;
  hipEvent_t ev_knots = nullptr, ev_k22 = nullptr;
  hipEvent_t ev_k22m = nullptr;           // K22 itself built (aux); ev_k22: K22 inverted too
  // phase 2's Bm-independent m x m work (K22inv S K22inv, tr(K22inv S)) also runs on `aux`,
  // concurrently with the latency-bound Bm inversion on the main stream
  hipEvent_t ev_s = nullptr, ev_m3 = nullptr, ev_bm = nullptr;
  hipEvent_t ev_lo = nullptr;             // VI phase 1: builder done (main) / side work done (aux_lo)
  bool vi_k22_ordered = true;             // VI phase 1 ordered main behind K22's build (ev_lo)
  // sgp_eval_vi (no reduction between the phases): at m_p = 256 t's row sums leave phase 1's
  // critical path for aux_lo in phase 2 (t is first read by the m-vectors, after the Bm chain)
  bool fused_vi = false, t_deferred = false;
  // sgp_eval_vi's phase 2: the contraction records' second pass is left to the readback kernel
  bool defer_rec = false;
  RecPass2 rec_defer{};
  int64_t t_rows_def = 0;
  hipEvent_t ev_t = nullptr;
  bool pack_red1 = false;                 // VI red1 carries S as packed lower 64-blocks
  bool borrowed_streams = false;          // own / aux / aux_lo belong to another context
  double* Sfull = nullptr;                // S unpacked from a packed red1 (mp_max^2)
  hipStream_t aux_lo = nullptr;           // ... at normal priority (the Bm chain keeps its CUs)
  double* slab_aux = nullptr;             // partials of the aux stream's small reductions
  double* rr_dev = nullptr;               // r^T r of the resident r (set with r)
  double* mmpart = nullptr;               // VI's m-vector row terms (mp), read on aux_lo
  unsigned* rsync = nullptr;              // the SYRK reduction's slice tickets (kept zeroed)
  // launch-bound Bm factorisation captured once per (mp, S pointer) and replayed
  // Poisson-Laplace state (row/knot vectors allocated on first use)
  double *y = nullptr, *mu = nullptr;     // per-row data (n_pad), kept for the Laplace path
  double* lv = nullptr;                   // LV_N x n_pad row vectors
  bool lap_gpsi_valid = false;            // LV_GPSI holds the last NR step's grad psi
  double* lm = nullptr;                   // LM_N x mp_max knot vectors
  double* lslab = nullptr;                // K^T V row-chunk partials
  double* Cprev = nullptr;                // (K22 + S_B)^-1 of the previous NR iterate
  int64_t lslab_cap = 0;
  double* lred[2] = {nullptr, nullptr};   // ping-pong reduction buffers of sgp_eval_laplace
  int lap_state = 0, lap_it = 0, lap_maxit = 0;
  double lap_obj = 0.0, lap_obj_prev = 0.0, lap_cnt = 0.0, lap_tol = 0.0, lap_expo = 1.0;
  bool lap_expo_rows = false;             // LV_AEXP holds a per-row exposure (sgp_lap_set_expo)
  const double* lap_av = nullptr;         // this NR run's per-row exposure (nullptr: lap_expo)
  std::vector<double> lap_objs;           // objective_function_values of the last NR run
  // timing
  bool timing = false;
  std::string timing_only;                // record only the scopes of this name ("" = all)
  int64_t timing_evals = 0;               // evaluations recorded since timing was enabled
  std::vector<Timer> timers;
  std::vector<hipEvent_t> pool;
  size_t pool_used = 0;
};

namespace {

constexpr int SC_LD22 = 0, SC_LDB = 1, SC_TU = 2, SC_TRKS = 3, SC_TRBS = 4, SC_RR = 5,
              SC_G22 = 16;  // SC_G22 .. SC_G22 + P - 1 (contract_kmm records)
constexpr int SC_N = 64;
// per-block partials of the small reductions: k_contract_kmm writes up to 1024 blocks x (P-1)
// records (P <= SGP_MAXD + 2), the dot/colsum helpers at most 1024 x 1
constexpr int SLAB_SMALL = 1024 * (SGP_MAXD + 2);
constexpr int KNOT_PART_ROWS = 256;   // row groups of the knot / t column-sum first pass
constexpr int RB_N = 256;             // pinned readback doubles at the end of c->pin

// The end-of-evaluation results are gathered by ONE small kernel straight into pinned host
// memory (device-visible, hipHostMalloc) and unpacked into the caller's host arrays after one
// synchronisation.  (Three hipMemcpyAsync D2H copies were three blit kernels plus their launch
// gaps on the critical path of every evaluation: ~15 us at C2.)
constexpr int RB_SEGS = SGP_RB_SEGS;

#ifdef SGP_HOST_PROBE
// host time of sgp_eval_vi: entry -> the readback's synchronisation (issue) and the wait in it;
// averages printed to stderr every 200 evaluations (variant builds only)
static double hp_now() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}
static double hp_t0 = 0.0, hp_issue = 0.0, hp_wait = 0.0, hp_tail = 0.0, hp_prev_end = 0.0,
              hp_gap = 0.0;
static long hp_n = 0;
#endif

struct Readback {
  sgp_ctx* c;
  double* base;
  size_t off = 0;   // doubles
  struct Item { void* host; size_t off, bytes; };
  std::vector<Item> items;
  GatherSegs segs{};
  explicit Readback(sgp_ctx* ctx)
      : c(ctx), base(ctx->pin + ctx->mp_max * ctx->d + ctx->m_max + (ctx->m_max + 1) / 2 + 8) {}
  // a readback abandoned before wait() (a failed add) drops the deferred record pass too: it
  // belongs to this readback's evaluation, and a later readback must not replay it
  ~Readback() { c->rec_defer = RecPass2{}; }
  // dev: device memory of `bytes` bytes, 8-byte aligned (copied as whole doubles)
  hipError_t add(void* host, const void* dev, size_t bytes) {
    const size_t nd = (bytes + 7) / 8;
    if (off + nd > (size_t)RB_N || segs.count == RB_SEGS) return hipErrorInvalidValue;
    items.push_back({host, off, bytes});
    segs.src[segs.count] = reinterpret_cast<const double*>(dev);
    segs.off[segs.count] = (int)off;
    segs.n[segs.count] = (int)nd;
    ++segs.count;
    off += nd;
    return hipSuccess;
  }
  hipError_t wait() {
    hipError_t e = launch_rec_gather(c->rec_defer, segs, base, c->stream);
    c->rec_defer = RecPass2{};
    if (e != hipSuccess) return e;
#ifdef SGP_HOST_PROBE
    const double t1 = hp_now();
    sgp_probe_t[1] = t1;
#endif
    e = hipStreamSynchronize(c->stream);
#ifdef SGP_HOST_PROBE
    const double t2 = hp_now();
    sgp_probe_t[2] = t2;
    if (hp_t0 > 0.0) {
      hp_issue += t1 - hp_t0;
      hp_wait += t2 - t1;
      hp_tail = t2;
    }
#endif
    if (e != hipSuccess) return e;
    for (const Item& it : items) memcpy(it.host, base + it.off, it.bytes);
    return hipSuccess;
  }
};

constexpr size_t kTimingPoolReserve = 1024;

hipEvent_t pool_event(sgp_ctx* c) {
  if (c->pool_used < c->pool.size()) return c->pool[c->pool_used++];
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  c->pool.push_back(e);
  c->pool_used++;
  return e;
}

struct Scope {
  sgp_ctx* c;
  hipStream_t s;
  size_t idx;
  Scope(sgp_ctx* ctx, const char* name, hipStream_t st = nullptr)
      : c(ctx), s(st ? st : ctx->stream), idx((size_t)-1) {
    if (!c->timing) return;
    if (!c->timing_only.empty() && c->timing_only != name) return;
    Timer t;
    t.name = name;
    t.a = pool_event(c);
    t.b = pool_event(c);
    if (!t.a || !t.b) return;
    (void)hipEventRecord(t.a, s);
    c->timers.push_back(t);
    idx = c->timers.size() - 1;
  }
  ~Scope() {
    if (idx != (size_t)-1) (void)hipEventRecord(c->timers[idx].b, s);
  }
};

// start of an evaluation: with timing on, its scopes are appended to those of the earlier
// evaluations (read out once, after the timed loop, by sgp_ctx_timings)
void timers_reset(sgp_ctx* c) {
  if (c->timing) {
    ++c->timing_evals;
    return;
  }
  c->timers.clear();
  c->pool_used = 0;
}

// a Gauss-Jordan chain whose watchdog expired (k_dense.hip: status -1; never expected)
static bool chain_watchdog(const int* status) {
  for (int q = 0; q < 3; ++q)
    if (status[q] < 0) {
      set_err("internal error: a Gauss-Jordan chain's wait watchdog expired");
      return true;
    }
  if (status[3] < 0) {
    set_err("internal error: the gradient contraction's hand-over wait watchdog expired");
    return true;
  }
  return false;
}

template <typename T>
int dalloc(T** p, int64_t count) {
  *p = nullptr;
  if (count <= 0) count = 1;
  hipError_t e = hipMalloc((void**)p, sizeof(T) * (size_t)count);
  if (e != hipSuccess) {
    set_err("hipMalloc of %lld bytes failed: %s", (long long)(sizeof(T) * count),
            hipGetErrorString(e));
    return SGP_ENOMEM;
  }
  return SGP_OK;
}

// Stored-product buffers for the FITC / Laplace passes; false (GEMM path) when HBM is short --
// the evaluation is the same either way.
bool tstore_ready(sgp_ctx* c) {
  if (c->tstore_state == 0) {
    // SGP_TSTORE=0: the recompute-everything passes, as when the memory is not there (tests)
    const char* env = getenv("SGP_TSTORE");
    if (env && env[0] == '0') {
      c->tstore_state = -1;
      return false;
    }
    const int64_t cnt = c->n_pad * c->mp_max;
    if (hipMalloc(reinterpret_cast<void**>(&c->tq), sizeof(double) * cnt) == hipSuccess &&
        hipMalloc(reinterpret_cast<void**>(&c->tp), sizeof(double) * cnt) == hipSuccess) {
      c->tstore_state = 1;
    } else {
      (void)hipGetLastError();
      if (c->tq) (void)hipFree(c->tq);
      if (c->tp) (void)hipFree(c->tp);
      c->tq = c->tp = nullptr;
      c->tstore_state = -1;
    }
  }
  return c->tstore_state == 1;
}

// FITC / Laplace: both stored products read in ONE gradient pass (ConArgs::tin2; d <= 8)
static bool fuse_tt(sgp_ctx* c) { return c->kp.d <= 8 && tstore_ready(c); }

void ctx_free(sgp_ctx* c) {
  void* ptrs[] = {c->X,      c->r,     c->K,      c->alpha,   c->zinv,  c->U,    c->K22,
                  c->K22inv, c->Bm,    c->Binv,   c->Pm,      c->Xt,    c->T1,   c->M3,
                  c->dinv,   c->logd22, c->logdB, c->uvec,    c->cdiag, c->status, c->red1,
                  c->red2,   c->slab_syrk, c->slab_con, c->slab_small, c->slab_aux, c->sc,
                  c->sk_ws,  c->sk_flags,
                  c->Xt22,   c->T22,    c->dinv22, c->omega, c->pvec, c->rowq, c->red2f,
                  c->y,      c->mu,     c->lv,     c->lm,    c->lslab, c->lred[0], c->lred[1],
                  c->Cprev,  c->knot_slab, c->knot_part, c->knot_kmm, c->tslab, c->tq, c->tp,
                  c->rr_dev, c->Sfull, c->gjs, c->mmpart, c->rsync};
  for (void* p : ptrs)
    if (p) hipFree(p);
  if (c->khash) hipFree(c->khash);
  if (c->kidx) hipFree(c->kidx);
  if (c->cflag) hipFree(c->cflag);
  if (c->ev_knots) hipEventDestroy(c->ev_knots);
  if (c->ev_pin) hipEventDestroy(c->ev_pin);
  if (c->pin) hipHostFree(c->pin);
  if (c->ev_k22) hipEventDestroy(c->ev_k22);
  if (c->ev_k22m) hipEventDestroy(c->ev_k22m);
  if (c->ev_s) hipEventDestroy(c->ev_s);
  if (c->ev_m3) hipEventDestroy(c->ev_m3);
  if (c->ev_bm) hipEventDestroy(c->ev_bm);
  if (c->ev_lo) hipEventDestroy(c->ev_lo);
  if (c->ev_t) hipEventDestroy(c->ev_t);
  if (c->aux && !c->borrowed_streams) hipStreamDestroy(c->aux);
  if (c->aux_lo && !c->borrowed_streams) hipStreamDestroy(c->aux_lo);
  for (hipEvent_t e : c->pool) hipEventDestroy(e);
  if (c->own && !c->borrowed_streams) hipStreamDestroy(c->own);
}

// n host values -> device vector of n_pad (zero padded), synchronous
hipError_t upload_rows(double* dst, const double* src, int64_t n, int64_t n_pad) {
  std::vector<double> h((size_t)n_pad, 0.0);
  for (int64_t i = 0; i < n; ++i) h[(size_t)i] = src[i];
  return hipMemcpy(dst, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice);
}

// FNV-1a over the coordinates' bytes, +0/-0 canonicalised (k_mfma.hip coord_hash)
uint64_t coord_hash_host(const double* x, int64_t stride, int d) {
  uint64_t h = 1469598103934665603ull;
  for (int q = 0; q < d; ++q) {
    double v = x[q * stride];
    if (v == 0.0) v = 0.0;
    uint64_t b;
    memcpy(&b, &v, sizeof(b));
    for (int k = 0; k < 8; ++k) {
      h ^= (b >> (8 * k)) & 0xffu;
      h *= 1099511628211ull;
    }
  }
  return h;
}

// An evaluation that was begun but never finished (an error or an abandoned caller between
// the phases) can leave the K22 chain (aux: writes status[0], sc[SC_LD22], reads U) and aux_lo
// work queued.  Every entry that begins an evaluation (VI / FITC phase 1, Laplace begin, the
// full GP) calls this before it touches phase, U, status or sc, so the new evaluation's knot
// upload and resets on the main stream cannot overtake that work.  Only an abandoned
// evaluation (phase != 0) pays the two cross-stream waits.
int drain_abandoned(sgp_ctx* c) {
  if (c->phase != 0) {
    HIPCHK(hipStreamWaitEvent(c->stream, c->ev_k22, 0));
    HIPCHK(hipStreamWaitEvent(c->stream, c->ev_m3, 0));
    c->phase = 0;
  }
  return SGP_OK;
}

int upload_knots(sgp_ctx* c, const double* U, int64_t m, int64_t ldu) {
  // optimizer iterations with fixed knots (xu_opt = "fixed") pass the same U every time: keep
  // the resident copy and its hash table
  if (c->knots_valid && c->knots_mp == c->mp && (int64_t)c->hU.size() == m * c->d) {
    bool same = true;
    for (int q = 0; q < c->d && same; ++q)
      same = memcmp(&c->hU[(size_t)(q * m)], U + q * ldu, sizeof(double) * m) == 0;
    if (same) return SGP_OK;
  }
  c->knots_valid = false;
  ++c->knots_gen;
  // staging through pinned host memory, copies async on the context stream; the previous
  // upload's copies must have drained before the buffer is rewritten
  HIPCHK(hipEventSynchronize(c->ev_pin));
  double* hU_dev = c->pin;                                        // mp x d (device layout)
  uint64_t* hh = reinterpret_cast<uint64_t*>(c->pin + c->mp_max * c->d);
  int* hi = reinterpret_cast<int*>(hh + c->m_max);
  {
    std::vector<std::pair<uint64_t, int>> hk((size_t)m);
    for (int64_t j = 0; j < m; ++j) hk[(size_t)j] = {coord_hash_host(U + j, ldu, c->d), (int)j};
    std::sort(hk.begin(), hk.end());
    for (int64_t j = 0; j < m; ++j) {
      hh[j] = hk[(size_t)j].first;
      hi[j] = hk[(size_t)j].second;
    }
  }
  c->hU.assign((size_t)(m * c->d), 0.0);
  for (int q = 0; q < c->d; ++q)
    for (int64_t j = 0; j < m; ++j) c->hU[(size_t)(j + q * m)] = U[j + q * ldu];
  for (int q = 0; q < c->d; ++q)
    for (int64_t j = 0; j < c->mp; ++j) hU_dev[q * c->mp + j] = j < m ? U[j + q * ldu] : 0.0;
  HIPCHK(hipMemcpyAsync(c->khash, hh, sizeof(uint64_t) * m, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->kidx, hi, sizeof(int) * m, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->U, hU_dev, sizeof(double) * c->mp * c->d, hipMemcpyHostToDevice,
                        c->stream));
  HIPCHK(hipEventRecord(c->ev_pin, c->stream));
  c->knots_valid = true;
  c->knots_mp = c->mp;
  return SGP_OK;
}

int check_eval_args(sgp_ctx* c, int kernel, const double* theta, const double* U, int64_t m,
                    int64_t ldu, double delta, KernParams* kp) {
  if (!c) { set_err("context is NULL"); return SGP_EINVAL; }
  if (kernel == SGP_KERNEL_EXP) {
    set_err("fused evaluation supports 'sqexp' and 'ard' (optimize_gp.R:263 rejects others)");
    return SGP_EINVAL;
  }
  int st = make_params(kernel, c->d, theta, delta, kp);
  if (st) return st;
  if (!U || m < 1 || m > c->m_max || ldu < m) {
    set_err("invalid knots: m=%lld (m_max=%lld), ldu=%lld", (long long)m, (long long)c->m_max,
            (long long)ldu);
    return SGP_EINVAL;
  }
  if (!(kp->tau > 0.0) || !(kp->sigma > 0.0)) {
    set_err("sigma and tau must be positive");
    return SGP_EINVAL;
  }
  set_center(kp, U, m, ldu, c->xmin.data(), c->xmax.data());
  return SGP_OK;
}

}  // namespace

// multi.hip's hooks (sgp_multi.h)
void sgp_internal_set_err(const char* msg) { set_err("%s", msg); }

void sgp_internal_forget_eval(sgp_ctx* c) {
  c->last_mode = 0;
  c->lap_gpsi_valid = false;
}

hipStream_t sgp_internal_stream(sgp_ctx* c) { return c->stream; }

// c takes over src's three streams (same device; c's own are idle after creation): the shards
// of one device then use the streams of the first, not three more hardware-queue clients each
int sgp_internal_share_streams(sgp_ctx* c, sgp_ctx* src) {
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->own));
  HIPCHK(hipStreamSynchronize(c->aux));
  HIPCHK(hipStreamSynchronize(c->aux_lo));
  (void)hipStreamDestroy(c->own);
  (void)hipStreamDestroy(c->aux);
  (void)hipStreamDestroy(c->aux_lo);
  c->own = src->own;
  c->stream = src->stream;
  c->aux = src->aux;
  c->aux_lo = src->aux_lo;
  c->borrowed_streams = true;
  return SGP_OK;
}

// =========================================================================== public API
extern "C" {

const char* sgp_last_error(void) { return g_err.c_str(); }
int sgp_abi_version(void) { return SGP_ABI_VERSION; }

int sgp_device_count(int* count) {
  if (!count) return SGP_EINVAL;
  HIPCHK(hipGetDeviceCount(count));
  return SGP_OK;
}

int sgp_num_params(int kernel, int d) {
  if (kernel < 0 || kernel > 2 || d < 1) return -1;
  return num_ls(kernel, d) + 2;
}

double sgp_kernel_pair(int kernel, const double* x1, const double* x2, int d,
                       const double* theta) {
  KernParams kp;
  if (make_params(kernel, d, theta, 0.0, &kp)) return NAN;
  double s = 0.0;
  if (kernel == SGP_KERNEL_SQEXP) {
    for (int c = 0; c < d; ++c) { double t = x1[c] - x2[c]; s = fma(t, t, s); }
    return kp.sig2 * exp(kp.coef * s);
  } else if (kernel == SGP_KERNEL_ARD) {
    for (int c = 0; c < d; ++c) { double t = (x1[c] - x2[c]) * kp.rl[c]; s = fma(t, t, s); }
    return kp.sig2 * exp(-s / 2.0);
  }
  for (int c = 0; c < d; ++c) s += fabs(x1[c] - x2[c]);
  return kp.sig2 * exp(kp.coef * s);
}

double sgp_dkernel_pair(int kernel, const double* x1, const double* x2, int d,
                        const double* theta, int param) {
  KernParams kp;
  if (make_params(kernel, d, theta, 0.0, &kp)) return NAN;
  if (param < 0 || param >= kp.P) { set_err("invalid parameter index %d", param); return NAN; }
  if (param == kp.P - 1) {
    bool eq = true;
    for (int c = 0; c < d; ++c) eq = eq && (x1[c] == x2[c]);
    return eq ? 2.0 * kp.tau * kp.tau : 0.0;
  }
  double s = 0.0;
  if (kernel == SGP_KERNEL_SQEXP) {
    for (int c = 0; c < d; ++c) { double t = x1[c] - x2[c]; s = fma(t, t, s); }
    const double e = exp(kp.coef * s);
    if (param == 0) return 2.0 * kp.sigma * e * kp.sigma;
    return (kp.sig2 * e) * ((1.0 / (kp.l[0] * kp.l[0] * kp.l[0])) * s) * kp.l[0];
  } else if (kernel == SGP_KERNEL_ARD) {
    for (int c = 0; c < d; ++c) { double t = (x1[c] - x2[c]) * kp.rl[c]; s = fma(t, t, s); }
    const double e = exp(-(s / 2.0));
    if (param == 0) return 2.0 * kp.sigma * e * kp.sigma;
    const int c = param - 1;
    const double dc = x1[c] - x2[c], lc = kp.l[c];
    return (kp.sig2 * e) * ((1.0 / (lc * lc * lc)) * (dc * dc)) * lc;
  }
  for (int c = 0; c < d; ++c) { double t = x1[c] - x2[c]; s = fma(t, t, s); }
  const double dist = sqrt(s);
  const double e = exp(-(1.0 / kp.l[0]) * dist);
  if (param == 0) return 2.0 * kp.sigma * e * kp.sigma;
  return (kp.sig2 * e) * ((1.0 / (kp.l[0] * kp.l[0])) * dist) * kp.l[0];
}

static int fill_common(int device, int kernel, const double* x, int64_t n, int64_t ldx,
                       const double* xp, int64_t np, int64_t ldxp, int d, const double* theta,
                       double delta, int param, bool deriv, double* out, int64_t ldo) {
  KernParams kp;
  int st = make_params(kernel, d, theta, delta, &kp);
  if (st) return st;
  const bool sym = (xp == nullptr);
  if (sym) { xp = x; np = n; ldxp = ldx; }
  if (!x || !out || n < 0 || np < 0 || ldx < n || ldxp < np || ldo < n) {
    set_err("invalid matrix arguments");
    return SGP_EINVAL;
  }
  if (deriv && (param < 0 || param >= kp.P)) {
    set_err("invalid parameter name for chosen covariance function (index %d)", param);
    return SGP_EINVAL;
  }
  if (n == 0 || np == 0) return SGP_OK;
  HIPCHK(hipSetDevice(device));
  double *dx = nullptr, *dxp = nullptr, *dout = nullptr;
  st = dalloc(&dx, n * d);
  if (!st) st = dalloc(&dxp, np * d);
  if (!st) st = dalloc(&dout, n * np);
  if (st) { hipFree(dx); hipFree(dxp); hipFree(dout); return st; }
  std::vector<double> hx((size_t)(n * d)), hxp((size_t)(np * d));
  for (int c = 0; c < d; ++c) {
    for (int64_t i = 0; i < n; ++i) hx[(size_t)(i + c * n)] = x[i + c * ldx];
    for (int64_t j = 0; j < np; ++j) hxp[(size_t)(j + c * np)] = xp[j + c * ldxp];
  }
  hipError_t e = hipMemcpy(dx, hx.data(), sizeof(double) * n * d, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(dxp, hxp.data(), sizeof(double) * np * d, hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = deriv ? launch_fill_dcov(kp, dx, n, n, dxp, np, np, sym, param, dout, n, 0)
              : launch_fill_cov(kp, dx, n, n, dxp, np, np, sym, dout, n, 0);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  std::vector<double> ho;
  if (e == hipSuccess) {
    ho.resize((size_t)(n * np));
    e = hipMemcpy(ho.data(), dout, sizeof(double) * n * np, hipMemcpyDeviceToHost);
  }
  hipFree(dx);
  hipFree(dxp);
  hipFree(dout);
  if (e != hipSuccess) {
    set_err("HIP error '%s' in covariance fill", hipGetErrorString(e));
    return SGP_EHIP;
  }
  for (int64_t j = 0; j < np; ++j)
    memcpy(out + j * ldo, ho.data() + j * n, sizeof(double) * (size_t)n);
  return SGP_OK;
}

int sgp_make_cov(int device, int kernel, const double* x, int64_t n, int64_t ldx,
                 const double* xp, int64_t np, int64_t ldxp, int d, const double* theta,
                 double delta, double* out, int64_t ldo) {
  return fill_common(device, kernel, x, n, ldx, xp, np, ldxp, d, theta, delta, 0, false, out,
                     ldo);
}

int sgp_dsig_dtheta(int device, int kernel, const double* x, int64_t n, int64_t ldx,
                    const double* xp, int64_t np, int64_t ldxp, int d, const double* theta,
                    int param, double* out, int64_t ldo) {
  return fill_common(device, kernel, x, n, ldx, xp, np, ldxp, d, theta, 0.0, param, true, out,
                     ldo);
}

// The balanced (Stream-K) contraction launch, k_contract_sk: opt-in with SGP_CON_SK=1.  It is
// equivalent to the tile grid (tests/test_gpu_contract_sk.py) but measured no faster at C2 and
// slower on the n = 125 000 shard, so the product launches the grid by default and
// does not allocate the hand-over workspace.
static bool con_sk_enabled() {
  static const bool on = getenv("SGP_CON_SK") && atoi(getenv("SGP_CON_SK")) == 1;
  return on;
}
// SGP_CON_SK_DP=k: the balanced launch runs only k whole rounds as the grid (default: all but the
// last); 0 balances every tile's k-steps over the resident workgroups
static int con_sk_dp() {
  static const int dp = getenv("SGP_CON_SK_DP") ? atoi(getenv("SGP_CON_SK_DP")) : -1;
  return dp;
}

// ------------------------------------------------------------------------- context
int sgp_ctx_create(sgp_ctx** out, int device, const double* X, int64_t n, int64_t ldx, int d,
                   const double* y, const double* mu, int64_t m_max) {
  if (!out || !X || !y || !mu || n < 1 || ldx < n || d < 1 || d > SGP_MAXD || m_max < 1) {
    set_err("invalid sgp_ctx_create arguments (n=%lld, d=%d, m_max=%lld)", (long long)n, d,
            (long long)m_max);
    return SGP_EINVAL;
  }
  *out = nullptr;
  HIPCHK(hipSetDevice(device));
  sgp_ctx* c = new sgp_ctx();
  c->device = device;
  c->n = n;
  c->d = d;
  c->n_pad = round_up(n, SGP_TILE);
  c->m_max = m_max;
  c->mp_max = round_up(m_max, SGP_TILE);
  const int64_t np_ = c->n_pad, mp = c->mp_max, mm = mp * mp;
  int st = SGP_OK;
  if (hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
    set_err("hipStreamCreate failed");
    delete c;
    return SGP_EHIP;
  }
  c->stream = c->own;
  // aux at the highest priority: its K22 chain (a few hundred short workgroups per launch)
  // would otherwise queue behind the builder's tens of thousands
  int prio_least = 0, prio_greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest) != hipSuccess)
    prio_greatest = 0;
  if (hipStreamCreateWithPriority(&c->aux, hipStreamNonBlocking, prio_greatest) != hipSuccess ||
      hipStreamCreateWithPriority(&c->aux_lo, hipStreamNonBlocking, prio_least) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_knots, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_k22, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_k22m, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_s, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_m3, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_bm, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_lo, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_t, hipEventDisableTiming) != hipSuccess) {
    set_err("hipStream/hipEvent creation failed");
    ctx_free(c);
    delete c;
    return SGP_EHIP;
  }
  c->slab_syrk_cap = syrk_slab_doubles(np_, mp);
  c->slab_con_cap = (np_ / SGP_TILE) * (mp / SGP_TILE) * (SGP_MAXD + 5);   // nrec <= L + 5
  st = st ? st : dalloc(&c->X, np_ * d);
  st = st ? st : dalloc(&c->r, np_);
  st = st ? st : dalloc(&c->K, np_ * mp);
  st = st ? st : dalloc(&c->alpha, np_);
  st = st ? st : dalloc(&c->zinv, np_);
  st = st ? st : dalloc(&c->omega, np_);
  st = st ? st : dalloc(&c->pvec, np_);
  st = st ? st : dalloc(&c->rowq, np_ * (mp / SGP_TILE));
  st = st ? st : dalloc(&c->U, mp * d);
  st = st ? st : dalloc(&c->K22, mm);
  st = st ? st : dalloc(&c->K22inv, mm);
  st = st ? st : dalloc(&c->Bm, mm);
  st = st ? st : dalloc(&c->Binv, mm);
  st = st ? st : dalloc(&c->Pm, mm);
  st = st ? st : dalloc(&c->Xt, mm);
  st = st ? st : dalloc(&c->T1, mm);
  st = st ? st : dalloc(&c->M3, mm);
  st = st ? st : dalloc(&c->dinv, mm / SGP_DB * SGP_DB);
  st = st ? st : dalloc(&c->dinv22, mm / SGP_DB * SGP_DB);
  st = st ? st : dalloc(&c->Xt22, mm);
  st = st ? st : dalloc(&c->T22, mm);
  st = st ? st : dalloc(&c->gjs, 2 * SGP_GJ_SYNC_WORDS);
  if (!st && hipMemset(c->gjs, 0, sizeof(unsigned) * 2 * SGP_GJ_SYNC_WORDS) != hipSuccess) {
    set_err("hipMemset of the Gauss-Jordan sync words failed");
    st = SGP_EHIP;
  }
  st = st ? st : dalloc(&c->rsync, SGP_SYRK_RSYNC_WORDS);
  if (!st && hipMemset(c->rsync, 0, sizeof(unsigned) * SGP_SYRK_RSYNC_WORDS) != hipSuccess) {
    set_err("hipMemset of the SYRK reduction tickets failed");
    st = SGP_EHIP;
  }
  st = st ? st : dalloc(&c->logd22, mp / SGP_DB);
  st = st ? st : dalloc(&c->logdB, mp / SGP_DB);
  st = st ? st : dalloc(&c->uvec, mp);
  st = st ? st : dalloc(&c->cdiag, mp);
  st = st ? st : dalloc(&c->status, 4);
  st = st ? st : dalloc(&c->red1, sgp_vi_red1_count(m_max));
  // second reductions, with room for the knot partials (mp x d) after the records
  st = st ? st : dalloc(&c->red2, 64 + mp * d);
  st = st ? st : dalloc(&c->red2f, sgp_fitc_red2_count(SGP_KERNEL_ARD, SGP_MAXD, m_max) + mp * d);
  st = st ? st : dalloc(&c->slab_syrk, c->slab_syrk_cap);
  st = st ? st : dalloc(&c->slab_con, c->slab_con_cap);
  if (con_sk_enabled()) {   // resident workgroups of the balanced contraction: two per CU
    int cus = 0;
    if (!st && hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) ==
                   hipSuccess && cus > 0)
      c->sk_slots = 2 * cus;
    if (c->sk_slots > 0) {
      st = st ? st : dalloc(&c->sk_ws, sgp_con_sk_doubles(c->sk_slots));
      st = st ? st : dalloc(&c->sk_flags, c->sk_slots + 1);
      if (!st && hipMemset(c->sk_flags, 0, sizeof(unsigned) * (c->sk_slots + 1)) != hipSuccess) {
        set_err("hipMemset of the contraction hand-over flags failed");
        st = SGP_EHIP;
      }
    }
  }
  // small-reduction partials: the dot/colsum helpers, and k_contract_kmm's one record per knot
  c->slab_small_cap = std::max<int64_t>(SLAB_SMALL, mp * (SGP_MAXD + 2));
  st = st ? st : dalloc(&c->slab_small, c->slab_small_cap);
  st = st ? st : dalloc(&c->slab_aux, c->slab_small_cap);
  st = st ? st : dalloc(&c->rr_dev, 1);
  st = st ? st : dalloc(&c->mmpart, mp);
  st = st ? st : dalloc(&c->sc, SC_N);
  st = st ? st : dalloc(&c->y, np_);
  st = st ? st : dalloc(&c->mu, np_);
  st = st ? st : dalloc(&c->tslab, (np_ / 64) * mp);
  st = st ? st : dalloc(&c->khash, mp);
  st = st ? st : dalloc(&c->kidx, mp);
  st = st ? st : dalloc(&c->cflag, np_);
  if (!st && (hipHostMalloc(reinterpret_cast<void**>(&c->pin),
                            sizeof(double) * (mp * d + m_max + (m_max + 1) / 2 + 8 + RB_N),
                            hipHostMallocDefault) != hipSuccess ||
              hipEventCreateWithFlags(&c->ev_pin, hipEventDisableTiming) != hipSuccess)) {
    set_err("pinned staging allocation failed");
    st = SGP_ENOMEM;
  }
  if (st) {
    ctx_free(c);
    delete c;
    return st;
  }
  c->xmin.assign((size_t)d, 0.0);
  c->xmax.assign((size_t)d, 0.0);
  for (int q = 0; q < d; ++q) {
    double lo = X[q * ldx], hi = X[q * ldx];
    for (int64_t i = 1; i < n; ++i) {
      const double v = X[i + q * ldx];
      lo = v < lo ? v : lo;
      hi = v > hi ? v : hi;
    }
    c->xmin[(size_t)q] = lo;
    c->xmax[(size_t)q] = hi;
  }
  // X: column-major with ld = n_pad, zero padded
  std::vector<double> hx((size_t)(np_ * d), 0.0);
  for (int q = 0; q < d; ++q)
    for (int64_t i = 0; i < n; ++i) hx[(size_t)(i + q * np_)] = X[i + q * ldx];
  std::vector<double> hr((size_t)np_, 0.0);
  for (int64_t i = 0; i < n; ++i) hr[(size_t)i] = y[i] - mu[i];
  hipError_t e = hipMemcpy(c->X, hx.data(), sizeof(double) * hx.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(c->r, hr.data(), sizeof(double) * hr.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemset(c->K, 0, sizeof(double) * np_ * mp);
  if (e == hipSuccess) e = upload_rows(c->y, y, n, np_);
  if (e == hipSuccess) e = upload_rows(c->mu, mu, n, np_);
  if (e == hipSuccess) e = launch_dot(c->r, c->r, np_, c->slab_aux, c->rr_dev, c->stream);
  // the set-up's hipMemset calls (sync words, tickets, K) run on the null stream, which the
  // context's non-blocking streams do not wait for: finish them before the first evaluation
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    set_err("HIP error '%s' uploading data", hipGetErrorString(e));
    ctx_free(c);
    delete c;
    return SGP_EHIP;
  }
  *out = c;
  return SGP_OK;
}

int sgp_ctx_destroy(sgp_ctx* c) {
  if (!c) return SGP_OK;
  if (c->multi) {
    multi_destroy(c->multi);
    delete c;
    return SGP_OK;
  }
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->aux) (void)hipStreamSynchronize(c->aux);
  if (c->aux_lo) (void)hipStreamSynchronize(c->aux_lo);
  ctx_free(c);
  delete c;
  return SGP_OK;
}

// Row-sharded multi-device context: shards = contiguous row blocks as dist.shard_rows, one per
// entry of `devices` (NULL: 0 .. nshards - 1; entries may repeat), reductions inside the library
// (multi.hip: device-side sums over a device's shards, RCCL all-reduce over the devices)
int sgp_ctx_create_multi(sgp_ctx** out, const int* devices, int nshards, const double* X,
                         int64_t n, int64_t ldx, int d, const double* y, const double* mu,
                         int64_t m_max) {
  if (!out || !X || !y || !mu || n < 1 || ldx < n || d < 1 || d > SGP_MAXD || m_max < 1 ||
      nshards < 1 || nshards > SGP_MAX_SHARDS || n < nshards) {
    set_err("invalid sgp_ctx_create_multi arguments (n=%lld, d=%d, m_max=%lld, nshards=%d; "
            "1 <= nshards <= min(n, %d))", (long long)n, d, (long long)m_max, nshards,
            SGP_MAX_SHARDS);
    return SGP_EINVAL;
  }
  *out = nullptr;
  if (devices)
    for (int k = 0; k < nshards; ++k)
      if (devices[k] < 0) {
        set_err("sgp_ctx_create_multi: device %d of shard %d", devices[k], k);
        return SGP_EINVAL;
      }
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  for (int k = 0; k < nshards; ++k) {
    const int dv = devices ? devices[k] : k;
    if (dv >= ndev) {
      set_err("sgp_ctx_create_multi: shard %d on device %d, but %d device(s) are visible", k, dv,
              ndev);
      return SGP_EINVAL;
    }
  }
  MultiCtx* mc = nullptr;
  const int st = multi_create(&mc, devices, nshards, X, n, ldx, d, y, mu, m_max);
  if (st) return st;
  sgp_ctx* c = new sgp_ctx();
  c->multi = mc;
  c->n = n;
  c->d = d;
  c->m_max = m_max;
  *out = c;
  return SGP_OK;
}

int sgp_ctx_shards(const sgp_ctx* c, int* nshards, int* ndevices) {
  if (!c) { set_err("context is NULL"); return SGP_EINVAL; }
  if (c->multi) return multi_shards(c->multi, nshards, ndevices);
  if (nshards) *nshards = 1;
  if (ndevices) *ndevices = 1;
  return SGP_OK;
}

int sgp_ctx_set_stream(sgp_ctx* c, void* s) {
  MULTI_REFUSE(c, "sgp_ctx_set_stream");
  if (!c) { set_err("context is NULL"); return SGP_EINVAL; }
  c->stream = s ? (hipStream_t)s : c->own;
  return SGP_OK;
}

int sgp_ctx_set_data(sgp_ctx* c, const double* y, const double* mu) {
  MULTI_FWD(c, y && mu ? multi_set_data(c->multi, y, mu) : multi_bad_args());
  if (!c || !y || !mu) { set_err("invalid arguments"); return SGP_EINVAL; }
  HIPCHK(hipSetDevice(c->device));
  std::vector<double> hr((size_t)c->n_pad, 0.0);
  for (int64_t i = 0; i < c->n; ++i) hr[(size_t)i] = y[i] - mu[i];
  HIPCHK(hipMemcpyAsync(c->r, hr.data(), sizeof(double) * hr.size(), hipMemcpyHostToDevice,
                        c->stream));
  HIPCHK(launch_dot(c->r, c->r, c->n_pad, c->slab_aux, c->rr_dev, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(upload_rows(c->y, y, c->n, c->n_pad));
  HIPCHK(upload_rows(c->mu, mu, c->n, c->n_pad));
  return SGP_OK;
}

int64_t sgp_ctx_rows(const sgp_ctx* c) { return c ? c->n : -1; }

int sgp_ctx_enable_timing(sgp_ctx* c, int enable) {
  MULTI_FWD(c, sgp_ctx_enable_timing(multi_lead(c->multi), enable));
  if (!c) return SGP_EINVAL;
  c->timing = enable != 0;
  if (c->timing) {
    c->timers.clear();
    c->pool_used = 0;
    c->timing_evals = 0;
    // events for the timed evaluations created here, not one pair per scope inside them
    // (hipEventCreate on the host between evaluations showed up at C2's 0.66 ms per step)
    while (c->pool.size() < kTimingPoolReserve) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) break;
      c->pool.push_back(e);
    }
  }
  return SGP_OK;
}

int sgp_ctx_timing_filter(sgp_ctx* c, const char* name) {
  MULTI_FWD(c, sgp_ctx_timing_filter(multi_lead(c->multi), name));
  if (!c) return SGP_EINVAL;
  c->timing_only = name ? name : "";
  return SGP_OK;
}

int64_t sgp_ctx_timing_evals(const sgp_ctx* c) {
  if (c && c->multi) return sgp_ctx_timing_evals(multi_lead(c->multi));
  return c ? c->timing_evals : -1;
}

int sgp_ctx_timings(sgp_ctx* c, char* names, int64_t names_len, double* ms, int max_n,
                    int* count) {
  MULTI_FWD(c, sgp_ctx_timings(multi_lead(c->multi), names, names_len, ms, max_n, count));
  if (!c || !count) return SGP_EINVAL;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipStreamSynchronize(c->aux));
  HIPCHK(hipStreamSynchronize(c->aux_lo));
  // per-phase totals over the recorded evaluations, in first-seen order
  std::vector<std::string> nm;
  std::vector<double> tot;
  for (const Timer& t : c->timers) {
    float v = 0.f;
    HIPCHK(hipEventElapsedTime(&v, t.a, t.b));
    size_t q = 0;
    while (q < nm.size() && nm[q] != t.name) ++q;
    if (q == nm.size()) {
      nm.push_back(t.name);
      tot.push_back(0.0);
    }
    tot[q] += v;
  }
  std::string all;
  int k = 0;
  for (size_t q = 0; q < nm.size() && k < max_n; ++q, ++k) {
    if (ms) ms[k] = tot[q];
    all += nm[q];
    all += '\n';
  }
  *count = k;
  if (names && names_len > 0) {
    strncpy(names, all.c_str(), (size_t)names_len - 1);
    names[names_len - 1] = 0;
  }
  return SGP_OK;
}

// ------------------------------------------------------------------------- VI phases
int64_t sgp_vi_red1_count(int64_t m) {
  const int64_t mp = round_up(m, SGP_TILE);
  return mp * mp + mp + 8;
}

int64_t sgp_vi_red2_count(int kernel, int d) { return num_ls(kernel, d) + 5; }

int64_t sgp_vi_red1_packed_count(int64_t m) {
  const int64_t mp = round_up(m, SGP_TILE);
  return syrk_packed_doubles(mp) + mp + 8;
}

int sgp_ctx_set_packed_reduction(sgp_ctx* c, int enable) {
  MULTI_REFUSE(c, "sgp_ctx_set_packed_reduction");
  if (!c) { set_err("context is NULL"); return SGP_EINVAL; }
  if (c->phase != 0) { set_err("cannot change the reduction layout inside an evaluation"); return SGP_EINVAL; }
  if (enable && !c->Sfull) {
    HIPCHK(hipSetDevice(c->device));
    int st = dalloc(&c->Sfull, c->mp_max * c->mp_max);
    if (st) return st;
  }
  c->pack_red1 = enable != 0;
  return SGP_OK;
}

// offset of t in VI's red1 (after S, full or packed); r'r follows t
static int64_t vi_red1_toff(const sgp_ctx* c, int64_t mp) {
  return c->pack_red1 ? syrk_packed_doubles(mp) : mp * mp;
}

int64_t sgp_knot_red_extra(int d, int64_t m) { return round_up(m, SGP_TILE) * d; }

// One K12 contraction pass: per-tile records summed into rec_out (L + 5 doubles) and, with
// knot gradients on, the per-knot column sums summed (or accumulated) into knot_out (mp x d).
static int contract_pass(sgp_ctx* c, const double* M, ConArgs ca, double* rec_out,
                         double* knot_out, bool knot_acc) {
  int64_t nrec = 0, nwg = 0;
  if (c->knot_on) ca.knot_slab = c->knot_slab;
  const bool fused = ca.uvec != nullptr && ca.alpha_in == nullptr;
  if (fused) ca.alpha_out = c->alpha;   // k_coinc needs the fused alpha_i
  // the balanced launch where the tile grid leaves a mostly idle last round (opt-in, see
  // con_sk_enabled)
  if (c->sk_ws) {
    if (++c->sk_epoch == 0) ++c->sk_epoch;   // 0 is the flags' initial value
    ca.sk_ws = c->sk_ws;
    ca.sk_flags = c->sk_flags;
    ca.sk_epoch = c->sk_epoch;
    ca.sk_slots = c->sk_slots;
    ca.sk_status = c->status + 3;
    ca.sk_dp = con_sk_dp();
  }
  HIPCHK(launch_contract_args(c->kp, c->K, M, c->X, c->n_pad, c->n, c->n_pad, c->U, c->mp, c->m,
                              c->mp, ca, c->slab_con, &nrec, &nwg, c->stream));
  // the per-tile records summed, and tau's coincidence sums added to record fields 1+L .. 3+L
  // (two launches); the rows that equal some knot depend only on (X, knot set): found by
  // hashing once per knot set (cflag written), later evaluations only revisit the flagged rows
  const bool flags_known = c->cflag_gen == c->knots_gen;
  HIPCHK(launch_records(c->slab_con, nrec, nwg, c->X, c->n_pad, c->n, c->kp.d, c->U, c->mp, c->m,
                        c->khash, c->kidx, c->K, c->mp, M, ca, fused ? c->alpha : ca.alpha_in,
                        c->slab_small, c->slab_small_cap, 1 + c->kp.L, rec_out, c->cflag,
                        flags_known ? 2 : 1, c->stream, c->defer_rec ? &c->rec_defer : nullptr));
  c->cflag_gen = c->knots_gen;
  if (c->knot_on)
    HIPCHK(launch_knot_reduce(c->knot_slab, c->n_pad / SGP_TILE, c->mp, c->kp.d, c->knot_part,
                              KNOT_PART_ROWS * c->mp_max * c->d,
                              knot_out, knot_acc, c->stream));
  return SGP_OK;
}

// d F / d u_kc = sum_i G_ik dK12_ik/du_kc + <G22, dK22/du_kc> (the knot branches of
// delbo_dcov_par / dlogp_dcov_par / dlogq_dcov_par, vi_functions.R:425-593): combines the
// reduced K12 part (knot_red, device) with the m x m part into c->knot_raw.
static int knot_finish(sgp_ctx* c, const double* knot_red, const double* uvec, const double* Ainv,
                       const double* Binv, const double* M3, double a, double b, double cc,
                       const double* v, const double* w, double e2) {
  if (!c->knot_on) return SGP_OK;
  const KernParams& kp = c->kp;
  const int64_t m = c->m, d = kp.d;
  HIPCHK(launch_knot_kmm(kp, c->U, c->mp, m, c->mp, uvec, Ainv, Binv, M3, a, b, cc, v, w, e2,
                         c->knot_kmm, c->stream));
  std::vector<double> h12((size_t)(m * d)), h22((size_t)(m * d));
  HIPCHK(hipMemcpyAsync(h12.data(), knot_red, sizeof(double) * m * d, hipMemcpyDeviceToHost,
                        c->stream));
  HIPCHK(hipMemcpyAsync(h22.data(), c->knot_kmm, sizeof(double) * m * d, hipMemcpyDeviceToHost,
                        c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  c->knot_raw.assign((size_t)(m * d), 0.0);
  const bool ard = kp.kernel == SGP_KERNEL_ARD;
  for (int64_t k = 0; k < m; ++k)
    for (int q = 0; q < d; ++q) {
      // the K12 part carries (x - u)/l_c (ARD) or (x - u) (sqexp); the m x m part raw u - u
      const double f12 = ard ? kp.rl[q] : kp.rl2[0];
      c->knot_raw[(size_t)(k * d + q)] =
          h12[(size_t)(k * d + q)] * f12 + h22[(size_t)(k * d + q)] * kp.rl2[q];
    }
  return SGP_OK;
}

int sgp_ctx_enable_knot_grad(sgp_ctx* c, int enable) {
  MULTI_FWD(c, multi_enable_knot_grad(c->multi, enable));
  if (!c) { set_err("context is NULL"); return SGP_EINVAL; }
  if (!enable) { c->knot_on = false; return SGP_OK; }
  HIPCHK(hipSetDevice(c->device));
  if (!c->knot_slab) {
    int st = dalloc(&c->knot_slab, (c->n_pad / SGP_TILE) * c->mp_max * c->d);
    st = st ? st : dalloc(&c->knot_part, KNOT_PART_ROWS * c->mp_max * c->d);
    st = st ? st : dalloc(&c->knot_kmm, c->mp_max * c->d);
    if (st) return st;
  }
  c->knot_on = true;
  return SGP_OK;
}

int sgp_ctx_row_bounds(sgp_ctx* c, double* lo, double* hi) {
  MULTI_FWD(c, lo && hi ? multi_row_bounds(c->multi, lo, hi) : multi_bad_args());
  if (!c || !lo || !hi) { set_err("invalid arguments"); return SGP_EINVAL; }
  for (int q = 0; q < c->d; ++q) {
    lo[q] = c->xmin[(size_t)q];
    hi[q] = c->xmax[(size_t)q];
  }
  return SGP_OK;
}

int sgp_knot_gradient(sgp_ctx* c, const double* bounds, double* grad_knot) {
  MULTI_FWD(c, grad_knot ? multi_knot_gradient(c->multi, bounds, grad_knot) : multi_bad_args());
  if (!c || !grad_knot) { set_err("invalid arguments"); return SGP_EINVAL; }
  const int64_t m = c->m, d = c->d;
  if (c->knot_raw.size() != (size_t)(m * d) || c->last_mode == 0) {
    set_err("no knot gradient: enable it with sgp_ctx_enable_knot_grad before the evaluation");
    return SGP_EINVAL;
  }
  if (!bounds && c->last_mode != 3 && c->n_global > c->n) {
    // the default bounds are this context's row range, which differs between the ranks of a
    // row-sharded evaluation: the caller must pass the bounds of the whole data set
    set_err("row-sharded context (n_global %lld > local rows %lld): pass the global knot bounds",
            (long long)c->n_global, (long long)c->n);
    return SGP_EINVAL;
  }
  std::vector<double> lb((size_t)d), ub((size_t)d);
  for (int q = 0; q < d; ++q) {
    if (bounds) {
      lb[(size_t)q] = bounds[q];
      ub[(size_t)q] = bounds[d + q];
    } else {   // vi_functions.R:175-178: column range of xy widened by a tenth on each side
      const double diff = c->xmax[(size_t)q] - c->xmin[(size_t)q];
      lb[(size_t)q] = c->xmin[(size_t)q] - diff / 10;
      ub[(size_t)q] = c->xmax[(size_t)q] + diff / 10;
    }
  }
  // dsqexp_dx2(_ard) transform = TRUE factor dx2_dx2t (covariance_function_derivatives.R:186)
  for (int64_t k = 0; k < m; ++k)
    for (int q = 0; q < d; ++q) {
      const double u = c->hU[(size_t)(k + q * m)];
      const double chain = (ub[(size_t)q] - lb[(size_t)q]) /
                           (((u - lb[(size_t)q]) * (ub[(size_t)q] - u)) + 1e-4);
      grad_knot[k * d + q] = c->knot_raw[(size_t)(k * d + q)] * chain;
    }
  return SGP_OK;
}

static int k22_sync(sgp_ctx* c);
static int k22_launch(sgp_ctx* c, double diag_sub);
static int k22_build(sgp_ctx* c, double diag_sub);
static int k22_factor(sgp_ctx* c, bool after_main);
static int k22_stage(sgp_ctx* c, double diag_sub) {
  int st = k22_sync(c);
  return st ? st : k22_launch(c, diag_sub);
}

int sgp_vi_phase1(sgp_ctx* c, int kernel, const double* theta, const double* U, int64_t m,
                  int64_t ldu, double delta, double* red1) {
  MULTI_REFUSE(c, "sgp_vi_phase1");
  KernParams kp;
  int st = check_eval_args(c, kernel, theta, U, m, ldu, delta, &kp);
  if (st) return st;
  if (!red1) { set_err("red1 is NULL"); return SGP_EINVAL; }
  HIPCHK(hipSetDevice(c->device));
  st = drain_abandoned(c);
  if (st) return st;
  timers_reset(c);
  c->kp = kp;
  c->m = m;
  c->mp = round_up(m, SGP_TILE);
  c->delta = delta;
  st = upload_knots(c, U, m, ldu);
  if (st) return st;
  const int64_t mpv = c->mp, mmv = mpv * mpv;
  int64_t t_rows = 0;
  // mp = 256 (C2): the fragment-balanced SYRK finishes ~35 us sooner, and the side work that
  // the main stream waited for on aux_lo (t's partial sums, r^T r, red1's zeroing), starved of
  // CUs beside the SYRK, would then sit on the critical path; instead t is summed on the main
  // stream right after the SYRK (a free GPU: two short launches), r^T r is the context's
  // precomputed constant, red1 needs no zeroing (S, t, rr are all written), and phase 2 waits
  // for K22's build itself
  const bool small_syrk = syrk_use_s256(mpv, false);
  c->vi_k22_ordered = !small_syrk;
  c->t_deferred = false;
  {
    // K12, and t = K^T r riding along in the memory-bound builder (keeps the SYRK's
    // diagonal tiles as cheap as the others); the first HIP call of the evaluation, so the
    // GPU starts on it as soon as the host gets here
    Scope t(c, "build_knm");
    if (SGP_VI_BUILD_NO_T)
      HIPCHK(launch_build_knm(kp, c->X, c->n_pad, c->n, c->n_pad, c->U, mpv, m, mpv, c->K,
                              c->stream, false));
    else
      HIPCHK(launch_build_knm_t(kp, c->X, c->n_pad, c->n, c->n_pad, c->U, mpv, m, mpv, c->K,
                                c->r, c->tslab, &t_rows, c->stream, false));
  }
  // ev_knots after the builder: aux may build K22 from here on (first needed by phase 2), and
  // aux_lo may reduce the builder's t partials.  The SYRK goes right behind the builder (it
  // needs only K12); red1's reset and the small t / rr reductions run on aux_lo beside it
  // instead of between the two on the main stream, where at small n (C2) the GPU idled while
  // the host issued them one by one
  st = k22_sync(c);
  if (st) return st;
  {
    Scope t(c, "syrk");
    HIPCHK(launch_syrk_aug(c->K, c->n_pad, mpv, c->r, nullptr, c->slab_syrk, c->slab_syrk_cap,
                           red1, c->stream, 1, nullptr, 0));
  }
  // K22 itself only (aux); its inverse runs in phase 2 beside the Bm inverse -- nothing in
  // phase 1 needs it, and the latency-bound chain no longer gates the one-round SYRK or shares
  // the CUs with the builder
  // status / scalar resets on aux ahead of K22's build: the K22 chain (aux; at small n queued
  // right behind the build) is their first writer, phase 2 (main, behind ev_lo, which covers
  // ev_k22m) the next.  (On aux_lo they raced the small-n chain.)
  HIPCHK(hipMemsetAsync(c->status, 0, sizeof(int) * 4, c->aux));
  HIPCHK(hipMemsetAsync(c->sc, 0, sizeof(double) * SC_N, c->aux));
  st = k22_build(c, kp.tau2);
  if (st) return st;
  // red1 = [S (full, or its packed lower 64-blocks), t, r'r]
  const int64_t toff = vi_red1_toff(c, mpv);
  if (small_syrk && c->fused_vi) {
    c->t_deferred = true;   // summed on aux_lo in phase 2
    c->t_rows_def = t_rows;
  } else if (small_syrk) {
    HIPCHK(launch_knot_reduce(c->tslab, t_rows, mpv, 1, c->T1, c->mp_max * c->mp_max,
                              red1 + toff, false, c->stream));
  } else {
    // aux_lo, after the builder: red1's zeroing (before the SYRK reduction below writes S and
    // r^T r into it: the main stream waits for ev_lo) and t
    HIPCHK(hipStreamWaitEvent(c->aux_lo, c->ev_knots, 0));
    HIPCHK(hipMemsetAsync(red1, 0, sizeof(double) * (toff + mpv + 8), c->aux_lo));
    HIPCHK(launch_knot_reduce(c->tslab, t_rows, mpv, 1, c->T1, c->mp_max * c->mp_max,
                              red1 + toff, false, c->aux_lo));
    // ev_lo also covers K22's build (aux): the main stream, which waits for ev_lo here, needs
    // no second cross-stream wait before forming Bm = K22 + S/z in phase 2 (bm_stage)
    HIPCHK(hipStreamWaitEvent(c->aux_lo, c->ev_k22m, 0));
    HIPCHK(hipEventRecord(c->ev_lo, c->aux_lo));
    HIPCHK(hipStreamWaitEvent(c->stream, c->ev_lo, 0));
  }
  {
    // S into red1, and r^T r (the context's constant; the 7 words past it zeroed)
    Scope t(c, "syrk_reduce");
    HIPCHK(launch_syrk_aug(c->K, c->n_pad, mpv, c->r, nullptr, c->slab_syrk, c->slab_syrk_cap,
                           red1, c->stream, 2, nullptr, 0, c->rr_dev, c->pack_red1, false,
                           c->rsync));
  }
  // K22's inverse (aux) is queued behind the SYRK here rather than in phase 2: it needs only
  // theta and U, so with several ranks it runs while the first all-reduce is in flight (the
  // caller issues it on the main stream between the phases); alone it starts where it did
  // Small SYRKs (C2: n m^2 = 6.6e9): the chain is queued right behind K22's build, not behind
  // the SYRK; its workgroups still find no slots until the one-round SYRK ends, and the
  // cross-stream event wait it saves was ~20 us of C2's critical path (1376 -> 1423 evals/s,
  // profiles/r3/k22_nowait_ab.txt).  At C3 and the 8-GPU shard the same change was neutral
  // overall but slowed the phase-2 chains by ~0.03 ms, so they keep the wait.
  const bool k22_after_syrk = (double)c->n_pad * (double)mpv * (double)mpv > 3e10;
  st = k22_factor(c, k22_after_syrk);
  if (st) return st;
  c->phase = 1;
  return SGP_OK;
}

static int k22_factor_launches(sgp_ctx* c, hipStream_t s) {
  const int64_t mp = c->mp;
  // K22inv holds a copy of K22 already (k22_build writes both)
  HIPCHK(dense_spd_inverse(c->K22inv, mp, c->Xt22, c->dinv22, c->logd22, c->status,
                           c->gjs + SGP_GJ_SYNC_WORDS, s));
  HIPCHK(launch_sum_and_diag(c->logd22, mp / SGP_DB, c->sc + SC_LD22, c->K22inv, mp, mp,
                             c->cdiag, s));
  return SGP_OK;
}

// K22 = Kuu + (tau^2 + delta - diag_sub) I factored and inverted on the aux stream.  It
// depends only on (U, theta), so it runs concurrently with phase 1's memory-bound builder; the
// SYRK (whose grid fills exactly one residency round) waits for it.  A pristine copy of K22
// goes to Bm for phase 2.
// The aux stream's K22 work may start once the knots (and the status/scalar resets) are on
// the main stream.  Split from the launches so that callers can enqueue the K12 builder on the
// main stream first: the chain's ~20 launches cost the host ~0.2 ms, which otherwise delayed
// the builder's start by as much.
static int k22_sync(sgp_ctx* c) {
  HIPCHK(hipEventRecord(c->ev_knots, c->stream));
  HIPCHK(hipStreamWaitEvent(c->aux, c->ev_knots, 0));
  return SGP_OK;
}

// K22 = Kuu + (tau^2 + delta - diag_sub) I on aux (ev_k22m), and its factorisation/inverse
// after it on aux (ev_k22).  VI runs the two halves in different phases.
static int k22_build(sgp_ctx* c, double diag_sub) {
  HIPCHK(launch_build_kmm(c->kp, c->U, c->mp, c->m, c->mp, diag_sub, c->K22, c->aux,
                          c->K22inv));   // and the copy the in-place inverse starts from
  HIPCHK(hipEventRecord(c->ev_k22m, c->aux));
  return SGP_OK;
}

static int k22_factor(sgp_ctx* c, bool after_main = false) {
  if (after_main) {   // not before the main stream's queued work (VI: the one-round SYRK)
    HIPCHK(hipEventRecord(c->ev_s, c->stream));
    HIPCHK(hipStreamWaitEvent(c->aux, c->ev_s, 0));
  }
  Scope t(c, "k22_aux", c->aux);
  int st = k22_factor_launches(c, c->aux);
  if (st) return st;
  HIPCHK(hipEventRecord(c->ev_k22, c->aux));
  return SGP_OK;
}

static int k22_launch(sgp_ctx* c, double diag_sub) {
  int st = k22_build(c, diag_sub);
  return st ? st : k22_factor(c, false);
}

// Binv = (K22 + S * s_scale)^-1 (one Gauss-Jordan launch per pivot; the sum is formed by the
// chain's first pivot and step as they read K22 and S)
// logdet_later: the caller sums the pivots' log-determinants itself (VI: on aux_lo, where only
// the finish waits for it, instead of one more launch between the chain and the m-vectors)
static int bm_stage(sgp_ctx* c, const double* S, double s_scale, bool k22_ordered = false,
                    bool logdet_later = false) {
  const int64_t mp = c->mp;
  Scope t(c, "dense_bm");
  if (!k22_ordered)   // Bm needs K22, not its inverse (VI: ordered through phase 1's ev_lo)
    HIPCHK(hipStreamWaitEvent(c->stream, c->ev_k22m, 0));
  HIPCHK(dense_spd_inverse_sum(c->K22, s_scale, S, c->Binv, mp, c->Xt, c->dinv, c->logdB,
                               c->status + 1, c->gjs, c->stream));
  if (!logdet_later) HIPCHK(launch_sum_small(c->logdB, mp / SGP_DB, c->sc + SC_LDB, c->stream));
  return SGP_OK;
}

int sgp_vi_phase2(sgp_ctx* c, const double* red1, int64_t n_global, unsigned flags,
                  double* red2) {
  MULTI_REFUSE(c, "sgp_vi_phase2");
  if (!c || !red1 || !red2) { set_err("invalid arguments"); return SGP_EINVAL; }
  if (c->phase != 1) { set_err("sgp_vi_phase2 called before sgp_vi_phase1"); return SGP_EINVAL; }
  if (n_global < c->n) { set_err("n_global < local rows"); return SGP_EINVAL; }
  HIPCHK(hipSetDevice(c->device));
  const KernParams& kp = c->kp;
  const int64_t mp = c->mp, mm = mp * mp;
  const double z = kp.tau2 + c->delta;
  const double* S = red1;
  const int64_t toff = vi_red1_toff(c, mp);
  const double* t = red1 + toff;
  c->n_global = n_global;
  c->flags = flags;
  if (c->pack_red1) {   // the summed packed blocks -> full S (m x m consumers below)
    HIPCHK(launch_unpack_lower64(red1, mp, c->Sfull, c->stream));
    S = c->Sfull;
  }
  // K22's inverse (queued on aux at the end of phase 1) runs concurrently with Bm's on the
  // main stream.  The Bm chain is enqueued before the side work below: the host's issue of
  // the aux_lo launches first left the GPU idle ~20 us between phase 1's last kernel and the
  // chain at C2 (kernel trace)
  HIPCHK(hipEventRecord(c->ev_s, c->stream));   // S (red1, summed) is ready
  // K22's build ordered by phase 1's ev_lo (or waited for here when phase 1 had no side work)
  const bool obj_only = (flags & SGP_FLAG_OBJ_ONLY) != 0;
  int st = bm_stage(c, S, 1.0 / z, c->vi_k22_ordered, !obj_only);
  if (st) return st;
  {
    // tr(K22inv S) and M3 = K22inv S K22inv need S and K22inv only: on aux_lo beside the Bm
    // inversion (T22 and K22inv are final once the K22 chain on `aux` has finished).  Beside
    // the K12 contraction instead, the GEMMs' workgroups starved and slowed it more.
    HIPCHK(hipStreamWaitEvent(c->aux_lo, c->ev_s, 0));
    if (c->t_deferred) {   // t = K^T r from the builder's partials (phase 1 deferred it; only
                           // sgp_eval_vi does, whose red1 is the context's own)
      HIPCHK(launch_knot_reduce(c->tslab, c->t_rows_def, mp, 1, c->T1, c->mp_max * c->mp_max,
                                c->red1 + toff, false, c->aux_lo));
    }
    HIPCHK(hipStreamWaitEvent(c->aux_lo, c->ev_k22, 0));
    // ev_t: t summed AND K22's inverse done -- the m-vectors then wait on one event, not two
    // (each cross-stream wait in front of them cost the critical path several us at C2)
    if (c->t_deferred) HIPCHK(hipEventRecord(c->ev_t, c->aux_lo));
    Scope ta(c, "m3_aux", c->aux_lo);
    HIPCHK(launch_dot(c->K22inv, S, mm, c->slab_aux, c->sc + SC_TRKS, c->aux_lo));
    if (!(flags & SGP_FLAG_OBJ_ONLY)) {
      HIPCHK(launch_gemm64(false, false, false, mp, mp, mp, 1.0, c->K22inv, mp, S, mp, 0.0,
                           c->T22, mp, c->aux_lo));
      HIPCHK(launch_gemm64(false, false, false, mp, mp, mp, 1.0, c->T22, mp, c->K22inv, mp, 0.0,
                           c->M3, mp, c->aux_lo));
    } else {
      HIPCHK(hipEventRecord(c->ev_m3, c->aux_lo));
    }
  }
  {
    Scope tm(c, "mm_vectors");
    const bool k22_via_t = c->t_deferred;   // ev_t covers K22's inverse too
    if (c->t_deferred) {
      HIPCHK(hipStreamWaitEvent(c->stream, c->ev_t, 0));
      c->t_deferred = false;
    }
    if (flags & SGP_FLAG_OBJ_ONLY) {   // elbo_fun alone: no adjoint work
      HIPCHK(dense_gemv(c->Binv, mp, t, 1.0 / z, c->uvec, c->stream));       // u = Binv t / z
      HIPCHK(launch_dot(t, c->uvec, mp, c->slab_small, c->sc + SC_TU, c->stream));
      HIPCHK(hipMemcpyAsync(c->sc + SC_RR, red1 + toff + mp, sizeof(double),
                            hipMemcpyDeviceToDevice, c->stream));
      HIPCHK(hipStreamWaitEvent(c->stream, c->ev_m3, 0));
      c->phase = 2;
      return SGP_OK;
    }
    // u = Binv t / z, P = tau^-2 K22inv - z^-1 Binv and tr(Binv S)'s row terms in one launch
    // between the Bm chain and the contraction (the critical path); t.u, tr(Binv S) and r^T r
    // on aux_lo below (only the finish reads them)
    if (!k22_via_t) HIPCHK(hipStreamWaitEvent(c->stream, c->ev_k22, 0));
    HIPCHK(launch_vi_mm_rows(c->Binv, c->K22inv, S, t, mp, 1.0 / z, 1.0 / kp.tau2, -1.0 / z,
                             c->uvec, c->Pm, c->mmpart, c->stream));
    HIPCHK(hipEventRecord(c->ev_bm, c->stream));
  }
  {
    // sum G22 o dK22/dtheta needs only m x m operands: on aux_lo beside the K12 contraction
    // (off the critical path; joined before the phase ends)
    HIPCHK(hipStreamWaitEvent(c->aux_lo, c->ev_bm, 0));
    HIPCHK(launch_vi_mm_scalars(t, c->uvec, c->mmpart, mp, red1 + toff + mp, c->sc + SC_TU,
                                c->sc + SC_TRBS, c->sc + SC_RR, c->aux_lo));
    HIPCHK(launch_sum_small(c->logdB, mp / SGP_DB, c->sc + SC_LDB, c->aux_lo));   // bm_stage's
    Scope tm(c, "contract_kmm", c->aux_lo);
    int nb = 0;
    HIPCHK(launch_contract_kmm(kp, c->U, c->mp, c->m, mp, c->uvec, c->K22inv, c->Binv, c->M3,
                               -0.5, 0.5, -1.0 / (2.0 * kp.tau2), nullptr, nullptr, 0.0,
                               c->slab_aux, c->slab_small_cap, &nb, c->aux_lo));
    HIPCHK(launch_colsum(c->slab_aux, nb, kp.P, c->sc + SC_G22, c->aux_lo));
    HIPCHK(hipEventRecord(c->ev_m3, c->aux_lo));
  }
  {
    Scope tm(c, "contract_knm");
    ConArgs ca;
    ca.r = c->r;
    ca.invz = 1.0 / z;
    ca.uvec = c->uvec;
    ca.cdiag = c->cdiag;
    ca.count_a2 = 1;
    int st2 = contract_pass(c, c->Pm, ca, red2, red2 + sgp_vi_red2_count(kp.kernel, kp.d), false);
    if (st2) return st2;
  }
  HIPCHK(hipStreamWaitEvent(c->stream, c->ev_m3, 0));   // G22 records (aux_lo)
  c->phase = 2;
  return SGP_OK;
}

int sgp_vi_finish(sgp_ctx* c, const double* red2, double* obj, double* grad) {
  MULTI_REFUSE(c, "sgp_vi_finish");
  const bool obj_only = c && (c->flags & SGP_FLAG_OBJ_ONLY);
  if (!c || !red2 || !obj || (!grad && !obj_only)) {
    set_err("invalid arguments");
    return SGP_EINVAL;
  }
  if (c->phase != 2) { set_err("sgp_vi_finish called before sgp_vi_phase2"); return SGP_EINVAL; }
  {
    const hipError_t e = hipSetDevice(c->device);
    if (e != hipSuccess) {
      // the evaluation is abandoned: no later readback may replay its deferred record pass
      c->rec_defer = RecPass2{};
      c->phase = 0;
      set_err("HIP error '%s' in hipSetDevice", hipGetErrorString(e));
      return SGP_EHIP;
    }
  }
  const KernParams& kp = c->kp;
  const int L = kp.L;
  double sc[SC_N], r2[SGP_MAXD + 8];
  int status[4];
  const int64_t n2 = sgp_vi_red2_count(kp.kernel, kp.d);
  {
    Readback rb(c);
    HIPCHK(rb.add(sc, c->sc, sizeof(sc)));
    if (!obj_only) HIPCHK(rb.add(r2, red2, sizeof(double) * n2));
    HIPCHK(rb.add(status, c->status, sizeof(status)));
    HIPCHK(rb.wait());
  }
  c->phase = 0;
  if (chain_watchdog(status)) return SGP_EHIP;
  if (status[0] || status[1]) {
    set_err("chol(): the leading minor of order %d of %s is not positive definite",
            status[0] ? status[0] : status[1],
            status[0] ? "Sigma22" : "Sigma22 + t(Sigma12) %*% ZSig12");
    return SGP_ENOTPD;
  }
  c->last_mode = 1;
  if (getenv("SGP_DEBUG_SC")) {
    fprintf(stderr, "[sgp sc] ld22 %.17g ldB %.17g tu %.17g trKS %.17g trBS %.17g rr %.17g g22",
            sc[SC_LD22], sc[SC_LDB], sc[SC_TU], sc[SC_TRKS], sc[SC_TRBS], sc[SC_RR]);
    for (int q = 0; q < kp.P; ++q) fprintf(stderr, " %.17g", sc[SC_G22 + q]);
    fprintf(stderr, "\n");
  }
  const double n = (double)c->n_global;
  const double z = kp.tau2 + c->delta;
  const double ld22 = 2.0 * sc[SC_LD22], ldB = 2.0 * sc[SC_LDB];
  const double rr = sc[SC_RR], tu = sc[SC_TU], trKS = sc[SC_TRKS], trBS = sc[SC_TRBS];
  // elbo_fun (vi_functions.R:102-118)
  const double quad = -0.5 * rr / z + 0.5 * tu / z;
  const double logdet22 = (c->flags & SGP_FLAG_R_DET) ? log(exp(ld22)) : ld22;
  const double det_part = -0.5 * (n * log(z) - logdet22 + ldB);
  const double trace_term = -(1.0 / (2.0 * kp.tau2)) * (n * (kp.sig2 + c->delta) - trKS);
  *obj = quad + det_part - (n / 2.0) * log(2.0 * M_PI) + trace_term;
  if (obj_only) {
    c->knot_raw.clear();
    return SGP_OK;
  }
  // delbo_dcov_par (vi_functions.R:259-419) in adjoint form
  // red2 = [e_sig, e_l(L), c_sum, c_cnt, c_dg, alpha^T alpha]
  const double e_sig = r2[0];
  const double c_sum = r2[1 + L], c_cnt = r2[2 + L], c_dg = r2[3 + L], aTa = r2[4 + L];
  const double trSinv = n / z - trBS / (z * z);
  const double trW = 0.5 * (aTa - trSinv);
  grad[0] = 2.0 * e_sig + sc[SC_G22] - n * kp.sig2 / kp.tau2;
  for (int q = 0; q < L; ++q) grad[1 + q] = r2[1 + q] + sc[SC_G22 + 1 + q];
  grad[L + 1] = 2.0 * kp.tau2 * (c_sum - (c_cnt - c->delta * c_dg) / kp.tau2) +
                2.0 * kp.tau2 * trW - 2.0 * trace_term;
  return knot_finish(c, red2 + n2, c->uvec, c->K22inv, c->Binv, c->M3, -0.5, 0.5,
                     -1.0 / (2.0 * kp.tau2), nullptr, nullptr, 0.0);
}

int sgp_eval_vi(sgp_ctx* c, int kernel, const double* theta, const double* U, int64_t m,
                int64_t ldu, double delta, unsigned flags, double* obj, double* grad) {
  MULTI_FWD(c, obj && (grad || (flags & SGP_FLAG_OBJ_ONLY)) ? multi_eval_vi(c->multi, kernel, theta, U, m, ldu, delta, flags, obj, grad) : multi_bad_args());
  if (!c) { set_err("context is NULL"); return SGP_EINVAL; }
  // sgp_vi_finish's own argument checks must not be the first to fail: phase 2 below defers the
  // records' second pass to finish's readback, and an early return there would leave it queued
  if (!obj || (!grad && !(flags & SGP_FLAG_OBJ_ONLY))) {
    set_err("obj is NULL, or grad is NULL without SGP_FLAG_OBJ_ONLY");
    return SGP_EINVAL;
  }
#ifdef SGP_HOST_PROBE
  hp_t0 = hp_now();
  sgp_probe_t[0] = hp_t0;
  if (hp_prev_end > 0.0) hp_gap += hp_t0 - hp_prev_end;
#endif
  c->fused_vi = true;   // nothing reduces red1 between the phases
  int st = sgp_vi_phase1(c, kernel, theta, U, m, ldu, delta, c->red1);
  c->fused_vi = false;
  if (st) return st;
  c->rec_defer = RecPass2{};
  c->defer_rec = true;   // the records' pass 2 runs in sgp_vi_finish's readback kernel
  st = sgp_vi_phase2(c, c->red1, c->n, flags, c->red2);
  c->defer_rec = false;
  if (st) {
    c->rec_defer = RecPass2{};
    return st;
  }
#ifdef SGP_HOST_PROBE
  const int fst = sgp_vi_finish(c, c->red2, obj, grad);
  const double t3 = hp_now();
  sgp_probe_t[3] = t3;
  hp_prev_end = t3;
  hp_tail = t3 - hp_tail;
  static double tail_sum = 0.0;
  tail_sum += hp_tail;
  if (++hp_n % 200 == 0) {
    fprintf(stderr, "[host probe] %ld evals: issue %.1f us, sync wait %.1f us, after sync %.1f us, "
            "caller gap %.1f us per eval\n", hp_n, 1e6 * hp_issue / 200, 1e6 * hp_wait / 200,
            1e6 * tail_sum / 200, 1e6 * hp_gap / 200);
    hp_issue = hp_wait = hp_gap = tail_sum = 0.0;
  }
  return fst;
#else
  return sgp_vi_finish(c, c->red2, obj, grad);
#endif
}

// ------------------------------------------------------------------------- FITC phases
// obj_fun_norm (laplace_approx_obj_funs.R:6-52) + dlogp_dcov_par (laplace_approx_gradient.R:
// 720-971) in adjoint form.  Z = sigma^2 + tau^2 + delta - q,
// q_i = K_i K22^-1 K_i^T, D = diag(Z), S_D = K^T D^-1 K, Bm = K22 + S_D, u = Bm^-1 K^T D^-1 r,
// alpha = D^-1 (r - K u), omega_i = alpha_i^2 - (Sigma^-1)_ii,
// G = alpha u^T - D^-1 K Bm^-1 - diag(omega) K K22^-1,
// G22 = -1/2 u u^T + 1/2 (K22^-1 - Bm^-1) + 1/2 K22^-1 S_omega K22^-1.
// red1 = [S_D (mp^2), t (mp), r^T D^-1 r, sum log Z]
// red2 = [S_omega (mp^2), t_omega (mp), rr_omega, sum omega, rec_1 (L+5), rec_2 (L+5)]
int64_t sgp_fitc_red1_count(int64_t m) { return sgp_vi_red1_count(m); }

int64_t sgp_fitc_red2_count(int kernel, int d, int64_t m) {
  const int64_t mp = round_up(m, SGP_TILE);
  return mp * mp + mp + 8 + 2 * (num_ls(kernel, d) + 5);
}

static int64_t fitc_rec_off(int64_t mp) { return mp * mp + mp + 8; }

int sgp_fitc_phase1(sgp_ctx* c, int kernel, const double* theta, const double* U, int64_t m,
                    int64_t ldu, double delta, double* red1) {
  MULTI_REFUSE(c, "sgp_fitc_phase1");
  KernParams kp;
  int st = check_eval_args(c, kernel, theta, U, m, ldu, delta, &kp);
  if (st) return st;
  if (!red1) { set_err("red1 is NULL"); return SGP_EINVAL; }
  HIPCHK(hipSetDevice(c->device));
  st = drain_abandoned(c);
  if (st) return st;
  timers_reset(c);
  c->kp = kp;
  c->m = m;
  c->mp = round_up(m, SGP_TILE);
  c->delta = delta;
  const int64_t mp = c->mp, mm = mp * mp;
  st = upload_knots(c, U, m, ldu);
  if (st) return st;
  HIPCHK(hipMemsetAsync(c->status, 0, sizeof(int) * 4, c->stream));
  HIPCHK(hipMemsetAsync(c->sc, 0, sizeof(double) * SC_N, c->stream));
  st = k22_sync(c);
  if (st) return st;
  {
    Scope t(c, "build_knm");
    HIPCHK(launch_build_knm(kp, c->X, c->n_pad, c->n, c->n_pad, c->U, c->mp, m, mp, c->K,
                            c->stream, true));   // beside the K22 chain on aux
  }
  st = k22_launch(c, kp.tau2);   // K22 = Kuu + delta I, same as the VI path (laplace_gradient_ascent.R:1238-1257)
  if (st) return st;
  HIPCHK(hipMemsetAsync(red1, 0, sizeof(double) * sgp_fitc_red1_count(m), c->stream));
  HIPCHK(hipStreamWaitEvent(c->stream, c->ev_k22, 0));
  {
    Scope t(c, "rowquad_q");
    HIPCHK(launch_rowquad_knm(kp, c->K, c->K22inv, c->n, c->n_pad, m, mp, c->r, 0.0, nullptr,
                              nullptr, nullptr, c->rowq, c->pvec, c->stream,
                              tstore_ready(c) ? c->tq : nullptr));
    int nb = 0;
    HIPCHK(launch_fitc_z(c->pvec, c->n, c->n_pad, kp.sig2 + kp.tau2 + delta, c->zinv,
                         c->slab_small, &nb, c->stream));
    HIPCHK(launch_colsum(c->slab_small, nb, 1, red1 + mm + mp + 1, c->stream));
  }
  {
    Scope t(c, "syrk");
    HIPCHK(launch_syrk_aug(c->K, c->n_pad, mp, c->r, c->zinv, c->slab_syrk, c->slab_syrk_cap,
                           red1, c->stream, 3));
  }
  c->phase = 11;
  return SGP_OK;
}

int sgp_fitc_phase2(sgp_ctx* c, const double* red1, int64_t n_global, unsigned flags,
                    double* red2) {
  MULTI_REFUSE(c, "sgp_fitc_phase2");
  if (!c || !red1 || !red2) { set_err("invalid arguments"); return SGP_EINVAL; }
  if (c->phase != 11) { set_err("sgp_fitc_phase2 called before sgp_fitc_phase1"); return SGP_EINVAL; }
  if (n_global < c->n) { set_err("n_global < local rows"); return SGP_EINVAL; }
  HIPCHK(hipSetDevice(c->device));
  const KernParams& kp = c->kp;
  const int64_t mp = c->mp, mm = mp * mp;
  const double* S = red1;
  const double* t = red1 + mm;
  c->n_global = n_global;
  c->flags = flags;
  int st = bm_stage(c, S, 1.0);
  if (st) return st;
  HIPCHK(hipMemsetAsync(red2, 0, sizeof(double) * (sgp_fitc_red2_count(kp.kernel, kp.d, c->m) +
                                                    (c->knot_on ? mp * kp.d : 0)),
                        c->stream));
  {
    Scope tm(c, "mm_vectors");
    HIPCHK(dense_gemv(c->Binv, mp, t, 1.0, c->uvec, c->stream));             // u = Bm^-1 t
    HIPCHK(launch_dot(t, c->uvec, mp, c->slab_small, c->sc + SC_TU, c->stream));
    HIPCHK(hipMemcpyAsync(c->sc + SC_RR, red1 + mm + mp, 2 * sizeof(double),
                          hipMemcpyDeviceToDevice, c->stream));               // rr_w, sum log Z
  }
  if (flags & SGP_FLAG_OBJ_ONLY) {   // obj_fun_norm alone
    c->phase = 12;
    return SGP_OK;
  }
  {
    Scope tm(c, "rowquad_p");
    HIPCHK(launch_rowquad_knm(kp, c->K, c->Binv, c->n, c->n_pad, c->m, mp, c->r, 0.0, c->zinv,
                              c->uvec, c->alpha, c->rowq, c->pvec, c->stream,
                              tstore_ready(c) ? c->tp : nullptr));
    int nb = 0;
    HIPCHK(launch_fitc_omega(c->alpha, c->zinv, c->pvec, c->n, c->n_pad, c->omega,
                             c->slab_small, &nb, c->stream));
    HIPCHK(launch_colsum(c->slab_small, nb, 1, red2 + mm + mp + 1, c->stream));
  }
  {
    Scope tm(c, "syrk_omega");
    HIPCHK(launch_syrk_aug(c->K, c->n_pad, mp, c->r, c->omega, c->slab_syrk, c->slab_syrk_cap,
                           red2, c->stream, 3, nullptr, 0));
    // the SYRK reduce wrote rr_omega at mm + mp; keep sum(omega) at mm + mp + 1
  }
  const int64_t off = fitc_rec_off(mp);
  const int64_t nrec = kp.L + 5;
  double* kout = red2 + off + 2 * nrec;
  {
    Scope tm(c, "contract_knm");
    // pass 1: G1 = alpha u^T - diag(1/Z) K Bm^-1
    ConArgs a1;
    a1.r = c->r;
    a1.invz_vec = c->zinv;
    a1.uvec = c->uvec;
    a1.rs_vec = c->zinv;
    a1.rs = -1.0;
    if (tstore_ready(c)) {   // K Bm^-1 and alpha were produced by rowquad_p
      a1.tin = c->tp;
      a1.alpha_in = c->alpha;
    }
    if (fuse_tt(c)) {
      // with both products stored, pass 2's term -diag(omega) K K22^-1 joins this pass (one
      // read of K instead of two; its records stay zero -- the finish sums the two sets)
      a1.tin2 = c->tq;
      a1.M2 = c->K22inv;
      a1.rs_vec2 = c->omega;
      a1.rs2 = -1.0;
    }
    st = contract_pass(c, c->Binv, a1, red2 + off, kout, false);
    if (st) return st;
  }
  if (!fuse_tt(c)) {
    Scope tm(c, "contract_knm_b");
    // pass 2: G2 = -diag(omega) K K22^-1
    ConArgs a2;
    a2.rs_vec = c->omega;
    a2.rs = -1.0;
    if (tstore_ready(c)) a2.tin = c->tq;   // K K22^-1 from phase 1's rowquad_q
    st = contract_pass(c, c->K22inv, a2, red2 + off + nrec, kout, true);
    if (st) return st;
  }
  c->phase = 12;
  return SGP_OK;
}

int sgp_fitc_finish(sgp_ctx* c, const double* red2, double* obj, double* grad) {
  MULTI_REFUSE(c, "sgp_fitc_finish");
  const bool obj_only = c && (c->flags & SGP_FLAG_OBJ_ONLY);
  if (!c || !red2 || !obj || (!grad && !obj_only)) {
    set_err("invalid arguments");
    return SGP_EINVAL;
  }
  if (c->phase != 12) { set_err("sgp_fitc_finish called before sgp_fitc_phase2"); return SGP_EINVAL; }
  HIPCHK(hipSetDevice(c->device));
  const KernParams& kp = c->kp;
  const int L = kp.L;
  const int64_t mp = c->mp;
  if (!obj_only) {
    Scope tm(c, "contract_kmm");
    // M3 = K22^-1 S_omega K22^-1 ; G22 = -1/2 uu^T + 1/2 (K22^-1 - Bm^-1) + 1/2 M3
    HIPCHK(launch_gemm64(false, false, false, mp, mp, mp, 1.0, c->K22inv, mp, red2, mp, 0.0,
                         c->T1, mp, c->stream));
    HIPCHK(launch_gemm64(false, false, false, mp, mp, mp, 1.0, c->T1, mp, c->K22inv, mp, 0.0,
                         c->M3, mp, c->stream));
    int nb = 0;
    HIPCHK(launch_contract_kmm(kp, c->U, c->mp, c->m, mp, c->uvec, c->K22inv, c->Binv, c->M3,
                               -0.5, 0.5, 0.5, nullptr, nullptr, 0.0, c->slab_small,
                               c->slab_small_cap, &nb, c->stream));
    HIPCHK(launch_colsum(c->slab_small, nb, kp.P, c->sc + SC_G22, c->stream));
  }
  double sc[SC_N], r2[2 * (SGP_MAXD + 5) + 2];
  int status[4];
  const int64_t off = fitc_rec_off(mp);
  const int nrec = L + 5;
  {
    Readback rb(c);
    HIPCHK(rb.add(sc, c->sc, sizeof(sc)));
    if (!obj_only) {
      HIPCHK(rb.add(r2, red2 + mp * mp + mp + 1, sizeof(double)));
      HIPCHK(rb.add(r2 + 1, red2 + off, sizeof(double) * 2 * nrec));
    }
    HIPCHK(rb.add(status, c->status, sizeof(status)));
    HIPCHK(rb.wait());
  }
  c->phase = 0;
  if (chain_watchdog(status)) return SGP_EHIP;
  if (status[0] || status[1]) {
    set_err("chol(): the leading minor of order %d of %s is not positive definite",
            status[0] ? status[0] : status[1],
            status[0] ? "Sigma22" : "Sigma22 + t(Sigma12) %*% ZSig12");
    return SGP_ENOTPD;
  }
  c->last_mode = 2;
  const double n = (double)c->n_global;
  const double ld22 = 2.0 * sc[SC_LD22], ldB = 2.0 * sc[SC_LDB];
  const double rr = sc[SC_RR], sumlogz = sc[SC_RR + 1], tu = sc[SC_TU];
  const double logdet22 = (c->flags & SGP_FLAG_R_DET) ? log(exp(ld22)) : ld22;
  *obj = -0.5 * rr + 0.5 * tu - 0.5 * (sumlogz - logdet22 + ldB) - (n / 2.0) * log(2.0 * M_PI);
  if (obj_only) {
    c->knot_raw.clear();
    return SGP_OK;
  }
  const double sum_omega = r2[0];
  const double* a = r2 + 1;
  const double* b = r2 + 1 + nrec;
  grad[0] = 2.0 * (a[0] + b[0]) + sc[SC_G22] + kp.sig2 * sum_omega;
  for (int q = 0; q < L; ++q) grad[1 + q] = a[1 + q] + b[1 + q] + sc[SC_G22 + 1 + q];
  grad[L + 1] = 2.0 * kp.tau2 * (a[1 + L] + b[1 + L]) + kp.tau2 * sum_omega;
  return knot_finish(c, red2 + off + 2 * nrec, c->uvec, c->K22inv, c->Binv, c->M3, -0.5, 0.5, 0.5,
                     nullptr, nullptr, 0.0);
}

int sgp_eval_fitc(sgp_ctx* c, int kernel, const double* theta, const double* U, int64_t m,
                  int64_t ldu, double delta, unsigned flags, double* obj, double* grad) {
  MULTI_FWD(c, obj && (grad || (flags & SGP_FLAG_OBJ_ONLY)) ? multi_eval_fitc(c->multi, kernel, theta, U, m, ldu, delta, flags, obj, grad) : multi_bad_args());
  if (!c) { set_err("context is NULL"); return SGP_EINVAL; }
  int st = sgp_fitc_phase1(c, kernel, theta, U, m, ldu, delta, c->red1);
  if (st) return st;
  st = sgp_fitc_phase2(c, c->red1, c->n, flags, c->red2f);
  if (st) return st;
  return sgp_fitc_finish(c, c->red2f, obj, grad);
}


// ------------------------------------------------------------------------- Poisson Laplace
// State machine over the reduction points of newtrap_sparseGP + dlogq_dcov_par (adjoint form,
// DESIGN.md sec. 3.4; numpy twin: tests/adjoint_ref.py NumpyLaplaceRank).
//   begin   : K12, K22 = Kuu + (tau^2+delta) I, Z, S_Z;  obj partials at f0
//   OBJ(0)  : C = (K22+S_B)^-1, x1 = (K22+S_Z)^-1 t_Z, objective; NR part a -> [K^T v, cnt]
//             or, once the stop rule holds, gradient part a -> [K^T c2, K^T g, K^T (B sv)]
//   NRB     : f += ...; obj partials at the new f
//   GRADB   : h, a;  [S_a, sum a, contraction records]
//   FIN     : G22 contraction, gradient
enum { LS_NONE = 0, LS_OBJ0, LS_NRB, LS_OBJ, LS_GRADB, LS_FIN };
enum { LV_F = 0, LV_Z, LV_ZI, LV_B, LV_RF, LV_TV, LV_OMZW, LV_Y1, LV_Y2, LV_DMT, LV_SV, LV_H,
       LV_A, LV_V, LV_P, LV_C2, LV_G, LV_BSV, LV_GPSI, LV_AEXP, LV_N };   // C2, G, BSV adjacent (one K^T pass)
enum { LM_X1 = 0, LM_X2, LM_S, LM_GG, LM_NGG, LM_CW, LM_N };

static double* lvec(sgp_ctx* c, int k) { return c->lv + (int64_t)k * c->n_pad; }
static double* lmv(sgp_ctx* c, int k) { return c->lm + (int64_t)k * c->mp_max; }
static int64_t lap_obj_off(int64_t mp) { return mp * mp + mp + 8; }
static int64_t lap_rec_off(int64_t mp) { return mp * mp + mp + 8; }

int64_t sgp_lap_red_count(int kernel, int d, int64_t m) {
  const int64_t mp = round_up(m, SGP_TILE);
  return 2 * (mp * mp + mp + 8) + 2 * (num_ls(kernel, d) + 5) + 8 + mp * d;   // + knot partials
}

static int lap_ensure(sgp_ctx* c) {
  if (c->lv) return SGP_OK;
  const int64_t np_ = c->n_pad, mp = c->mp_max;
  int st = dalloc(&c->lv, LV_N * np_);
  st = st ? st : dalloc(&c->lm, LM_N * mp);
  c->lslab_cap = 4 * 128 * 4096;
  if (c->lslab_cap < 4 * mp) c->lslab_cap = 4 * mp;
  st = st ? st : dalloc(&c->lslab, c->lslab_cap);
  const int64_t rc = sgp_lap_red_count(SGP_KERNEL_ARD, SGP_MAXD, c->m_max);
  st = st ? st : dalloc(&c->lred[0], rc);
  st = st ? st : dalloc(&c->lred[1], rc);
  st = st ? st : dalloc(&c->Cprev, mp * mp);
  if (st) return st;
  HIPCHK(hipMemset(c->lv, 0, sizeof(double) * LV_N * np_));
  HIPCHK(hipMemset(c->lm, 0, sizeof(double) * LM_N * mp));
  // (null-stream memsets: done before the Laplace kernels run on the context's streams)
  HIPCHK(hipDeviceSynchronize());
  return SGP_OK;
}

int sgp_lap_set_f(sgp_ctx* c, const double* f, double fill) {
  MULTI_FWD(c, multi_lap_set_f(c->multi, f, fill));
  if (!c) { set_err("context is NULL"); return SGP_EINVAL; }
  HIPCHK(hipSetDevice(c->device));
  int st = lap_ensure(c);
  if (st) return st;
  std::vector<double> h((size_t)c->n_pad, 0.0);
  for (int64_t i = 0; i < c->n; ++i) h[(size_t)i] = f ? f[i] : fill;
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipMemcpy(lvec(c, LV_F), h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice));
  c->lap_gpsi_valid = false;
  return SGP_OK;
}

// the reference's `m` per row ("a vector of the areas of each grid cell",
// R/derivative_functions_of_data_likelihoods.R:38; optimize_gp.R:461-468 passes `a` through as m)
int sgp_lap_set_expo(sgp_ctx* c, const double* a, double fill) {
  MULTI_FWD(c, multi_lap_set_expo(c->multi, a, fill));
  if (!c) { set_err("context is NULL"); return SGP_EINVAL; }
  if (!a && !(fill > 0.0 && std::isfinite(fill))) {
    set_err("sgp_lap_set_expo: the fill exposure %g is not a positive finite number", fill);
    return SGP_EINVAL;
  }
  for (int64_t i = 0; a && i < c->n; ++i)
    if (!(a[i] > 0.0 && std::isfinite(a[i]))) {
      set_err("sgp_lap_set_expo: exposure a[%lld] = %g is not a positive finite number",
              (long long)i, a[i]);
      return SGP_EINVAL;
    }
  HIPCHK(hipSetDevice(c->device));
  int st = lap_ensure(c);
  if (st) return st;
  std::vector<double> h((size_t)c->n_pad, 1.0);
  for (int64_t i = 0; i < c->n; ++i) h[(size_t)i] = a ? a[i] : fill;
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipMemcpy(lvec(c, LV_AEXP), h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice));
  c->lap_expo_rows = true;
  return SGP_OK;
}

int sgp_lap_get_grad_psi(sgp_ctx* c, double* out) {
  MULTI_FWD(c, out ? multi_lap_get_grad_psi(c->multi, out) : multi_bad_args());
  if (!c || !out) { set_err("invalid arguments"); return SGP_EINVAL; }
  if (!c->lap_gpsi_valid) {
    set_err("no Newton-Raphson step has run since the mode was last set");
    return SGP_EINVAL;
  }
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipMemcpy(out, lvec(c, LV_GPSI), sizeof(double) * c->n, hipMemcpyDeviceToHost));
  return SGP_OK;
}

int sgp_lap_get_f(sgp_ctx* c, double* f) {
  MULTI_FWD(c, f ? multi_lap_get_f(c->multi, f) : multi_bad_args());
  if (!c || !f) { set_err("invalid arguments"); return SGP_EINVAL; }
  HIPCHK(hipSetDevice(c->device));
  int st = lap_ensure(c);
  if (st) return st;
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipMemcpy(f, lvec(c, LV_F), sizeof(double) * c->n, hipMemcpyDeviceToHost));
  return SGP_OK;
}

// objective partials at the current f into red[o ..]: [S_B, t_Z, r'Z^-1 r, log p(y|f), log Z2]
static int lap_obj_partials(sgp_ctx* c, double* red, int64_t o) {
  const int64_t mp = c->mp, mm = mp * mp;
  Scope t(c, "lap_obj");
  int nb = 0;
  HIPCHK(launch_lap_obj(c->n, c->n_pad, lvec(c, LV_F), c->y, c->mu, lvec(c, LV_Z),
                        lvec(c, LV_ZI), c->lap_expo, c->lap_av, lvec(c, LV_B), lvec(c, LV_RF),
                        lvec(c, LV_TV), c->slab_small, &nb, c->stream));
  HIPCHK(launch_syrk_aug(c->K, c->n_pad, mp, lvec(c, LV_RF), lvec(c, LV_B), c->slab_syrk,
                         c->slab_syrk_cap, red + o, c->stream, 3, lvec(c, LV_TV)));
  HIPCHK(launch_colsum(c->slab_small, nb, 2, red + o + mm + mp + 1, c->stream));
  return SGP_OK;
}

int sgp_lap_begin(sgp_ctx* c, int kernel, const double* theta, const double* U, int64_t m,
                  int64_t ldu, double delta, double expo, double tol, int maxit, unsigned flags,
                  double* red_out, int64_t* count) {
  MULTI_REFUSE(c, "sgp_lap_begin");
  KernParams kp;
  int st = check_eval_args(c, kernel, theta, U, m, ldu, delta, &kp);
  if (st) return st;
  if (!red_out || !count) { set_err("red_out/count is NULL"); return SGP_EINVAL; }
  if (!(expo >= 0.0) || !std::isfinite(expo) || !(tol >= 0.0) || maxit < 0) {
    set_err("invalid Laplace controls (expo=%g, tol=%g, maxit=%d)", expo, tol, maxit);
    return SGP_EINVAL;
  }
  if (expo == SGP_EXPO_ROWS && !c->lap_expo_rows) {
    set_err("expo = SGP_EXPO_ROWS but no per-row exposure was set (sgp_lap_set_expo)");
    return SGP_EINVAL;
  }
  HIPCHK(hipSetDevice(c->device));
  st = drain_abandoned(c);
  if (st) return st;
  st = lap_ensure(c);
  if (st) return st;
  timers_reset(c);
  c->kp = kp;
  c->m = m;
  c->mp = round_up(m, SGP_TILE);
  c->delta = delta;
  c->lap_expo = expo == SGP_EXPO_ROWS ? 1.0 : expo;
  c->lap_av = expo == SGP_EXPO_ROWS ? lvec(c, LV_AEXP) : nullptr;
  c->lap_tol = tol;
  c->lap_maxit = maxit;
  c->flags = flags;
  c->lap_it = 0;
  c->lap_cnt = 0.0;
  c->lap_gpsi_valid = false;   // grad psi belongs to the NR run that starts here
  c->lap_objs.clear();
  const int64_t mp = c->mp;
  st = upload_knots(c, U, m, ldu);
  if (st) return st;
  HIPCHK(hipMemsetAsync(c->status, 0, sizeof(int) * 4, c->stream));
  HIPCHK(hipMemsetAsync(c->sc, 0, sizeof(double) * SC_N, c->stream));
  st = k22_sync(c);
  if (st) return st;
  {
    Scope t(c, "build_knm");
    HIPCHK(launch_build_knm(kp, c->X, c->n_pad, c->n, c->n_pad, c->U, c->mp, m, mp, c->K,
                            c->stream, true));   // beside the K22 chain on aux
  }
  st = k22_launch(c, 0.0);   // K22 = Kuu + (tau^2 + delta) I (newtrap_sparseGP.R:51-59)
  if (st) return st;
  HIPCHK(hipStreamWaitEvent(c->stream, c->ev_k22, 0));
  {
    Scope t(c, "rowquad_q");
    HIPCHK(launch_rowquad_knm(kp, c->K, c->K22inv, c->n, c->n_pad, m, mp, c->r, 0.0, nullptr,
                              nullptr, nullptr, c->rowq, lvec(c, LV_P), c->stream,
                              tstore_ready(c) ? c->tq : nullptr));
    HIPCHK(launch_lap_z(lvec(c, LV_P), c->n, c->n_pad, kp.sig2 + kp.tau2 + delta, lvec(c, LV_Z),
                        lvec(c, LV_ZI), c->stream));
  }
  {
    Scope t(c, "syrk_z");
    HIPCHK(launch_syrk_aug(c->K, c->n_pad, mp, c->r, lvec(c, LV_ZI), c->slab_syrk,
                           c->slab_syrk_cap, red_out, c->stream, 3, nullptr, 0, nullptr, false,
                           true));   // 1/Z > 0
  }
  st = lap_obj_partials(c, red_out, lap_obj_off(mp));
  if (st) return st;
  *count = lap_obj_off(mp) + mp * mp + mp + 3;
  c->lap_state = LS_OBJ0;
  return SGP_OK;
}

// consume objective sums: factor, solve, evaluate obj_fun_pois; returns the objective
static int lap_consume_obj(sgp_ctx* c, const double* red, int64_t o, bool first, double* obj) {
  const int64_t mp = c->mp, mm = mp * mp;
  {
    Scope t(c, "lap_dense");
    if (first)   // (K22 + S_Z)^-1 is fixed for the whole NR run (Z depends on theta only)
      HIPCHK(dense_spd_inverse_sum(c->K22, 1.0, red, c->Bm, mp, c->Xt, c->dinv, c->logdB,
                                   c->status + 1, c->gjs, c->stream));
    if (!first)   // newtrap_sparseGP's u posterior uses the W of the last update's start
      HIPCHK(hipMemcpyAsync(c->Cprev, c->Binv, sizeof(double) * mm, hipMemcpyDeviceToDevice,
                            c->stream));
    HIPCHK(dense_spd_inverse_sum(c->K22, 1.0, red + o, c->Binv, mp, c->Xt, c->dinv, c->logdB,
                                 c->status + 2, c->gjs, c->stream));
    HIPCHK(launch_sum_small(c->logdB, mp / SGP_DB, c->sc + SC_LDB, c->stream));
    HIPCHK(dense_gemv(c->Bm, mp, red + o + mm, 1.0, lmv(c, LM_X1), c->stream));
    HIPCHK(launch_dot(red + o + mm, lmv(c, LM_X1), mp, c->slab_small, c->sc + SC_TU, c->stream));
    HIPCHK(hipMemcpyAsync(c->sc + SC_RR, red + o + mm + mp, 3 * sizeof(double),
                          hipMemcpyDeviceToDevice, c->stream));
  }
  double sc[SC_N];
  int status[4];
  HIPCHK(hipMemcpyAsync(sc, c->sc, sizeof(sc), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(status, c->status, sizeof(status), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (chain_watchdog(status)) return SGP_EHIP;
  if (status[0] || status[1] || status[2]) {
    c->lap_state = LS_NONE;
    set_err("chol(): the leading minor of order %d of %s is not positive definite",
            status[0] ? status[0] : (status[1] ? status[1] : status[2]),
            status[0] ? "Sigma22" : (status[1] ? "Sigma22 + t(Sigma12) %*% ZSig12"
                                               : "Sigma22 + t(Sigma12) %*% (B * Sigma12)"));
    return SGP_ENOTPD;
  }
  if (!first) c->lap_cnt = sc[SC_RR + 3];   // the count of the step that led here (nr_b)
  const double ld22 = 2.0 * sc[SC_LD22], ldB = 2.0 * sc[SC_LDB];
  const double rr = sc[SC_RR], logpy = sc[SC_RR + 1], logz2 = sc[SC_RR + 2], tu = sc[SC_TU];
  // laplace_approx_obj_funs.R:158-172: quad + log p(y|f) + det_part_1 + det_part_2
  *obj = (-0.5 * rr + 0.5 * tu) + logpy + (-0.5 * (-ld22 + ldB)) + (-0.5 * logz2);
  return SGP_OK;
}

int sgp_lap_step(sgp_ctx* c, const double* red_in, double* red_out, int64_t* count, int* done,
                 double* obj, double* grad, int* nr_iters) {
  MULTI_REFUSE(c, "sgp_lap_step");
  if (!c || !red_in || !red_out || !count || !done || red_in == red_out) {
    set_err("invalid arguments (red_in and red_out must be distinct device buffers)");
    return SGP_EINVAL;
  }
  HIPCHK(hipSetDevice(c->device));
  *done = 0;
  const KernParams& kp = c->kp;
  const int64_t n = c->n, n_pad = c->n_pad, mp = c->mp, mm = mp * mp;
  const int st_in = c->lap_state;
  if (st_in == LS_OBJ0 || st_in == LS_OBJ) {
    double o = 0.0;
    int st = lap_consume_obj(c, red_in, st_in == LS_OBJ0 ? lap_obj_off(mp) : 0, st_in == LS_OBJ0,
                             &o);
    if (st) return st;
    c->lap_obj_prev = c->lap_obj;
    c->lap_obj = o;
    c->lap_it += 1;
    c->lap_objs.push_back(o);
    // maxit = 0 is this ABI's "evaluate at the given f" mode (sgp.h); any maxit >= 1 performs
    // the first update before the loop as newtrap_sparseGP.R:79-96 does (iter >= 2)
    // maxit = 0 is the C ABI's "objective and gradient at the given f" mode (dlogq_dcov_par);
    // every reference-facing caller passes maxit >= 1, so the first update always runs there,
    // as newtrap_sparseGP.R:79-96 run it before the loop whatever maxit is
    const bool go = (st_in == LS_OBJ0 && c->lap_maxit > 0) ||
                    (c->lap_it < c->lap_maxit &&
                     (fabs(c->lap_obj - c->lap_obj_prev) > c->lap_tol || c->lap_cnt > 0.0));
    if (go) {   // NR part a: grad_psi and K^T (grad_psi / omzw)
      Scope t(c, "lap_nr_a");
      if (mp <= 2048 && lap_rowpass_slab(n_pad, mp) <= c->lslab_cap) {
        // one pass over K12: y1 = K x1, the row update and K^T v from the same staged rows
        HIPCHK(launch_lap_nr_a_fused(c->K, n, n_pad, mp, lmv(c, LM_X1), lvec(c, LV_F), c->y,
                                     c->mu, lvec(c, LV_Z), lvec(c, LV_ZI), c->lap_expo,
                                     c->lap_av, c->lap_tol, lvec(c, LV_Y1), lvec(c, LV_G), lvec(c, LV_OMZW),
                                     lvec(c, LV_V), lvec(c, LV_GPSI), c->lslab, c->lslab_cap,
                                     red_out, red_out + mp, c->stream));
      } else {
        HIPCHK(launch_gemv_rows(c->K, n_pad, mp, lmv(c, LM_X1), nullptr, lvec(c, LV_Y1), nullptr,
                                c->stream));
        int nb = 0;
        HIPCHK(launch_lap_nr_a(n, n_pad, lvec(c, LV_F), c->y, c->mu, lvec(c, LV_Z),
                               lvec(c, LV_ZI), c->lap_expo, c->lap_av, lvec(c, LV_Y1), c->lap_tol,
                               lvec(c, LV_G), lvec(c, LV_OMZW), lvec(c, LV_V), lvec(c, LV_GPSI),
                               c->slab_small, &nb, c->stream));
        HIPCHK(launch_gemv_cols(c->K, n_pad, mp, lvec(c, LV_V), n_pad, 1, c->lslab, c->lslab_cap,
                                red_out, c->stream));
        HIPCHK(launch_colsum(c->slab_small, nb, 1, red_out + mp, c->stream));
      }
      c->lap_gpsi_valid = true;
      *count = mp + 1;
      c->lap_state = LS_NRB;
      return SGP_OK;
    }
    if (c->flags & SGP_FLAG_OBJ_ONLY) {   // newtrap_sparseGP alone: stop at the mode
      if (obj) *obj = c->lap_obj;
      if (nr_iters) *nr_iters = c->lap_it;
      c->last_mode = 3;
      c->knot_raw.clear();
      *count = 0;
      *done = 1;
      c->lap_state = LS_NONE;
      return SGP_OK;
    }
    // gradient part a (dlogq_dcov_par at the final f)
    Scope t(c, "lap_grad_a");
    // c2 = (rf - K x1) / Z rides in the row-quadratic pass's k-loop as its fused alpha (the
    // K x1 dot products from the staged K values): no separate K x1 pass
    HIPCHK(launch_rowquad_knm(kp, c->K, c->Binv, n, n_pad, c->m, mp, lvec(c, LV_RF), 0.0,
                              lvec(c, LV_ZI), lmv(c, LM_X1), lvec(c, LV_C2), c->rowq,
                              lvec(c, LV_P), c->stream, tstore_ready(c) ? c->tp : nullptr));
    HIPCHK(launch_lap_grad_a(n, n_pad, lvec(c, LV_F), c->y, c->mu, lvec(c, LV_Z), lvec(c, LV_ZI),
                             c->lap_expo, c->lap_av, nullptr, lvec(c, LV_P), lvec(c, LV_C2),
                             lvec(c, LV_G), lvec(c, LV_B), lvec(c, LV_DMT), lvec(c, LV_SV),
                             lvec(c, LV_BSV), c->stream));
    HIPCHK(launch_gemv_cols(c->K, n_pad, mp, lvec(c, LV_C2), n_pad, 3, c->lslab, c->lslab_cap,
                            red_out, c->stream));
    *count = 3 * mp;
    c->lap_state = LS_GRADB;
    return SGP_OK;
  }
  if (st_in == LS_NRB) {
    // NR part b and the next objective's rows fused into one K pass where the knot count allows
    const bool fused = mp <= 2048 && lap_rowpass_slab(n_pad, mp) <= c->lslab_cap;
    {
      Scope t(c, "lap_nr_b");
      // the stop-rule count rides to the host with the next objective's scalars (sc is read
      // back by lap_consume_obj): no host round trip inside the Newton step
      HIPCHK(hipMemcpyAsync(c->sc + SC_RR + 3, red_in + mp, sizeof(double),
                            hipMemcpyDeviceToDevice, c->stream));
      HIPCHK(dense_gemv(c->Binv, mp, red_in, 1.0, lmv(c, LM_X2), c->stream));
      if (!fused) {
        HIPCHK(launch_gemv_rows(c->K, n_pad, mp, lmv(c, LM_X2), nullptr, lvec(c, LV_Y2),
                                nullptr, c->stream));
        HIPCHK(launch_lap_nr_b(n, n_pad, lvec(c, LV_F), c->mu, lvec(c, LV_Z), lvec(c, LV_G),
                               lvec(c, LV_OMZW), lvec(c, LV_Y1), lvec(c, LV_Y2), c->stream));
      }
    }
    if (fused) {
      // one K pass: y2 = K x2, the f update and t = K^T tv at the new f (red_out + mm) with
      // tv'(f - mu) (red_out + mm + mp); k_lap_obj's rows (B, rf, tv, the likelihood sums) and
      // S_B by the weighted SYRK without t (red_out)
      Scope t(c, "lap_obj");
      HIPCHK(launch_lap_nr_b_t_fused(c->K, n, n_pad, mp, lmv(c, LM_X2), lvec(c, LV_F), c->y,
                                     c->mu, lvec(c, LV_Z), lvec(c, LV_ZI), lvec(c, LV_G),
                                     lvec(c, LV_OMZW), lvec(c, LV_Y1), c->lslab, c->lslab_cap,
                                     red_out + mm, red_out + mm + mp, c->stream));
      int nb = 0;
      HIPCHK(launch_lap_obj(n, n_pad, lvec(c, LV_F), c->y, c->mu, lvec(c, LV_Z), lvec(c, LV_ZI),
                            c->lap_expo, c->lap_av, lvec(c, LV_B), lvec(c, LV_RF), lvec(c, LV_TV),
                            c->slab_small, &nb, c->stream));
      // B = W / (Z W - 1) >= 0 (W = -a e^f <= 0, Z > 0)
      HIPCHK(launch_syrk_aug(c->K, n_pad, mp, lvec(c, LV_RF), lvec(c, LV_B), c->slab_syrk,
                             c->slab_syrk_cap, red_out, c->stream, 3, nullptr, 0, nullptr, false,
                             true));
      HIPCHK(launch_colsum(c->slab_small, nb, 2, red_out + mm + mp + 1, c->stream));
      *count = mm + mp + 3;
      c->lap_state = LS_OBJ;
      return SGP_OK;
    }
    int st = lap_obj_partials(c, red_out, 0);
    if (st) return st;
    *count = mm + mp + 3;
    c->lap_state = LS_OBJ;
    return SGP_OK;
  }
  if (st_in == LS_GRADB) {
    Scope t(c, "lap_grad_b");
    const double* sr = red_in;
    const double* ggr = red_in + mp;
    const double* w = red_in + 2 * mp;
    HIPCHK(dense_gemv(c->K22inv, mp, sr, 1.0, lmv(c, LM_S), c->stream));
    HIPCHK(dense_gemv(c->K22inv, mp, ggr, 1.0, lmv(c, LM_GG), c->stream));
    HIPCHK(dense_gemv(c->K22inv, mp, ggr, -1.0, lmv(c, LM_NGG), c->stream));
    HIPCHK(dense_gemv(c->Binv, mp, w, 1.0, lmv(c, LM_CW), c->stream));
    HIPCHK(launch_gemv_rows(c->K, n_pad, mp, lmv(c, LM_CW), nullptr, lvec(c, LV_Y2), nullptr,
                            c->stream));
    int nb = 0;
    HIPCHK(launch_lap_grad_b(n, n_pad, lvec(c, LV_B), lvec(c, LV_SV), lvec(c, LV_Y2),
                             lvec(c, LV_DMT), lvec(c, LV_C2), lvec(c, LV_G), lvec(c, LV_H),
                             lvec(c, LV_A), c->slab_small, &nb, c->stream));
    const int64_t off = lap_rec_off(mp);
    HIPCHK(hipMemsetAsync(red_out, 0, sizeof(double) * (off + 2 * (kp.L + 5)), c->stream));
    HIPCHK(launch_syrk_aug(c->K, n_pad, mp, c->r, lvec(c, LV_A), c->slab_syrk, c->slab_syrk_cap,
                           red_out, c->stream, 3, nullptr, 0));
    HIPCHK(launch_colsum(c->slab_small, nb, 1, red_out + mm + mp + 1, c->stream));
    int64_t nrec = kp.L + 5;
    double* kout = red_out + off + 2 * nrec;
    // G1 = c2 s^T - h GG^T - diag(B) K C
    ConArgs a1;
    a1.alpha_in = lvec(c, LV_C2);
    a1.uvec = lmv(c, LM_S);
    a1.beta_in = lvec(c, LV_H);
    a1.vvec = lmv(c, LM_NGG);
    a1.rs_vec = lvec(c, LV_B);
    a1.rs = -1.0;
    if (tstore_ready(c)) a1.tin = c->tp;   // K C from lap_grad_a's row-quadratic pass
    if (fuse_tt(c)) {
      // and G2 = -diag(2a) K K22^-1 from lap_begin's rowquad_q in the same pass (one read of
      // K; the second record set stays zero -- the finish sums the two)
      a1.tin2 = c->tq;
      a1.M2 = c->K22inv;
      a1.rs_vec2 = lvec(c, LV_A);
      a1.rs2 = -2.0;
    }
    int st = contract_pass(c, c->Binv, a1, red_out + off, kout, false);
    if (st) return st;
    if (fuse_tt(c)) {
      *count = off + 2 * nrec + (c->knot_on ? mp * kp.d : 0);
      c->lap_state = LS_FIN;
      return SGP_OK;
    }
    // G2 = -diag(2a) K K22^-1
    ConArgs a2;
    a2.rs_vec = lvec(c, LV_A);
    a2.rs = -2.0;
    if (tstore_ready(c)) a2.tin = c->tq;   // K K22^-1 from lap_begin's rowquad_q
    st = contract_pass(c, c->K22inv, a2, red_out + off + nrec, kout, true);
    if (st) return st;
    *count = off + 2 * nrec + (c->knot_on ? mp * kp.d : 0);
    c->lap_state = LS_FIN;
    return SGP_OK;
  }
  if (st_in == LS_FIN) {
    const int L = kp.L;
    {
      Scope t(c, "contract_kmm");
      // G22 = (K22^-1 - C)/2 - s s^T/2 + (Cw GG^T + GG Cw^T)/4 + K22^-1 S_a K22^-1
      HIPCHK(launch_gemm64(false, false, false, mp, mp, mp, 1.0, c->K22inv, mp, red_in, mp, 0.0,
                           c->T1, mp, c->stream));
      HIPCHK(launch_gemm64(false, false, false, mp, mp, mp, 1.0, c->T1, mp, c->K22inv, mp, 0.0,
                           c->M3, mp, c->stream));
      int nb = 0;
      HIPCHK(launch_contract_kmm(kp, c->U, c->mp, c->m, mp, lmv(c, LM_S), c->K22inv, c->Binv,
                                 c->M3, -0.5, 0.5, 1.0, lmv(c, LM_CW), lmv(c, LM_GG), 0.25,
                                 c->slab_small, c->slab_small_cap, &nb, c->stream));
      HIPCHK(launch_colsum(c->slab_small, nb, kp.P, c->sc + SC_G22, c->stream));
    }
    const int64_t off = lap_rec_off(mp);
    const int nrec = L + 5;
    double sc[SC_N], r2[2 * (SGP_MAXD + 5) + 2];
    HIPCHK(hipMemcpyAsync(sc, c->sc, sizeof(sc), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(r2, red_in + mm + mp + 1, sizeof(double), hipMemcpyDeviceToHost,
                          c->stream));
    HIPCHK(hipMemcpyAsync(r2 + 1, red_in + off, sizeof(double) * 2 * nrec, hipMemcpyDeviceToHost,
                          c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    const double suma = r2[0];
    const double* a = r2 + 1;
    const double* b = r2 + 1 + nrec;
    const double* g22 = sc + SC_G22;
    if (grad) {
      grad[0] = 2.0 * (a[0] + b[0]) + g22[0] + 2.0 * kp.sig2 * suma;
      for (int q = 0; q < L; ++q) grad[1 + q] = a[1 + q] + b[1 + q] + g22[1 + q];
      grad[L + 1] = 2.0 * kp.tau2 * (a[1 + L] + b[1 + L]) + 2.0 * kp.tau2 * g22[kp.P - 1] +
                    2.0 * kp.tau2 * suma;
    }
    if (obj) *obj = c->lap_obj;
    if (nr_iters) *nr_iters = c->lap_it;
    c->last_mode = 3;
    int st = knot_finish(c, red_in + off + 2 * nrec, lmv(c, LM_S), c->K22inv, c->Binv, c->M3,
                         -0.5, 0.5, 1.0, lmv(c, LM_CW), lmv(c, LM_GG), 0.25);
    if (st) return st;
    *count = 0;
    *done = 1;
    c->lap_state = LS_NONE;
    return SGP_OK;
  }
  set_err("sgp_lap_step called without sgp_lap_begin");
  return SGP_EINVAL;
}

int sgp_lap_objective_values(sgp_ctx* c, double* out, int max_n, int* count) {
  MULTI_FWD(c, sgp_lap_objective_values(multi_lead(c->multi), out, max_n, count));
  if (!c || !count) { set_err("invalid arguments"); return SGP_EINVAL; }
  int k = 0;
  for (double v : c->lap_objs) {
    if (k >= max_n) break;
    if (out) out[k] = v;
    ++k;
  }
  *count = (int)c->lap_objs.size();
  return SGP_OK;
}

int sgp_eval_laplace(sgp_ctx* c, int kernel, const double* theta, const double* U, int64_t m,
                     int64_t ldu, double delta, double expo, double tol, int maxit, double* obj,
                     double* grad, int* nr_iters) {
  MULTI_FWD(c, multi_eval_laplace(c->multi, kernel, theta, U, m, ldu, delta, expo, tol, maxit, 0u, obj, grad, nr_iters));
  if (!c) { set_err("context is NULL"); return SGP_EINVAL; }
  HIPCHK(hipSetDevice(c->device));
  int st = lap_ensure(c);
  if (st) return st;
  int64_t count = 0;
  st = sgp_lap_begin(c, kernel, theta, U, m, ldu, delta, expo, tol, maxit, 0u, c->lred[0],
                     &count);
  if (st) return st;
  int cur = 0, done = 0;
  while (!done) {
    st = sgp_lap_step(c, c->lred[cur], c->lred[cur ^ 1], &count, &done, obj, grad, nr_iters);
    if (st) return st;
    cur ^= 1;
  }
  return SGP_OK;
}

int sgp_lap_nr(sgp_ctx* c, int kernel, const double* theta, const double* U, int64_t m,
               int64_t ldu, double delta, double expo, double tol, int maxit, double* obj,
               int* nr_iters) {
  MULTI_FWD(c, multi_eval_laplace(c->multi, kernel, theta, U, m, ldu, delta, expo, tol, maxit, SGP_FLAG_OBJ_ONLY, obj, nullptr, nr_iters));
  if (!c) { set_err("context is NULL"); return SGP_EINVAL; }
  HIPCHK(hipSetDevice(c->device));
  int st = lap_ensure(c);
  if (st) return st;
  int64_t count = 0;
  st = sgp_lap_begin(c, kernel, theta, U, m, ldu, delta, expo, tol, maxit, SGP_FLAG_OBJ_ONLY,
                     c->lred[0], &count);
  if (st) return st;
  int cur = 0, done = 0;
  while (!done) {
    st = sgp_lap_step(c, c->lred[cur], c->lred[cur ^ 1], &count, &done, obj, nullptr, nr_iters);
    if (st) return st;
    cur ^= 1;
  }
  return SGP_OK;
}


// ------------------------------------------------------------------------- full GP
// Config 1 (norm_grad_ascent_full, R/laplace_gradient_ascent.R:1700-2011): the n x n system
// Sigma11 = k(xy, xy) + (tau^2 + delta) I over the context's own rows, factored like K22.
//   obj  = obj_fun_norm_full = log dmvnorm(y; mu, Sigma11)  (R/laplace_approx_obj_funs.R:56-61)
//   grad = dlogp_dcov_par_full (R/laplace_approx_gradient.R:1140-1269):
//          1/2 tr((a a^T - Sigma11^-1) dSigma11/dlog theta) with a = Sigma11^-1 y -- y, not
//          y - mu (the reference's quirk) -- contracted by k_contract_kmm with
//          G = 1/2 a a^T - 1/2 Sigma11^-1; tau's derivative is 2 tau^2 on coincident pairs.
int sgp_eval_full(sgp_ctx* c, int kernel, const double* theta, double delta, unsigned flags,
                  double* obj, double* grad) {
  MULTI_REFUSE(c, "sgp_eval_full (the full GP needs every row on one device)");
  if (!c) { set_err("context is NULL"); return SGP_EINVAL; }
  const bool obj_only = (flags & SGP_FLAG_OBJ_ONLY) != 0;
  if (!obj || (!grad && !obj_only)) { set_err("invalid arguments"); return SGP_EINVAL; }
  if (kernel == SGP_KERNEL_EXP) {
    set_err("fused evaluation supports 'sqexp' and 'ard' (optimize_gp.R:263 rejects others)");
    return SGP_EINVAL;
  }
  if (c->n > c->m_max) {
    set_err("the full GP needs m_max >= n (n = %lld, m_max = %lld)", (long long)c->n,
            (long long)c->m_max);
    return SGP_EINVAL;
  }
  KernParams kp;
  int st = make_params(kernel, c->d, theta, delta, &kp);
  if (st) return st;
  HIPCHK(hipSetDevice(c->device));
  st = drain_abandoned(c);   // before U is overwritten below
  if (st) return st;
  timers_reset(c);
  c->kp = kp;
  c->m = c->n;
  c->mp = round_up(c->n, SGP_TILE);
  c->delta = delta;
  c->flags = flags;
  c->phase = 0;
  c->last_mode = 0;
  c->knot_raw.clear();
  const int64_t mp = c->mp, mm = mp * mp;
  // the rows are the "knots": X (ld n_pad) -> U (ld mp), zero padded alike (mp == n_pad)
  HIPCHK(hipMemcpy2DAsync(c->U, sizeof(double) * mp, c->X, sizeof(double) * c->n_pad,
                          sizeof(double) * mp, (size_t)c->d, hipMemcpyDeviceToDevice, c->stream));
  c->knots_valid = false;
  ++c->knots_gen;
  HIPCHK(hipMemsetAsync(c->status, 0, sizeof(int) * 4, c->stream));
  HIPCHK(hipMemsetAsync(c->sc, 0, sizeof(double) * SC_N, c->stream));
  st = k22_stage(c, 0.0);   // Sigma11 = k(xy, xy) + (tau^2 + delta) I and its inverse
  if (st) return st;
  HIPCHK(hipStreamWaitEvent(c->stream, c->ev_k22, 0));
  {
    Scope t(c, "full_vectors");
    HIPCHK(dense_gemv(c->K22inv, mp, c->y, 1.0, c->uvec, c->stream));    // a = Sigma11^-1 y
    HIPCHK(dense_gemv(c->K22inv, mp, c->r, 1.0, c->alpha, c->stream));   // Sigma11^-1 (y - mu)
    HIPCHK(launch_dot(c->r, c->alpha, mp, c->slab_small, c->sc + SC_RR, c->stream));
  }
  if (!obj_only) {
    Scope t(c, "contract_kmm");
    HIPCHK(hipMemsetAsync(c->T1, 0, sizeof(double) * mm, c->stream));
    int nb = 0;
    HIPCHK(launch_contract_kmm(kp, c->U, mp, c->m, mp, c->uvec, c->T1, c->K22inv, c->T1, 0.5,
                               0.5, 0.0, nullptr, nullptr, 0.0, c->slab_small, c->slab_small_cap, &nb,
                               c->stream));
    HIPCHK(launch_colsum(c->slab_small, nb, kp.P, c->sc + SC_G22, c->stream));
  }
  double sc[SC_N];
  int status[4];
  {
    Readback rb(c);
    HIPCHK(rb.add(sc, c->sc, sizeof(sc)));
    HIPCHK(rb.add(status, c->status, sizeof(status)));
    HIPCHK(rb.wait());
  }
  if (chain_watchdog(status)) return SGP_EHIP;
  if (status[0]) {
    set_err("Sigma11 is not positive definite (leading minor of order %d)", status[0]);
    return SGP_ENOTPD;
  }
  const double n = (double)c->n;
  *obj = -0.5 * sc[SC_RR] - sc[SC_LD22] - (n / 2.0) * log(2.0 * M_PI);   // sc: 1/2 log det
  if (!obj_only) {
    const double* g22 = sc + SC_G22;
    grad[0] = g22[0];
    for (int q = 0; q < kp.L; ++q) grad[1 + q] = g22[1 + q];
    grad[kp.L + 1] = 2.0 * kp.tau2 * g22[kp.P - 1];
  }
  return SGP_OK;
}

// ------------------------------------------------------------------------- knot posterior
// u | y at the end of the drivers, from the replicated state of the last evaluation:
//   VI / FITC (vi_functions.R:1161-1180, laplace_gradient_ascent.R:1635-1655):
//     u_mean = muu + K22 Bm^-1 t,  u_var = K22 Bm^-1 K22   (= Sigma22 - S + S Bm^-1 S)
//   Laplace (newtrap_sparseGP.R:137-176): u_mean = muu + K22 (K22+S_Z)^-1 t_Z(f_hat),
//     u_var = K22 (K22 + S_B(W_prev))^-1 K22   (= Sigma22 + TT + TT (Sigma22 - TT)^-1 TT)
int sgp_posterior_u(sgp_ctx* c, const double* muu, double* u_mean, double* u_var) {
  MULTI_FWD(c, sgp_posterior_u(multi_lead(c->multi), muu, u_mean, u_var));
  if (!c || !muu || !u_mean || !u_var) { set_err("invalid arguments"); return SGP_EINVAL; }
  if (c->last_mode == 0) { set_err("no completed evaluation in this context"); return SGP_EINVAL; }
  HIPCHK(hipSetDevice(c->device));
  const int64_t mp = c->mp, m = c->m;
  const double* vec = c->uvec;
  const double* inv = c->Binv;
  if (c->last_mode == 3) {
    vec = lmv(c, LM_X1);
    if (c->lap_it >= 2) inv = c->Cprev;
  }
  HIPCHK(dense_gemv(c->K22, mp, vec, 1.0, c->T22, c->stream));   // T22 row 0 as scratch
  HIPCHK(launch_gemm64(false, false, false, mp, mp, mp, 1.0, c->K22, mp, inv, mp, 0.0, c->T1, mp,
                       c->stream));
  HIPCHK(launch_gemm64(false, false, false, mp, mp, mp, 1.0, c->T1, mp, c->K22, mp, 0.0, c->M3,
                       mp, c->stream));
  std::vector<double> hv((size_t)mp), hm((size_t)(mp * mp));
  HIPCHK(hipMemcpyAsync(hv.data(), c->T22, sizeof(double) * mp, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(hm.data(), c->M3, sizeof(double) * mp * mp, hipMemcpyDeviceToHost,
                        c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  for (int64_t j = 0; j < m; ++j) u_mean[j] = muu[j] + hv[(size_t)j];
  for (int64_t j = 0; j < m; ++j)
    for (int64_t i = 0; i < m; ++i) u_var[i + j * m] = hm[(size_t)(i * mp + j)];
  return SGP_OK;
}

// ------------------------------------------------------------------------- prediction
namespace {
struct DevBuf {
  double* p = nullptr;
  ~DevBuf() { if (p) (void)hipFree(p); }
};
struct StreamGuard {
  hipStream_t s = nullptr;
  ~StreamGuard() {
    if (s) {
      (void)hipStreamSynchronize(s);
      (void)hipStreamDestroy(s);
    }
  }
};
struct IntBuf {
  int* p = nullptr;
  ~IntBuf() { if (p) (void)hipFree(p); }
};
}  // namespace

int sgp_predict(int device, int kernel, const double* theta, double delta, int method,
                int gaussian, const double* U, int64_t m, int64_t ldu, const double* u_mean,
                const double* muu, const double* u_var, int64_t ldv, const double* x_pred,
                int64_t np, int64_t ldxp, int d, const double* mu_pred, int full_cov,
                double* pred_mean, double* pred_var, int64_t ldpv) {
  KernParams kp;
  int st = make_params(kernel, d, theta, delta, &kp);
  if (st) return st;
  const bool full = method == SGP_PRED_FULL;   // u_var unused (zero): Sigma22 = the data block
  if (!U || m < 1 || ldu < m || !u_mean || !muu || (!u_var && !full) || (!full && ldv < m) ||
      !x_pred || np < 1 ||
      ldxp < np || !mu_pred || !pred_mean || !pred_var || (full_cov && ldpv < np)) {
    set_err("invalid sgp_predict arguments");
    return SGP_EINVAL;
  }
  {
    std::vector<double> plo, phi;
    col_range(x_pred, np, ldxp, d, &plo, &phi);
    set_center(&kp, U, m, ldu, plo.data(), phi.data());
  }
  if (method != SGP_PRED_VI && method != SGP_PRED_LAPLACE && method != SGP_PRED_FULL) {
    set_err("invalid prediction method %d", method);
    return SGP_EINVAL;
  }
  if (method == SGP_PRED_VI && !gaussian) {
    set_err("Error: VI not supported for non-gaussian data.");   // predict_gp, l.424-427
    return SGP_EINVAL;
  }
  HIPCHK(hipSetDevice(device));
  StreamGuard sg;
  HIPCHK(hipStreamCreateWithFlags(&sg.s, hipStreamNonBlocking));
  hipStream_t s = sg.s;
  const int64_t mp = round_up(m, SGP_TILE), npp = round_up(np, SGP_TILE), mm = mp * mp;
  DevBuf dU, K22, Kinv, R, Pb, logd, V, T1, T22, wv, Xp, Kp, yv, rowq, q, S, Y;
  IntBuf status, gsync;
  st = dalloc(&dU.p, mp * d);
  st = st ? st : dalloc(&K22.p, mm);
  st = st ? st : dalloc(&Kinv.p, mm);
  st = st ? st : dalloc(&R.p, mm);
  st = st ? st : dalloc(&Pb.p, mp * 64);
  st = st ? st : dalloc(&logd.p, mp / SGP_DB);
  st = st ? st : dalloc(&V.p, mm);
  st = st ? st : dalloc(&T1.p, mm);
  st = st ? st : dalloc(&T22.p, mm);
  st = st ? st : dalloc(&wv.p, 2 * mp);
  st = st ? st : dalloc(&Xp.p, npp * d);
  st = st ? st : dalloc(&Kp.p, npp * mp);
  st = st ? st : dalloc(&yv.p, npp);
  st = st ? st : dalloc(&rowq.p, npp * (mp / SGP_TILE));
  st = st ? st : dalloc(&q.p, npp);
  st = st ? st : dalloc(&status.p, 4);
  st = st ? st : dalloc(&gsync.p, SGP_GJ_SYNC_WORDS);
  if (!st && full_cov) {
    st = dalloc(&S.p, npp * npp);
    st = st ? st : dalloc(&Y.p, npp * mp);
  }
  if (st) return st;
  {
    std::vector<double> hU((size_t)(mp * d), 0.0), hX((size_t)(npp * d), 0.0);
    for (int c = 0; c < d; ++c) {
      for (int64_t j = 0; j < m; ++j) hU[(size_t)(c * mp + j)] = U[j + c * ldu];
      for (int64_t i = 0; i < np; ++i) hX[(size_t)(c * npp + i)] = x_pred[i + c * ldxp];
    }
    std::vector<double> hd((size_t)mp, 0.0), hV((size_t)mm, 0.0);
    for (int64_t j = 0; j < m; ++j) hd[(size_t)j] = u_mean[j] - muu[j];
    if (!full)
      for (int64_t i = 0; i < m; ++i)
        for (int64_t j = 0; j < m; ++j) hV[(size_t)(i * mp + j)] = u_var[i + j * ldv];
    HIPCHK(hipMemcpy(dU.p, hU.data(), sizeof(double) * hU.size(), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(Xp.p, hX.data(), sizeof(double) * hX.size(), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(wv.p + mp, hd.data(), sizeof(double) * mp, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(V.p, hV.data(), sizeof(double) * mm, hipMemcpyHostToDevice));
    // on the launch stream: the null stream's hipMemset is not ordered before a non-blocking
    // stream's kernels (the chain's sync words must be zero when it starts)
    HIPCHK(hipMemsetAsync(status.p, 0, sizeof(int) * 4, s));
    HIPCHK(hipMemsetAsync(gsync.p, 0, sizeof(int) * SGP_GJ_SYNC_WORDS, s));
  }
  // Sigma22: the gaussian family subtracts tau^2 I again (vi_functions.R:1246-1260,
  // laplace_approx_prediction.R:25-43) -> diagonal sigma^2 + delta; otherwise Kuu+(tau^2+delta)I
  // (predict_gp_full, laplace_approx_prediction.R:281-405: Sigma22 = k(xy, xy) + (tau^2+delta) I)
  const double diag_sub = (gaussian && !full) ? kp.tau2 : 0.0;
  HIPCHK(launch_build_kmm(kp, dU.p, mp, m, mp, diag_sub, K22.p, s));
  HIPCHK(hipMemcpyAsync(Kinv.p, K22.p, sizeof(double) * mm, hipMemcpyDeviceToDevice, s));
  HIPCHK(dense_spd_inverse(Kinv.p, mp, R.p, Pb.p, logd.p, status.p,
                           reinterpret_cast<unsigned*>(gsync.p), s));
  HIPCHK(dense_gemv(Kinv.p, mp, wv.p + mp, 1.0, wv.p, s));          // Sigma22^-1 (u_mean - muu)
  HIPCHK(launch_gemm64(false, false, false, mp, mp, mp, 1.0, Kinv.p, mp, V.p, mp, 0.0, T1.p, mp,
                       s));
  HIPCHK(launch_gemm64(false, false, false, mp, mp, mp, 1.0, T1.p, mp, Kinv.p, mp, 0.0, T22.p, mp,
                       s));                                           // Sigma22^-1 u_var Sigma22^-1
  const bool lap_full = (method == SGP_PRED_LAPLACE) && full_cov;
  if (!lap_full) HIPCHK(dense_axpby(1.0, T22.p, -1.0, Kinv.p, T22.p, mm, s));   // temp22
  HIPCHK(launch_build_knm(kp, Xp.p, npp, np, npp, dU.p, mp, m, mp, Kp.p, s));
  HIPCHK(launch_gemv_rows(Kp.p, npp, mp, wv.p, nullptr, yv.p, nullptr, s));
  std::vector<double> hy((size_t)npp), hq((size_t)npp, 0.0);
  if (!full_cov) {
    HIPCHK(launch_rowquad_knm(kp, Kp.p, T22.p, np, npp, m, mp, nullptr, 0.0, nullptr, nullptr,
                              nullptr, rowq.p, q.p, s));
  } else {
    if (lap_full)
      HIPCHK(launch_rowquad_knm(kp, Kp.p, Kinv.p, np, npp, m, mp, nullptr, 0.0, nullptr, nullptr,
                                nullptr, rowq.p, q.p, s));
    if (method == SGP_PRED_VI || full)   // Sigma11 of x_pred with its tau^2 + delta diagonal
      HIPCHK(launch_fill_cov(kp, Xp.p, np, npp, Xp.p, np, npp, true, S.p, npp, s));
    else
      HIPCHK(hipMemsetAsync(S.p, 0, sizeof(double) * npp * npp, s));
    HIPCHK(launch_gemm64(false, false, false, npp, mp, mp, 1.0, Kp.p, mp, T22.p, mp, 0.0, Y.p, mp,
                         s));
    HIPCHK(launch_gemm64(false, true, false, npp, npp, mp, 1.0, Y.p, mp, Kp.p, mp, 1.0, S.p, npp,
                         s));
  }
  int hst[4];
  HIPCHK(hipMemcpyAsync(hy.data(), yv.p, sizeof(double) * npp, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(hq.data(), q.p, sizeof(double) * npp, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(hst, status.p, sizeof(hst), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (hst[0]) {
    set_err("Sigma22 is not positive definite (leading minor of order %d)", hst[0]);
    return SGP_ENOTPD;
  }
  for (int64_t i = 0; i < np; ++i) pred_mean[i] = mu_pred[i] + hy[(size_t)i];
  if (!full_cov) {
    // vi_functions.R:1321: tau^2 + sigma^2 + delta; laplace_approx_prediction.R:114: sigma^2 + tau^2
    // predict_gp_full: diag(Sigma11) = sigma^2 + tau^2 + delta
    const double c0 = (method == SGP_PRED_VI) ? (kp.tau2 + kp.sig2) + delta
                                              : (full ? (kp.sig2 + kp.tau2) + delta
                                                      : kp.sig2 + kp.tau2);
    for (int64_t i = 0; i < np; ++i) pred_var[i] = c0 + hq[(size_t)i];
    return SGP_OK;
  }
  std::vector<double> hS((size_t)(npp * npp));
  HIPCHK(hipMemcpyAsync(hS.data(), S.p, sizeof(double) * hS.size(), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  for (int64_t j = 0; j < np; ++j)
    for (int64_t i = 0; i < np; ++i) pred_var[i + j * ldpv] = hS[(size_t)(i * npp + j)];
  if (lap_full) {   // diag(diag(Sigma11 - Q)) + Q with Sigma11_ii = sigma^2 + tau^2 + delta
    const double c11 = (kp.sig2 + kp.tau2) + delta;
    for (int64_t i = 0; i < np; ++i) pred_var[i + i * ldpv] += c11 - hq[(size_t)i];
  }
  return SGP_OK;
}


// ------------------------------------------------------------------------- OAT candidates
// ELBO of the knot sets [U; x*_t] for T candidate knots at fixed theta, as the meta-model
// y values of knot_prop_random_norm_vi / knot_prop_ego_norm_vi (R/vi_functions.R:2196-2300)
// compute them -- but without rebuilding K12 per candidate: a candidate borders K22, S and
// Bm by one row/column, so its ELBO follows from the base evaluation plus Schur complements
// (DESIGN.md sec. 3.5).  Work per 128 candidates: one K(X, x*) build and one n x m x 128 TN
// GEMM (K^T Kc) instead of 128 SYRKs.
int sgp_vi_candidates(sgp_ctx* c, int kernel, const double* theta, const double* U, int64_t m,
                      int64_t ldu, double delta, unsigned flags, const double* cand, int64_t T,
                      int64_t ldc, double* obj_out) {
  MULTI_FWD(c, U && cand && T >= 1 && ldc >= T && obj_out && m >= 1 && ldu >= m ? multi_vi_candidates(c->multi, kernel, theta, U, m, ldu, delta, flags, cand, T, ldc, obj_out) : multi_bad_args());
  if (!c || !cand || T < 1 || ldc < T || !obj_out) {
    set_err("invalid sgp_vi_candidates arguments");
    return SGP_EINVAL;
  }
  int st = sgp_vi_phase1(c, kernel, theta, U, m, ldu, delta, c->red1);
  if (st) return st;
  const KernParams& kp = c->kp;
  const int64_t mp = c->mp, mm = mp * mp, n_pad = c->n_pad, d = kp.d;
  const double z = kp.tau2 + delta;
  const double* S = c->red1;
  const int64_t toff = vi_red1_toff(c, mp);
  const double* t = c->red1 + toff;
  if (c->pack_red1) {
    HIPCHK(launch_unpack_lower64(c->red1, mp, c->Sfull, c->stream));
    S = c->Sfull;
  }
  // K22's inverse was queued on aux by sgp_vi_phase1; it runs beside Bm's
  st = bm_stage(c, S, 1.0 / z, c->vi_k22_ordered);   // as sgp_vi_phase2
  if (st) return st;
  HIPCHK(hipStreamWaitEvent(c->stream, c->ev_k22, 0));
  {
    Scope tm(c, "mm_vectors");
    HIPCHK(dense_gemv(c->Binv, mp, t, 1.0 / z, c->uvec, c->stream));
    HIPCHK(launch_dot(t, c->uvec, mp, c->slab_small, c->sc + SC_TU, c->stream));
    HIPCHK(launch_dot(c->K22inv, S, mm, c->slab_small, c->sc + SC_TRKS, c->stream));
    HIPCHK(hipMemcpyAsync(c->sc + SC_RR, c->red1 + toff + mp, sizeof(double),
                          hipMemcpyDeviceToDevice, c->stream));
  }
  // the candidate builds' parameters: phase 1's (same centre), with the accuracy guard's span
  // widened to the candidates, which may lie outside the data box (knot bounds, Q9)
  KernParams kpc = kp;
  set_center(&kpc, U, m, ldu, c->xmin.data(), c->xmax.data(), cand, T, ldc);
  constexpr int64_t TP = 128;
  DevBuf Kc, slab, P, part, rk, cc, Uc, K22c, W, SW, Bt, BB, base, out;
  const int64_t slab_cap = gemm_tn_slab_doubles(n_pad, mp, TP);
  const int64_t part_cap = lap_gemv_cols_slab(n_pad, TP, 1);
  st = dalloc(&Kc.p, n_pad * TP);
  st = st ? st : dalloc(&slab.p, slab_cap);
  st = st ? st : dalloc(&P.p, mp * TP);
  st = st ? st : dalloc(&part.p, part_cap);
  st = st ? st : dalloc(&rk.p, TP);
  st = st ? st : dalloc(&cc.p, TP);
  st = st ? st : dalloc(&Uc.p, TP * d);
  st = st ? st : dalloc(&K22c.p, mp * TP);
  st = st ? st : dalloc(&W.p, mp * TP);
  st = st ? st : dalloc(&SW.p, mp * TP);
  st = st ? st : dalloc(&Bt.p, mp * TP);
  st = st ? st : dalloc(&BB.p, mp * TP);
  st = st ? st : dalloc(&base.p, 2);
  st = st ? st : dalloc(&out.p, TP * 4);
  if (st) return st;
  // Sigma22' diagonal entry of the new knot: make_cov (sigma^2 + tau^2 + delta) - tau^2
  const double kxx = ((kp.sig2 + kp.tau2) + delta) - kp.tau2;
  const double hb[2] = {kxx, z};
  HIPCHK(hipMemcpyAsync(base.p, hb, sizeof(hb), hipMemcpyHostToDevice, c->stream));
  double sc[SC_N];
  int status[4];
  HIPCHK(hipMemcpyAsync(sc, c->sc, sizeof(sc), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(status, c->status, sizeof(status), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  c->phase = 0;
  if (chain_watchdog(status)) return SGP_EHIP;
  if (status[0] || status[1]) {
    set_err("chol(): the leading minor of order %d of %s is not positive definite",
            status[0] ? status[0] : status[1],
            status[0] ? "Sigma22" : "Sigma22 + t(Sigma12) %*% ZSig12");
    return SGP_ENOTPD;
  }
  const double n = (double)c->n;
  const double ld22 = 2.0 * sc[SC_LD22], ldB = 2.0 * sc[SC_LDB];
  const double quad = -0.5 * sc[SC_RR] / z + 0.5 * sc[SC_TU] / z;   // u = Bm^-1 t / z
  const double trKS = sc[SC_TRKS];
  std::vector<double> hU((size_t)(TP * d)), ho((size_t)(TP * 4));
  for (int64_t t0 = 0; t0 < T; t0 += TP) {
    const int64_t tc = (T - t0 < TP) ? T - t0 : TP;
    std::fill(hU.begin(), hU.end(), 0.0);
    for (int q = 0; q < d; ++q)
      for (int64_t j = 0; j < tc; ++j) hU[(size_t)(q * TP + j)] = cand[(t0 + j) + q * ldc];
    HIPCHK(hipMemcpyAsync(Uc.p, hU.data(), sizeof(double) * hU.size(), hipMemcpyHostToDevice,
                          c->stream));
    Scope tm(c, "candidates");
    HIPCHK(launch_build_knm(kpc, c->X, n_pad, c->n, n_pad, Uc.p, TP, tc, TP, Kc.p, c->stream));
    HIPCHK(launch_gemm_tn(c->K, mp, mp, Kc.p, TP, TP, n_pad, slab.p, slab_cap, P.p, c->stream));
    HIPCHK(launch_gemv_cols(Kc.p, n_pad, TP, c->r, n_pad, 1, part.p, part_cap, rk.p, c->stream));
    HIPCHK(launch_colnorm2(Kc.p, n_pad, TP, part.p, part_cap, cc.p, c->stream));
    HIPCHK(launch_build_knm(kpc, c->U, mp, m, mp, Uc.p, TP, tc, TP, K22c.p, c->stream));
    HIPCHK(launch_gemm64(false, false, false, mp, TP, mp, 1.0, c->K22inv, mp, K22c.p, TP, 0.0,
                         W.p, TP, c->stream));
    HIPCHK(launch_gemm64(false, false, false, mp, TP, mp, 1.0, S, mp, W.p, TP, 0.0, SW.p, TP,
                         c->stream));
    HIPCHK(dense_axpby(1.0, K22c.p, 1.0 / z, P.p, Bt.p, mp * TP, c->stream));
    HIPCHK(launch_gemm64(false, false, false, mp, TP, mp, 1.0, c->Binv, mp, Bt.p, TP, 0.0, BB.p,
                         TP, c->stream));
    HIPCHK(launch_vi_cand_scalars(m, mp, tc, TP, K22c.p, W.p, SW.p, P.p, Bt.p, BB.p, c->uvec,
                                  rk.p, cc.p, base.p, out.p, c->stream));
    HIPCHK(hipMemcpyAsync(ho.data(), out.p, sizeof(double) * tc * 4, hipMemcpyDeviceToHost,
                          c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (int64_t j = 0; j < tc; ++j) {
      const double sK = ho[(size_t)(j * 4)], sB = ho[(size_t)(j * 4 + 1)];
      const double dq = ho[(size_t)(j * 4 + 2)], trinc = ho[(size_t)(j * 4 + 3)];
      if (!(sK > 0.0) || !(sB > 0.0)) {   // the reference's chol() would fail (try-error)
        obj_out[t0 + j] = NAN;
        continue;
      }
      const double ld22c = ld22 + log(sK), ldBc = ldB + log(sB);
      const double logdet22 = (flags & SGP_FLAG_R_DET) ? log(exp(ld22c)) : ld22c;
      const double qd = quad + 0.5 * dq * dq / (z * z * sB);
      const double det_part = -0.5 * (n * log(z) - logdet22 + ldBc);
      const double tt = -(1.0 / (2.0 * kp.tau2)) * (n * (kp.sig2 + delta) - (trKS + trinc / sK));
      obj_out[t0 + j] = qd + det_part - (n / 2.0) * log(2.0 * M_PI) + tt;
    }
  }
  return SGP_OK;
}

// [U; cand_t] (m + 1) x d column-major on the host
static void bordered_knots(const double* U, int64_t m, int64_t ldu, int d, const double* cand,
                           int64_t t, int64_t ldc, std::vector<double>& Ub) {
  Ub.resize((size_t)((m + 1) * d));
  for (int q = 0; q < d; ++q) {
    for (int64_t k = 0; k < m; ++k) Ub[(size_t)(k + q * (m + 1))] = U[k + q * ldu];
    Ub[(size_t)(m + q * (m + 1))] = cand[t + q * ldc];
  }
}

// FITC meta-model values (knot_proposal_functions.R:1292-1319 per candidate): obj_fun_norm at
// [U; cand_t].  Each candidate changes Z for every row, so unlike VI there is no bordered
// shortcut for the weighted Gram matrix; each one is an objective-only FITC evaluation
// (builder, row-quadratic, SYRK, m x m inverse) on the resident rows.
int sgp_fitc_candidates(sgp_ctx* c, int kernel, const double* theta, const double* U, int64_t m,
                        int64_t ldu, double delta, unsigned flags, const double* cand, int64_t T,
                        int64_t ldc, double* obj_out) {
  MULTI_FWD(c, U && cand && T >= 1 && ldc >= T && obj_out && m >= 1 && ldu >= m ? multi_fitc_candidates(c->multi, kernel, theta, U, m, ldu, delta, flags, cand, T, ldc, obj_out) : multi_bad_args());
  if (!c || !U || !cand || T < 1 || ldc < T || !obj_out || m < 1 || ldu < m) {
    set_err("invalid sgp_fitc_candidates arguments");
    return SGP_EINVAL;
  }
  if (m + 1 > c->m_max) {
    set_err("m + 1 = %lld knots exceed the context's m_max = %lld", (long long)(m + 1),
            (long long)c->m_max);
    return SGP_EINVAL;
  }
  std::vector<double> Ub;
  for (int64_t t = 0; t < T; ++t) {
    bordered_knots(U, m, ldu, c->d, cand, t, ldc, Ub);
    double o = 0.0;
    int st = sgp_eval_fitc(c, kernel, theta, Ub.data(), m + 1, m + 1, delta,
                           flags | SGP_FLAG_OBJ_ONLY, &o, nullptr);
    if (st == SGP_ENOTPD) {   // the reference's try-error
      obj_out[t] = NAN;
      continue;
    }
    if (st) return st;
    obj_out[t] = o;
  }
  c->last_mode = 0;   // the context's posterior state belongs to the last candidate
  return SGP_OK;
}

// Laplace meta-model values (knot_proposal_functions.R:1116-1160 per candidate): the last NR
// objective value of newtrap_sparseGP at [U; cand_t], started from the same f every time.
int sgp_lap_candidates(sgp_ctx* c, int kernel, const double* theta, const double* U, int64_t m,
                       int64_t ldu, double delta, double expo, double tol, int maxit,
                       const double* cand, int64_t T, int64_t ldc, double* obj_out) {
  MULTI_FWD(c, U && cand && T >= 1 && ldc >= T && obj_out && m >= 1 && ldu >= m ? multi_lap_candidates(c->multi, kernel, theta, U, m, ldu, delta, expo, tol, maxit, cand, T, ldc, obj_out) : multi_bad_args());
  if (!c || !U || !cand || T < 1 || ldc < T || !obj_out || m < 1 || ldu < m) {
    set_err("invalid sgp_lap_candidates arguments");
    return SGP_EINVAL;
  }
  if (m + 1 > c->m_max) {
    set_err("m + 1 = %lld knots exceed the context's m_max = %lld", (long long)(m + 1),
            (long long)c->m_max);
    return SGP_EINVAL;
  }
  HIPCHK(hipSetDevice(c->device));
  int st = lap_ensure(c);
  if (st) return st;
  DevBuf f0;
  st = dalloc(&f0.p, c->n_pad);
  if (st) return st;
  HIPCHK(hipMemcpyAsync(f0.p, lvec(c, LV_F), sizeof(double) * c->n_pad, hipMemcpyDeviceToDevice,
                        c->stream));
  std::vector<double> Ub;
  for (int64_t t = 0; t < T && st == SGP_OK; ++t) {
    bordered_knots(U, m, ldu, c->d, cand, t, ldc, Ub);
    if (t > 0)
      HIPCHK(hipMemcpyAsync(lvec(c, LV_F), f0.p, sizeof(double) * c->n_pad,
                            hipMemcpyDeviceToDevice, c->stream));
    double o = 0.0;
    int it = 0;
    st = sgp_lap_nr(c, kernel, theta, Ub.data(), m + 1, m + 1, delta, expo, tol, maxit, &o, &it);
    if (st == SGP_ENOTPD) {
      obj_out[t] = NAN;
      st = SGP_OK;
      continue;
    }
    if (st == SGP_OK) obj_out[t] = o;
  }
  HIPCHK(hipMemcpyAsync(lvec(c, LV_F), f0.p, sizeof(double) * c->n_pad, hipMemcpyDeviceToDevice,
                        c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  c->last_mode = 0;   // the context's posterior state belongs to the last candidate
  c->lap_gpsi_valid = false;
  return st;
}

// ------------------------------------------------------------------------- diagnostics
// (include/sgp_diag.h)

int sgp_diag_gj_pair(int device, int64_t m, const double* A, const double* B, double beta,
                     int per_step, double* invA, double* invS, double* logdet) {
  if (m < 1 || m > 16384 || !A || !B || !invA || !invS || !logdet ||
      !(beta == beta) || (per_step != 0 && per_step != 1)) {
    set_err("invalid sgp_diag_gj_pair arguments (m=%lld, per_step=%d)", (long long)m, per_step);
    return SGP_EINVAL;
  }
  const int64_t mp = round_up(m, SGP_TILE), mm = mp * mp, nb = mp / SGP_DB;
  if (!per_step && nb > 64) {
    set_err("sgp_diag_gj_pair: the persistent chain takes m <= 4096 (m = %lld)", (long long)m);
    return SGP_EINVAL;
  }
  HIPCHK(hipSetDevice(device));
  StreamGuard s_main, s_aux;
  HIPCHK(hipStreamCreateWithFlags(&s_main.s, hipStreamNonBlocking));
  HIPCHK(hipStreamCreateWithFlags(&s_aux.s, hipStreamNonBlocking));
  DevBuf dA, dB, dInvA, dInvS, R1, R2, P1, P2, L1, L2;
  IntBuf status, sync;
  int st = dalloc(&dA.p, mm);
  st = st ? st : dalloc(&dB.p, mm);
  st = st ? st : dalloc(&dInvA.p, mm);
  st = st ? st : dalloc(&dInvS.p, mm);
  st = st ? st : dalloc(&R1.p, mm);
  st = st ? st : dalloc(&R2.p, mm);
  st = st ? st : dalloc(&P1.p, mp * 64);
  st = st ? st : dalloc(&P2.p, mp * 64);
  st = st ? st : dalloc(&L1.p, nb);
  st = st ? st : dalloc(&L2.p, nb);
  st = st ? st : dalloc(&status.p, 4);
  st = st ? st : dalloc(&sync.p, 2 * SGP_GJ_SYNC_WORDS);
  if (st) return st;
  // row-major padded as the contexts hold them: A padded with the identity, B with zeros
  std::vector<double> hA((size_t)mm, 0.0), hB((size_t)mm, 0.0);
  for (int64_t i = 0; i < mp; ++i)
    for (int64_t j = 0; j < mp; ++j) {
      const bool in = i < m && j < m;
      hA[(size_t)(i * mp + j)] = in ? A[i + j * m] : (i == j ? 1.0 : 0.0);
      hB[(size_t)(i * mp + j)] = in ? B[i + j * m] : 0.0;
    }
  HIPCHK(hipMemcpy(dA.p, hA.data(), sizeof(double) * mm, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dB.p, hB.data(), sizeof(double) * mm, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dInvA.p, hA.data(), sizeof(double) * mm, hipMemcpyHostToDevice));
  HIPCHK(hipMemset(status.p, 0, sizeof(int) * 4));
  HIPCHK(hipMemset(sync.p, 0, sizeof(int) * 2 * SGP_GJ_SYNC_WORDS));
  // hipMemset runs on the null stream, which non-blocking streams do not wait for: the chains'
  // sync words must be zero before either chain starts
  HIPCHK(hipDeviceSynchronize());
  unsigned* sy = reinterpret_cast<unsigned*>(sync.p);
  // both chains in flight together, as VI's phase 2 issues them
  HIPCHK(dense_spd_inverse_chain(dInvA.p, mp, R1.p, P1.p, L1.p, status.p, sy + SGP_GJ_SYNC_WORDS,
                                 s_aux.s, per_step != 0));
  HIPCHK(dense_spd_inverse_sum_chain(dA.p, beta, dB.p, dInvS.p, mp, R2.p, P2.p, L2.p,
                                     status.p + 1, sy, s_main.s, per_step != 0));
  HIPCHK(hipStreamSynchronize(s_aux.s));
  HIPCHK(hipStreamSynchronize(s_main.s));
  int hs[4];
  std::vector<double> ld1((size_t)nb), ld2((size_t)nb);
  HIPCHK(hipMemcpy(hs, status.p, sizeof(hs), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(ld1.data(), L1.p, sizeof(double) * nb, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(ld2.data(), L2.p, sizeof(double) * nb, hipMemcpyDeviceToHost));
  if (chain_watchdog(hs)) return SGP_EHIP;
  if (hs[0] || hs[1]) {
    set_err("chol(): the leading minor of order %d of %s is not positive definite",
            hs[0] ? hs[0] : hs[1], hs[0] ? "A" : "A + beta B");
    return SGP_ENOTPD;
  }
  HIPCHK(hipMemcpy(hA.data(), dInvA.p, sizeof(double) * mm, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(hB.data(), dInvS.p, sizeof(double) * mm, hipMemcpyDeviceToHost));
  for (int64_t i = 0; i < m; ++i)
    for (int64_t j = 0; j < m; ++j) {
      invA[i + j * m] = hA[(size_t)(i * mp + j)];
      invS[i + j * m] = hB[(size_t)(i * mp + j)];
    }
  // block log-determinant halves summed in block order (the evaluations' order)
  double a = 0.0, b = 0.0;
  for (int64_t k = 0; k < nb; ++k) {
    a += ld1[(size_t)k];
    b += ld2[(size_t)k];
  }
  logdet[0] = 2.0 * a;
  logdet[1] = 2.0 * b;
  return SGP_OK;
}

namespace {
typedef double sgp_d2 __attribute__((ext_vector_type(2)));
// pattern 0: one linear stream, 16 B per lane per instruction
__global__ void __launch_bounds__(256) k_diag_store_lin(sgp_d2* __restrict__ p, int64_t n2,
                                                        double v) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256)
    __builtin_nontemporal_store(sgp_d2{v, v}, &p[i]);
}
// pattern 1: the K12 builder's store shape -- per wave instruction 4 rows x 256 B of a
// row-major matrix with mp = 1024 doubles per row; a workgroup owns 128 columns and walks 64-row
// blocks
__global__ void __launch_bounds__(256) k_diag_store_tile(double* __restrict__ K, int64_t nrb,
                                                         int64_t mp, double v) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, ln = lane & 15, lq = lane >> 4;
  const int64_t j0 = (int64_t)blockIdx.x * 128;
  for (int64_t rb = blockIdx.y; rb < nrb; rb += gridDim.y) {
    const int64_t ib = rb * 64 + 16 * w;
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t i = ib + lq + 4 * r;
        __builtin_nontemporal_store(sgp_d2{v, v},
                                    reinterpret_cast<sgp_d2*>(&K[i * mp + j0 + 32 * p + 2 * ln]));
      }
  }
}
}  // namespace

int sgp_diag_store_bw(int device, int64_t bytes, int reps, int pattern, double* gbs) {
  if (!gbs || bytes < (int64_t)(1 << 20) || reps < 1 || (pattern != 0 && pattern != 1)) {
    set_err("invalid sgp_diag_store_bw arguments");
    return SGP_EINVAL;
  }
  HIPCHK(hipSetDevice(device));
  const int64_t mp = 1024;
  const int64_t nrb = bytes / (64 * mp * 8);
  if (nrb < 1) { set_err("sgp_diag_store_bw: bytes < one 64-row block"); return SGP_EINVAL; }
  const int64_t used = nrb * 64 * mp * 8;
  DevBuf buf;
  int st = dalloc(&buf.p, used / 8);
  if (st) return st;
  int cus = 0;
  HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  StreamGuard sg;
  HIPCHK(hipStreamCreateWithFlags(&sg.s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&e1));
  double best = 0.0;
  hipError_t err = hipSuccess;
  for (int r = 0; r <= reps && err == hipSuccess; ++r) {   // pass 0 warms up
    err = hipEventRecord(e0, sg.s);
    if (pattern == 0)
      hipLaunchKernelGGL(k_diag_store_lin, dim3((unsigned)(cus * 16)), dim3(256), 0, sg.s,
                         reinterpret_cast<sgp_d2*>(buf.p), used / 16, (double)r);
    else
      hipLaunchKernelGGL(k_diag_store_tile, dim3((unsigned)(mp / 128), (unsigned)(cus * 2)),
                         dim3(256), 0, sg.s, buf.p, nrb, mp, (double)r);
    if (err == hipSuccess) err = hipGetLastError();
    if (err == hipSuccess) err = hipEventRecord(e1, sg.s);
    if (err == hipSuccess) err = hipEventSynchronize(e1);
    float ms = 0.0f;
    if (err == hipSuccess) err = hipEventElapsedTime(&ms, e0, e1);
    if (err == hipSuccess && r > 0 && ms > 0.0f) best = std::max(best, (double)used / (ms * 1e6));
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  HIPCHK(err);
  *gbs = best;
  return SGP_OK;
}

}  // extern "C"
