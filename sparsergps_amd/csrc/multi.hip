// Row-sharded multi-device contexts: one process, several GPUs of one node, RCCL over xGMI.
//
// BASELINE.json north_star / SURVEY.md sec. 8(b) and config C4: "sharding the n observation
// rows across the 8 GPUs of one node with an RCCL all-reduce over xGMI for the Qnn-diag trace
// term and log-likelihood accumulators", driven from host-side R through the C ABI
// (R/optimize_gp.R:297-315 -> R/vi_functions.R:733-771 for VI, R/laplace_gradient_ascent.R:
// 1568-1603 for FITC, R/newtrap_sparseGP.R:6-186 for Laplace).  Every n-indexed sum of the
// reference's objective and gradient (R/vi_functions.R:87-118, 227-253;
// R/laplace_approx_obj_funs.R:6-52; R/laplace_approx_gradient.R:25-553, 720-1135) is
// row-separable, so an evaluation is the one-device evaluation split at its reduction points
// (the sgp_vi_phase* / sgp_fitc_phase* / sgp_lap_begin+step entry points of capi.hip) with the
// partial sums added up between them:
//
//   shard s (rows [r0_s, r1_s) on device dev_s)   phase / step -> partial buffer
//   device g: k_sum_parts over its shards, fixed shard order    -> red_g   (on g's stream)
//   all devices: ncclAllReduce(red_g, in place, sum)            -> every device holds the total
//   shard s: the next phase / step reads red_g
//
// One host worker thread per distinct device issues its shards' work and its collective, so the
// devices start together (a single issuing thread would stagger them by the host cost of each
// phase); a host barrier before every collective lets all workers abandon an evaluation together
// when one fails (none is then left waiting inside a collective).  A device may hold several
// shards (a repeated entry in `devices`): their partials are summed by k_sum_parts before the
// collective, which is how the 8-shard composition of C4 is tested on a one-GPU box.  All
// decisions (the Laplace NR stop rule) are functions of the summed buffers, so every shard takes
// the same path; the replicated m x m state of shard 0 answers the posterior, knot-gradient and
// objective-history queries.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <cmath>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "sgp_internal.h"
#include "sgp_multi.h"
#include "sgp_pool.h"

namespace {

// RCCL, bound at the first multi-device context rather than at load time: a process that also
// runs torch.distributed carries torch's own librccl (NEEDED as "librccl.so", SONAME
// librccl.so.1).  Linking ROCm's librccl.so.1 into libsgp put a second copy in such a process
// whenever libsgp was loaded first (the names differ, so the loader does not share them); with
// the symbols interposed across the two copies their exit-time destructors freed the same
// objects ("double free or corruption" after a GPU test run).  Here an already loaded RCCL is
// reused (RTLD_NOLOAD), and otherwise ROCm's is opened RTLD_LOCAL, so it never interposes.
struct Rccl {
  ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  bool ok = false;
  std::string err;
};

const Rccl& rccl() {
  static Rccl r = [] {
    Rccl x;
    void* h = nullptr;
    for (const char* nm : {"librccl.so.1", "librccl.so"})
      if (!h) h = dlopen(nm, RTLD_NOW | RTLD_NOLOAD);
    for (const char* nm : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"})
      if (!h) h = dlopen(nm, RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      const char* e = dlerror();
      x.err = std::string("cannot load librccl (the multi-device context's collectives): ") +
              (e ? e : "unknown error");
      return x;
    }
    x.comm_init_all = reinterpret_cast<decltype(x.comm_init_all)>(dlsym(h, "ncclCommInitAll"));
    x.all_reduce = reinterpret_cast<decltype(x.all_reduce)>(dlsym(h, "ncclAllReduce"));
    x.comm_destroy = reinterpret_cast<decltype(x.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    x.comm_abort = reinterpret_cast<decltype(x.comm_abort)>(dlsym(h, "ncclCommAbort"));
    x.error_string = reinterpret_cast<decltype(x.error_string)>(dlsym(h, "ncclGetErrorString"));
    x.ok = x.comm_init_all && x.all_reduce && x.comm_destroy && x.comm_abort && x.error_string;
    if (!x.ok)
      x.err = "librccl lacks ncclCommInitAll / ncclAllReduce / ncclCommDestroy / ncclCommAbort";
    return x;
  }();
  return r;
}

struct Shard {
  sgp_ctx* ctx = nullptr;
  int device = 0;
  int group = 0;
  int64_t row0 = 0, rows = 0;
  double* part = nullptr;     // partial sums (only when its device holds more than one shard)
};

struct Group {
  int device = 0;
  std::vector<int> shards;
  hipStream_t stream = nullptr;
  ncclComm_t comm = nullptr;
  double* red[2] = {nullptr, nullptr};   // summed buffers (ping-pong)
};

struct PartPtrs {
  const double* p[SGP_MAX_SHARDS];
  int k;
};

// out[i] = sum_q parts[q][i] in shard order (deterministic)
__global__ void __launch_bounds__(256) k_sum_parts(PartPtrs pp, int64_t count, double* out) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < count;
       i += (int64_t)gridDim.x * 256) {
    double v = pp.p[0][i];
    for (int q = 1; q < pp.k; ++q) v += pp.p[q][i];
    out[i] = v;
  }
}

std::string hip_msg(hipError_t e, const char* what) {
  char b[256];
  snprintf(b, sizeof(b), "HIP error '%s' in %s", hipGetErrorString(e), what);
  return b;
}

}  // namespace

struct MultiCtx {
  std::vector<Shard> shards;
  std::vector<Group> groups;
  int64_t n = 0, m_max = 0, cap = 0;
  int d = 0;
  bool knot_on = false;
  std::vector<double> xmin, xmax;   // column ranges of all rows
  // the host workers (sgp_pool.h: one per distinct device, barriers with votes, the job bodies)
  std::unique_ptr<sgp_pool::Pool> pool;
  std::vector<sgp_pool::Result> res;   // per group; every group computes the same, group 0's
                                       // are returned
  // a collective failed to enqueue on one device after its peers' were queued: the
  // communicators are aborted and rebuilt before any stream of this context is synchronised
  std::atomic<bool> broken{false};
  bool dead = false;   // the rebuild failed: every evaluation is refused
  std::string dead_msg;

  sgp_ctx* ctx(const Group& g, int q) { return shards[(size_t)g.shards[(size_t)q]].ctx; }
  // where shard q of group g writes its partial sums (straight into the summed buffer when
  // it is the device's only shard)
  double* out_of(Group& g, int q, double* red) {
    return g.shards.size() == 1 ? red : shards[(size_t)g.shards[(size_t)q]].part;
  }

  // the device's shards' partials -> red (fixed shard order)
  int sum_parts(Group& g, double* red, int64_t count) {
    PartPtrs pp{};
    pp.k = (int)g.shards.size();
    for (int q = 0; q < pp.k; ++q) pp.p[q] = shards[(size_t)g.shards[(size_t)q]].part;
    int64_t nb = (count + 255) / 256;
    if (nb > 4096) nb = 4096;
    hipLaunchKernelGGL(k_sum_parts, dim3((unsigned)nb), dim3(256), 0, g.stream, pp, count, red);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      sgp_internal_set_err(hip_msg(e, "k_sum_parts").c_str());
      return SGP_EHIP;
    }
    return SGP_OK;
  }

  // the all-reduce over the devices, in place on the device's stream
  int all_reduce(Group& g, double* red, int64_t count) {
#ifdef SGP_PROBE_BUILD
    // fault injection (probe builds only): SGP_PROBE_FAIL_COLLECTIVE=<device> makes that
    // device's next collective fail to enqueue after its peers' were queued
    static const char* fail = getenv("SGP_PROBE_FAIL_COLLECTIVE");
    if (fail && atoi(fail) == g.device) {
      sgp_internal_set_err("RCCL all-reduce failed: injected (SGP_PROBE_FAIL_COLLECTIVE)");
      return SGP_EHIP;
    }
#endif
    const ncclResult_t r = rccl().all_reduce(red, red, (size_t)count, ncclDouble, ncclSum, g.comm,
                                             g.stream);
    if (r != ncclSuccess) {
      char b[256];
      snprintf(b, sizeof(b), "RCCL all-reduce failed: %s", rccl().error_string(r));
      sgp_internal_set_err(b);
      return SGP_EHIP;
    }
    return SGP_OK;
  }

  int set_dev(const Group& g) {
    const hipError_t e = hipSetDevice(g.device);
    if (e != hipSuccess) {
      sgp_internal_set_err(hip_msg(e, "hipSetDevice").c_str());
      return SGP_EHIP;
    }
    return SGP_OK;
  }

  // one communicator per distinct device, all in this process
  int init_comms() {
    std::vector<ncclComm_t> comms(groups.size());
    std::vector<int> devs;
    for (const Group& g : groups) devs.push_back(g.device);
    const ncclResult_t r = rccl().comm_init_all(comms.data(), (int)devs.size(), devs.data());
    if (r != ncclSuccess) {
      char b[256];
      snprintf(b, sizeof(b), "ncclCommInitAll over %d devices failed: %s", (int)devs.size(),
               rccl().error_string(r));
      sgp_internal_set_err(b);
      return SGP_EHIP;
    }
    for (size_t g = 0; g < comms.size(); ++g) groups[g].comm = comms[g];
    return SGP_OK;
  }

  // after a broken collective: abort every communicator (its queued collectives exit), drain
  // the streams, rebuild the communicators.  The evaluation's own error stays the reported one.
  void recover() {
    if (!broken.load()) return;
    broken.store(false);
    for (Group& g : groups) {
      (void)hipSetDevice(g.device);
      if (g.comm) (void)rccl().comm_abort(g.comm);
      g.comm = nullptr;
    }
    for (Group& g : groups) {
      (void)hipSetDevice(g.device);
      if (g.stream) (void)hipStreamSynchronize(g.stream);
    }
    const std::string keep = sgp_last_error();
    if (init_comms() != SGP_OK) {
      dead = true;
      dead_msg = std::string("multi-device context unusable: rebuilding its communicators after "
                             "a failed collective failed (") + sgp_last_error() + ")";
    }
    sgp_internal_set_err(keep.c_str());
  }

  // run a job on every group (sgp_pool.h), then the communicator repair it may need
  int run(const std::function<int(int)>& job) {
    if (dead) {
      sgp_internal_set_err(dead_msg.c_str());
      return SGP_EHIP;
    }
    std::string msg;
    const int st = pool->run_all(job, &msg);
    if (st) sgp_internal_set_err(msg.c_str());
    recover();
    return st;
  }

  void release() {
    pool.reset();   // joins the workers
    for (Group& g : groups) {
      (void)hipSetDevice(g.device);
      if (g.stream) (void)hipStreamSynchronize(g.stream);
    }
    // (an evaluation's aux-stream work is joined into the launch stream before it returns)
    // reverse order: a device's first shard owns the streams its other shards borrow
    for (size_t k = shards.size(); k-- > 0;) {
      if (shards[k].ctx) sgp_ctx_destroy(shards[k].ctx);
      shards[k].ctx = nullptr;
    }
    for (Group& g : groups) {
      (void)hipSetDevice(g.device);
      if (g.comm) rccl().comm_destroy(g.comm);
      for (double*& p : g.red)
        if (p) (void)hipFree(p);
      g.stream = nullptr;   // the first shard's, destroyed with it
    }
    for (Shard& s : shards)
      if (s.part) {
        (void)hipSetDevice(s.device);
        (void)hipFree(s.part);
      }
    groups.clear();
    shards.clear();
  }
};

namespace {
std::string last_error_copy() { return sgp_last_error(); }
}  // namespace

// ------------------------------------------------------------------------------ creation
int multi_create(MultiCtx** out, const int* devices, int nshards, const double* X, int64_t n,
                 int64_t ldx, int d, const double* y, const double* mu, int64_t m_max) {
  *out = nullptr;
  MultiCtx* mc = new MultiCtx();
  mc->n = n;
  mc->d = d;
  mc->m_max = m_max;
  // every reduction an evaluation issues fits one buffer (ARD has the most parameters)
  const int64_t extra = sgp_knot_red_extra(d, m_max);
  int64_t cap = sgp_lap_red_count(SGP_KERNEL_ARD, d, m_max);
  cap = std::max<int64_t>(cap, sgp_fitc_red2_count(SGP_KERNEL_ARD, d, m_max) + extra);
  cap = std::max<int64_t>(cap, sgp_vi_red1_count(m_max));
  cap = std::max<int64_t>(cap, sgp_vi_red2_count(SGP_KERNEL_ARD, d) + extra);
  mc->cap = cap;
  // shards: contiguous row blocks as dist.shard_rows(n, N, k); groups: distinct devices in
  // order of first appearance
  const int64_t base = n / nshards, rem = n % nshards;
  int64_t r0 = 0;
  for (int k = 0; k < nshards; ++k) {
    Shard s;
    s.device = devices ? devices[k] : k;
    s.row0 = r0;
    s.rows = base + (k < rem ? 1 : 0);
    r0 += s.rows;
    int g = 0;
    while (g < (int)mc->groups.size() && mc->groups[(size_t)g].device != s.device) ++g;
    if (g == (int)mc->groups.size()) {
      Group gr;
      gr.device = s.device;
      mc->groups.push_back(gr);
    }
    s.group = g;
    mc->groups[(size_t)g].shards.push_back(k);
    mc->shards.push_back(s);
  }
  mc->xmin.assign((size_t)d, 0.0);
  mc->xmax.assign((size_t)d, 0.0);
  for (int q = 0; q < d; ++q) {
    double lo = X[q * ldx], hi = X[q * ldx];
    for (int64_t i = 1; i < n; ++i) {
      const double v = X[i + q * ldx];
      lo = v < lo ? v : lo;
      hi = v > hi ? v : hi;
    }
    mc->xmin[(size_t)q] = lo;
    mc->xmax[(size_t)q] = hi;
  }
  // per device: summed buffers, the shards' partial buffers (the launch stream is the first
  // shard's own: no extra hardware-queue client -- with more streams than the process's hardware
  // queues (GPU_MAX_HW_QUEUES, 4) the latency-bound Gauss-Jordan steps ran 2.4x slower)
  int st = SGP_OK;
  for (Group& g : mc->groups) {
    hipError_t e = hipSetDevice(g.device);
    for (int b = 0; b < 2 && e == hipSuccess; ++b)
      e = hipMalloc(reinterpret_cast<void**>(&g.red[b]), sizeof(double) * (size_t)cap);
    for (size_t q = 0; q < g.shards.size() && g.shards.size() > 1 && e == hipSuccess; ++q)
      e = hipMalloc(reinterpret_cast<void**>(&mc->shards[(size_t)g.shards[q]].part),
                    sizeof(double) * (size_t)cap);
    for (int b = 0; b < 2 && e == hipSuccess; ++b)
      e = hipMemset(g.red[b], 0, sizeof(double) * (size_t)cap);
    if (e != hipSuccess) {
      sgp_internal_set_err(hip_msg(e, "multi-device context set-up").c_str());
      st = e == hipErrorOutOfMemory ? SGP_ENOMEM : SGP_EHIP;
      break;
    }
  }
  // one RCCL communicator per distinct device, all in this process
  if (!st && !rccl().ok) {
    sgp_internal_set_err(rccl().err.c_str());
    st = SGP_EHIP;
  }
  if (!st) st = mc->init_comms();
  if (st) {
    mc->release();
    delete mc;
    return st;
  }
  mc->pool.reset(new sgp_pool::Pool((int)mc->groups.size(), last_error_copy));
  mc->res.assign(mc->groups.size(), sgp_pool::Result{});
  // the shards' contexts, created by their device's worker (uploads run side by side)
  st = mc->run([&](int gi) {
    Group& g = mc->groups[(size_t)gi];
    int s2 = mc->set_dev(g);
    for (size_t q = 0; q < g.shards.size() && !s2; ++q) {
      Shard& s = mc->shards[(size_t)g.shards[q]];
      s2 = sgp_ctx_create(&s.ctx, s.device, X + s.row0, s.rows, ldx, d, y + s.row0, mu + s.row0,
                          m_max);
      if (!s2 && q == 0) g.stream = sgp_internal_stream(s.ctx);
      // the device's other shards use the first one's streams (one worker issues them in turn)
      if (!s2 && q > 0) s2 = sgp_internal_share_streams(s.ctx, mc->shards[(size_t)g.shards[0]].ctx);
      if (!s2) s2 = sgp_ctx_set_packed_reduction(s.ctx, 1);   // all-reduce #1: 53 % of S
    }
    return s2;
  });
  if (st) {
    mc->release();
    delete mc;
    return st;
  }
  *out = mc;
  return SGP_OK;
}

void multi_destroy(MultiCtx* mc) {
  if (!mc) return;
  mc->release();
  delete mc;
}

int multi_shards(const MultiCtx* mc, int* nshards, int* ndevices) {
  if (nshards) *nshards = (int)mc->shards.size();
  if (ndevices) *ndevices = (int)mc->groups.size();
  return SGP_OK;
}

sgp_ctx* multi_lead(MultiCtx* mc) { return mc->shards[0].ctx; }

int multi_set_data(MultiCtx* mc, const double* y, const double* mu) {
  for (Shard& s : mc->shards) {
    const int st = sgp_ctx_set_data(s.ctx, y + s.row0, mu + s.row0);
    if (st) return st;
  }
  return SGP_OK;
}

// ------------------------------------------------------------------------------ evaluations
namespace {

struct EvalArgs {
  int kernel;
  const double* theta;
  const double* U;
  int64_t m, ldu;
  double delta;
  unsigned flags;
  // Laplace
  double expo = 1.0, tol = 0.0;
  int maxit = 0;
};

// sgp_pool.h's operations on the HIP contexts and the RCCL communicators
struct HipOps {
  MultiCtx* mc;
  const EvalArgs& a;
  bool fitc;

  int begin(int g) { return mc->set_dev(mc->groups[(size_t)g]); }
  int shards(int g) { return (int)mc->groups[(size_t)g].shards.size(); }
  double* red(int g, int b) { return mc->groups[(size_t)g].red[b]; }
  double* out_of(int g, int q, double* r) { return mc->out_of(mc->groups[(size_t)g], q, r); }
  sgp_ctx* ctx(int g, int q) { return mc->ctx(mc->groups[(size_t)g], q); }
  int phase1(int g, int q, double* out) {
    return fitc ? sgp_fitc_phase1(ctx(g, q), a.kernel, a.theta, a.U, a.m, a.ldu, a.delta, out)
                : sgp_vi_phase1(ctx(g, q), a.kernel, a.theta, a.U, a.m, a.ldu, a.delta, out);
  }
  int phase2(int g, int q, const double* red1, double* out) {
    return fitc ? sgp_fitc_phase2(ctx(g, q), red1, mc->n, a.flags, out)
                : sgp_vi_phase2(ctx(g, q), red1, mc->n, a.flags, out);
  }
  int finish(int g, int q, const double* red2, double* obj, double* grad) {
    return fitc ? sgp_fitc_finish(ctx(g, q), red2, obj, grad)
                : sgp_vi_finish(ctx(g, q), red2, obj, grad);
  }
  int lap_begin(int g, int q, double* out, int64_t* count) {
    return sgp_lap_begin(ctx(g, q), a.kernel, a.theta, a.U, a.m, a.ldu, a.delta, a.expo, a.tol,
                         a.maxit, a.flags, out, count);
  }
  int lap_step(int g, int q, const double* in, double* out, int64_t* count, int* done,
               double* obj, double* grad, int* nr_iters) {
    return sgp_lap_step(ctx(g, q), in, out, count, done, obj, grad, nr_iters);
  }
  int sum_parts(int g, double* r, int64_t count) {
    return mc->sum_parts(mc->groups[(size_t)g], r, count);
  }
  int all_reduce(int g, double* r, int64_t count) {
    return mc->all_reduce(mc->groups[(size_t)g], r, count);
  }
  void collective_broken() { mc->broken.store(true); }
  void set_err(const char* msg) { sgp_internal_set_err(msg); }
};

// VI (fitc = false) or FITC: phase 1 -> all-reduce #1 -> phase 2 -> all-reduce #2 -> finish
int two_phase(MultiCtx* mc, const EvalArgs& a, bool fitc, double* obj, double* grad) {
  const bool obj_only = (a.flags & SGP_FLAG_OBJ_ONLY) != 0;
  const int npar = sgp_num_params(a.kernel, mc->d);
  const int64_t c1 = fitc ? sgp_fitc_red1_count(a.m) : sgp_vi_red1_packed_count(a.m);
  // the objective alone leaves the second buffer unwritten: nothing to sum
  const int64_t extra = mc->knot_on ? sgp_knot_red_extra(mc->d, a.m) : 0;
  const int64_t c2 = obj_only ? 0
                              : (fitc ? sgp_fitc_red2_count(a.kernel, mc->d, a.m)
                                      : sgp_vi_red2_count(a.kernel, mc->d)) + extra;
  HipOps ops{mc, a, fitc};
  const int st = mc->run([&](int gi) {
    return sgp_pool::two_phase_job(ops, *mc->pool, gi, c1, c2, obj_only ? 0 : npar,
                                   mc->res[(size_t)gi]);
  });
  if (st) return st;
  const sgp_pool::Result& r = mc->res[0];
  *obj = r.obj;
  if (grad && !obj_only)
    for (int p = 0; p < npar; ++p) grad[p] = r.grad[(size_t)p];
  return SGP_OK;
}

}  // namespace

int multi_eval_vi(MultiCtx* mc, int kernel, const double* theta, const double* U, int64_t m,
                  int64_t ldu, double delta, unsigned flags, double* obj, double* grad) {
  const EvalArgs a{kernel, theta, U, m, ldu, delta, flags};
  return two_phase(mc, a, false, obj, grad);
}

int multi_eval_fitc(MultiCtx* mc, int kernel, const double* theta, const double* U, int64_t m,
                    int64_t ldu, double delta, unsigned flags, double* obj, double* grad) {
  const EvalArgs a{kernel, theta, U, m, ldu, delta, flags};
  return two_phase(mc, a, true, obj, grad);
}

// sgp_lap_begin -> all-reduce -> (sgp_lap_step -> all-reduce)* until done (sgp_pool.h)
int multi_eval_laplace(MultiCtx* mc, int kernel, const double* theta, const double* U,
                       int64_t m, int64_t ldu, double delta, double expo, double tol, int maxit,
                       unsigned flags, double* obj, double* grad, int* nr_iters) {
  EvalArgs a{kernel, theta, U, m, ldu, delta, flags};
  a.expo = expo;
  a.tol = tol;
  a.maxit = maxit;
  const int npar = sgp_num_params(kernel, mc->d);
  HipOps ops{mc, a, false};
  const int st = mc->run([&](int gi) {
    return sgp_pool::laplace_job(ops, *mc->pool, gi, npar, mc->res[(size_t)gi]);
  });
  if (st) return st;
  const sgp_pool::Result& r = mc->res[0];
  if (obj) *obj = r.obj;
  if (nr_iters) *nr_iters = r.nr_iters;
  if (grad && !(flags & SGP_FLAG_OBJ_ONLY))
    for (int p = 0; p < npar; ++p) grad[p] = r.grad[(size_t)p];
  return SGP_OK;
}

// the latent vector f in the global row order
int multi_lap_set_f(MultiCtx* mc, const double* f, double fill) {
  for (Shard& s : mc->shards) {
    const int st = sgp_lap_set_f(s.ctx, f ? f + s.row0 : nullptr, fill);
    if (st) return st;
  }
  return SGP_OK;
}

// the per-row exposure in the global row order: every value is checked before any shard
// changes, so a rejected vector leaves the context as it was
int multi_lap_set_expo(MultiCtx* mc, const double* a, double fill) {
  if (!a && !(fill > 0.0 && std::isfinite(fill))) {
    char b[160];
    snprintf(b, sizeof(b), "sgp_lap_set_expo: the fill exposure %g is not a positive finite number",
             fill);
    sgp_internal_set_err(b);
    return SGP_EINVAL;
  }
  for (int64_t i = 0; a && i < mc->n; ++i)
    if (!(a[i] > 0.0 && std::isfinite(a[i]))) {
      char b[160];
      snprintf(b, sizeof(b), "sgp_lap_set_expo: exposure a[%lld] = %g is not a positive finite "
               "number", (long long)i, a[i]);
      sgp_internal_set_err(b);
      return SGP_EINVAL;
    }
  for (Shard& s : mc->shards) {
    const int st = sgp_lap_set_expo(s.ctx, a ? a + s.row0 : nullptr, fill);
    if (st) return st;
  }
  return SGP_OK;
}

int multi_lap_get_f(MultiCtx* mc, double* f) {
  for (Shard& s : mc->shards) {
    const int st = sgp_lap_get_f(s.ctx, f + s.row0);
    if (st) return st;
  }
  return SGP_OK;
}

int multi_lap_get_grad_psi(MultiCtx* mc, double* out) {
  for (Shard& s : mc->shards) {
    const int st = sgp_lap_get_grad_psi(s.ctx, out + s.row0);
    if (st) return st;
  }
  return SGP_OK;
}

// ------------------------------------------------------------------------------ knots
int multi_enable_knot_grad(MultiCtx* mc, int enable) {
  for (Shard& s : mc->shards) {
    const int st = sgp_ctx_enable_knot_grad(s.ctx, enable);
    if (st) return st;
  }
  mc->knot_on = enable != 0;
  return SGP_OK;
}

int multi_row_bounds(MultiCtx* mc, double* lo, double* hi) {
  for (int q = 0; q < mc->d; ++q) {
    lo[q] = mc->xmin[(size_t)q];
    hi[q] = mc->xmax[(size_t)q];
  }
  return SGP_OK;
}

// bounds NULL: the reference's knot_bounds over ALL rows (vi_functions.R:175-178), not shard 0's
int multi_knot_gradient(MultiCtx* mc, const double* bounds, double* grad_knot) {
  std::vector<double> b;
  if (!bounds) {
    const int d = mc->d;
    b.assign((size_t)(2 * d), 0.0);
    for (int q = 0; q < d; ++q) {
      const double diff = mc->xmax[(size_t)q] - mc->xmin[(size_t)q];
      b[(size_t)q] = mc->xmin[(size_t)q] - diff / 10;
      b[(size_t)(d + q)] = mc->xmax[(size_t)q] + diff / 10;
    }
    bounds = b.data();
  }
  return sgp_knot_gradient(multi_lead(mc), bounds, grad_knot);
}

// ------------------------------------------------------------------------------ candidates
namespace {

void bordered(const double* U, int64_t m, int64_t ldu, int d, const double* cand, int64_t t,
              int64_t ldc, std::vector<double>& Ub) {
  Ub.resize((size_t)((m + 1) * d));
  for (int q = 0; q < d; ++q) {
    for (int64_t k = 0; k < m; ++k) Ub[(size_t)(k + q * (m + 1))] = U[k + q * ldu];
    Ub[(size_t)(m + q * (m + 1))] = cand[t + q * ldc];
  }
}

void forget_all(MultiCtx* mc) {
  for (Shard& s : mc->shards) sgp_internal_forget_eval(s.ctx);
}

}  // namespace

// VI / FITC meta-model values: the objective-only evaluation at [U; cand_t] over all shards
// (NaN = the reference's try-error).  A VI candidate costs one objective-only evaluation here
// rather than the bordered Schur update of the one-device scorer.
static int cand_loop(MultiCtx* mc, bool fitc, int kernel, const double* theta, const double* U,
                     int64_t m, int64_t ldu, double delta, unsigned flags, const double* cand,
                     int64_t T, int64_t ldc, double* obj_out) {
  if (m + 1 > mc->m_max) {
    char b[160];
    snprintf(b, sizeof(b), "m + 1 = %lld knots exceed the context's m_max = %lld",
             (long long)(m + 1), (long long)mc->m_max);
    sgp_internal_set_err(b);
    return SGP_EINVAL;
  }
  std::vector<double> Ub;
  int st = SGP_OK;
  for (int64_t t = 0; t < T && !st; ++t) {
    bordered(U, m, ldu, mc->d, cand, t, ldc, Ub);
    double o = 0.0;
    st = fitc ? multi_eval_fitc(mc, kernel, theta, Ub.data(), m + 1, m + 1, delta,
                                flags | SGP_FLAG_OBJ_ONLY, &o, nullptr)
              : multi_eval_vi(mc, kernel, theta, Ub.data(), m + 1, m + 1, delta,
                              flags | SGP_FLAG_OBJ_ONLY, &o, nullptr);
    if (st == SGP_ENOTPD) {
      obj_out[t] = NAN;
      st = SGP_OK;
    } else if (!st) {
      obj_out[t] = o;
    }
  }
  forget_all(mc);
  return st;
}

int multi_vi_candidates(MultiCtx* mc, int kernel, const double* theta, const double* U,
                        int64_t m, int64_t ldu, double delta, unsigned flags, const double* cand,
                        int64_t T, int64_t ldc, double* obj_out) {
  return cand_loop(mc, false, kernel, theta, U, m, ldu, delta, flags, cand, T, ldc, obj_out);
}

int multi_fitc_candidates(MultiCtx* mc, int kernel, const double* theta, const double* U,
                          int64_t m, int64_t ldu, double delta, unsigned flags,
                          const double* cand, int64_t T, int64_t ldc, double* obj_out) {
  return cand_loop(mc, true, kernel, theta, U, m, ldu, delta, flags, cand, T, ldc, obj_out);
}

// Laplace: newtrap_sparseGP at [U; cand_t] from the same f every time (the fit's fmax), f
// restored afterwards
int multi_lap_candidates(MultiCtx* mc, int kernel, const double* theta, const double* U,
                         int64_t m, int64_t ldu, double delta, double expo, double tol,
                         int maxit, const double* cand, int64_t T, int64_t ldc,
                         double* obj_out) {
  if (m + 1 > mc->m_max) {
    char b[160];
    snprintf(b, sizeof(b), "m + 1 = %lld knots exceed the context's m_max = %lld",
             (long long)(m + 1), (long long)mc->m_max);
    sgp_internal_set_err(b);
    return SGP_EINVAL;
  }
  std::vector<double> f0((size_t)mc->n);
  int st = multi_lap_get_f(mc, f0.data());
  if (st) return st;
  std::vector<double> Ub;
  for (int64_t t = 0; t < T && !st; ++t) {
    bordered(U, m, ldu, mc->d, cand, t, ldc, Ub);
    if (t > 0) st = multi_lap_set_f(mc, f0.data(), 0.0);
    if (st) break;
    double o = 0.0;
    int it = 0;
    st = multi_eval_laplace(mc, kernel, theta, Ub.data(), m + 1, m + 1, delta, expo, tol, maxit,
                            SGP_FLAG_OBJ_ONLY, &o, nullptr, &it);
    if (st == SGP_ENOTPD) {
      obj_out[t] = NAN;
      st = SGP_OK;
    } else if (!st) {
      obj_out[t] = o;
    }
  }
  const int st2 = multi_lap_set_f(mc, f0.data(), 0.0);
  forget_all(mc);
  return st ? st : st2;
}
