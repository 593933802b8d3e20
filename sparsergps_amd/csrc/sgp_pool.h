// Host-side orchestration of a row-sharded multi-device evaluation (multi.hip), kept free of
// HIP and RCCL so the CPU test suite can drive it with G > 1 fake device groups under
// ThreadSanitizer (tests/pool/pool_driver.cc, tests/test_pool.py).
//
// An evaluation is the one-device evaluation split at its row-sum reductions (the reference's
// n-indexed sums, R/vi_functions.R:87-118, 227-253; R/laplace_approx_obj_funs.R:6-52;
// R/laplace_approx_gradient.R:25-553, 720-1135); between two phases every device group sums its
// shards' partials and then joins an all-reduce over the groups.  Two things can go wrong that a
// single-device evaluation never meets:
//   * one group fails before a collective: its peers must not enter that collective (they would
//     wait in it for ever) -- a barrier with a vote in front of every collective;
//   * one group's collective fails to enqueue after its peers' were queued: the peers' next host
//     synchronisation would wait for ever on their queued collectives -- a second vote right
//     after every collective, before any host synchronisation, and the caller aborts the
//     communicators (Ops::collective_broken) before touching the streams again.
// The Newton-Raphson stop rule of newtrap_sparseGP (R/newtrap_sparseGP.R:77-150) is decided by
// every group from the summed buffers; a disagreement ends every group with SGP_EINVAL instead
// of leaving one waiting at a barrier the others do not reach.
//
// Invariant the job bodies keep: every group performs the same sequence of Pool::arrive calls
// until a vote tells all of them to stop, and a group leaves a job only right after a vote (or
// before its first one when it fails alone -- it then still arrives once with `false`).
#ifndef SGP_POOL_H
#define SGP_POOL_H

#include <stdint.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sgp.h"

namespace sgp_pool {

constexpr int ABORTED = -1;   // a group that stopped because another one failed

inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
  __builtin_ia32_pause();
#endif
}

// One host worker per device group: the calling thread runs group 0, one thread each the
// others.  Hand-offs spin (bounded, then yield / sleep on a condition variable): a
// condition-variable wake-up costs tens to hundreds of microseconds, paid at the start of every
// evaluation and at every barrier.
class Pool {
 public:
  using Job = std::function<int(int)>;
  using ErrFn = std::string (*)();   // the calling thread's last error message

  Pool(int groups, ErrFn err) : G_(groups < 1 ? 1 : groups), err_fn_(err),
                                status_((size_t)G_, SGP_OK), err_((size_t)G_) {
    for (int g = 1; g < G_; ++g) threads_.emplace_back([this, g] { worker(g); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      quit_.store(true);
    }
    cv_job_.notify_all();
    for (std::thread& t : threads_) t.join();
  }
  Pool(const Pool&) = delete;
  Pool& operator=(const Pool&) = delete;

  int groups() const { return G_; }

  // job(g) for every group, group 0 on this thread; waits for all.  Returns the first real
  // error in group order (its message in *msg), SGP_EHIP "aborted" when groups only aborted,
  // SGP_OK otherwise.
  int run_all(const Job& job, std::string* msg) {
    if (G_ > 1) {
      {
        std::lock_guard<std::mutex> lk(mu_);
        job_ = job;
        pending_.store(G_ - 1, std::memory_order_release);
        job_gen_.fetch_add(1, std::memory_order_acq_rel);
      }
      cv_job_.notify_all();
    }
    run_group(0, job);
    int spins = 0;
    while (pending_.load(std::memory_order_acquire) > 0) relax(spins);
    for (int g = 0; g < G_; ++g)
      if (status_[(size_t)g] != SGP_OK && status_[(size_t)g] != ABORTED) {
        if (msg) *msg = err_[(size_t)g];
        return status_[(size_t)g];
      }
    for (int g = 0; g < G_; ++g)
      if (status_[(size_t)g] == ABORTED) {
        if (msg) *msg = "multi-device evaluation aborted";
        return SGP_EHIP;
      }
    return SGP_OK;
  }

  // the status each group's job returned in the last run_all
  int status(int g) const { return status_[(size_t)g]; }

  // Barrier with a vote: every group arrives with ok (and a done flag); returns false for all
  // when any group voted !ok, and sets *any_done / *all_done from the done flags.
  bool arrive(bool ok, bool done = false, bool* any_done = nullptr, bool* all_done = nullptr) {
    if (G_ == 1) {
      if (any_done) *any_done = done;
      if (all_done) *all_done = done;
      return ok;
    }
    uint64_t gen;
    bool last = false;
    {
      std::lock_guard<std::mutex> lk(bmu_);
      gen = b_gen_.load(std::memory_order_relaxed);
      b_all_ok_ = b_all_ok_ && ok;
      b_any_ = b_any_ || done;
      b_all_ = b_all_ && done;
      if (++b_count_ == G_) {
        r_ok_ = b_all_ok_;
        r_any_ = b_any_;
        r_all_ = b_all_;
        b_all_ok_ = true;
        b_any_ = false;
        b_all_ = true;
        b_count_ = 0;
        last = true;
        b_gen_.store(gen + 1, std::memory_order_release);
      }
    }
    if (!last) {
      int spins = 0;
      while (b_gen_.load(std::memory_order_acquire) == gen) relax(spins);
    }
    // r_* still hold this round's votes: the next round cannot complete before this group
    // arrives at it
    std::lock_guard<std::mutex> lk(bmu_);
    if (any_done) *any_done = r_any_;
    if (all_done) *all_done = r_all_;
    return r_ok_;
  }

 private:
  static constexpr int SPIN = 1 << 16;

  static void relax(int& spins) {
    if (++spins < SPIN)
      cpu_relax();
    else
      std::this_thread::yield();
  }

  void run_group(int g, const Job& f) {
    err_[(size_t)g].clear();
    const int st = f(g);
    status_[(size_t)g] = st;
    if (st != SGP_OK && st != ABORTED && err_fn_) err_[(size_t)g] = err_fn_();
  }

  void worker(int g) {
    uint64_t seen = 0;
    for (;;) {
      int spins = 0;
      while (job_gen_.load(std::memory_order_acquire) == seen && !quit_.load()) {
        if (spins < SPIN) {
          relax(spins);
        } else {   // idle for long: sleep until the next job (a system_clock deadline: a
                   // steady_clock wait is a pthread_cond_clockwait, which gcc 11's
                   // ThreadSanitizer does not intercept, so the CPU test could not check it)
          std::unique_lock<std::mutex> lk(mu_);
          cv_job_.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(2), [&] {
            return quit_.load() || job_gen_.load(std::memory_order_acquire) != seen;
          });
        }
      }
      if (quit_.load()) return;
      seen = job_gen_.load(std::memory_order_acquire);
      Job job;
      {
        std::lock_guard<std::mutex> lk(mu_);
        job = job_;
      }
      run_group(g, job);
      pending_.fetch_sub(1, std::memory_order_acq_rel);
    }
  }

  const int G_;
  ErrFn err_fn_;
  std::vector<int> status_;
  std::vector<std::string> err_;
  std::vector<std::thread> threads_;
  std::mutex mu_;
  std::condition_variable cv_job_;
  Job job_;
  std::atomic<uint64_t> job_gen_{0};
  std::atomic<int> pending_{0};
  std::atomic<bool> quit_{false};
  std::mutex bmu_;
  std::atomic<uint64_t> b_gen_{0};
  int b_count_ = 0;
  bool b_all_ok_ = true, b_any_ = false, b_all_ = true;
  bool r_ok_ = true, r_any_ = false, r_all_ = true;
};

// ------------------------------------------------------------------------------ job bodies
// Ops (multi.hip's HIP/RCCL operations, or the CPU test's fakes) provides, for group g and its
// q-th shard:
//   int    begin(int g)                        per-job set-up on the group's thread (device)
//   int    shards(int g)                       shards on the group's device
//   double* red(int g, int b)                  the group's summed buffer b (0 / 1)
//   double* out_of(int g, int q, double* red)  where shard q writes partials bound for `red`
//   int    phase1(g, q, double* out)           VI / FITC phase 1 -> partials
//   int    phase2(g, q, const double* red1, double* out)
//   int    finish(g, q, const double* red2, double* obj, double* grad /* NULL: discard */)
//   int    lap_begin(g, q, double* out, int64_t* count)
//   int    lap_step(g, q, const double* in, double* out, int64_t* count, int* done, double* obj,
//                   double* grad, int* nr_iters)
//   int    sum_parts(g, double* red, int64_t count)   the shards' partials -> red (fixed order)
//   int    all_reduce(g, double* red, int64_t count)  enqueue the in-place sum over the groups
//   void   collective_broken()                        some group's collective failed after its
//                                                     peers' were queued
//   void   set_err(const char*)                       the calling thread's error message
// All status returns are sgp_status values.

struct Result {
  double obj = 0.0;
  std::vector<double> grad;
  int nr_iters = 0;
};

// partials summed on the device, a vote, the collective, a vote.  false: stop now (returning
// st, or ABORTED when this group did not fail itself)
template <class Ops>
bool reduce(Ops& o, Pool& p, int g, double* red, int64_t count, int& st) {
  if (st == SGP_OK && count > 0 && o.shards(g) > 1) st = o.sum_parts(g, red, count);
  if (!p.arrive(st == SGP_OK)) return false;   // someone failed before it: nobody enters
  if (count > 0) st = o.all_reduce(g, red, count);
  if (!p.arrive(st == SGP_OK)) {
    // some group's collective did not enqueue; this group's own (if any) waits for it on the
    // device, so no stream of any group may be synchronised before the communicators go
    if (p.groups() > 1) o.collective_broken();
    return false;
  }
  return true;
}

// VI (fitc = false) or FITC: phase 1 -> all-reduce #1 -> phase 2 -> all-reduce #2 -> finish.
// c1 / c2: the two reduction sizes (c2 = 0 for the objective alone); npar: gradient length
// (0: objective only).
template <class Ops>
int two_phase_job(Ops& o, Pool& p, int g, int64_t c1, int64_t c2, int npar, Result& res) {
  int st = o.begin(g);
  const int k = o.shards(g);
  for (int q = 0; q < k && !st; ++q) st = o.phase1(g, q, o.out_of(g, q, o.red(g, 0)));
  if (!reduce(o, p, g, o.red(g, 0), c1, st)) return st ? st : ABORTED;
  for (int q = 0; q < k && !st; ++q) st = o.phase2(g, q, o.red(g, 0), o.out_of(g, q, o.red(g, 1)));
  if (!reduce(o, p, g, o.red(g, 1), c2, st)) return st ? st : ABORTED;
  res.grad.assign((size_t)(npar > 0 ? npar : 1), 0.0);
  std::vector<double> tmp(res.grad.size());
  for (int q = 0; q < k && !st; ++q) {
    double ob = 0.0;
    double* gp = npar > 0 ? (q == 0 ? res.grad.data() : tmp.data()) : nullptr;
    st = o.finish(g, q, o.red(g, 1), &ob, gp);
    if (q == 0) res.obj = ob;
  }
  return st;
}

// Laplace: begin -> all-reduce -> (step -> all-reduce)* until done (the NR iterations' two
// exchanges and the gradient's two).  Every group stops at the same step:
// the stop rule reads summed buffers only, and the done flags are voted on.
template <class Ops>
int laplace_job(Ops& o, Pool& p, int g, int npar, Result& res) {
  int st = o.begin(g);
  const int k = o.shards(g);
  int64_t count = -1;
  for (int q = 0; q < k && !st; ++q) {
    int64_t cq = 0;
    st = o.lap_begin(g, q, o.out_of(g, q, o.red(g, 0)), &cq);
    if (!st && count >= 0 && cq != count) {
      o.set_err("Laplace shards disagree on the reduction size");
      st = SGP_EINVAL;
    }
    count = cq;
  }
  if (!reduce(o, p, g, o.red(g, 0), count, st)) return st ? st : ABORTED;
  res.grad.assign((size_t)(npar > 0 ? npar : 1), 0.0);
  std::vector<double> tmp(res.grad.size());
  int cur = 0;
  for (;;) {
    bool done = false;
    int64_t cnt = -1;
    for (int q = 0; q < k && !st; ++q) {
      int64_t cq = 0;
      int dq = 0, it = 0;
      double ob = 0.0;
      st = o.lap_step(g, q, o.red(g, cur), o.out_of(g, q, o.red(g, cur ^ 1)), &cq, &dq, &ob,
                      q == 0 ? res.grad.data() : tmp.data(), &it);
      if (st) break;
      if (q > 0 && ((dq != 0) != done || cq != cnt)) {
        o.set_err("Laplace shards disagree on the NR state");
        st = SGP_EINVAL;
        break;
      }
      done = dq != 0;
      cnt = cq;
      if (q == 0) {
        res.obj = ob;
        res.nr_iters = it;
      }
    }
    if (st) {
      p.arrive(false, done);
      return st;
    }
    if (done) {
      // every group must stop here too
      bool any = false, all = false;
      if (!p.arrive(true, true, &any, &all)) return ABORTED;
      if (!all) {
        o.set_err("Laplace devices disagree on the NR stop rule");
        return SGP_EINVAL;
      }
      return SGP_OK;
    }
    // the partials -> the other buffer, summed over the group's shards and the groups; this
    // group votes "not done" at the first barrier
    if (cnt > 0 && k > 1) st = o.sum_parts(g, o.red(g, cur ^ 1), cnt);
    bool any = false;
    if (!p.arrive(st == SGP_OK, false, &any)) return st ? st : ABORTED;
    if (any) {
      o.set_err("Laplace devices disagree on the NR stop rule");
      return SGP_EINVAL;
    }
    if (cnt > 0) st = o.all_reduce(g, o.red(g, cur ^ 1), cnt);
    if (!p.arrive(st == SGP_OK)) {
      if (p.groups() > 1) o.collective_broken();
      return st ? st : ABORTED;
    }
    cur ^= 1;
  }
}

}  // namespace sgp_pool

#endif  // SGP_POOL_H
