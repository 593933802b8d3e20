// CPU driver of the multi-device orchestration (sparsergps_amd/csrc/sgp_pool.h) with G > 1 fake
// device groups -- the part of the in-library multi-GPU context (multi.hip) that no one-GPU box
// can exercise: the worker pool, the barriers with votes, and the VI / FITC and Laplace job
// bodies with their failure paths.  Built and run by tests/test_pool.py, once under
// ThreadSanitizer.
//
// The fakes keep the properties of the real operations that the orchestration depends on:
//   * a shard's phases write partial sums of its rows; the group sums its shards' partials in
//     fixed order (sum_parts);
//   * all_reduce only ENQUEUES: the sum lands in every group's buffer once the last group has
//     enqueued its part, and a group's next phase first waits for everything it enqueued (the
//     stream synchronisation of the real readbacks).  That wait has a deadline: a group left
//     waiting on a collective its peers never join is reported as a hang, not a stuck test;
//   * the Laplace stop rule is a function of the summed buffers (newtrap_sparseGP's loop,
//     R/newtrap_sparseGP.R:77-150), so every group stops at the same step unless a fault says
//     otherwise.
// Faults: a phase / step / sum failing on one group, one group's collective failing to enqueue
// after its peers' were queued (the post-collective vote must stop the peers before their
// next wait), and one group disagreeing on the NR stop rule.  After each faulted evaluation the
// harness does what MultiCtx::run does (abort + rebuild the "communicators" when a collective
// broke) and a clean evaluation must give the right answer again.
//
// Values are small integers, so every sum is exact and the expected results are computed
// serially.  Exit status 0 = all checks passed.
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <mutex>
#include <random>
#include <string>
#include <vector>

#include "../../sparsergps_amd/csrc/sgp_pool.h"

namespace {

int failures = 0;
#define CHECK(cond, ...)                                  \
  do {                                                    \
    if (!(cond)) {                                        \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                       \
      fprintf(stderr, "\n");                              \
      ++failures;                                         \
    }                                                     \
  } while (0)

thread_local std::string t_err;
std::string last_err() { return t_err; }

enum Where { NONE, BEGIN, PHASE1, PHASE2, FINISH, SUM, COLLECTIVE, LAP_BEGIN, LAP_STEP, STOP_VOTE };
const char* where_name(int w) {
  static const char* n[] = {"none", "begin", "phase1", "phase2", "finish", "sum_parts",
                            "collective", "lap_begin", "lap_step", "stop_vote"};
  return n[w];
}

struct Fault {
  int group = -1, where = NONE, index = 0;   // index: the occurrence within one evaluation
  int status = SGP_ENOMEM;                   // a code no healthy path returns
};

// an asynchronous in-place all-reduce over G groups (sequence-numbered per group)
class Coll {
 public:
  explicit Coll(int G) : G_(G), issued_((size_t)G, 0) {}
  void issue(int g, double* buf, int64_t count) {
    std::lock_guard<std::mutex> lk(mu_);
    const size_t k = issued_[(size_t)g]++;
    if (slots_.size() <= k) slots_.resize(k + 1);
    Slot& s = slots_[k];
    if (s.sum.empty()) s.sum.assign((size_t)count, 0.0);
    if ((int64_t)s.sum.size() != count) mismatch_ = true;
    for (int64_t i = 0; i < count && i < (int64_t)s.sum.size(); ++i) s.sum[(size_t)i] += buf[i];
    s.dst.push_back(buf);
    if (++s.arrived == G_) {
      for (double* d : s.dst) std::copy(s.sum.begin(), s.sum.end(), d);
      s.done = true;
      cv_.notify_all();
    }
  }
  // the host waits for everything group g enqueued
  int sync(int g) {
    std::unique_lock<std::mutex> lk(mu_);
    // (a system_clock deadline: gcc 11's ThreadSanitizer does not intercept the
    // pthread_cond_clockwait a steady_clock wait compiles to)
    const auto deadline = std::chrono::system_clock::now() + std::chrono::seconds(5);
    for (;;) {
      bool ok = true;
      for (size_t k = 0; k < issued_[(size_t)g]; ++k) ok = ok && slots_[k].done;
      if (ok) return SGP_OK;
      if (cv_.wait_until(lk, deadline) == std::cv_status::timeout) {
        ++hangs_;
        t_err = "hang: waited on a collective its peers never joined";
        return SGP_EHIP;
      }
    }
  }
  // ncclCommAbort + ncclCommInitAll: queued collectives are dropped, counters restart
  void abort_and_reset() {
    std::lock_guard<std::mutex> lk(mu_);
    slots_.clear();
    issued_.assign((size_t)G_, 0);
    cv_.notify_all();
  }
  int hangs() {
    std::lock_guard<std::mutex> lk(mu_);
    return hangs_;
  }
  bool mismatch() {
    std::lock_guard<std::mutex> lk(mu_);
    return mismatch_;
  }

 private:
  struct Slot {
    int arrived = 0;
    bool done = false;
    std::vector<double> sum;
    std::vector<double*> dst;
  };
  const int G_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<Slot> slots_;
  std::vector<size_t> issued_;
  int hangs_ = 0;
  bool mismatch_ = false;
};

constexpr int64_t C1 = 3, C2 = 4, CL = 2, NPAR = 3, CAP = 8;

// the fake NR loop's length: 2..4 steps, a function of the summed data
int steps_for(double total) { return 2 + (int)((((int64_t)total % 3) + 3) % 3); }

struct Shard {
  std::vector<double> x;
  std::vector<double> part = std::vector<double>(CAP, 0.0);
  int lap_it = 0;
};

struct Group {
  std::vector<int> shards;
  double red[2][CAP] = {};
  int count[16] = {};   // occurrences of each Where in the current evaluation
  bool forced_done = false;
};

struct FakeOps {
  std::vector<Shard>& sh;
  std::vector<Group>& gr;
  Coll& coll;
  Fault fault;
  bool broken = false;   // set by collective_broken (any group thread)
  std::mutex bmu;
  unsigned jitter_seed;

  bool hit(int g, int where) {
    const int k = gr[(size_t)g].count[where]++;
    if (g == fault.group && where == fault.where && k == fault.index) {
      char b[128];
      snprintf(b, sizeof(b), "injected %s failure in group %d", where_name(where), g);
      t_err = b;
      return true;
    }
    return false;
  }
  void jitter(int g) {   // vary the interleaving
    thread_local std::mt19937 rng;
    static thread_local bool seeded = false;
    if (!seeded) {
      rng.seed(jitter_seed + 7919u * (unsigned)g);
      seeded = true;
    }
    const unsigned r = rng() % 8;
    if (r == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 200));
    else if (r < 3) std::this_thread::yield();
  }
  Shard& shard(int g, int q) { return sh[(size_t)gr[(size_t)g].shards[(size_t)q]]; }

  int begin(int g) {
    for (int& c : gr[(size_t)g].count) c = 0;
    return hit(g, BEGIN) ? fault.status : SGP_OK;
  }
  int shards(int g) { return (int)gr[(size_t)g].shards.size(); }
  double* red(int g, int b) { return gr[(size_t)g].red[b]; }
  double* out_of(int g, int q, double* r) {
    return gr[(size_t)g].shards.size() == 1 ? r : shard(g, q).part.data();
  }
  int phase1(int g, int q, double* out) {
    jitter(g);
    if (hit(g, PHASE1)) return fault.status;
    const Shard& s = shard(g, q);
    double a = 0, b = 0;
    for (double v : s.x) {
      a += v;
      b += v * v;
    }
    out[0] = a;
    out[1] = b;
    out[2] = (double)s.x.size();
    return SGP_OK;
  }
  int phase2(int g, int q, const double* red1, double* out) {
    const int st = coll.sync(g);   // phase 2 reads the summed red1
    if (st) return st;
    jitter(g);
    if (hit(g, PHASE2)) return fault.status;
    const Shard& s = shard(g, q);
    out[0] = out[1] = out[2] = 0.0;
    for (double v : s.x) {
      out[0] += v * red1[0];
      out[1] += v + red1[1];
      out[2] += v * red1[2];
    }
    out[3] = (double)s.x.size();
    return SGP_OK;
  }
  int finish(int g, int q, const double* red2, double* obj, double* grad) {
    (void)q;
    const int st = coll.sync(g);   // the readback
    if (st) return st;
    if (hit(g, FINISH)) return fault.status;
    *obj = red2[0] + red2[1];
    if (grad)
      for (int p = 0; p < NPAR; ++p) grad[p] = red2[1 + p];
    return SGP_OK;
  }
  int lap_begin(int g, int q, double* out, int64_t* count) {
    jitter(g);
    if (hit(g, LAP_BEGIN)) return fault.status;
    Shard& s = shard(g, q);
    s.lap_it = 0;
    double a = 0;
    for (double v : s.x) a += v;
    out[0] = a;
    out[1] = 0.0;
    *count = CL;
    return SGP_OK;
  }
  int lap_step(int g, int q, const double* in, double* out, int64_t* count, int* done,
               double* obj, double* grad, int* nr_iters) {
    const int st = coll.sync(g);   // the NR step reads the summed objective sums
    if (st) return st;
    jitter(g);
    if (hit(g, LAP_STEP)) return fault.status;
    Shard& s = shard(g, q);
    s.lap_it += 1;
    const int nsteps = steps_for(in[0]);   // decided from the summed buffer
    *done = s.lap_it >= nsteps;
    // a stop-rule fault: this group alone (all its shards) believes the loop is over
    Group& G0 = gr[(size_t)g];
    if (q == 0) G0.forced_done = hit(g, STOP_VOTE);
    if (G0.forced_done) *done = 1;
    *obj = in[0] * s.lap_it + in[1];
    *nr_iters = s.lap_it;
    if (*done) {
      for (int p = 0; p < NPAR; ++p) grad[p] = in[0] + p;
      *count = 0;
      return SGP_OK;
    }
    double a = 0;
    for (double v : s.x) a += v;
    out[0] = a;
    out[1] = (double)s.x.size();
    *count = CL;
    return SGP_OK;
  }
  int sum_parts(int g, double* r, int64_t count) {
    if (hit(g, SUM)) return fault.status;
    for (int64_t i = 0; i < count; ++i) {
      double v = 0.0;
      for (int q = 0; q < shards(g); ++q) v += shard(g, q).part[(size_t)i];
      r[i] = v;
    }
    return SGP_OK;
  }
  int all_reduce(int g, double* r, int64_t count) {
    jitter(g);
    if (hit(g, COLLECTIVE)) return SGP_EHIP;   // fails to enqueue; the peers' are queued
    coll.issue(g, r, count);
    return SGP_OK;
  }
  void collective_broken() {
    std::lock_guard<std::mutex> lk(bmu);
    broken = true;
  }
  void set_err(const char* m) { t_err = m; }
};

struct Expect {
  double obj;
  double grad[NPAR];
  int nr_iters;
};

Expect expect_vi(const std::vector<Shard>& sh) {
  double A = 0, B = 0, N = 0;
  for (const Shard& s : sh)
    for (double v : s.x) {
      A += v;
      B += v * v;
      N += 1;
    }
  double r[4] = {0, 0, 0, 0};
  for (const Shard& s : sh)
    for (double v : s.x) {
      r[0] += v * A;
      r[1] += v + B;
      r[2] += v * N;
      r[3] += 1;
    }
  return {r[0] + r[1], {r[1], r[2], r[3]}, 0};
}

Expect expect_lap(const std::vector<Shard>& sh) {
  double A = 0, N = 0;
  for (const Shard& s : sh)
    for (double v : s.x) {
      A += v;
      N += 1;
    }
  // begin sums [A, 0]; every later step sums [A, N]
  const int nsteps = steps_for(A);
  Expect e{};
  e.nr_iters = nsteps;
  e.obj = A * nsteps + (nsteps == 1 ? 0.0 : N);
  for (int p = 0; p < NPAR; ++p) e.grad[p] = A + p;
  return e;
}

// one evaluation on every group, as MultiCtx::run: run_all, then the communicator repair
struct Harness {
  int G;
  std::vector<Shard> sh;
  std::vector<Group> gr;
  Coll coll;
  sgp_pool::Pool pool;
  std::vector<sgp_pool::Result> res;
  unsigned seed;

  Harness(int G_, int shards_per_group, unsigned s)
      : G(G_), gr((size_t)G_), coll(G_), pool(G_, last_err), res((size_t)G_), seed(s) {
    std::mt19937 rng(s);
    int id = 0;
    for (int g = 0; g < G; ++g)
      for (int q = 0; q < shards_per_group + (g % 2 == 1 && shards_per_group > 1); ++q) {
        Shard x;
        const int rows = 1 + (int)(rng() % 9);
        for (int i = 0; i < rows; ++i) x.x.push_back((double)(rng() % 7) - 3.0);
        sh.push_back(x);
        gr[(size_t)g].shards.push_back(id++);
      }
  }

  // returns the run's status; *msg its message; statuses[g] each group's
  int eval(bool laplace, const Fault& f, std::string* msg, std::vector<int>* statuses,
           bool* broken) {
    FakeOps ops{sh, gr, coll, f, false, {}, seed++};
    int st = pool.run_all(
        [&](int g) {
          return laplace ? sgp_pool::laplace_job(ops, pool, g, NPAR, res[(size_t)g])
                         : sgp_pool::two_phase_job(ops, pool, g, C1, C2, NPAR, res[(size_t)g]);
        },
        msg);
    statuses->clear();
    for (int g = 0; g < G; ++g) statuses->push_back(pool.status(g));
    {
      std::lock_guard<std::mutex> lk(ops.bmu);
      *broken = ops.broken;
    }
    // MultiCtx::recover: abort and rebuild the communicators only after every worker returned;
    // every run starts from fresh communicators as after ncclCommInitAll
    coll.abort_and_reset();
    return st;
  }
};

void check_clean(Harness& h, bool laplace, const char* what) {
  std::string msg;
  std::vector<int> stv;
  bool broken = false;
  const int st = h.eval(laplace, Fault{}, &msg, &stv, &broken);
  CHECK(st == SGP_OK, "%s G=%d clean %s: status %d (%s)", what, h.G, laplace ? "laplace" : "vi",
        st, msg.c_str());
  CHECK(!broken, "%s G=%d: collective_broken on a clean run", what, h.G);
  if (st) return;
  const Expect e = laplace ? expect_lap(h.sh) : expect_vi(h.sh);
  for (int g = 0; g < h.G; ++g) {
    const sgp_pool::Result& r = h.res[(size_t)g];
    CHECK(r.obj == e.obj, "%s G=%d group %d obj %g != %g", what, h.G, g, r.obj, e.obj);
    for (int p = 0; p < NPAR; ++p)
      CHECK(r.grad[(size_t)p] == e.grad[p], "%s G=%d group %d grad[%d] %g != %g", what, h.G, g, p,
            r.grad[(size_t)p], e.grad[p]);
    if (laplace)
      CHECK(r.nr_iters == e.nr_iters, "%s G=%d group %d nr_iters %d != %d", what, h.G, g,
            r.nr_iters, e.nr_iters);
  }
}

void check_fault(Harness& h, bool laplace, const Fault& f) {
  std::string msg;
  std::vector<int> stv;
  bool broken = false;
  const int st = h.eval(laplace, f, &msg, &stv, &broken);
  const char* w = where_name(f.where);
  const int hangs = h.coll.hangs();
  CHECK(hangs == 0, "G=%d fault %s@%d in group %d (%s): %d hang(s)", h.G, w, f.index, f.group,
        laplace ? "laplace" : "vi", hangs);
  if (f.where == STOP_VOTE) {
    // a stop-rule disagreement ends every group with SGP_EINVAL (none waits at a barrier)
    CHECK(st == SGP_EINVAL, "G=%d stop-vote disagreement: status %d (%s)", h.G, st, msg.c_str());
    CHECK(msg.find("disagree") != std::string::npos, "G=%d stop-vote message '%s'", h.G,
          msg.c_str());
    for (int g = 0; g < h.G; ++g)
      CHECK(stv[(size_t)g] == SGP_EINVAL, "G=%d stop vote: group %d status %d", h.G, g,
            stv[(size_t)g]);
  } else {
    const int want = f.where == COLLECTIVE ? SGP_EHIP : f.status;
    CHECK(st == want, "G=%d fault %s@%d in group %d: status %d, want %d (%s)", h.G, w, f.index,
          f.group, st, want, msg.c_str());
    CHECK(msg.find("injected") != std::string::npos && msg.find(w) != std::string::npos,
          "G=%d fault %s: message '%s' does not name the failing group's error", h.G, w,
          msg.c_str());
    for (int g = 0; g < h.G; ++g) {
      const int s = stv[(size_t)g];
      if (g == f.group)
        CHECK(s == want, "G=%d fault %s: failing group %d status %d", h.G, w, g, s);
      else if (f.where == FINISH)   // after the last vote: the peers may finish normally
        CHECK(s == sgp_pool::ABORTED || s == SGP_OK, "G=%d finish fault: group %d status %d",
              h.G, g, s);
      else
        CHECK(s == sgp_pool::ABORTED, "G=%d fault %s in group %d: group %d status %d (want "
              "ABORTED)", h.G, w, f.group, g, s);
    }
    CHECK(broken == (f.where == COLLECTIVE && h.G > 1),
          "G=%d fault %s: collective_broken = %d", h.G, w, (int)broken);
  }
  CHECK(!h.coll.mismatch(), "G=%d: collective sizes differ across groups", h.G);
  // the context is usable again
  check_clean(h, laplace, "after fault");
}

}  // namespace

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 3;
  int cases = 0;
  for (int G : {1, 2, 3, 8}) {
    for (int spg : {1, 2}) {
      for (int rep = 0; rep < reps; ++rep) {
        Harness h(G, spg, 1000u * (unsigned)G + 17u * (unsigned)spg + (unsigned)rep);
        check_clean(h, false, "first");
        check_clean(h, true, "first");
        ++cases;
        for (int fg : {0, G - 1, G / 2}) {
          // VI / FITC: before the first collective, between the two, after the second
          for (int w : {BEGIN, PHASE1, PHASE2, FINISH}) {
            Fault f;
            f.group = fg;
            f.where = w;
            check_fault(h, false, f);
            ++cases;
          }
          if (spg > 1 && fg % 2 == 1) {   // groups with two or more shards sum partials
            Fault f;
            f.group = fg;
            f.where = SUM;
            f.index = rep % 2;
            check_fault(h, false, f);
            ++cases;
          }
          for (int k : {0, 1}) {   // the first or the second collective fails to enqueue
            Fault f;
            f.group = fg;
            f.where = COLLECTIVE;
            f.index = k;
            check_fault(h, false, f);
            ++cases;
          }
          // Laplace: begin, an NR step, an NR collective, the stop vote
          for (int w : {LAP_BEGIN, LAP_STEP, COLLECTIVE}) {
            Fault f;
            f.group = fg;
            f.where = w;
            f.index = w == LAP_BEGIN ? 0 : rep % 2;
            check_fault(h, true, f);
            ++cases;
          }
          if (G > 1) {
            Fault f;
            f.group = fg;
            f.where = STOP_VOTE;
            f.index = 0;   // the first step, where no group is done yet
            check_fault(h, true, f);
            ++cases;
          }
        }
        // many evaluations back to back on the same workers
        for (int k = 0; k < 20; ++k) check_clean(h, k % 2 == 1, "repeat");
      }
    }
  }
  if (failures) {
    fprintf(stderr, "%d check(s) failed over %d cases\n", failures, cases);
    return 1;
  }
  printf("pool driver: %d fault / clean cases passed (G = 1, 2, 3, 8)\n", cases);
  return 0;
}
