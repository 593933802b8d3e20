// Timeline probe (stamps from the last launch: the normal 2-workgroups-per-CU grid) of the K12 contraction kernel (k_contract<8, EPI_GRAD>): thread 0 of every
// workgroup records s_memtime at entry, after the k-loop and at the end, plus its CU / XCD, so
// the per-tile fixed cost (prologue + epilogue) and the phase relation of the workgroups that
// share a CU can be read off.  Synthetic operands; default n = 131072 rows, m = 1024, d = 8
// (ARD); C2's shape is n = 100000, m = 256.
//   build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o con_trace con_trace.hip
//   run:   ./con_trace out.csv [n m]
#include <cstdio>
#include <vector>
#include <random>
#include <algorithm>
#include <cstdlib>
__device__ unsigned long long* g_trace;
#define SGP_PROBE_BUILD 1
#define SGP_CON_TRACE(k)                                                                   \
  do {                                                                                     \
    unsigned long long* t_ = g_trace + (int64_t)blockIdx.x * 8;                            \
    t_[k] = __builtin_amdgcn_s_memtime();                                                  \
    if ((k) == 0) t_[7] = ((unsigned long long)__builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11)) << 32) | \
                          (unsigned long long)__builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11)); \
  } while (0)
#include "../../sparsergps_amd/csrc/k_mfma.hip"

// medians of the per-workgroup phases of the last launch (s_memtime ticks: shader clock)
static void report(const char* tag, const unsigned long long* tr, int64_t nwg, int64_t n,
                   int64_t m, const char* csv) {
  std::vector<unsigned long long> ht(nwg * 8);
  hipMemcpy(ht.data(), tr, ht.size() * 8, hipMemcpyDeviceToHost);
  if (csv) {
    FILE* f = fopen(csv, "w");
    fprintf(f, "wg,t0,t1,t4,t3,t5,t6,t2,hwid,xcc\n");
    for (int64_t w = 0; w < nwg; ++w) {
      const unsigned long long* t = &ht[w * 8];
      fprintf(f, "%lld,%llu,%llu,%llu,%llu,%llu,%llu,%llu,%llu,%llu\n", (long long)w, t[0], t[1],
              t[4], t[3], t[5], t[6], t[2], t[7] & 0xffffffffull, t[7] >> 32);
    }
    fclose(f);
  }
  std::vector<double> kl, ep;
  for (int64_t w = 0; w < nwg; ++w) {
    const unsigned long long* t = &ht[w * 8];
    kl.push_back((double)(t[1] - t[0]));
    ep.push_back((double)(t[2] - t[1]));
  }
  std::sort(kl.begin(), kl.end());
  std::sort(ep.begin(), ep.end());
  // epilogue phases: 1 -> 4 setup (alpha, u / cdiag, first K stages, coordinate staging, wait),
  // 4 -> 5 the eight K half-stages (W and its MFMA products), 5 -> 6 column sums / E /
  // records into LDS, 6 -> 2 the record reduction and store
  const int idx[5] = {1, 4, 5, 6, 2};
  for (int p = 0; p < 4; ++p) {
    std::vector<double> ph;
    for (int64_t w = 0; w < nwg; ++w) {
      const unsigned long long* t = &ht[w * 8];
      ph.push_back((double)(t[idx[p + 1]] - t[idx[p]]));
    }
    std::sort(ph.begin(), ph.end());
    printf("  [%s] epilogue phase t%d->t%d: median %.0f ticks\n", tag, idx[p], idx[p + 1],
           ph[ph.size() / 2]);
  }
  printf("[%s] n=%lld m=%lld nwg=%lld  median k-loop %.0f ticks (%.0f per k-step), epilogue %.0f "
         "ticks\n", tag, (long long)n, (long long)m, (long long)nwg, kl[kl.size() / 2],
         kl[kl.size() / 2] / (double)(m / 16), ep[ep.size() / 2]);
}

int main(int argc, char** argv) {
  const int64_t n = argc > 3 ? atoll(argv[2]) : 131072, n_pad = (n + 127) / 128 * 128;
  const int64_t m = argc > 3 ? atoll(argv[3]) : 1024, mp = (m + 127) / 128 * 128;
  const int d = 8;
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> U01(0.0, 1.0);
  std::vector<double> hK(n_pad * mp), hM(mp * mp), hX(n_pad * d), hU(mp * d), hr(n_pad), hu(mp),
      hc(mp, 0.0);
  for (auto& v : hK) v = U01(g);
  for (auto& v : hM) v = U01(g) - 0.5;
  for (auto& v : hX) v = 10 * U01(g);
  for (auto& v : hU) v = 10 * U01(g);
  for (auto& v : hr) v = U01(g);
  for (auto& v : hu) v = U01(g);
  double *K, *M, *X, *Uu, *r, *uv, *cd, *slab, *alpha;
  unsigned long long* tr;
  const int64_t nwg = (n_pad / 128) * (mp / 128);
  hipMalloc(&K, hK.size() * 8); hipMalloc(&M, hM.size() * 8); hipMalloc(&X, hX.size() * 8);
  hipMalloc(&Uu, hU.size() * 8); hipMalloc(&r, hr.size() * 8); hipMalloc(&uv, hu.size() * 8);
  hipMalloc(&cd, hc.size() * 8); hipMalloc(&slab, nwg * 16 * 8); hipMalloc(&alpha, n_pad * 8);
  hipMalloc(&tr, nwg * 8 * 8);
  hipMemcpy(K, hK.data(), hK.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(M, hM.data(), hM.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(X, hX.data(), hX.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(Uu, hU.data(), hU.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(r, hr.data(), hr.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(uv, hu.data(), hu.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(cd, hc.data(), hc.size() * 8, hipMemcpyHostToDevice);
  hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &tr, sizeof(tr));
  KernParams kp{};
  kp.kernel = 1; kp.d = d; kp.L = d; kp.P = d + 2;
  kp.sigma = 1; kp.sig2 = 1; kp.tau = 0.5; kp.tau2 = 0.25; kp.delta = 1e-6;
  for (int c = 0; c < d; ++c) { kp.l[c] = 3; kp.rl[c] = 1.0 / 3; kp.rl2[c] = 1.0 / 9; }
  ConArgs ca;
  ca.r = r; ca.invz = 4.0; ca.uvec = uv; ca.cdiag = cd; ca.count_a2 = 1; ca.alpha_out = alpha;
  int64_t nrec, nw;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  // one workgroup per CU: pad the launch with dynamic LDS so a second one cannot fit
  for (int it = 0; it < 3; ++it) {
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL((k_contract<8, EPI_GRAD>), dim3((unsigned)nwg), dim3(256), 80 * 1024, 0,
                       kp, K, M, X, n_pad, n, n_pad, Uu, mp, m, mp, ca, slab, (int)(kp.L + 5),
                       (double*)nullptr);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("1 WG/CU run %d: %.3f ms  %.2f TF/s\n", it, ms, 2.0 * n * m * m / (ms * 1e-3) / 1e12);
  }
  report("1 WG/CU", tr, nwg, n, m, nullptr);
  for (int it = 0; it < 3; ++it) {
    hipEventRecord(e0, 0);
    launch_contract_args(kp, K, M, X, n_pad, n, n_pad, Uu, mp, m, mp, ca, slab, &nrec, &nw, 0);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("run %d: %.3f ms  %.2f TF/s\n", it, ms, 2.0 * n * m * m / (ms * 1e-3) / 1e12);
  }
  report("2 WG/CU", tr, nwg, n, m, argc > 1 ? argv[1] : "con_trace.csv");
  return 0;
}
