// Timeline probe of the Gauss-Jordan SPD inverse (k_dense.hip dense_spd_inverse) at m = 1024:
// s_memtime stamps of each step's look-ahead workgroup (entry, operands staged, first product,
// update stored, next pivot done) plus event timing of the whole inverse, alone and as two
// concurrent chains (the VI phase-2 situation: K22's and Bm's inverses side by side).
//   build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o gj_trace gj_trace.hip
#include <cmath>
#include <cstdio>
#include <vector>
__device__ unsigned long long g_gj[64][8];
#define SGP_PROBE_BUILD 1
#define SGP_GJ_TRACE(k_, p_) (g_gj[(k_)][(p_)] = __builtin_amdgcn_s_memtime())
#include "../../sparsergps_amd/csrc/k_dense.hip"

int main() {
  const int64_t m = 1024, mp = 1024;
  std::vector<double> hU(m * 8), hA(mp * mp);
  unsigned long long st = 88172645463325252ull;
  auto rnd = [&]() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return (double)(st >> 11) / 9007199254740992.0; };
  for (auto& v : hU) v = 10.0 * rnd();
  for (int64_t a = 0; a < m; ++a)
    for (int64_t b = 0; b < m; ++b) {
      double s = 0.0;
      for (int c = 0; c < 8; ++c) { const double t = (hU[a * 8 + c] - hU[b * 8 + c]) / 3.0; s += t * t; }
      hA[a * mp + b] = exp(-0.5 * s) + (a == b ? 1e-3 : 0.0);
    }
  double *A0, *A, *R, *P, *logd, *A2, *R2, *P2, *logd2;
  int* status;
  hipMalloc(&A0, mp * mp * 8); hipMalloc(&A, mp * mp * 8); hipMalloc(&R, mp * mp * 8);
  hipMalloc(&P, mp * 64 * 8); hipMalloc(&logd, 64 * 8); hipMalloc(&status, 16);
  hipMalloc(&A2, mp * mp * 8); hipMalloc(&R2, mp * mp * 8); hipMalloc(&P2, mp * 64 * 8);
  hipMalloc(&logd2, 64 * 8);
  hipMemcpy(A0, hA.data(), mp * mp * 8, hipMemcpyHostToDevice);
  hipStream_t s1, s2;
  hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  hipEvent_t e0, e1, e2;
  hipEventCreate(&e0); hipEventCreate(&e1); hipEventCreate(&e2);
  for (int it = 0; it < 4; ++it) {
    hipMemcpyAsync(A, A0, mp * mp * 8, hipMemcpyDeviceToDevice, s1);
    hipEventRecord(e0, s1);
    dense_spd_inverse(A, mp, R, nullptr, P, logd, status, s1);
    hipEventRecord(e1, s1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("one chain: %.1f us\n", ms * 1e3);
  }
  std::vector<unsigned long long> tr(64 * 8);
  hipMemcpyFromSymbol(tr.data(), HIP_SYMBOL(g_gj), tr.size() * 8);
  printf("step  staged  prod1  stored  pivot  (s_memtime ticks from entry; next entry)\n");
  for (int k = 0; k < 15; ++k) {
    const unsigned long long* t = &tr[k * 8];
    printf("%2d %7lld %7lld %7lld %7lld  next %7lld\n", k, (long long)(t[1] - t[0]),
           (long long)(t[2] - t[0]), (long long)(t[3] - t[0]), (long long)(t[4] - t[0]),
           k < 14 ? (long long)(tr[(k + 1) * 8] - t[0]) : 0LL);
  }
  for (int it = 0; it < 3; ++it) {
    hipMemcpyAsync(A, A0, mp * mp * 8, hipMemcpyDeviceToDevice, s1);
    hipMemcpyAsync(A2, A0, mp * mp * 8, hipMemcpyDeviceToDevice, s2);
    hipDeviceSynchronize();
    hipEventRecord(e0, s1);
    hipStreamWaitEvent(s2, e0, 0);
    dense_spd_inverse(A, mp, R, nullptr, P, logd, status, s1);
    dense_spd_inverse(A2, mp, R2, nullptr, P2, logd2, status + 1, s2);
    hipEventRecord(e1, s1);
    hipEventRecord(e2, s2);
    hipEventSynchronize(e1);
    hipEventSynchronize(e2);
    float a_ms, b_ms; hipEventElapsedTime(&a_ms, e0, e1); hipEventElapsedTime(&b_ms, e0, e2);
    printf("two chains: %.1f / %.1f us\n", a_ms * 1e3, b_ms * 1e3);
  }
  return 0;
}
