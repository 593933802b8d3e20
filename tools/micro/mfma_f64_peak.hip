// Microbenchmark: achievable v_mfma_f64_16x16x4_f64 throughput on one MI355X (no memory
// traffic).  Each wave keeps NACC independent accumulators in flight; the grid covers every
// SIMD with `waves_per_simd` waves.  Prints TFLOP/s per configuration.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef double v4d __attribute__((ext_vector_type(4)));

// RND: operands with random mantissas, re-drawn every iteration (switching activity like a
// real GEMM; DVFS lowers the clock more than for near-constant operands)
template <int NACC, bool RND>
__global__ __launch_bounds__(256) void k_peak(int iters, double* out) {
  v4d acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = (v4d){0.0, 0.0, 0.0, 0.0};
  unsigned long long st = 0x9E3779B97F4A7C15ull * (threadIdx.x + 1 + blockIdx.x * 977ull);
  double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
  for (int it = 0; it < iters; ++it) {
    if (RND) {
      st = st * 6364136223846793005ull + 1442695040888963407ull;
      a = __longlong_as_double((long long)((st >> 12) | 0x3FE0000000000000ull));
      b = __longlong_as_double((long long)(((st << 20) >> 12) | 0x3FE0000000000000ull));
    }
    // inline asm keeps the accumulators in place: with the builtin, hipcc round-trips every
    // accumulator through AGPRs each iteration (64 v_accvgpr moves per 8 MFMAs)
#pragma unroll
    for (int i = 0; i < NACC; ++i)
      asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b));
  }
  asm volatile("s_nop 15\n s_nop 15" ::: "memory");
  double s = 0.0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.678) out[threadIdx.x] = s;   // keep the work alive
}

template <int NACC, bool RND = false>
static void run(int wgs_per_cu, int iters) {
  double* out;
  (void)hipMalloc(&out, 4096);
  const int cus = 256;
  dim3 grid(cus * wgs_per_cu), block(256);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL((k_peak<NACC, RND>), grid, block, 0, 0, iters / 10, out);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL((k_peak<NACC, RND>), grid, block, 0, 0, iters, out);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 16 * 16 * 4 * (double)NACC * iters * grid.x * 4;
  printf("NACC=%d wgs/cu=%d (waves/simd=%d) %s: %.3f ms  %.2f TFLOP/s\n", NACC, wgs_per_cu,
         wgs_per_cu, RND ? "random operands" : "near-constant operands", ms,
         flops / (ms * 1e-3) / 1e12);
  (void)hipFree(out);
}

int main() {
  run<4>(1, 20000 * 5);
  run<8>(1, 10000 * 5);
  run<16>(1, 5000 * 5);
  run<4>(2, 20000 * 5);
  run<8>(2, 10000 * 5);
  run<16>(2, 5000 * 5);
  run<8>(4, 10000 * 5);
  run<8, true>(1, 10000 * 5);
  run<8, true>(2, 10000 * 5);
  run<16, true>(2, 5000 * 5);
  return 0;
}
