// Microbenchmark of the Gauss-Jordan 64x64 pivot (k_dense.hip gj_pivot_body) against the
// previous one-barrier-per-sweep version: one workgroup runs the pivot `reps` times on an SPD
// block held in global memory (L2-resident), timed with events.
// MI355X (r1): block-sweep 10.8 us/pivot, scalar-sweep 17.9 us; of the block-sweep's first
// version (13.4 us) the single-wave sweeps were ~9.3 us and the MFMA block products ~4 us.
//   build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o gj_pivot gj_pivot.hip
#include <cstdio>
#include <vector>
#include <random>
#include <cmath>
#include "../../sparsergps_amd/csrc/k_dense.hip"
namespace {



__device__ __forceinline__ void gj_pivot_old(const double* B, int64_t ldb, int64_t gofs,
                                              double* __restrict__ P,
                                              double* __restrict__ logd_slot,
                                              int* __restrict__ status, double* lds) {
  double (*colv)[64] = reinterpret_cast<double (*)[64]>(lds);
  double* piv_s = lds + 128;
  const int tid = threadIdx.x;
  const int bi = tid >> 4, bj = tid & 15;
  double a[4][4];
#pragma unroll
  for (int ii = 0; ii < 4; ++ii)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) a[ii][jj] = B[(4 * bi + ii) * ldb + 4 * bj + jj];
  for (int kb4 = 0; kb4 < 16; ++kb4) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int kc = 4 * kb4 + kk;
      const int b = kc & 1;
      if (bj == kb4) {
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) colv[b][4 * bi + ii] = a[ii][kk];
      }
      __syncthreads();
      const double d = colv[b][kc];
      const double r = rcp_nr(d);
      if (tid == 0) {
        piv_s[kc] = d;
        if (!(d > 0.0) || !isfinite(d)) atomicCAS(status, 0, (int)(gofs + kc + 1));
      }
      // sweep: a_ij <- a_ij - v_i v_j / d with v = column kc and v_kc = -1, row/col kc
      // zeroed first (gives a_ik = a_ik / d, a_kk = -1/d); the result is -inv(B)
      double vi[4], vj[4];
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int i = 4 * bi + ii;
        vi[ii] = (i == kc) ? -r : colv[b][i] * r;
      }
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int j = 4 * bj + jj;
        vj[jj] = (j == kc) ? -1.0 : colv[b][j];
      }
      if (bi == kb4) {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) a[kk][jj] = 0.0;
      }
      if (bj == kb4) {
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) a[ii][kk] = 0.0;
      }
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) a[ii][jj] = fma(-vi[ii], vj[jj], a[ii][jj]);
    }
  }
#pragma unroll
  for (int ii = 0; ii < 4; ++ii)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) P[(4 * bi + ii) * 64 + 4 * bj + jj] = -a[ii][jj];
  __syncthreads();
  double lg = (tid < 64) ? log(piv_s[tid]) : 0.0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) lg += __shfl_xor(lg, off, 64);
  if (tid == 0) *logd_slot = 0.5 * lg;
}

template <int V>
__global__ void __launch_bounds__(256) k_piv_bench(const double* B, double* P, double* logd,
                                                   int* status, int reps) {
  __shared__ double lds[GJ_PIVOT_LDS > 192 ? GJ_PIVOT_LDS : 192];
  for (int r = 0; r < reps; ++r) {
    if (V == 0) gj_pivot_body(B, 64, 0, P, logd, status, lds);
    else gj_pivot_old(B, 64, 0, P, logd, status, lds);
    __syncthreads();
  }
}
}  // namespace

int main() {
  std::mt19937_64 g(3);
  std::normal_distribution<double> N01;
  std::vector<double> G(64 * 64), B(64 * 64, 0.0), P(64 * 64);
  for (auto& v : G) v = N01(g);
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 64; ++j) {
      double s = 0; for (int k = 0; k < 64; ++k) s += G[i * 64 + k] * G[j * 64 + k];
      B[i * 64 + j] = s / 64 + (i == j ? 1.0 : 0.0);
    }
  double *dB, *dP, *dl; int* ds;
  hipMalloc(&dB, 64 * 64 * 8); hipMalloc(&dP, 64 * 64 * 8); hipMalloc(&dl, 8); hipMalloc(&ds, 4);
  hipMemcpy(dB, B.data(), 64 * 64 * 8, hipMemcpyHostToDevice);
  hipMemset(ds, 0, 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const char* names[2] = {"block-sweep", "scalar-sweep"};
  for (int v = 0; v < 2; ++v) {
    for (int it = 0; it < 2; ++it) {
      const int reps = 2000;
      hipEventRecord(e0, 0);
      if (v == 0) hipLaunchKernelGGL(k_piv_bench<0>, dim3(1), dim3(256), 0, 0, dB, dP, dl, ds, reps);
      else hipLaunchKernelGGL(k_piv_bench<1>, dim3(1), dim3(256), 0, 0, dB, dP, dl, ds, reps);
      hipEventRecord(e1, 0); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      hipMemcpy(P.data(), dP, 64 * 64 * 8, hipMemcpyDeviceToHost);
      double err = 0;   // || B P - I ||_max
      for (int i = 0; i < 64; ++i)
        for (int j = 0; j < 64; ++j) {
          double s = 0; for (int k = 0; k < 64; ++k) s += B[i * 64 + k] * P[k * 64 + j];
          err = fmax(err, fabs(s - (i == j ? 1.0 : 0.0)));
        }
      double ld; hipMemcpy(&ld, dl, 8, hipMemcpyDeviceToHost);
      printf("%s: %.2f us/pivot  |BP-I| %.2e  logd %.12f\n", names[v],
             ms * 1e3 / reps, err, ld);
    }
  }
  return 0;
}
