// Microbenchmark of the Gauss-Jordan 64x64 pivot (k_dense.hip gj_pivot_body) against the
// previous one-barrier-per-sweep version: one workgroup runs the pivot `reps` times on an SPD
// block held in global memory (L2-resident), timed with events.
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

template <int MODE>
__device__ __forceinline__ void gj_pivot_var(const double* B, int64_t ldb, int64_t gofs,
                                              double* __restrict__ P,
                                              double* __restrict__ logd_slot,
                                              int* __restrict__ status, double* lds) {
  double* Es0 = lds;                          // [2][64][GJP_LD]  column panel W_:K (old)
  double* Fs = lds + 2 * 64 * GJP_LD;         // [64][GJP_LD]     F = W_:K Q (own rows per wave)
  double* Qs = Fs + 64 * GJP_LD;              // [16][GJP_LD]     Q = -inv(W_KK)
  double* piv = Qs + 16 * GJP_LD;             // [64]             sweep pivots
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int lr = lane >> 4, lc = lane & 15;
  d4 acc[4];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[ct][q] = B[(16 * wv + lr + 4 * q) * ldb + 16 * ct + lc];
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    double* Es = Es0 + (kb & 1) * 64 * GJP_LD;
    // publish the column panel E = W_:K (every wave's tile kb)
#pragma unroll
    for (int q = 0; q < 4; ++q) Es[(16 * wv + lr + 4 * q) * GJP_LD + lc] = acc[kb][q];
    __syncthreads();
    if (MODE != 2 && wv == kb) {
      // 16 scalar sweeps of W_KK in registers: lane (lr, lc) holds rows lr + 4q of column lc
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int kq = k >> 2, kr = k & 3;
        const double vc = __shfl(acc[kb][kq], lc + 16 * kr, 64);          // W_k,lc
        const double d = readlane_f64(acc[kb][kq], k + 16 * kr);          // W_kk (uniform)
        double vr[4];                                                      // W_i,k: lane k
#pragma unroll                                                             // of each row
        for (int q = 0; q < 4; ++q) vr[q] = row_bcast_f64(acc[kb][q], k);
        const double r = rcp_nr(d);
        if (lane == 0) {
          piv[16 * kb + k] = d;
          if (!(d > 0.0) || !isfinite(d)) atomicCAS(status, 0, (int)(gofs + 16 * kb + k + 1));
        }
        const double vj = (lc == k) ? -1.0 : vc;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = lr + 4 * q;
          const double vi = (i == k) ? -r : vr[q] * r;
          const double base = (i == k || lc == k) ? 0.0 : acc[kb][q];
          acc[kb][q] = fma(-vi, vj, base);
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) Qs[(lr + 4 * q) * GJP_LD + lc] = acc[kb][q];
    }
    __syncthreads();
    if (MODE == 1) {
    } else if (wv == kb) {
      // W_KR <- -Q E_R^T  (tiles ct != kb of the pivot rows)
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        if (ct == kb) continue;
        d4 t = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int sk = 0; sk < 4; ++sk) {
          const double af = -Qs[lc * GJP_LD + 4 * sk + lr];
          const double bf = Es[(16 * ct + lc) * GJP_LD + 4 * sk + lr];
          t = __builtin_amdgcn_mfma_f64_16x16x4f64(af, bf, t, 0, 0, 0);
        }
        acc[ct] = t;
      }
    } else {
      // F_w = E_w Q; W_wK <- -F_w; W_wR <- W_wR + F_w E_R^T
      d4 f = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int sk = 0; sk < 4; ++sk) {
        const double af = Es[(16 * wv + lc) * GJP_LD + 4 * sk + lr];
        const double bf = Qs[(4 * sk + lr) * GJP_LD + lc];
        f = __builtin_amdgcn_mfma_f64_16x16x4f64(af, bf, f, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) Fs[(16 * wv + lr + 4 * q) * GJP_LD + lc] = f[q];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        if (ct == kb) continue;
#pragma unroll
        for (int sk = 0; sk < 4; ++sk) {
          const double af = Fs[(16 * wv + lc) * GJP_LD + 4 * sk + lr];
          const double bf = Es[(16 * ct + lc) * GJP_LD + 4 * sk + lr];
          acc[ct] = __builtin_amdgcn_mfma_f64_16x16x4f64(af, bf, acc[ct], 0, 0, 0);
        }
      }
      acc[kb] = -f;
    }
  }
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int q = 0; q < 4; ++q) P[(16 * wv + lr + 4 * q) * 64 + 16 * ct + lc] = -acc[ct][q];
  __syncthreads();
  double lg = (tid < 64) ? log(piv[tid]) : 0.0;
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
    else if (V == 1) gj_pivot_old(B, 64, 0, P, logd, status, lds);
    else if (V == 2) gj_pivot_var<1>(B, 64, 0, P, logd, status, lds);
    else gj_pivot_var<2>(B, 64, 0, P, logd, status, lds);
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
  const char* names[4] = {"block-sweep", "scalar-sweep", "block-sweep: sweeps only",
                          "block-sweep: block products only"};
  for (int v = 0; v < 4; ++v) {
    for (int it = 0; it < 2; ++it) {
      const int reps = 2000;
      hipEventRecord(e0, 0);
      if (v == 0) hipLaunchKernelGGL(k_piv_bench<0>, dim3(1), dim3(256), 0, 0, dB, dP, dl, ds, reps);
      else if (v == 1) hipLaunchKernelGGL(k_piv_bench<1>, dim3(1), dim3(256), 0, 0, dB, dP, dl, ds, reps);
      else if (v == 2) hipLaunchKernelGGL(k_piv_bench<2>, dim3(1), dim3(256), 0, 0, dB, dP, dl, ds, reps);
      else hipLaunchKernelGGL(k_piv_bench<3>, dim3(1), dim3(256), 0, 0, dB, dP, dl, ds, reps);
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
