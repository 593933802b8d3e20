// Experiment (no product change): an fp64-accurate split-integer (Ozaki-style) GEMM of the
// contraction's shape on gfx950's int8 MFMA, against native v_mfma_f64 on the same operands.
//
// Operands: C3's contraction C = K12 P (tools: n_s = 32768 sampled rows of K12, m = k = 1024),
// built here from the SURVEY 8(d) C3 recipe -- X, U ~ U(0,10)^8 (xorshift, not numpy's PCG64:
// the statistics matter, not the values), ARD l_c = 3, sigma = 1, tau = 0.5, delta = 1e-6 --
// with P = tau^-2 K22^-1 - z^-1 Bm^-1, Bm = K22 + S/z, S = (1e6 / n_s) K12^T K12 (the n = 1e6
// Gram matrix estimated from the sample), inverses by a host Cholesky.
//
// Split-integer scheme (Ozaki scheme I with integer slices): every row i of A is scaled by
// 2^-(e_i + 1) (max |A_i.| < 2^e_i) and written as S signed 7-bit digits,
//   A_ik = 2^(e_i + 1) sum_t d_t,ik 128^-(t + 1) + O(128^-S),   |d| <= 64 (int8),
// likewise every column j of B with f_j.  The product's level L = t + u terms are one int8 GEMM
// with K' = (L + 1) k (int32-exact: (L + 1) k 64^2 < 2^31 for k = 1024, L < 8), so
//   C_ij = 2^(e_i + f_j + 2) sum_{L < S} 128^-(L + 2) sum_{t + u = L} D^A_t D^B_u,
// S (S + 1) / 2 int8 GEMMs of n m k MACs; levels >= S are dropped (their size is below
// 128^-(S+1) max|A_i.| max|B_.j| k).  Each 128 x 128 output tile keeps its fp64 result in
// registers and folds each level's exact int32 sum in with one power-of-two multiply-add.
//
// Reported: time and TF/s-equivalent (2 n m k / t) of the native fp64 GEMM (a plain MFMA tile
// kernel; the product contraction itself runs at ~67 TF/s) and of the int8 scheme for S = 7..9
// (splits included and separately), and for 128 sampled rows x 1024 columns the error against a
// long-double reference: max |C - C_ref| / sum_k |A_ik| |B_kj| (the normwise bound's unit;
// native fp64 sits near 2^-53 k-scaled) and max |C - C_ref| / max |C_ref|.
//   build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o ozaki ozaki.hip
//   run:   ./ozaki
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                           \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

typedef double d4 __attribute__((ext_vector_type(4)));
typedef int v4i __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ native fp64 GEMM
// C (M x N, row-major ldc) = A B with A(i, k) = A[i * ars + k * acs], B(k, j) = B[k * brs + j];
// 64 x 64 tiles, 4 waves of 32 x 32, BK = 16, LDS-staged (M, N multiples of 64, K of 16).
__global__ void __launch_bounds__(256) k_dgemm(int64_t M, int64_t N, int64_t K, const double* A,
                                               int64_t ars, int64_t acs, const double* B,
                                               int64_t brs, double* C, int64_t ldc) {
  __shared__ double As[64][17];
  __shared__ double Bs[16][66];
  const int64_t i0 = (int64_t)blockIdx.y * 64, j0 = (int64_t)blockIdx.x * 64;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wr = wv >> 1, wc = wv & 1;
  d4 acc[2][2];
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b) acc[a][b] = d4{0, 0, 0, 0};
  for (int64_t k0 = 0; k0 < K; k0 += 16) {
    for (int e = tid; e < 64 * 16; e += 256) {
      const int r = e >> 4, kk = e & 15;
      As[r][kk] = A[(i0 + r) * ars + (k0 + kk) * acs];
      const int kb = e >> 6, c = e & 63;
      Bs[kb][c] = B[(k0 + kb) * brs + j0 + c];
    }
    __syncthreads();
    for (int kk = 0; kk < 4; ++kk) {
      const int kx = kk * 4 + (lane >> 4);
      double af[2], bf[2];
      for (int f = 0; f < 2; ++f) {
        af[f] = As[wr * 32 + f * 16 + (lane & 15)][kx];
        bf[f] = Bs[kx][wc * 32 + f * 16 + (lane & 15)];
      }
      for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[a], bf[b], acc[a][b], 0, 0, 0);
    }
    __syncthreads();
  }
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b)
      for (int q = 0; q < 4; ++q)
        C[(i0 + wr * 32 + a * 16 + (lane >> 4) + 4 * q) * ldc + j0 + wc * 32 + b * 16 +
          (lane & 15)] = acc[a][b][q];
}

// ------------------------------------------------------------------ splitting
// rows of A (n x k, row-major) -> S digit planes D[t][i][k] (int8) and exponents e[i]
// (transpose = true: columns of B (k x m, row-major) -> D[t][j][k], i.e. stored transposed so
// that an MFMA lane reads 16 consecutive k of its column)
__global__ void __launch_bounds__(256) k_split(const double* X, int64_t rows, int64_t len,
                                               int64_t rs, int64_t cs, int S, int8_t* D,
                                               int* ex) {
  __shared__ double red[4];
  const int64_t i = blockIdx.x;
  double mx = 0.0;
  for (int64_t k = threadIdx.x; k < len; k += 256) mx = fmax(mx, fabs(X[i * rs + k * cs]));
  for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
  int e = 0;
  if (mx > 0.0) frexp(mx, &e);   // mx < 2^e
  if (threadIdx.x == 0) ex[i] = e;
  const double sc = ldexp(1.0, -(e + 1));   // |x sc| < 1/2
  for (int64_t k = threadIdx.x; k < len; k += 256) {
    double r = X[i * rs + k * cs] * sc;
    for (int t = 0; t < S; ++t) {
      r *= 128.0;
      const double dv = rint(r);
      r -= dv;
      D[((int64_t)t * rows + i) * len + k] = (int8_t)dv;
    }
  }
}

// ------------------------------------------------------------------ int8 level GEMM
// One 128 x 128 tile of C = A B per workgroup (4 waves, 64 x 64 each as 4 x 4 fragments of
// v_mfma_i32_16x16x64_i8).  For each level L < S: int32 acc = sum_{t <= L} D^A_t D^B_{L-t}
// over k (K step 64, LDS rows padded to 80 bytes: conflict-free ds_read_b128), then
// out += acc * 128^-(L + 2) in fp64; finally C = out * 2^(e_i + f_j + 2).
constexpr int KS = 64;     // k per step (one MFMA depth)
constexpr int LROW = 80;   // LDS row stride (bytes)

__global__ void __launch_bounds__(256) k_ozaki(int64_t n, int64_t m, int64_t k, int S,
                                               const int8_t* DA, const int8_t* DB, const int* ea,
                                               const int* fb, double* C) {
  __shared__ __attribute__((aligned(16))) int8_t As[2][128 * LROW];
  __shared__ __attribute__((aligned(16))) int8_t Bs[2][128 * LROW];
  const int64_t i0 = (int64_t)blockIdx.y * 128, j0 = (int64_t)blockIdx.x * 128;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wr = wv >> 1, wc = wv & 1;
  d4 out[4][4];
  for (int a = 0; a < 4; ++a)
    for (int b = 0; b < 4; ++b) out[a][b] = d4{0, 0, 0, 0};
  // staging: 128 rows x 64 bytes per operand = 512 x 16 B chunks, two per thread
  const int sr0 = tid >> 2, sc0 = (tid & 3) * 16;          // chunk tid and tid + 256
  const int nks = (int)(k / KS);
  for (int L = 0; L < S; ++L) {
    v4i acc[4][4];
    for (int a = 0; a < 4; ++a)
      for (int b = 0; b < 4; ++b) acc[a][b] = v4i{0, 0, 0, 0};
    const int nsteps = (L + 1) * nks;
    v4i ra[2], rb[2];
    auto gload = [&](int s) {
      const int t = s / nks, kk = (s % nks) * KS, u = L - t;
      const int8_t* pa = DA + ((int64_t)t * n + i0) * k + kk;
      const int8_t* pb = DB + ((int64_t)u * m + j0) * k + kk;
      for (int h = 0; h < 2; ++h) {
        const int r = sr0 + 64 * h;
        ra[h] = *reinterpret_cast<const v4i*>(pa + (int64_t)r * k + sc0);
        rb[h] = *reinterpret_cast<const v4i*>(pb + (int64_t)r * k + sc0);
      }
    };
    auto sstore = [&](int buf) {
      for (int h = 0; h < 2; ++h) {
        const int r = sr0 + 64 * h;
        *reinterpret_cast<v4i*>(&As[buf][r * LROW + sc0]) = ra[h];
        *reinterpret_cast<v4i*>(&Bs[buf][r * LROW + sc0]) = rb[h];
      }
    };
    gload(0);
    sstore(0);
    __syncthreads();
    for (int s = 0; s < nsteps; ++s) {
      const int cur = s & 1;
      if (s + 1 < nsteps) gload(s + 1);
      v4i af[4], bf[4];
      for (int f = 0; f < 4; ++f) {
        af[f] = *reinterpret_cast<const v4i*>(
            &As[cur][(wr * 64 + f * 16 + (lane & 15)) * LROW + 16 * (lane >> 4)]);
        bf[f] = *reinterpret_cast<const v4i*>(
            &Bs[cur][(wc * 64 + f * 16 + (lane & 15)) * LROW + 16 * (lane >> 4)]);
      }
      for (int a = 0; a < 4; ++a)
        for (int b = 0; b < 4; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[a], bf[b], acc[a][b], 0, 0, 0);
      if (s + 1 < nsteps) sstore(cur ^ 1);
      __syncthreads();
    }
    const double lsc = ldexp(1.0, -7 * (L + 2));
    for (int a = 0; a < 4; ++a)
      for (int b = 0; b < 4; ++b)
        for (int q = 0; q < 4; ++q) out[a][b][q] = fma((double)acc[a][b][q], lsc, out[a][b][q]);
  }
  for (int a = 0; a < 4; ++a)
    for (int b = 0; b < 4; ++b)
      for (int q = 0; q < 4; ++q) {
        const int64_t i = i0 + wr * 64 + a * 16 + (lane >> 4) * 4 + q;   // C/D map: row
        const int64_t j = j0 + wc * 64 + b * 16 + (lane & 15);            // (l>>4)*4 + q
        C[i * m + j] = ldexp(out[a][b][q], ea[i] + fb[j] + 2);
      }
}

// ------------------------------------------------------------------ host helpers
static uint64_t g_s = 0x9E3779B97F4A7C15ull;
static double urand() {
  g_s ^= g_s >> 12;
  g_s ^= g_s << 25;
  g_s ^= g_s >> 27;
  return (double)((g_s * 2685821657736338717ull) >> 11) * (1.0 / 9007199254740992.0);
}

// in-place SPD inverse (row-major m x m): Cholesky, then inv(L)^T inv(L)
static void spd_inverse(std::vector<double>& A, int m) {
  std::vector<double> L((size_t)m * m, 0.0);
  for (int j = 0; j < m; ++j) {
    double s = A[(size_t)j * m + j];
    for (int p = 0; p < j; ++p) s -= L[(size_t)j * m + p] * L[(size_t)j * m + p];
    if (s <= 0) { fprintf(stderr, "not SPD at %d\n", j); exit(1); }
    const double d = std::sqrt(s);
    L[(size_t)j * m + j] = d;
    for (int i = j + 1; i < m; ++i) {
      double t = A[(size_t)i * m + j];
      for (int p = 0; p < j; ++p) t -= L[(size_t)i * m + p] * L[(size_t)j * m + p];
      L[(size_t)i * m + j] = t / d;
    }
  }
  std::vector<double> Li((size_t)m * m, 0.0);   // inv(L), lower
  for (int j = 0; j < m; ++j) {
    Li[(size_t)j * m + j] = 1.0 / L[(size_t)j * m + j];
    for (int i = j + 1; i < m; ++i) {
      double t = 0.0;
      for (int p = j; p < i; ++p) t += L[(size_t)i * m + p] * Li[(size_t)p * m + j];
      Li[(size_t)i * m + j] = -t / L[(size_t)i * m + i];
    }
  }
  for (int i = 0; i < m; ++i)
    for (int j = 0; j <= i; ++j) {
      double t = 0.0;
      for (int p = i; p < m; ++p) t += Li[(size_t)p * m + i] * Li[(size_t)p * m + j];
      A[(size_t)i * m + j] = A[(size_t)j * m + i] = t;
    }
}

int main() {
  const int64_t n = 32768, m = 1024, k = 1024, d = 8, nsamp = 128;
  const double ell = 3.0, tau = 0.5, delta = 1e-6, z = tau * tau + delta;
  std::vector<double> X(n * d), U(m * d);
  for (auto& v : X) v = 10.0 * urand();
  for (auto& v : U) v = 10.0 * urand();
  std::vector<double> K12(n * m), K22(m * m);
  for (int64_t i = 0; i < n; ++i)
    for (int64_t j = 0; j < m; ++j) {
      double s = 0.0;
      for (int c = 0; c < d; ++c) {
        const double t = (X[i * d + c] - U[j * d + c]) / ell;
        s += t * t;
      }
      K12[i * m + j] = std::exp(-0.5 * s);
    }
  for (int64_t i = 0; i < m; ++i)
    for (int64_t j = 0; j < m; ++j) {
      double s = 0.0;
      for (int c = 0; c < d; ++c) {
        const double t = (U[i * d + c] - U[j * d + c]) / ell;
        s += t * t;
      }
      K22[i * m + j] = std::exp(-0.5 * s) + (i == j ? delta : 0.0);
    }
  double *dK, *dP, *dS, *dC, *dCo;
  CHK(hipMalloc(&dK, sizeof(double) * n * m));
  CHK(hipMalloc(&dP, sizeof(double) * m * m));
  CHK(hipMalloc(&dS, sizeof(double) * m * m));
  CHK(hipMalloc(&dC, sizeof(double) * n * m));
  CHK(hipMalloc(&dCo, sizeof(double) * n * m));
  CHK(hipMemcpy(dK, K12.data(), sizeof(double) * n * m, hipMemcpyHostToDevice));
  // S = K^T K over the sample, scaled to n = 1e6 rows
  hipLaunchKernelGGL(k_dgemm, dim3(m / 64, m / 64), dim3(256), 0, 0, m, m, n, dK, (int64_t)1, m,
                     dK, m, dS, m);
  CHK(hipDeviceSynchronize());
  std::vector<double> S(m * m);
  CHK(hipMemcpy(S.data(), dS, sizeof(double) * m * m, hipMemcpyDeviceToHost));
  std::vector<double> K22i = K22, Bi(m * m);
  for (int64_t e = 0; e < m * m; ++e) Bi[e] = K22[e] + S[e] * (1e6 / (double)n) / z;
  spd_inverse(K22i, (int)m);
  spd_inverse(Bi, (int)m);
  std::vector<double> P(m * m);
  for (int64_t e = 0; e < m * m; ++e) P[e] = K22i[e] / (tau * tau) - Bi[e] / z;
  CHK(hipMemcpy(dP, P.data(), sizeof(double) * m * m, hipMemcpyHostToDevice));

  // long-double reference on sampled rows
  std::vector<int64_t> rows(nsamp);
  for (int64_t s = 0; s < nsamp; ++s) rows[s] = (s * (n / nsamp) + 7 * s) % n;
  std::vector<long double> ref(nsamp * m), bnd(nsamp * m);
  for (int64_t s = 0; s < nsamp; ++s)
    for (int64_t j = 0; j < m; ++j) {
      long double a = 0.0L, b = 0.0L;
      for (int64_t q = 0; q < k; ++q) {
        const long double x = K12[rows[s] * m + q], y = P[q * m + j];
        a += x * y;
        b += std::fabs(x * y);
      }
      ref[s * m + j] = a;
      bnd[s * m + j] = b;
    }
  long double refmax = 0.0L;
  for (auto v : ref) refmax = std::max(refmax, std::fabs(v));
  auto errors = [&](const double* dev, double* e_norm, double* e_max) {
    std::vector<double> row(m);
    long double en = 0.0L, em = 0.0L;
    for (int64_t s = 0; s < nsamp; ++s) {
      CHK(hipMemcpy(row.data(), dev + rows[s] * m, sizeof(double) * m, hipMemcpyDeviceToHost));
      for (int64_t j = 0; j < m; ++j) {
        const long double diff = std::fabs((long double)row[j] - ref[s * m + j]);
        en = std::max(en, diff / bnd[s * m + j]);
        em = std::max(em, diff);
      }
    }
    *e_norm = (double)en;
    *e_max = (double)(em / refmax);
  };
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const double flops = 2.0 * n * m * k;
  // native fp64
  float ms = 0.f;
  for (int rep = 0; rep < 2; ++rep) {
    CHK(hipEventRecord(e0));
    for (int it = 0; it < 5; ++it)
      hipLaunchKernelGGL(k_dgemm, dim3(m / 64, n / 64), dim3(256), 0, 0, n, m, k, dK, m,
                         (int64_t)1, dP, m, dC, m);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    CHK(hipEventElapsedTime(&ms, e0, e1));
  }
  double en, em;
  errors(dC, &en, &em);
  printf("native fp64 (plain MFMA tile kernel): %.3f ms = %.1f TF/s; err/bound %.3e, "
         "err/max|C| %.3e\n", ms / 5, flops / (ms / 5 * 1e-3) / 1e12, en, em);
  // split-integer
  for (int S = 6; S <= 9; ++S) {
    int8_t *DA, *DB;
    int *ea, *fb;
    CHK(hipMalloc(&DA, (size_t)S * n * k));
    CHK(hipMalloc(&DB, (size_t)S * m * k));
    CHK(hipMalloc(&ea, sizeof(int) * n));
    CHK(hipMalloc(&fb, sizeof(int) * m));
    float ms_split = 0.f, ms_gemm = 0.f;
    for (int rep = 0; rep < 2; ++rep) {
      CHK(hipEventRecord(e0));
      hipLaunchKernelGGL(k_split, dim3(n), dim3(256), 0, 0, dK, n, k, m, (int64_t)1, S, DA, ea);
      hipLaunchKernelGGL(k_split, dim3(m), dim3(256), 0, 0, dP, m, k, (int64_t)1, m, S, DB, fb);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      CHK(hipEventElapsedTime(&ms_split, e0, e1));
      CHK(hipEventRecord(e0));
      for (int it = 0; it < 3; ++it)
        hipLaunchKernelGGL(k_ozaki, dim3(m / 128, n / 128), dim3(256), 0, 0, n, m, k, S, DA, DB,
                           ea, fb, dCo);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      CHK(hipEventElapsedTime(&ms_gemm, e0, e1));
      ms_gemm /= 3;
    }
    CHK(hipGetLastError());
    errors(dCo, &en, &em);
    const double t_all = (ms_gemm + ms_split) * 1e-3;
    printf("int8 split S=%d (%d int8 GEMMs): gemm %.3f ms + splits %.3f ms = %.1f TF/s-equiv "
           "(gemm alone %.1f, int8 %.0f TOP/s); err/bound %.3e, err/max|C| %.3e\n",
           S, S * (S + 1) / 2, ms_gemm, ms_split, flops / t_all / 1e12,
           flops / (ms_gemm * 1e-3) / 1e12, flops * S * (S + 1) / 2 / (ms_gemm * 1e-3) / 1e12,
           en, em);
    CHK(hipFree(DA));
    CHK(hipFree(DB));
    CHK(hipFree(ea));
    CHK(hipFree(fb));
  }
  return 0;
}
