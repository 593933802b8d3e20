// Round 5: the 16 scalar sweeps of a 16x16 SPD diagonal block (the serial core of the
// Gauss-Jordan pivot, k_dense.hip gj_pivot_body) in two register layouts, one wave, timed over
// many repetitions (the block L2-resident):
//   cur: lane (lr, lc) holds rows lr + 4q of column lc (MFMA accumulator layout); row k by
//        ds_bpermute, column k by DPP row_newbcast, the pivot by readlane (k_dense.hip today);
//   col: every 16-lane row holds the whole block, lane c column c (16 registers); a sweep is one
//        v_fmac_f64_dpp per element (src0 = lane k's register by row_newbcast), the pivot lane's
//        column kept unscaled with a pending factor (applied once after the 16 sweeps).
//   pipe: cur pipelined one sweep ahead (measured, not kept);
//   dpp: cur with one DPP64 v_fmac_f64_dpp per register instead of DPP moves and selects;
//   pair: dpp with the sweeps taken two at a time (2x2 block pivots, k_dense.hip gj_sweep2_dpp);
//   build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form -o gj_sweep gj_sweep.hip
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "../../sparsergps_amd/csrc/k_dense.hip"

namespace {
#include "gj_fmac_bcast.inc"

// the current sweep (gj_pivot_body's wave-kb loop), on a tile in accumulator layout
__device__ __forceinline__ void sweep_cur(d4& t, double (&dk)[16]) {
  const int lane = threadIdx.x & 63, lr = lane >> 4, lc = lane & 15;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int kq = k >> 2, kr = k & 3;
    const double vc = __shfl(t[kq], lc + 16 * kr, 64);
    const double d = readlane_f64(t[kq], k + 16 * kr);
    double vr[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) vr[q] = row_bcast_f64(t[q], k);
    const double r = rcp_nr(d);
    dk[k] = d;
    const double vj = (lc == k) ? -1.0 : vc;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = lr + 4 * q;
      const double vi = (i == k) ? -r : vr[q] * r;
      const double base = (i == k || lc == k) ? 0.0 : t[q];
      t[q] = fma(-vi, vj, base);
    }
  }
}

// round 5, second form (k_dense.hip today): pipelined one sweep ahead -- the next pivot and
// row k+1 from their pre-sweep values with sweep k's own arithmetic
__device__ __forceinline__ void sweep_pipe(d4& t, double (&dk)[16]) {
  const int lane = threadIdx.x & 63, lr = lane >> 4, lc = lane & 15;
  double vc = __shfl(t[0], lc, 64);
  double d = readlane_f64(t[0], 0);
  double r = rcp_nr(d);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int kq = k >> 2, kr = k & 3;
    const int k1 = k + 1 < 16 ? k + 1 : 15, k1q = k1 >> 2, k1r = k1 & 3;
    dk[k] = d;
    const double wnext = __shfl(t[k1q], lc + 16 * k1r, 64);
    const double a = readlane_f64(t[k1q], k + 16 * k1r);
    const double b = readlane_f64(t[kq], k1 + 16 * kr);
    const double cdg = readlane_f64(t[k1q], k1 + 16 * k1r);
    double vr[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) vr[q] = row_bcast_f64(t[q], k);
    const double vj = (lc == k) ? -1.0 : vc;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = lr + 4 * q;
      const double vi = (i == k) ? -r : vr[q] * r;
      const double base = (i == k || lc == k) ? 0.0 : t[q];
      t[q] = fma(-vi, vj, base);
    }
    if (k + 1 < 16) {
      const double ar = a * r;
      d = fma(-ar, b, cdg);
      vc = (lc == k) ? ar : fma(-ar, vc, wnext);
      r = rcp_nr(d);
    }
  }
}

// dpp: the accumulator layout with one DPP64 v_fmac_f64_dpp per register (W_iK read from lane K
// of the row, nvj = -r W_Kj per lane, r - 1 on column K), row K set apart afterwards
template <int K>
__device__ __forceinline__ void sweep_dpp_step(d4& t, double (&dk)[16], int lr, int lc) {
  constexpr int kq = K >> 2, kr = K & 3;
  const double vc = __shfl(t[kq], lc + 16 * kr, 64);
  const double d = readlane_f64(t[kq], K + 16 * kr);
  const double r = rcp_nr(d);
  dk[K] = d;
  const double rowk = t[kq];
  const double nvj = (lc == K) ? r - 1.0 : -(r * vc);
  double a0 = t[0], a1 = t[1], a2 = t[2], a3 = t[3];
  asm volatile("s_nop 1\n"
               "v_fmac_f64_dpp %0, %0, %4 row_newbcast:%5 row_mask:0xf bank_mask:0xf\n"
               "v_fmac_f64_dpp %1, %1, %4 row_newbcast:%5 row_mask:0xf bank_mask:0xf\n"
               "v_fmac_f64_dpp %2, %2, %4 row_newbcast:%5 row_mask:0xf bank_mask:0xf\n"
               "v_fmac_f64_dpp %3, %3, %4 row_newbcast:%5 row_mask:0xf bank_mask:0xf\n"
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)
               : "v"(nvj), "i"(K));
  t[0] = a0; t[1] = a1; t[2] = a2; t[3] = a3;
  const double rk = (lc == K) ? -r : r * rowk;
  t[kq] = (lr == kr) ? rk : t[kq];
}

__device__ __forceinline__ void sweep_dpp(d4& t, double (&dk)[16]) {
  const int lane = threadIdx.x & 63, lr = lane >> 4, lc = lane & 15;
  sweep_dpp_step<0>(t, dk, lr, lc);   sweep_dpp_step<1>(t, dk, lr, lc);
  sweep_dpp_step<2>(t, dk, lr, lc);   sweep_dpp_step<3>(t, dk, lr, lc);
  sweep_dpp_step<4>(t, dk, lr, lc);   sweep_dpp_step<5>(t, dk, lr, lc);
  sweep_dpp_step<6>(t, dk, lr, lc);   sweep_dpp_step<7>(t, dk, lr, lc);
  sweep_dpp_step<8>(t, dk, lr, lc);   sweep_dpp_step<9>(t, dk, lr, lc);
  sweep_dpp_step<10>(t, dk, lr, lc);  sweep_dpp_step<11>(t, dk, lr, lc);
  sweep_dpp_step<12>(t, dk, lr, lc);  sweep_dpp_step<13>(t, dk, lr, lc);
  sweep_dpp_step<14>(t, dk, lr, lc);  sweep_dpp_step<15>(t, dk, lr, lc);
}

template <int K>
__device__ __forceinline__ void sweep_col_step(double (&R)[16], double (&dk)[16], double& sig,
                                               int c) {
  const double d = row_bcast_f64<K>(R[K]);
  dk[K] = d;
  const double r = rcp_nr(d);
  const bool piv = c == K;
  const double f = piv ? 0.0 : R[K] * r;
  fmac_bcast<K>(R, -f);
  R[K] = piv ? -1.0 : f;
  sig = piv ? r : sig;
}

__device__ __forceinline__ void sweep_col(double (&R)[16], double (&dk)[16]) {
  const int c = threadIdx.x & 15;
  double sig = 1.0;
  sweep_col_step<0>(R, dk, sig, c);   sweep_col_step<1>(R, dk, sig, c);
  sweep_col_step<2>(R, dk, sig, c);   sweep_col_step<3>(R, dk, sig, c);
  sweep_col_step<4>(R, dk, sig, c);   sweep_col_step<5>(R, dk, sig, c);
  sweep_col_step<6>(R, dk, sig, c);   sweep_col_step<7>(R, dk, sig, c);
  sweep_col_step<8>(R, dk, sig, c);   sweep_col_step<9>(R, dk, sig, c);
  sweep_col_step<10>(R, dk, sig, c);  sweep_col_step<11>(R, dk, sig, c);
  sweep_col_step<12>(R, dk, sig, c);  sweep_col_step<13>(R, dk, sig, c);
  sweep_col_step<14>(R, dk, sig, c);  sweep_col_step<15>(R, dk, sig, c);
#pragma unroll
  for (int i = 0; i < 16; ++i) R[i] *= sig;
}

// Sweeps K and K + 1 (K even) as one 2x2 block sweep: Q = inv(W_SS) for S = {K, K + 1} from the
// four pivot-block values (one reciprocal on the dependency chain instead of two, and no second
// cross-lane fetch of an updated row), then W_RR -= W_RS Q W_SR as two DPP64 fmacs per register:
// t += W_iK g_j (g on column K + 1 = Q01, so the second fmac's broadcast source becomes
// W_i,K+1 + Q01 W_iK) and t += (W_i,K+1 + Q01 W_iK) h_j, with h_j = -(Q10 W_Kj + Q11 W_K+1,j)
// and g_j = -(Q00 W_Kj + Q01 W_K+1,j) - Q01 h_j (both 0 on the pivot columns but g's K + 1).
// The pivot columns then get W_RS Q from their quad neighbour (DPP quad_perm swap), the pivot
// rows Q W_SR and -Q.  Rows K, K + 1 sit in one register (lane rows kr, kr + 1).  The pivots
// recorded are the sequential sweep's: d_K = W_KK and d_K+1 = det / W_KK.
// Measured: 1.90 against 1.10 us per 16 sweeps -- one wave's sweeps are bound by VALU issue, not by
// the dependency chain, and the pair issues more than two single sweeps (not kept).
template <int K>
__device__ __forceinline__ void gj_sweep2_dpp(d4& t, double (&dk)[16], int lr, int lc) {
  static_assert((K & 1) == 0, "pairs start on even pivots");
  constexpr int kq = K >> 2, kr = K & 3;
  const double v0 = __shfl(t[kq], lc + 16 * kr, 64);          // W_K,lc
  const double v1 = __shfl(t[kq], lc + 16 * (kr + 1), 64);    // W_K+1,lc
  const double a = readlane_f64(t[kq], K + 16 * kr);
  const double b = readlane_f64(t[kq], K + 1 + 16 * kr);
  const double b2 = readlane_f64(t[kq], K + 16 * (kr + 1));
  const double c = readlane_f64(t[kq], K + 1 + 16 * (kr + 1));
  const double det = fma(a, c, -(b * b2));
  const double rd = rcp_nr(det);
  const double q00 = c * rd, q01 = -b * rd, q10 = -b2 * rd, q11 = a * rd;
  dk[K] = a;
  dk[K + 1] = det;   // the caller turns it into det / W_KK after the sweeps (off the chain)
  const bool p0 = lc == K, p1 = lc == K + 1;
  const double h = (p0 || p1) ? 0.0 : -fma(q10, v0, q11 * v1);
  const double g = p1 ? q01 : p0 ? 0.0 : fma(-q01, h, -fma(q00, v0, q01 * v1));
  double a0 = t[0], a1 = t[1], a2 = t[2], a3 = t[3];
  asm volatile("s_nop 1\n"
               "v_fmac_f64_dpp %0, %0, %4 row_newbcast:%6 row_mask:0xf bank_mask:0xf\n"
               "v_fmac_f64_dpp %1, %1, %4 row_newbcast:%6 row_mask:0xf bank_mask:0xf\n"
               "v_fmac_f64_dpp %2, %2, %4 row_newbcast:%6 row_mask:0xf bank_mask:0xf\n"
               "v_fmac_f64_dpp %3, %3, %4 row_newbcast:%6 row_mask:0xf bank_mask:0xf\n"
               "s_nop 1\n"
               "v_fmac_f64_dpp %0, %0, %5 row_newbcast:%7 row_mask:0xf bank_mask:0xf\n"
               "v_fmac_f64_dpp %1, %1, %5 row_newbcast:%7 row_mask:0xf bank_mask:0xf\n"
               "v_fmac_f64_dpp %2, %2, %5 row_newbcast:%7 row_mask:0xf bank_mask:0xf\n"
               "v_fmac_f64_dpp %3, %3, %5 row_newbcast:%7 row_mask:0xf bank_mask:0xf\n"
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)
               : "v"(g), "v"(h), "i"(K), "i"(K + 1));
  // pivot columns: lane K holds W_iK, lane K + 1 holds W_i,K+1 + Q01 W_iK
  const double cA = p0 ? fma(-q10, q01, q00) : p1 ? q11 : 1.0;
  const double cB = p0 ? q10 : p1 ? q01 * (1.0 - q11) : 0.0;
  // t = cA t + cB t[quad neighbour] (DPP64 ALU ops take only row_newbcast: the swap is two
  // 32-bit DPP moves, quad_perm [1,0,3,2])
  const double r[4] = {a0, a1, a2, a3};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const long long bits = __double_as_longlong(r[q]);
    const int lo = __builtin_amdgcn_mov_dpp((int)bits, 0xB1, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(bits >> 32), 0xB1, 0xF, 0xF, false);
    const double nb = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
    t[q] = fma(cB, nb, cA * r[q]);
  }
  // pivot rows: Q W_SR off the pivot columns, -Q on them
  const double rK = p0 ? -q00 : p1 ? -q01 : fma(q00, v0, q01 * v1);
  const double rK1 = p0 ? -q10 : p1 ? -q11 : fma(q10, v0, q11 * v1);
  t[kq] = (lr == kr) ? rK : (lr == kr + 1) ? rK1 : t[kq];
}
__device__ __forceinline__ void gj_sweeps16_pair(d4& t, double (&dk)[16], int lr, int lc) {
  gj_sweep2_dpp<0>(t, dk, lr, lc);   gj_sweep2_dpp<2>(t, dk, lr, lc);
  gj_sweep2_dpp<4>(t, dk, lr, lc);   gj_sweep2_dpp<6>(t, dk, lr, lc);
  gj_sweep2_dpp<8>(t, dk, lr, lc);   gj_sweep2_dpp<10>(t, dk, lr, lc);
  gj_sweep2_dpp<12>(t, dk, lr, lc);  gj_sweep2_dpp<14>(t, dk, lr, lc);
}
// B: 16 x 16 row-major; out: the swept block (-inv(B)); piv: the 16 pivots
__global__ void __launch_bounds__(64) k_cur(const double* B, double* out, double* piv, int reps) {
  const int lane = threadIdx.x, lr = lane >> 4, lc = lane & 15;
  double dk[16];
  d4 t;
  for (int r = 0; r < reps; ++r) {
#pragma unroll
    for (int q = 0; q < 4; ++q) t[q] = B[(lr + 4 * q) * 16 + lc];
    sweep_cur(t, dk);
#pragma unroll
    for (int q = 0; q < 4; ++q) out[(lr + 4 * q) * 16 + lc] = t[q];
  }
  if (lane < 16) {
    double v = dk[0];
#pragma unroll
    for (int k = 1; k < 16; ++k) v = (lane == k) ? dk[k] : v;
    piv[lane] = v;
  }
}

__global__ void __launch_bounds__(64) k_pipe(const double* B, double* out, double* piv, int reps) {
  const int lane = threadIdx.x, lr = lane >> 4, lc = lane & 15;
  double dk[16];
  d4 t;
  for (int r = 0; r < reps; ++r) {
#pragma unroll
    for (int q = 0; q < 4; ++q) t[q] = B[(lr + 4 * q) * 16 + lc];
    sweep_pipe(t, dk);
#pragma unroll
    for (int q = 0; q < 4; ++q) out[(lr + 4 * q) * 16 + lc] = t[q];
  }
  if (lane < 16) {
    double v = dk[0];
#pragma unroll
    for (int k = 1; k < 16; ++k) v = (lane == k) ? dk[k] : v;
    piv[lane] = v;
  }
}

__global__ void __launch_bounds__(64) k_dpp(const double* B, double* out, double* piv, int reps) {
  const int lane = threadIdx.x, lr = lane >> 4, lc = lane & 15;
  double dk[16];
  d4 t;
  for (int r = 0; r < reps; ++r) {
#pragma unroll
    for (int q = 0; q < 4; ++q) t[q] = B[(lr + 4 * q) * 16 + lc];
    sweep_dpp(t, dk);
#pragma unroll
    for (int q = 0; q < 4; ++q) out[(lr + 4 * q) * 16 + lc] = t[q];
  }
  if (lane < 16) {
    double v = dk[0];
#pragma unroll
    for (int k = 1; k < 16; ++k) v = (lane == k) ? dk[k] : v;
    piv[lane] = v;
  }
}

__global__ void __launch_bounds__(64) k_pair(const double* B, double* out, double* piv, int reps) {
  const int lane = threadIdx.x, lr = lane >> 4, lc = lane & 15;
  double dk[16];
  d4 t;
  for (int r = 0; r < reps; ++r) {
#pragma unroll
    for (int q = 0; q < 4; ++q) t[q] = B[(lr + 4 * q) * 16 + lc];
    gj_sweeps16_pair(t, dk, lr, lc);
#pragma unroll
    for (int k = 1; k < 16; k += 2) dk[k] = dk[k] * rcp_nr(dk[k - 1]);
#pragma unroll
    for (int q = 0; q < 4; ++q) out[(lr + 4 * q) * 16 + lc] = t[q];
  }
  if (lane < 16) {
    double v = dk[0];
#pragma unroll
    for (int k = 1; k < 16; ++k) v = (lane == k) ? dk[k] : v;
    piv[lane] = v;
  }
}

__global__ void __launch_bounds__(64) k_col(const double* B, double* out, double* piv, int reps) {
  const int lane = threadIdx.x, g = lane >> 4, c = lane & 15;
  double dk[16], R[16];
  for (int r = 0; r < reps; ++r) {
#pragma unroll
    for (int i = 0; i < 16; ++i) R[i] = B[i * 16 + c];
    sweep_col(R, dk);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      // row group g writes rows 4g .. 4g + 3 (static register indices via a select chain)
      const double v = g == 0 ? R[q] : g == 1 ? R[4 + q] : g == 2 ? R[8 + q] : R[12 + q];
      out[(4 * g + q) * 16 + c] = v;
    }
  }
  if (lane < 16) {
    double v = dk[0];
#pragma unroll
    for (int k = 1; k < 16; ++k) v = (lane == k) ? dk[k] : v;
    piv[lane] = v;
  }
}
}  // namespace

int main() {
  std::mt19937_64 gen(5);
  std::normal_distribution<double> N01;
  std::vector<double> G(16 * 16), B(16 * 16, 0.0), O(16 * 16), pv(16);
  for (auto& v : G) v = N01(gen);
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double s = 0;
      for (int k = 0; k < 16; ++k) s += G[i * 16 + k] * G[j * 16 + k];
      B[i * 16 + j] = s / 16 + (i == j ? 0.5 : 0.0) + (i == j ? 3e3 * (i % 3) : 0.0);
    }
  double *dB, *dO, *dP;
  hipMalloc(&dB, 16 * 16 * 8); hipMalloc(&dO, 16 * 16 * 8); hipMalloc(&dP, 16 * 8);
  hipMemcpy(dB, B.data(), 16 * 16 * 8, hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const char* names[5] = {"cur (accumulator layout)", "col (v_fmac_f64_dpp)", "pipe (one sweep ahead)",
                          "dpp (DPP64 fmac, acc layout)", "pair (2x2 block sweeps)"};
  std::vector<double> O0(16 * 16), P0(16);
  for (int it = 0; it < 3; ++it)
    for (int v = 0; v < 5; ++v) {
      const int reps = 20000;
      hipEventRecord(e0, 0);
      if (v == 0) hipLaunchKernelGGL(k_cur, dim3(1), dim3(64), 0, 0, dB, dO, dP, reps);
      else if (v == 1) hipLaunchKernelGGL(k_col, dim3(1), dim3(64), 0, 0, dB, dO, dP, reps);
      else if (v == 2) hipLaunchKernelGGL(k_pipe, dim3(1), dim3(64), 0, 0, dB, dO, dP, reps);
      else if (v == 3) hipLaunchKernelGGL(k_dpp, dim3(1), dim3(64), 0, 0, dB, dO, dP, reps);
      else hipLaunchKernelGGL(k_pair, dim3(1), dim3(64), 0, 0, dB, dO, dP, reps);
      hipEventRecord(e1, 0); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      hipMemcpy(O.data(), dO, 16 * 16 * 8, hipMemcpyDeviceToHost);
      hipMemcpy(pv.data(), dP, 16 * 8, hipMemcpyDeviceToHost);
      double err = 0, ld = 0;   // || B (-O) - I ||_max
      for (int i = 0; i < 16; ++i) {
        ld += log(pv[i]);
        for (int j = 0; j < 16; ++j) {
          double s = 0;
          for (int k = 0; k < 16; ++k) s -= B[i * 16 + k] * O[k * 16 + j];
          err = fmax(err, fabs(s - (i == j ? 1.0 : 0.0)));
        }
      }
      if (v == 0) { O0 = O; P0 = pv; }
      const bool same = v == 1 || v >= 3 || (O == O0 && pv == P0);
      printf("%-26s %7.3f us per 16 sweeps (%6.1f ns/sweep)  |B inv - I| %.2e  sum log piv %.15f%s\n",
             names[v], ms * 1e3 / reps, ms * 1e6 / reps / 16, err, ld,
             v == 2 ? (same ? "  bit-identical to cur" : "  DIFFERS from cur") : "");
    }
  return 0;
}
